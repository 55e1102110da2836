#!/usr/bin/env python3
"""Input-conv (space-to-depth folded) GEMM throughput per tile: GoogLeNet conv1/7x7_s2
(batch 128) and CaffeNet conv1 (batch 256), forward and weight gradient."""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

from scripts.tile_probe import med  # noqa: E402
from sparknet_amd.ops import gemm as G, hip  # noqa: E402
from sparknet_amd.ops.spec import ConvSpec  # noqa: E402

for name, s in {"googlenet conv1": ConvSpec(128, 224, 224, 3, 64, 7, 7, 2, 2, 3, 3),
                "caffenet conv1": ConvSpec(256, 227, 227, 3, 96, 11, 11, 4, 4, 0, 0)}.items():
    x = torch.randn(s.N, s.H, s.W, s.C, device="cuda").to(torch.bfloat16)
    w = (torch.randn(s.K, s.R, s.S, s.C, device="cuda") * 0.05).to(torch.bfloat16)
    dy = torch.randn(s.N, s.P, s.Q, s.K, device="cuda").to(torch.bfloat16)
    dw = torch.zeros(s.K, s.R, s.S, s.C, device="cuda")
    plan = hip.s2d_plan(s)
    x2 = hip._s2d_input(x, s, plan)
    s2 = plan[4]
    w2 = torch.randn(s2.K, s2.R, s2.S, s2.C, device="cuda").to(torch.bfloat16)
    fl = 2.0 * s.N * s.P * s.Q * s.K * s2.R * s2.S * s2.C
    for t in (0, 1, 2, 4, 5, 7):
        G._FORCE_TILE = t
        try:
            ms = med(lambda: hip.conv_forward(x2, w2, None, s2))
            msw = med(lambda: hip.conv_backward(dy, x, w, s, False, dw, None))
            print(f"{name} tile {t}: fwd {ms * 1e3:7.1f} us ({fl / ms / 1e9:6.1f} TF/s)  wgrad {msw * 1e3:7.1f} us",
                  flush=True)
        except Exception as e:  # noqa: BLE001
            print(f"{name} tile {t}: n/a {str(e)[:60]}", flush=True)
    G._FORCE_TILE = -1
