#!/usr/bin/env python3
"""A/B of GEMM tiles on dense NT products and CaffeNet-shaped implicit convs, interleaved
in one process (median of reps).  python scripts/tile_probe.py [tiles...]"""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

from sparknet_amd.ops import _lib, gemm as G, hip  # noqa: E402
from sparknet_amd.ops.spec import ConvSpec  # noqa: E402

_lib.kernels()
tiles = [int(t) for t in sys.argv[1:]] or [0, 2, 6, 7]


def med(fn, reps=15):
    for _ in range(3):
        fn()
    torch.cuda.synchronize()
    ts = []
    for _ in range(reps):
        a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        a.record()
        fn()
        b.record()
        b.synchronize()
        ts.append(a.elapsed_time(b))
    ts.sort()
    return ts[len(ts) // 2]


cases = []
for n in (4096, 8192):
    a = (torch.rand(n, n, device="cuda") * 2 - 1).to(torch.bfloat16)
    b = (torch.rand(n, n, device="cuda") * 2 - 1).to(torch.bfloat16)
    c = torch.empty(n, n, device="cuda", dtype=torch.bfloat16)
    cases.append((f"NT {n}^3", 2.0 * n ** 3, lambda a=a, b=b, c=c: G.linear_fwd(a, b, out=c)))
for name, (N, H, W, Cc, K, R, S, st, pd, g) in {
        "conv2 fwd": (256, 27, 27, 96, 256, 5, 5, 1, 2, 2), "conv3 fwd": (256, 13, 13, 256, 384, 3, 3, 1, 1, 1),
        "conv4 fwd": (256, 13, 13, 384, 384, 3, 3, 1, 1, 2), "conv5 fwd": (256, 13, 13, 384, 256, 3, 3, 1, 1, 2),
        "vgg conv3_2": (64, 56, 56, 256, 256, 3, 3, 1, 1, 1), "vgg conv4_2": (64, 28, 28, 512, 512, 3, 3, 1, 1, 1)}.items():
    s = ConvSpec(N, H, W, Cc, K, R, S, st, st, pd, pd, 1, 1, g)
    x = (torch.randn(N, H, W, Cc, device="cuda")).to(torch.bfloat16)
    w = (torch.randn(K, R, S, Cc // g, device="cuda") * 0.05).to(torch.bfloat16)
    fl = 2.0 * N * s.P * s.Q * K * R * S * Cc // g
    cases.append((name, fl, lambda x=x, w=w, s=s: hip.conv_forward(x, w, None, s)))
    dy = torch.randn(N, s.P, s.Q, K, device="cuda").to(torch.bfloat16)
    dw = torch.zeros(K, R, S, Cc // g, device="cuda")
    cases.append((name.replace("fwd", "") + " wgrad", fl, lambda x=x, w=w, s=s, dy=dy, dw=dw:
                  hip.conv_backward(dy, x, w, s, False, dw, None)))
for name, fl, fn in cases:
    res = []
    for t in tiles:
        G._FORCE_TILE = t
        try:
            ms = med(fn)
            res.append(f"t{t}:{fl / ms / 1e9:7.1f}")
        except Exception as e:  # noqa: BLE001
            res.append(f"t{t}:  n/a ({str(e)[:30]})")
    G._FORCE_TILE = -1
    ms = med(fn)
    res.append(f"auto:{fl / ms / 1e9:7.1f}")
    print(f"{name:18s} TF/s " + "  ".join(res), flush=True)
