#!/usr/bin/env python3
"""One conv GEMM (CaffeNet conv3 forward: M=43264, N=384, K=2304) launched 10x per tile in
TILES (env, comma list; SN GEMM tile ids) for rocprofv3 --pmc A/B of mainloop variants."""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

from sparknet_amd.ops import _lib, gemm, hip  # noqa: E402
from sparknet_amd.ops.spec import ConvSpec  # noqa: E402

_lib.kernels()
s = ConvSpec(256, 13, 13, 256, 384, 3, 3, 1, 1, 1, 1)
x = (torch.rand(s.N, s.H, s.W, s.C, device="cuda") * 2 - 1).to(torch.bfloat16)
w = ((torch.rand(s.K, s.R, s.S, s.Cg, device="cuda") * 2 - 1) * 0.05).to(torch.bfloat16)
for t in [int(v) for v in os.environ.get("TILES", "0,13,30,39").split(",")]:
    gemm._FORCE_TILE = t
    for _ in range(10):
        hip.conv_forward(x, w, None, s)
    torch.cuda.synchronize()
# WGRAD_TILES: the weight gradient of the same conv (MC dense dy x MC implicit im2col of x,
# split-K slabs + reduce), 10x per tile
dy = (torch.rand(s.N, s.P, s.Q, s.K, device="cuda") * 2 - 1).to(torch.bfloat16)
dw = torch.zeros(s.K, s.R, s.S, s.Cg, device="cuda")
for t in [int(v) for v in os.environ.get("WGRAD_TILES", "").split(",") if v]:
    gemm._FORCE_TILE = t
    for _ in range(10):
        hip.conv_backward(dy, x, w, s, False, dw, None)
    torch.cuda.synchronize()
print("done")
