#!/usr/bin/env python3
"""One GEMM case for rocprofv3 --pmc: CaffeNet conv3 forward (M=43264, N=384, K=2304) or
its weight gradient, 20 launches (CASE=fwd|wgrad)."""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

from sparknet_amd.ops import _lib, hip  # noqa: E402
from sparknet_amd.ops.spec import ConvSpec  # noqa: E402

_lib.kernels()
s = ConvSpec(256, 13, 13, 256, 384, 3, 3, 1, 1, 1, 1)
x = torch.randn(s.N, s.H, s.W, s.C, device="cuda").to(torch.bfloat16)
w = (torch.randn(s.K, s.R, s.S, s.Cg, device="cuda") * 0.05).to(torch.bfloat16)
dy = torch.randn(s.N, s.P, s.Q, s.K, device="cuda").to(torch.bfloat16)
dw = torch.zeros(s.K, s.R, s.S, s.Cg, device="cuda")
case = os.environ.get("CASE", "fwd")
fn = (lambda: hip.conv_forward(x, w, None, s)) if case == "fwd" else (lambda: hip.conv_backward(dy, x, w, s, False, dw, None))
for _ in range(20):
    fn()
torch.cuda.synchronize()
print("done", case)
