#!/usr/bin/env python3
"""Run a few GEMM layouts back to back (for rocprofv3 --pmc): dense 4096^3 NT (KC/KC),
NN (KC/MC), TN (MC/MC), and CaffeNet conv3 fwd / wgrad / dgrad, 5 launches each."""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

from sparknet_amd.ops import _lib, gemm, hip  # noqa: E402
from sparknet_amd.ops.spec import ConvSpec  # noqa: E402

_lib.kernels()
dev = "cuda"
n = 4096
a = torch.randn(n, n, device=dev).to(torch.bfloat16)
b = torch.randn(n, n, device=dev).to(torch.bfloat16)
c = torch.empty(n, n, device=dev, dtype=torch.bfloat16)
dw = torch.zeros(n, n, device=dev)
s = ConvSpec(256, 13, 13, 256, 384, 3, 3, 1, 1, 1, 1)
x = torch.randn(s.N, s.H, s.W, s.C, device=dev).to(torch.bfloat16)
w = (torch.randn(s.K, s.R, s.S, s.Cg, device=dev) * 0.05).to(torch.bfloat16)
dy = torch.randn(s.N, s.P, s.Q, s.K, device=dev).to(torch.bfloat16)
cdw = torch.zeros(s.K, s.R, s.S, s.Cg, device=dev)
cases = [("NT", lambda: gemm.linear_fwd(a, b, out=c)), ("NN", lambda: gemm.linear_dgrad(a, b)),
         ("TN", lambda: gemm.linear_wgrad(a, b, dw)), ("conv3_fwd", lambda: hip.conv_forward(x, w, None, s)),
         ("conv3_wgrad", lambda: hip.conv_backward(dy, x, w, s, False, cdw, None)),
         ("conv3_dgrad", lambda: hip.conv_backward(dy, x, w, s, True, None, None))]
for name, fn in cases:
    for _ in range(5):
        fn()
    torch.cuda.synchronize()
    print(name, flush=True)
