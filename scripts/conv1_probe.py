#!/usr/bin/env python3
"""AlexNet conv1 after the space-to-depth fold (3x3/1 on 57x57x48, 96 filters, batch 256):
implicit-GEMM conv vs a dense GEMM of the same M/N/K vs variants of K (channel pad)."""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

from sparknet_amd.ops import _lib, gemm, hip  # noqa: E402
from sparknet_amd.ops.spec import ConvSpec  # noqa: E402
from scripts.bench_kernels import timeit  # noqa: E402

_lib.kernels()
dev = "cuda"
for C in (48, 64):
    s = ConvSpec(256, 57, 57, C, 96, 3, 3, 1, 1, 0, 0)
    x = torch.randn(s.N, s.H, s.W, s.C, device=dev).to(torch.bfloat16)
    w = (torch.randn(s.K, s.R, s.S, s.Cg, device=dev) * 0.05).to(torch.bfloat16)
    b = torch.zeros(s.K, device=dev)
    fl = 2.0 * s.N * s.P * s.Q * s.K * s.R * s.S * s.Cg
    ms = timeit(lambda: hip.conv_forward(x, w, b, s, relu=True))
    print(f"implicit C={C}: {ms * 1e3:7.1f} us {fl / ms / 1e9:7.1f} TF", flush=True)
    M, N, K = s.N * s.P * s.Q, 96, 9 * C
    a = torch.randn(M, K, device=dev).to(torch.bfloat16)
    bb = torch.randn(N, K, device=dev).to(torch.bfloat16)
    c = torch.empty(M, N, device=dev, dtype=torch.bfloat16)
    ms = timeit(lambda: gemm.linear_fwd(a, bb, out=c))
    print(f"dense    K={K}: {ms * 1e3:7.1f} us {2 * M * N * K / ms / 1e9:7.1f} TF", flush=True)
