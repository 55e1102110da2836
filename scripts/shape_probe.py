#!/usr/bin/env python3
"""Dense NT GEMMs with the CaffeNet conv GEMM shapes (implicit im2col vs explicit dense
operands of the same M/N/K) — separates gather cost from shape/quantization cost."""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

from sparknet_amd.ops import _lib, gemm  # noqa: E402
from scripts.bench_kernels import timeit  # noqa: E402

_lib.kernels()
for name, (M, N, K) in {"conv3-like": (43264, 384, 2304), "conv2-like/g": (186624, 128, 1200),
                        "conv4-like/g": (43264, 192, 1728), "conv5-like/g": (43264, 128, 1728),
                        "sq4096": (4096, 4096, 4096), "sq8192": (8192, 8192, 8192)}.items():
    a = torch.randn(M, K, device="cuda").to(torch.bfloat16)
    b = torch.randn(N, K, device="cuda").to(torch.bfloat16)
    c = torch.empty(M, N, device="cuda", dtype=torch.bfloat16)
    ms = timeit(lambda: gemm.linear_fwd(a, b, out=c))
    print(f"{name:14s} M={M} N={N} K={K}: {ms * 1e3:8.1f} us {2 * M * N * K / ms / 1e9:7.1f} TF", flush=True)
