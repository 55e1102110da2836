#!/usr/bin/env python3
"""The same dense bf16 products on hipBLASLt (torch.matmul) and on gemm_kernel, for
rocprofv3 --pmc passes (scripts/pmc_blas.sh): 8192^3 NT and the VGG-16
conv4_2 shape as a dense NT product (M = 64 x 28 x 28 pixels, N 512, K 4608), 5 launches each."""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

from sparknet_amd.ops import _lib, gemm  # noqa: E402

_lib.kernels()
dev = "cuda"
SHAPES = {"8192^3": (8192, 8192, 8192), "conv4_2": (64 * 28 * 28, 512, 4608)}
for name, (M, N, K) in SHAPES.items():
    a = torch.randn(M, K, device=dev).to(torch.bfloat16)
    b = torch.randn(N, K, device=dev).to(torch.bfloat16)
    c = torch.empty(M, N, device=dev, dtype=torch.bfloat16)
    for label, fn in (("hipblaslt", lambda: torch.matmul(a, b.t(), out=c)),
                      ("gemm_kernel", lambda: gemm.linear_fwd(a, b, out=c))):
        for _ in range(5):
            fn()
        torch.cuda.synchronize()
        print(name, label, flush=True)
