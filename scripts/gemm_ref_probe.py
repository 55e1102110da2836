#!/usr/bin/env python3
"""Headroom probe: our MFMA GEMM vs the vendor library (torch.mm -> hipBLASLt) on the
dense NT equivalents of the conv shapes that dominate CaffeNet / VGG-16 training.
Random bf16 operands, interleaved repetitions in one process (cdna_hip_programming.md
§5.4 rules 24/25).  Prints TFLOP/s per (shape, implementation).

    python scripts/gemm_ref_probe.py
"""
from __future__ import annotations

import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import torch  # noqa: E402


def timeit(fn, reps=15, warm=3):
    for _ in range(warm):
        fn()
    torch.cuda.synchronize()
    ev = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)) for _ in range(reps)]
    for a, b in ev:
        a.record()
        fn()
        b.record()
    torch.cuda.synchronize()
    ts = sorted(a.elapsed_time(b) for a, b in ev)
    return ts[len(ts) // 2]


SHAPES = {  # name: (M, N, K) for C[M,N] = A[M,K] B[N,K]^T
    "square 8192": (8192, 8192, 8192),
    "square 4096": (4096, 4096, 4096),
    "caffenet conv2 (per group)": (186624, 128, 1200),
    "caffenet conv3": (43264, 384, 2304),
    "caffenet conv4 (per group)": (43264, 192, 1728),
    "vgg conv3_2": (200704, 256, 2304),
    "vgg conv4_2": (50176, 512, 4608),
    "vgg conv1_2": (3211264, 64, 576),
    "fc6 fwd": (256, 4096, 9216),
}


def main():
    from sparknet_amd.ops import _lib, gemm
    _lib.kernels()
    torch.manual_seed(0)
    for name, (M, N, K) in SHAPES.items():
        a = (torch.rand(M, K, device="cuda") * 2 - 1).to(torch.bfloat16)
        b = (torch.rand(N, K, device="cuda") * 2 - 1).to(torch.bfloat16)
        c = torch.empty(M, N, device="cuda", dtype=torch.bfloat16)
        fl = 2.0 * M * N * K
        t_ours = timeit(lambda: gemm.linear_fwd(a, b, out=c))
        t_lib = timeit(lambda: torch.mm(a, b.t(), out=c))
        t_ours2 = timeit(lambda: gemm.linear_fwd(a, b, out=c))
        t_o = min(t_ours, t_ours2)
        print(f"{name:30s} M={M:8d} N={N:5d} K={K:5d}  ours {fl / t_o / 1e9:7.1f} TF  "
              f"hipBLASLt {fl / t_lib / 1e9:7.1f} TF", flush=True)
        del a, b, c


if __name__ == "__main__":
    main()
