#!/usr/bin/env python3
"""Micro-benchmarks of the MFMA GEMM / implicit-GEMM conv kernels on MI355X.

Times each case with HIP events over interleaved repetitions in ONE process (random
bf16 data, cdna_hip_programming.md §5.4 rules 24/25) and prints TFLOP/s.

    python scripts/bench_kernels.py [--quick]
"""
from __future__ import annotations

import argparse
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import torch  # noqa: E402


def timeit(fn, reps=20, warm=3):
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


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--quick", action="store_true")
    ap.add_argument("--json", default=None)
    args = ap.parse_args()
    from sparknet_amd.ops import _lib, gemm, hip
    from sparknet_amd.ops.spec import ConvSpec
    _lib.kernels()
    dev = "cuda"
    out = []

    def rec(name, ms, flops):
        tf = flops / ms / 1e9
        out.append({"case": name, "ms": round(ms, 4), "tflops": round(tf, 1)})
        print(f"{name:48s} {ms * 1000:9.1f} us  {tf:8.1f} TFLOP/s", flush=True)

    # dense square GEMMs (kernel-structure ceiling)
    for n in ([4096] if args.quick else [2048, 4096, 8192]):
        a = torch.randn(n, n, device=dev).to(torch.bfloat16)
        b = torch.randn(n, n, device=dev).to(torch.bfloat16)
        c = torch.empty(n, n, device=dev, dtype=torch.bfloat16)
        rec(f"NT dense {n}^3", timeit(lambda: gemm.linear_fwd(a, b, out=c)), 2 * n ** 3)
        dw = torch.zeros(n, n, device=dev)
        rec(f"TN dense (wgrad) {n}^3", timeit(lambda: gemm.linear_wgrad(a, b, dw)), 2 * n ** 3)
        rec(f"NN dense (dgrad) {n}^3", timeit(lambda: gemm.linear_dgrad(a, b)), 2 * n ** 3)

    # AlexNet/CaffeNet conv layers at batch 256 (NHWC)
    convs = {
        "conv1": ConvSpec(256, 227, 227, 3, 96, 11, 11, 4, 4, 0, 0),
        "conv2": ConvSpec(256, 27, 27, 96, 256, 5, 5, 1, 1, 2, 2, groups=2),
        "conv3": ConvSpec(256, 13, 13, 256, 384, 3, 3, 1, 1, 1, 1),
        "conv4": ConvSpec(256, 13, 13, 384, 384, 3, 3, 1, 1, 1, 1, groups=2),
        "conv5": ConvSpec(256, 13, 13, 384, 256, 3, 3, 1, 1, 1, 1, groups=2),
    }
    for name, s in convs.items():
        x = torch.randn(s.N, s.H, s.W, s.C, device=dev).to(torch.bfloat16)
        w = (torch.randn(s.K, s.R, s.S, s.Cg, device=dev) * 0.05).to(torch.bfloat16)
        b = torch.zeros(s.K, device=dev)
        dy = torch.randn(s.N, s.P, s.Q, s.K, device=dev).to(torch.bfloat16)
        dw = torch.zeros(s.K, s.R, s.S, s.Cg, device=dev)
        fl = 2.0 * s.N * s.P * s.Q * s.K * s.R * s.S * s.Cg
        rec(f"{name} fwd", timeit(lambda: hip.conv_forward(x, w, b, s, relu=True)), fl)
        rec(f"{name} wgrad", timeit(lambda: hip.conv_backward(dy, x, w, s, False, dw, None)), fl)
        if name != "conv1":
            rec(f"{name} dgrad", timeit(lambda: hip.conv_backward(dy, x, w, s, True, None, None)), fl)
    # FC layers
    for name, (M, K, N) in {"fc6": (256, 9216, 4096), "fc7": (256, 4096, 4096), "fc8": (256, 4096, 1000)}.items():
        x = torch.randn(M, K, device=dev).to(torch.bfloat16)
        w = (torch.randn(N, K, device=dev) * 0.01).to(torch.bfloat16)
        dy = torch.randn(M, N, device=dev).to(torch.bfloat16)
        dw = torch.zeros(N, K, device=dev)
        fl = 2.0 * M * N * K
        rec(f"{name} fwd", timeit(lambda: gemm.linear_fwd(x, w)), fl)
        rec(f"{name} wgrad", timeit(lambda: gemm.linear_wgrad(dy, x, dw)), fl)
        rec(f"{name} dgrad", timeit(lambda: gemm.linear_dgrad(dy, w)), fl)
    if args.json:
        with open(args.json, "w") as f:
            json.dump(out, f, indent=1)


if __name__ == "__main__":
    main()
