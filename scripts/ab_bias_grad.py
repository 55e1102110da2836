#!/usr/bin/env python3
"""A/B in one process: conv / FC weight+bias gradient with the bias column folded into the
wgrad GEMM vs the separate two-pass column sum (CaffeNet shapes, batch 256).

    python scripts/ab_bias_grad.py
"""
from __future__ import annotations

import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import torch  # noqa: E402

from bench_kernels import timeit  # noqa: E402


def main():
    from sparknet_amd.ops import _lib, gemm, hip
    from sparknet_amd.ops.spec import ConvSpec
    _lib.kernels()
    dev = "cuda"
    convs = {
        "conv1": ConvSpec(256, 227, 227, 3, 96, 11, 11, 4, 4, 0, 0),
        "conv2": ConvSpec(256, 27, 27, 96, 256, 5, 5, 1, 1, 2, 2, groups=2),
        "conv3": ConvSpec(256, 13, 13, 256, 384, 3, 3, 1, 1, 1, 1),
        "conv4": ConvSpec(256, 13, 13, 384, 384, 3, 3, 1, 1, 1, 1, groups=2),
        "conv5": ConvSpec(256, 13, 13, 384, 256, 3, 3, 1, 1, 1, 1, groups=2),
    }
    orig_gemm = hip.gemm

    def unfused_gemm(*a, **kw):
        bg = kw.pop("bias_grad", None)
        acc = kw.pop("bias_acc", True)
        if bg is not None:  # A is the [pixels, K] output gradient (all groups)
            gemm.colsum(a[3].t, bg, accumulate=acc)
        return orig_gemm(*a, **kw)

    for name, s in convs.items():
        x = torch.randn(s.N, s.H, s.W, s.C, device=dev).to(torch.bfloat16)
        w = (torch.randn(s.K, s.R, s.S, s.Cg, device=dev) * 0.05).to(torch.bfloat16)
        dy = torch.randn(s.N, s.P, s.Q, s.K, device=dev).to(torch.bfloat16)
        dw = torch.zeros(s.K, s.R, s.S, s.Cg, device=dev)
        db = torch.zeros(s.K, device=dev)
        res = {}
        for rnd in range(3):
            for mode in ("fused", "colsum"):
                hip.gemm = orig_gemm if mode == "fused" else unfused_gemm
                t = timeit(lambda: hip.conv_backward(dy, x, w, s, False, dw, db, dw_acc=False, db_acc=False))
                res.setdefault(mode, []).append(t)
        hip.gemm = orig_gemm
        print(f"{name}: fused {min(res['fused']) * 1000:7.1f} us   colsum+wgrad {min(res['colsum']) * 1000:7.1f} us",
              flush=True)
    for name, (M, K, N) in {"fc6": (256, 9216, 4096), "fc7": (256, 4096, 4096), "fc8": (256, 4096, 1000)}.items():
        x = torch.randn(M, K, device=dev).to(torch.bfloat16)
        dy = torch.randn(M, N, device=dev).to(torch.bfloat16)
        dw = torch.zeros(N, K, device=dev)
        db = torch.zeros(N, device=dev)
        tf = min(timeit(lambda: gemm.linear_wgrad(dy, x, dw, db=db)) for _ in range(3))
        tu = min(timeit(lambda: (gemm.linear_wgrad(dy, x, dw), gemm.colsum(dy, db))) for _ in range(3))
        print(f"{name}: fused {tf * 1000:7.1f} us   colsum+wgrad {tu * 1000:7.1f} us", flush=True)


if __name__ == "__main__":
    main()
