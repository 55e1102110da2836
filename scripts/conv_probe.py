#!/usr/bin/env python3
"""One implicit-GEMM convolution forward at a model's real geometry, every tile (splits 1), with
and without the fused bias + ReLU epilogue, and the same product as a plain dense GEMM of equal
M / N / K — separating the im2col staging cost from the mainloop / epilogue.

    python scripts/conv_probe.py [--case gn_conv2]
"""
from __future__ import annotations

import argparse
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import torch  # noqa: E402

CASES = {  # N, H, W, C, K, R, S, stride, pad
    "gn_conv2": (128, 56, 56, 64, 192, 3, 3, 1, 1),
    "gn_3b_3x3": (128, 28, 28, 128, 192, 3, 3, 1, 1),
    "cn_conv3": (256, 13, 13, 256, 384, 3, 3, 1, 1),
    "cn_conv4g": (256, 13, 13, 192, 192, 3, 3, 1, 1),
    "cn_conv2g": (256, 27, 27, 48, 128, 5, 5, 1, 2),  # CaffeNet conv2, one of its two groups
    "cn_conv5g": (256, 13, 13, 192, 128, 3, 3, 1, 1),
    "vgg_conv3_2": (128, 56, 56, 256, 256, 3, 3, 1, 1),  # VGG-16 at 1/16 of its b2048 batch
    "vgg_conv4_2": (256, 28, 28, 512, 512, 3, 3, 1, 1),
}


def timed(fn, reps=10, passes=5):
    fn()
    torch.cuda.synchronize()
    best = []
    for _ in range(passes):
        torch.cuda._sleep(1 << 18)
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        for _ in range(reps):
            fn()
        e1.record()
        e1.synchronize()
        best.append(e0.elapsed_time(e1) * 1e3 / reps)
    best.sort()
    return best[len(best) // 2]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--case", default="gn_conv2,cn_conv3")
    ap.add_argument("--tiles", default="-1,0,1,2,4,11,12,13,15,16,17,18,19")
    ap.add_argument("--reps", type=int, default=10)
    ap.add_argument("--no-dense", action="store_true")
    args = ap.parse_args()
    from sparknet_amd.ops import gemm as G, hip
    from sparknet_amd.ops.spec import ConvSpec
    dev = torch.device("cuda", 0)
    for case in args.case.split(","):
        N, H, W, C, K, R, S, st, pd = CASES[case]
        s = ConvSpec(N, H, W, C, K, R, S, st, st, pd, pd, 1, 1, 1)
        x = torch.randn(N, H, W, C, device=dev).to(torch.bfloat16)
        w = (torch.randn(K, R, S, C, device=dev) * 0.05).to(torch.bfloat16)
        b = torch.randn(K, device=dev)
        M, Kr = N * s.P * s.Q, R * S * C
        fl = 2.0 * M * K * Kr
        a = torch.randn(M, Kr, device=dev).to(torch.bfloat16)
        wf = w.reshape(K, Kr)
        res = []
        for t in [int(v) for v in args.tiles.split(",")]:
            G._FORCE_TILE = t
            try:
                tc = timed(lambda: hip.conv_forward(x, w, b, s, relu=True), args.reps)
            except (RuntimeError, AssertionError, TypeError):
                tc = None
            try:
                if args.no_dense:
                    raise RuntimeError("skipped")
                y = torch.empty(M, K, device=dev, dtype=torch.bfloat16)
                td = timed(lambda: G.gemm(M, K, Kr, G.Dense(a, Kr, True), G.Dense(wf, Kr, True), y, K,
                                          epi=G.EPI_BF16, bias=b, relu=True, splits=None if t < 0 else 1))
            except (RuntimeError, AssertionError):
                td = None
            res.append(f"{t}: conv {fl / tc / 1e6 if tc else 0:.0f} dense {fl / td / 1e6 if td else 0:.0f}")
        G._FORCE_TILE = -1
        print(f"{case} M={M} N={K} K={Kr} ({fl / 1e9:.1f} GF), TF/s: " + " | ".join(res), flush=True)


if __name__ == "__main__":
    main()
