#!/usr/bin/env python3
"""Max-pooling kernels at VGG-16's five 2x2 / stride-2 shapes (and GoogLeNet's 3x3 ones):
forward (pooled output + argmax mask) and backward (gradient scatter through the mask), timed
in isolation, with the effective HBM rate of the bytes each must move.

    python scripts/pool_probe.py [--batch 256]
"""
from __future__ import annotations

import argparse
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import torch  # noqa: E402


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
    ap.add_argument("--batch", type=int, default=256)
    ap.add_argument("--only", default="", help="comma-separated substrings of the shape names to run")
    ap.add_argument("--reps", type=int, default=10)
    args = ap.parse_args()
    from sparknet_amd.ops import _lib
    from sparknet_amd.ops import hip  # noqa: F401
    dev = torch.device("cuda", 0)
    lib = _lib.kernels()
    B = args.batch
    shapes = [("vgg pool1", 224, 64, 2, 2, 0), ("vgg pool2", 112, 128, 2, 2, 0), ("vgg pool3", 56, 256, 2, 2, 0),
              ("vgg pool4", 28, 512, 2, 2, 0), ("vgg pool5", 14, 512, 2, 2, 0),
              ("gn 3a pool 3x3/1", 28, 192, 3, 1, 1), ("gn 3b pool 3x3/1", 28, 256, 3, 1, 1),
              ("gn 4a pool 3x3/1", 14, 480, 3, 1, 1), ("gn 5a pool 3x3/1", 7, 832, 3, 1, 1),
              ("gn pool3 3x3/2", 28, 480, 3, 2, 0)]
    if args.only:
        shapes = [sh for sh in shapes if any(o in sh[0] for o in args.only.split(","))]
    for name, H, C, k, s, pad in shapes:
        P = (H + 2 * pad - k + s - 1) // s + 1
        if (P - 1) * s >= H + pad:
            P -= 1
        x = torch.randn(B, H, H, C, device=dev).to(torch.bfloat16)
        y = torch.empty(B, P, P, C, device=dev, dtype=torch.bfloat16)
        mask = torch.empty(B, P, P, C, device=dev, dtype=torch.uint8)
        dy = torch.randn(B, P, P, C, device=dev).to(torch.bfloat16)
        dx = torch.empty_like(x)
        st = _lib.stream_ptr()

        def fwd():
            _lib.check(lib.sn_pool_fwd(*[_lib.C.c_void_p(t.data_ptr()) for t in (x, y, mask)],
                                       *[_lib.C.c_longlong(v) for v in (B, H, H, C, P, P, k, k, s, s, pad, pad, 0, 0)],
                                       None, None, None, _lib.C.c_longlong(0), _lib.C.c_void_p(st)), "pool_fwd")

        def bwd():
            _lib.check(lib.sn_pool_bwd(*[_lib.C.c_void_p(t.data_ptr()) for t in (dy, mask, dx)],
                                       *[_lib.C.c_longlong(v) for v in (B, H, H, C, P, P, k, k, s, s, pad, pad, 0)],
                                       None, None, None, _lib.C.c_longlong(0), _lib.C.c_void_p(st)), "pool_bwd")
        tf, tb = timed(fwd, args.reps), timed(bwd, args.reps)
        bf = x.numel() * 2 + y.numel() * 3
        bb = dy.numel() * 3 + dx.numel() * 2
        print(f"{name:18s} B={B} {H}x{H}x{C} -> {P}x{P}: fwd {tf:8.1f} us {bf / tf / 1e6:5.2f} TB/s | "
              f"bwd {tb:8.1f} us {bb / tb / 1e6:5.2f} TB/s", flush=True)
        del x, y, mask, dy, dx


if __name__ == "__main__":
    main()
