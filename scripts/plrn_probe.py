#!/usr/bin/env python3
"""Isolated timing of the fused max-pool + LRN kernels (csrc/kernels/pool_lrn.hip) at the
CaffeNet shapes, with the backward's forms A/B'd (sn_plrn_bwd_variant: 0 block form, 1 / 2
whole-pixel form with a 32 / 64 KB tile) and checked bitwise equal to form 0.

    python scripts/plrn_probe.py [--iters 50]
"""
import argparse
import ctypes as C
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

from sparknet_amd.ops import _lib, hip  # noqa: E402
from sparknet_amd.ops.spec import PoolSpec  # noqa: E402

p = argparse.ArgumentParser()
p.add_argument("--iters", type=int, default=50)
args = p.parse_args()
dev = torch.device("cuda:0")
SHAPES = {"pool1/norm1": (256, 55, 55, 96), "pool2/norm2": (256, 27, 27, 256)}
setv = _lib.kernels().sn_plrn_bwd_variant
setv.argtypes = [C.c_int]


def timed(fn):
    for _ in range(3):
        fn()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(args.iters):
        fn()
    e1.record()
    torch.cuda.synchronize()
    return e0.elapsed_time(e1) * 1000.0 / args.iters


for name, (n, h, w, c) in SHAPES.items():
    s = PoolSpec(n, h, w, c, 3, 3, 2, 2)
    g = torch.Generator(device=dev).manual_seed(0)
    x = torch.randn((n, h, w, c), device=dev, generator=g).relu_().to(torch.bfloat16)
    pooled, mask, y = hip.pool_lrn_forward(x, s, True, 5, 1e-4, 0.75, 1.0)
    dy = torch.randn(y.shape, device=dev, generator=g).to(torch.bfloat16)
    t_f = timed(lambda: hip.pool_lrn_forward(x, s, True, 5, 1e-4, 0.75, 1.0))
    fbytes = x.numel() * 2 + pooled.numel() * 5
    print(f"{name}: forward {t_f:7.1f} us  {fbytes / t_f / 1e6:5.2f} TB/s", flush=True)
    ref = None
    bbytes = x.numel() * 2 + pooled.numel() * 5
    for v in (0, 1, 2):
        setv(v)
        dx = hip.lrn_pool_backward(dy, pooled, mask, s, 5, 1e-4, 0.75, 1.0)
        torch.cuda.synchronize()
        same = "ref" if ref is None else ("bitwise equal" if torch.equal(dx, ref) else
                                          f"DIFFERS max {float((dx.float() - ref.float()).abs().max()):.3g}")
        ref = dx if ref is None else ref
        t_b = timed(lambda: hip.lrn_pool_backward(dy, pooled, mask, s, 5, 1e-4, 0.75, 1.0))
        print(f"{name}: backward form {v} {t_b:7.1f} us  {bbytes / t_b / 1e6:5.2f} TB/s  {same}", flush=True)
    setv(0)
