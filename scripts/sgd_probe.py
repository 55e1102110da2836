#!/usr/bin/env python3
"""CaffeNet's fused InnerProduct weight-gradient + solver-update products (EPI_SGD, batch 256)
on every tile with an EPI_SGD instance: time and the HBM rate of the 18 B/parameter update
stream (fp32 master + history read and written, bf16 shadow written).

    python scripts/sgd_probe.py
"""
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
    from sparknet_amd.ops import gemm as G
    dev = torch.device("cuda", 0)
    B = 256
    for name, O, I in (("fc6", 4096, 9216), ("fc7", 4096, 4096), ("fc8", 1000, 4096)):
        dy = (torch.randn(B, O, device=dev) * 0.1).to(torch.bfloat16)
        x = torch.randn(B, I, device=dev).to(torch.bfloat16)
        w = torch.randn(O, I, device=dev) * 0.05
        h = torch.zeros(O, I, device=dev)
        sh = torch.zeros(O, I, dtype=torch.bfloat16, device=dev)
        hyper = torch.tensor([1e-6, 0.9, 5e-4, 0.0, 1.0, 0, 0, 0], dtype=torch.float32, device=dev)
        db = torch.zeros(O, device=dev)
        sgd = dict(w=w, h=h, shadow=sh, hyper=hyper, lr_mult=1.0, decay_mult=1.0, flags=0)
        res = []
        for t in (0, 1, 2, 3, 10):
            G._FORCE_TILE = t
            try:
                us = timed(lambda: G.linear_wgrad_sgd(dy, x, sgd, db, db_acc=False))
            except (RuntimeError, AssertionError) as e:
                res.append(f"{t}:-")
                continue
            res.append(f"{t}:{us:.1f}us/{O * I * 18 / us / 1e6:.2f}TB/s")
        G._FORCE_TILE = -1
        print(f"{name} {O}x{I}: " + "  ".join(res), flush=True)


if __name__ == "__main__":
    main()
