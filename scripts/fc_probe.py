#!/usr/bin/env python3
"""InnerProduct products of CaffeNet at batch 256 (fc6 / fc7 / fc8 forward with bias + ReLU,
data gradient with the ReLU gate): every gemm_kernel-family tile x split-K factor, timed as
the whole product (GEMM + reduce launch), against the tuned-database choice.  Prints the best
configurations so the database can be updated where a better one exists.

    python scripts/fc_probe.py [--tiles 0,1,2,...] [--splits 1,2,3,...]
"""
from __future__ import annotations

import argparse
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import torch  # noqa: E402


def timed(fn, reps=20, passes=5):
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
    ap.add_argument("--tiles", default="0,1,2,3,4,5,10,12,13,16,17,18,19,20,21,22")
    ap.add_argument("--splits", default="1,2,3,4,6,8,12,16")
    args = ap.parse_args()
    from sparknet_amd.ops import gemm as G
    dev = torch.device("cuda", 0)
    tiles = [int(t) for t in args.tiles.split(",")]
    splits = [int(s) for s in args.splits.split(",")]
    B = 256
    shapes = [("fc6", 9216, 4096), ("fc7", 4096, 4096), ("fc8", 4096, 1000)]
    for name, I, O in shapes:
        x = torch.randn(B, I, device=dev).to(torch.bfloat16)
        w = (torch.randn(O, I, device=dev) * 0.02).to(torch.bfloat16)
        b = torch.randn(O, device=dev)
        dy = torch.randn(B, O, device=dev).to(torch.bfloat16)
        gate = torch.randn(B, I, device=dev).to(torch.bfloat16)
        y = torch.empty(B, O, device=dev, dtype=torch.bfloat16)
        dx = torch.empty(B, I, device=dev, dtype=torch.bfloat16)
        ref_y = torch.relu(x.float() @ w.float().t() + b)
        ref_dx = (dy.float() @ w.float()) * (gate.float() > 0)
        for kind, M, N, K in (("fwd", B, O, I), ("dgrad", B, I, O)):
            if kind == "fwd":
                def prod(s=None):
                    G.gemm(M, N, K, G.Dense(x, K, True), G.Dense(w, K, True), y, N, epi=G.EPI_BF16, bias=b,
                           relu=True, splits=s)
                    return y, ref_y
            else:
                def prod(s=None):
                    G.gemm(M, N, K, G.Dense(dy, K, True), G.Dense(w, N, False), dx, N, epi=G.EPI_BF16, splits=s,
                           gate=gate)
                    return dx, ref_dx
            G._FORCE_TILE = -1
            t_db = timed(lambda: prod())
            fl = 2.0 * M * N * K
            res = []
            best = (t_db, "db")
            for t in tiles:
                G._FORCE_TILE = t
                for s in splits:
                    try:
                        out, ref = prod(s)
                        torch.cuda.synchronize()
                    except (RuntimeError, AssertionError):
                        continue
                    err = float((out.float() - ref).abs().max() / (ref.abs().max() + 1e-6))
                    if err > 2e-2:
                        res.append(f"{t}/{s}:ERR{err:.2g}")
                        continue
                    us = timed(lambda: prod(s))
                    res.append(f"{t}/{s}:{us:.1f}")
                    if us < best[0]:
                        best = (us, f"{t}/{s}")
            G._FORCE_TILE = -1
            print(f"{name} {kind:5s} M={M} N={N} K={K}: db {t_db:.1f} us ({fl / t_db / 1e6:.0f} TF/s)  best {best[1]} "
                  f"{best[0]:.1f} us ({fl / best[0] / 1e6:.0f} TF/s) | " + " ".join(res), flush=True)


if __name__ == "__main__":
    main()
