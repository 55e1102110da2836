#!/usr/bin/env python3
"""Anatomy of the conv weight-gradient product: the CaffeNet b256 wgrad
shapes as (a) the implicit MC x MC(im2col) product the engine runs, (b) the same product
with an explicit im2col matrix (dense MC x dense MC: no im2col addressing), (c) the dense
K-contiguous product of the pre-transposed operands (KC x KC: no transposed LDS reads), each
over tiles x split-K, fp32 slab + reduce included.  Separates the im2col staging cost and
the transposed-read cost from the mainloop.

    python scripts/wgrad_probe.py [--case conv3,conv2] [--tiles 0,10,...] [--splits ...]
"""
from __future__ import annotations

import argparse
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import torch  # noqa: E402

CASES = {  # N, H, W, C(per group), K(per group), R, S, stride, pad
    "conv1f": (256, 57, 57, 48, 96, 3, 3, 1, 0),  # CaffeNet conv1 after the 4x4 space-to-depth fold
    "conv2": (256, 27, 27, 48, 128, 5, 5, 1, 2),
    "conv3": (256, 13, 13, 256, 384, 3, 3, 1, 1),
    "conv4": (256, 13, 13, 192, 192, 3, 3, 1, 1),
    "conv5": (256, 13, 13, 192, 128, 3, 3, 1, 1),
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
    ap.add_argument("--case", default="conv3,conv2,conv5")
    ap.add_argument("--tiles", default="0,10,2,3,12,13,15,16,20")
    ap.add_argument("--splits", default="2,4,6,8,12,16,24")
    ap.add_argument("--forms", default="implicit,mcmc,kckc")
    args = ap.parse_args()
    from sparknet_amd.ops import gemm as G
    from sparknet_amd.ops.hip import _geom
    from sparknet_amd.ops.spec import ConvSpec
    dev = torch.device("cuda", 0)
    tiles = [int(t) for t in args.tiles.split(",")]
    splits = [int(s) for s in args.splits.split(",")]
    for case in args.case.split(","):
        N, H, W, C, K, R, S, st, pd = CASES[case]
        s = ConvSpec(N, H, W, C, K, R, S, st, st, pd, pd, 1, 1, 1)
        x = torch.randn(N, H, W, C, device=dev).to(torch.bfloat16)
        dy = torch.randn(N, s.P, s.Q, K, device=dev).to(torch.bfloat16)
        Mr, kred = N * s.P * s.Q, R * S * C  # reduction (pixels), output columns
        fl = 2.0 * Mr * K * kred
        dy2 = dy.view(Mr, K)
        dw = torch.empty(K, kred, device=dev)
        col = torch.randn(Mr, kred, device=dev).to(torch.bfloat16)  # explicit im2col stand-in
        dyT = dy2.t().contiguous()
        colT = col.t().contiguous()
        forms = {
            "implicit": (G.Dense(dy2, K, kcontig=False), G.Im2col(x, _geom(s), kcontig=False)),
            "mcmc": (G.Dense(dy2, K, kcontig=False), G.Dense(col, kred, kcontig=False)),
            "kckc": (G.Dense(dyT, Mr, kcontig=True), G.Dense(colT, Mr, kcontig=True)),
        }
        print(f"== {case}: M {K} N {kred} K {Mr}  ({fl / 1e9:.1f} GFLOP)", flush=True)
        for fname in args.forms.split(","):
            A, B = forms[fname]
            G._FORCE_TILE = -1
            try:
                us = timed(lambda: G.gemm(K, kred, Mr, A, B, dw, kred, epi=G.EPI_F32))
                print(f"  {fname:9s} tuned/auto      {us:8.1f} us  {fl / us / 1e6:7.1f} TF/s", flush=True)
            except Exception as e:  # noqa: BLE001
                print(f"  {fname:9s} tuned/auto      n/a ({str(e)[:60]})", flush=True)
            best = None
            for t in tiles:
                row = []
                G._FORCE_TILE = t
                for sp in splits:
                    try:
                        us = timed(lambda: G.gemm(K, kred, Mr, A, B, dw, kred, epi=G.EPI_F32, splits=sp))
                    except Exception:  # noqa: BLE001
                        row.append("   n/a")
                        continue
                    row.append(f"{us:6.1f}")
                    if best is None or us < best[0]:
                        best = (us, t, sp)
                print(f"  {fname:9s} t{t:<3d} " + " ".join(row), flush=True)
            G._FORCE_TILE = -1
            if best:
                print(f"  {fname:9s} BEST t{best[1]} s{best[2]}: {best[0]:.1f} us {fl / best[0] / 1e6:.1f} TF/s",
                      flush=True)


if __name__ == "__main__":
    main()
