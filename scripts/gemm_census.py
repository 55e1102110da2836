#!/usr/bin/env python3
"""Per-layer GEMM census of one training iteration: every MFMA GEMM launch of an eager
step (after autotuning) is recorded with its layer / pass, then re-launched on its own
and timed (median of interleaved repetitions).  Prints one line per launch with the
shape, tile / split-K choice, time and TF/s, plus per-pass totals.

    python scripts/gemm_census.py [--model caffenet] [--batch 256] [--reps 20]
"""
from __future__ import annotations

import argparse
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import torch  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--model", default="caffenet")
    ap.add_argument("--batch", type=int, default=0)
    ap.add_argument("--reps", type=int, default=20)
    args = ap.parse_args()

    import bench
    from sparknet_amd import models
    from sparknet_amd.core.solver import Solver
    from sparknet_amd.data.prefetch import DeviceFeeder, SyntheticSource
    from sparknet_amd.engine import LocalSGDTrainer, fuse_input_fold, fuse_relu
    from sparknet_amd.ops import _lib, gemm

    _lib.kernels()
    dev = torch.device("cuda", 0)
    B, C, HW, crop, classes, mean, in_scale = bench.DEFAULTS[args.model]
    B = args.batch or B
    kw = dict(train_batch=B, test_batch=max(1, min(B, 50)))
    if args.model in ("caffenet", "alexnet", "googlenet", "vgg16"):
        kw["crop"] = crop
    solver = Solver(models.solver_for(args.model, **kw), device=dev, seed=1701, build_test_nets=False)
    net = solver.net
    fuse_relu(net)
    src = SyntheticSource(B, C, HW, HW, classes=classes, pool=3, seed=0)
    feeder = DeviceFeeder(src, net.blob_by_name("data"), net.blob_by_name("label"), crop=crop, mean=mean,
                          scale=in_scale, mirror=True, train=True, rng_state=net.ctx.rng_state, device=dev)
    fuse_input_fold(net, feeder)
    trainer = LocalSGDTrainer(solver, None, tau=50, feeder=feeder, use_graph=False)
    trainer.local_step()  # autotune every shape
    torch.cuda.synchronize()

    where = ["?"]
    for layer in net.layers:
        f, b = layer.forward, layer.backward

        def fw(*a, _f=f, _n=layer.name):
            where[0] = _n + ":fwd"
            return _f(*a)

        def bw(*a, _b=b, _n=layer.name):
            where[0] = _n + ":bwd"
            return _b(*a)
        layer.forward, layer.backward = fw, bw

    rec = []
    orig = gemm._launch

    def spy(*a, **k):
        rec.append((where[0], a, k))
        return orig(*a, **k)
    gemm._launch = spy
    trainer.local_step()
    torch.cuda.synchronize()
    gemm._launch = orig

    rows = []
    for name, a, k in rec:
        M, N, K, groups = a[0], a[1], a[2], a[3]
        ops = a[4]
        epi = a[5]
        tile, splits, kchunk = a[16], a[17], a[18]
        fn = (lambda a=a, k=k: orig(*a, **k))
        for _ in range(3):
            fn()
        torch.cuda.synchronize()
        ts = []
        for _ in range(args.reps):
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record()
            fn()
            e1.record()
            e1.synchronize()
            ts.append(e0.elapsed_time(e1))
        ts.sort()
        us = ts[len(ts) // 2] * 1e3
        fl = 2.0 * M * N * K * groups
        kind = {(0, 1, 0, 0): "fwd", (1, 0, 1, 1): "wgrad", (0, 1, 1, 2): "dgrad"}.get(
            (ops[1], ops[2], ops[4], ops[5]), f"{ops[1]}{ops[2]}/{ops[4]}{ops[5]}")
        rows.append((name, kind, M, N, K, groups, tile, splits, epi, us, fl / us / 1e6))
    tot = 0.0
    print(f"{'layer:pass':24s} {'kind':7s} {'M':>8s} {'N':>5s} {'K':>6s} {'g':>2s} tile spl epi {'us':>8s} {'TF/s':>7s}")
    for r in rows:
        tot += r[9]
        print(f"{r[0]:24s} {r[1]:7s} {r[2]:8d} {r[3]:5d} {r[4]:6d} {r[5]:2d} {r[6]:4d} {r[7]:3d} {r[8]:3d} "
              f"{r[9]:8.1f} {r[10]:7.1f}")
    flops = sum(2.0 * r[2] * r[3] * r[4] * r[5] for r in rows)
    print(f"total GEMM time (isolated launches): {tot:.1f} us, {flops / 1e12:.3f} TFLOP, {flops / tot / 1e6:.1f} TF/s")


if __name__ == "__main__":
    main()
