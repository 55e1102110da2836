#!/usr/bin/env python3
"""In-process A/B of a GEMM code-path switch on every GEMM launch of one training step.

Records the launches of an eager step (as scripts/gemm_census.py), then replays each one
under two settings of a module-level switch of ops.gemm (default ``_ADDR_LEGACY``: the
scalar-offset DMA fast paths vs the general per-lane decode), interleaved over rounds
(cdna_hip_programming.md §5.4 rule 24), and prints per-launch medians and totals.

    python scripts/gemm_ab.py [--model caffenet] [--switch _ADDR_LEGACY] [--a 0] [--b 1]
"""
from __future__ import annotations

import argparse
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import torch  # noqa: E402


def record(model, batch):
    import bench
    from sparknet_amd import models
    from sparknet_amd.core.solver import Solver
    from sparknet_amd.data.prefetch import DeviceFeeder, SyntheticSource
    from sparknet_amd.engine import LocalSGDTrainer, fuse_input_fold, fuse_relu
    from sparknet_amd.ops import _lib, gemm

    _lib.kernels()
    dev = torch.device("cuda", 0)
    B, C, HW, crop, classes, mean, in_scale = bench.DEFAULTS[model]
    B = batch or B
    kw = dict(train_batch=B, test_batch=max(1, min(B, 50)))
    if model in ("caffenet", "alexnet", "googlenet", "vgg16"):
        kw["crop"] = crop
    solver = Solver(models.solver_for(model, **kw), device=dev, seed=1701, build_test_nets=False)
    net = solver.net
    fuse_relu(net)
    src = SyntheticSource(B, C, HW, HW, classes=classes, pool=3, seed=0)
    feeder = DeviceFeeder(src, net.blob_by_name("data"), net.blob_by_name("label"), crop=crop, mean=mean,
                          scale=in_scale, mirror=True, train=True, rng_state=net.ctx.rng_state, device=dev)
    fuse_input_fold(net, feeder)
    trainer = LocalSGDTrainer(solver, None, tau=50, feeder=feeder, use_graph=False)
    trainer.local_step()
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
    return rec, orig


def med(fn, reps):
    ts = []
    for _ in range(reps):
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        fn()
        e1.record()
        e1.synchronize()
        ts.append(e0.elapsed_time(e1))
    ts.sort()
    return ts[len(ts) // 2] * 1e3


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--model", default="caffenet")
    ap.add_argument("--batch", type=int, default=0)
    ap.add_argument("--switch", default="_ADDR_LEGACY")
    ap.add_argument("--a", type=int, default=0)
    ap.add_argument("--b", type=int, default=1)
    ap.add_argument("--rounds", type=int, default=5)
    ap.add_argument("--reps", type=int, default=7)
    args = ap.parse_args()
    from sparknet_amd.ops import gemm
    rec, orig = record(args.model, args.batch)
    tot = {args.a: 0.0, args.b: 0.0}
    print(f"{'layer:pass':24s} {'M':>8s} {'N':>5s} {'K':>6s} g tile spl  {'A us':>8s} {'B us':>8s}  B/A")
    for name, a, k in rec:
        fn = (lambda a=a, k=k: orig(*a, **k))
        res = {args.a: [], args.b: []}
        for _ in range(args.rounds):
            for v in (args.a, args.b):
                setattr(gemm, args.switch, v)
                fn()
                res[v].append(med(fn, args.reps))
        setattr(gemm, args.switch, args.a)
        ua, ub = sorted(res[args.a])[len(res[args.a]) // 2], sorted(res[args.b])[len(res[args.b]) // 2]
        tot[args.a] += ua
        tot[args.b] += ub
        print(f"{name:24s} {a[0]:8d} {a[1]:5d} {a[2]:6d} {a[3]} {a[16]:4d} {a[17]:3d}  {ua:8.1f} {ub:8.1f}  {ub / ua:.3f}",
              flush=True)
    print(f"total: A({args.switch}={args.a}) {tot[args.a]:.1f} us   B({args.switch}={args.b}) {tot[args.b]:.1f} us"
          f"   B/A {tot[args.b] / tot[args.a]:.3f}")


if __name__ == "__main__":
    main()
