#!/usr/bin/env python3
"""CPU list-scheduling simulation of engine.BranchStreams plans (no GPU): each layer costs its
estimated GEMM FLOPs at a fixed rate (conv / InnerProduct) or its blob bytes at a fixed HBM
rate, plus a per-launch overhead; a layer starts when its stream is free and the layers it
waits on have ended.  Prints the simulated forward / backward span and per-stream busy time
for 2 / 3 / 4 streams — a quick way to compare planner policies before a GPU A/B.

    python scripts/branch_sim.py [--model googlenet] [--batch 128]
"""
from __future__ import annotations

import argparse
import collections
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import torch  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--model", default="googlenet")
    ap.add_argument("--batch", type=int, default=128)
    ap.add_argument("--gemm-tfs", type=float, default=550.0)
    ap.add_argument("--hbm-tbs", type=float, default=3.0)
    ap.add_argument("--launch-us", type=float, default=5.0)
    args = ap.parse_args()
    from sparknet_amd import models
    from sparknet_amd.core.solver import Solver
    from sparknet_amd.engine import BranchStreams
    kw = dict(train_batch=2, test_batch=2)
    if args.model in ("caffenet", "alexnet", "googlenet", "vgg16"):
        kw["crop"] = 224 if args.model != "caffenet" else 227
    net = Solver(models.solver_for(args.model, **kw), device=torch.device("cpu"), seed=1, build_test_nets=False).net
    B = args.batch
    free_types = ("ReLU", "Concat", "Split") if True else ()

    def cost(li, bwd):
        lay = net.layers[li]
        t = lay.type_name
        if t in ("ReLU", "Concat"):
            return 0.0  # fused into producers / zero-copy on the GPU path
        if t == "Convolution":
            b, tp = net.bottom_vecs[li][0], net.top_vecs[li][0]
            s = lay.spec(b)
            fl = 2.0 * B * tp.shape[2] * tp.shape[3] * tp.shape[1] * s.R * s.S * s.Cg
            return (2 if bwd else 1) * fl / (args.gemm_tfs * 1e12) * 1e6 + args.launch_us
        if t == "InnerProduct":
            fl = 2.0 * B * net.bottom_vecs[li][0].count_range(1) * lay.N
            return (2 if bwd else 1) * fl / (args.gemm_tfs * 0.5e12) * 1e6 + args.launch_us
        nb = sum(x.count_range(1) for x in net.bottom_vecs[li]) + sum(x.count_range(1) for x in net.top_vecs[li])
        return (2 if bwd else 1) * nb * B * 2 / (args.hbm_tbs * 1e12) * 1e6 + args.launch_us

    def simulate(plan, bwd, n):
        free, end, busy = [0.0] * n, {}, collections.Counter()
        for pos, (li, sid, waits, _) in enumerate(plan):
            d = cost(li, bwd)
            end[pos] = max([free[sid]] + [end[w] for w in waits]) + d
            free[sid] = end[pos]
            busy[sid] += d
        return max(free), busy

    for n in (2, 3, 4):
        bs = BranchStreams(net, n, star=n > 2)
        f, fb = simulate(bs.fwd_plan, False, n)
        b, bb = simulate(bs.bwd_plan, True, n)
        print(f"{n} streams: forward {f:7.0f} us (busy {[round(fb[s]) for s in range(n)]}), "
              f"backward {b:7.0f} us (busy {[round(bb[s]) for s in range(n)]})")
    del free_types


if __name__ == "__main__":
    main()
