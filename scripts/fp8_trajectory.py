#!/usr/bin/env python3
"""200-step VGG-16 loss trajectories: bf16 vs e4m3 forward (fp8) vs e4m3 forward + e4m3
data gradients (fp8dg) vs e4m3 forward + e5m2 data gradients (fp8dg5), on the production path (GraphStep: one hipGraph per iteration, fused ReLU,
delayed per-tensor fp8 scaling), same seeds, same data stream.

The data is a learnable synthetic task (no datasets on the box): 10 fixed random class
templates plus Gaussian noise, so the loss falls from ln(10) and the trajectories say
whether the fp8 products train like bf16.  Prints one JSON line per mode and a summary
(max |smoothed loss - bf16 smoothed loss| over 20-step windows).

    python scripts/fp8_trajectory.py [--steps 200] [--batch 64] [--crop 64] [--modes bf16,fp8,fp8dg,fp8dg5]
"""
import argparse
import json
import math
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

from sparknet_amd import models  # noqa: E402
from sparknet_amd.core.solver import Solver  # noqa: E402
from sparknet_amd.engine import GraphStep, enable_fp8, fuse_relu  # noqa: E402

p = argparse.ArgumentParser()
p.add_argument("--steps", type=int, default=200)
p.add_argument("--batch", type=int, default=64)
p.add_argument("--crop", type=int, default=64)
p.add_argument("--classes", type=int, default=10)
p.add_argument("--lr", type=float, default=0.005)
p.add_argument("--modes", default="bf16,fp8,fp8dg,fp8dg5", help="bf16, bf16alt (chaos floor), fp8, fp8dg, fp8dg5, "
               "and fp8dgw / fp8dg5w (+ fp8 weight gradients)")
p.add_argument("--window", type=int, default=20)
p.add_argument("--noise", type=float, default=0.8)
p.add_argument("--seed", type=int, default=12)
args = p.parse_args()
dev = torch.device("cuda:0")

g0 = torch.Generator().manual_seed(11)
templates = torch.randn(args.classes, 3, args.crop, args.crop, generator=g0)


def batches():
    g = torch.Generator().manual_seed(args.seed)
    while True:
        y = torch.randint(0, args.classes, (args.batch,), generator=g)
        x = templates[y] + args.noise * torch.randn(args.batch, 3, args.crop, args.crop, generator=g)
        yield x, y.float().view(-1, 1)


def run(mode):
    net_p = models.vgg16(train_batch=args.batch, test_batch=args.batch, crop=args.crop, classes=args.classes)
    sp = models.zoo.vgg16_solver(net_p)
    sp.base_lr = args.lr
    solver = Solver(sp, device=dev, seed=5, build_test_nets=False)
    fuse_relu(solver.net)
    n8 = 0
    # bf16alt: bf16 with every GEMM on the 128x128 tile and cost-model split-K (a different
    # fp32 accumulation order): how far two bf16 runs drift apart on their own (chaos floor)
    from sparknet_amd.ops import gemm as _G
    _G._FORCE_TILE = 0 if mode == "bf16alt" else -1
    if mode not in ("bf16", "bf16alt"):
        n8 = enable_fp8(solver.net, 0.0, dgrad=mode.startswith("fp8dg"),
                        dgrad_format="e5m2" if mode.startswith("fp8dg5") else "e4m3", wgrad=mode.endswith("w"))
    it = batches()

    def pre():
        x, y = next(it)
        solver.net.blob_by_name("data").set_nchw(x)
        solver.net.blob_by_name("label").set_nchw(y)
    st = GraphStep(solver, warmup=2, pre=pre, overlap=False)
    losses = [float(st.step()) for _ in range(args.steps)]
    return losses, n8


def smooth(v, w):
    return [sum(v[i:i + w]) / w for i in range(0, len(v) - w + 1, w)]


res = {}
for mode in args.modes.split(","):
    losses, n8 = run(mode)
    res[mode] = losses
    sm = smooth(losses, args.window)
    print(json.dumps({"mode": mode, "fp8_products": n8, "first": round(losses[0], 4), "last": round(losses[-1], 4),
                      f"smoothed_{args.window}": [round(v, 4) for v in sm],
                      "finite": all(math.isfinite(v) for v in losses)}), flush=True)
if "bf16" in res:
    ref = smooth(res["bf16"], args.window)
    for mode, v in res.items():
        if mode == "bf16":
            continue
        sm = smooth(v, args.window)
        d = max(abs(a - b) for a, b in zip(sm, ref))
        print(f"{mode}: max |smoothed loss - bf16| = {d:.4f} (bf16 smoothed {ref[0]:.3f} -> {ref[-1]:.3f}; "
              f"{mode} {sm[0]:.3f} -> {sm[-1]:.3f})", flush=True)
