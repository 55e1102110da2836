#!/usr/bin/env python3
"""Within-process throughput stability of the CaffeNet bench step: 10 chunks of 100
graph-replayed steps, img/s per chunk (is run-to-run variance inside or across processes?)."""
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

import bench  # noqa: E402
from sparknet_amd import models  # noqa: E402
from sparknet_amd.core.solver import Solver  # noqa: E402
from sparknet_amd.data.prefetch import DeviceFeeder, SyntheticSource  # noqa: E402
from sparknet_amd.engine import LocalSGDTrainer, fuse_input_fold, fuse_relu  # noqa: E402
from sparknet_amd.ops import _lib  # noqa: E402

_lib.kernels()
dev = torch.device("cuda", 0)
B, C, HW, crop, classes, mean, sc = bench.DEFAULTS["caffenet"]
solver = Solver(models.solver_for("caffenet", train_batch=B, test_batch=50, crop=crop), device=dev, seed=1701,
                build_test_nets=False)
fuse_relu(solver.net)
feeder = DeviceFeeder(SyntheticSource(B, C, HW, HW, classes=classes, pool=3, seed=0), solver.net.blob_by_name("data"),
                      solver.net.blob_by_name("label"), crop=crop, mean=mean, scale=sc, mirror=True, train=True,
                      rng_state=solver.net.ctx.rng_state, device=dev,
                      group=int(os.environ.get("GROUP", "2")))
fuse_input_fold(solver.net, feeder)
tr = LocalSGDTrainer(solver, None, tau=50, feeder=feeder, use_graph=True)
for _ in range(20):
    tr.local_step()
torch.cuda.synchronize()
fine = []
for c in range(15):  # the ramp in 10-step slices
    t = time.perf_counter()
    for _ in range(10):
        tr.local_step()
    torch.cuda.synchronize()
    fine.append(B * 10 / (time.perf_counter() - t))
print("10-step slices img/s:", " ".join(f"{v / 1e3:.0f}k" for v in fine), flush=True)
if os.environ.get("SPIN"):
    torch.cuda._sleep(int(float(os.environ["SPIN"]) * 2.0e9))
    torch.cuda.synchronize()
if os.environ.get("NOFEED"):  # replay without the per-step H2D minibatch copies (timing only)
    tr.step_fn.pre = None
f = tr.feeder
mode = os.environ.get("FEED", "")
if mode == "nocopy":  # augment from the staged slots every step, no new H2D copy
    def _pf():
        f._pending = f.k % len(f.slots)
        f.events[f._pending] = None
        f.k += 1
    f.prefetch = _pf
elif mode == "samestream":  # the copy on the compute stream itself (no cross-stream events)
    def _pf():
        x, y = f.source.next_batch()
        slot = f.k % len(f.slots)
        dx, dy = f.slots[slot]
        dx.copy_(x, non_blocking=True)
        dy.copy_(y, non_blocking=True)
        f.events[slot] = None
        f._pending = slot
        f.k += 1
    f.prefetch = _pf
# GPU-side timing of 10-step slices inside one long un-synchronised run
evs = [torch.cuda.Event(enable_timing=True) for _ in range(31)]
evs[0].record()
for c in range(30):
    for _ in range(10):
        tr.local_step()
    evs[c + 1].record()
torch.cuda.synchronize()
print("in-stream 10-step slices img/s:",
      " ".join(f"{B * 10 / (evs[c].elapsed_time(evs[c + 1]) / 1e3) / 1e3:.0f}k" for c in range(30)), flush=True)
out = []
for c in range(10):
    t = time.perf_counter()
    for _ in range(100):
        tr.local_step()
    torch.cuda.synchronize()
    out.append(B * 100 / (time.perf_counter() - t))
print("chunks img/s:", " ".join(f"{v / 1e3:.1f}k" for v in out), flush=True)
