"""Chunk-table size and isolated time of the fused solver update for a bench model
(GPU): python scripts/solver_probe.py googlenet"""
import sys
import time

import torch

from sparknet_amd import models
from sparknet_amd.core.solver import Solver
from sparknet_amd.engine import fuse_fc_updates, fuse_relu

model = sys.argv[1] if len(sys.argv) > 1 else "googlenet"
dev = torch.device("cuda", 0)
sp = models.solver_for(model, train_batch=8, test_batch=8, crop=224 if model != "caffenet" else 227)
s = Solver(sp, device=dev, seed=1, build_test_nets=False)
fuse_relu(s.net)
print("segments", len(s.net.param_segments()), "params", s.net.num_param_elems)
print("table chunks before fc fusion", s._tables["n"])
print("fused fc layers", fuse_fc_updates(s))
print("table chunks", s._tables["n"])
for _ in range(3):
    s.update_params_segments(s._tables) if hasattr(s, "update_params_segments") else None
torch.cuda.synchronize()
t = time.perf_counter()
for _ in range(50):
    s.update_params_segments(s._tables)
torch.cuda.synchronize()
print(f"update: {(time.perf_counter() - t) / 50 * 1e6:.1f} us per call")
