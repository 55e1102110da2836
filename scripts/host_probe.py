import os, sys, time
sys.path.insert(0, os.getcwd())
import torch
from sparknet_amd import models
from sparknet_amd.core.solver import Solver
from sparknet_amd.data.prefetch import DeviceFeeder, SyntheticSource
from sparknet_amd.engine import LocalSGDTrainer, fuse_input_fold, fuse_relu
from sparknet_amd.ops import _lib
_lib.kernels()
dev = torch.device("cuda", 0)
sp = models.solver_for("caffenet", train_batch=256, test_batch=50, crop=227)
solver = Solver(sp, device=dev, seed=1701, build_test_nets=False)
net = solver.net
fuse_relu(net)
src = SyntheticSource(256, 3, 256, 256, classes=1000, pool=3, seed=0)
feeder = DeviceFeeder(src, net.blob_by_name("data"), net.blob_by_name("label"), crop=227, mean=[104.0, 117.0, 123.0], mirror=True, train=True, rng_state=net.ctx.rng_state, device=dev)
fuse_input_fold(net, feeder)
tr = LocalSGDTrainer(solver, None, tau=50, feeder=feeder)
for _ in range(5): tr.local_step()
torch.cuda.synchronize()
st = tr.step_fn
T = {"pre": 0.0, "hyper": 0.0, "replay": 0.0}
N = 100
t0 = time.perf_counter()
for _ in range(N):
    a = time.perf_counter(); st.pre(); b = time.perf_counter(); solver.stage_hyper(); c = time.perf_counter(); st.graph.replay(); solver.iter += 1; d = time.perf_counter()
    T["pre"] += b - a; T["hyper"] += c - b; T["replay"] += d - c
t1 = time.perf_counter()
torch.cuda.synchronize()
t2 = time.perf_counter()
print({k: round(v / N * 1e3, 3) for k, v in T.items()}, "host ms/step", round((t1 - t0) / N * 1e3, 3), "total ms/step", round((t2 - t0) / N * 1e3, 3))
