"""Bisect the thin-tile (21 / 22) cifar10_quick learning failure.

python scripts/dbg_thin.py graph|eager [only=<M>x<N>x<K>] [tile=21|22]
Trains cifar10_quick 300 steps exactly as tests/test_training_gpu.py does, with the thin
tiles offered to the first-call tuner (SN_GEMM_THIN=1) for every M <= 64 product, or only
for the one product named by only=, and prints every tuning decision and the loss curve."""
import os
import sys

os.environ.setdefault("SN_GEMM_THIN", "1")
os.environ.setdefault("SN_GEMM_TUNE_LOG", "1")
sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), ".."))

import torch  # noqa: E402

from sparknet_amd import models  # noqa: E402
from sparknet_amd.ops import gemm as G  # noqa: E402

args = dict(a.split("=", 1) for a in sys.argv[2:] if "=" in a)
only = args.get("only")
force = int(args.get("tile", "-1"))
_orig = G._candidates


def cands(M, N, K, groups, b_kc_dense, epi):
    out = _orig(M, N, K, groups, b_kc_dense, epi)
    name = f"{M}x{N}x{K}"
    if only is not None and name != only:
        out = [c for c in out if c[0] not in (21, 22)]
    if force >= 0 and (only is None or name == only) and M <= 64:
        keep = [c for c in out if c[0] == force]
        out = keep or out
    return out


G._candidates = cands
# cfg=MxNxK:tile:splits forces that product's tile / split-K (summation-order experiments)
forced = {}
for item in args.get("cfg", "").split(","):
    if item:
        name, t, sp = item.split(":")
        forced[name] = (int(t), int(sp))
_raw = G._tuned_config_raw


def raw(M, N, K, *a, **k):
    f = forced.get(f"{M}x{N}x{K}")
    if f is not None:
        kc = -(-(-(-K // f[1])) // 64) * 64
        print(f"[forced] {M}x{N}x{K} -> tile {f[0]} splits {-(-K // kc)} kchunk {kc}", flush=True)
        return (f[0], -(-K // kc), kc)
    return _raw(M, N, K, *a, **k)


G._tuned_config_raw = raw
sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "tests"))
from test_training_gpu import _patterns  # noqa: E402

from sparknet_amd.core.solver import Solver  # noqa: E402
from sparknet_amd.data.prefetch import DeviceFeeder, TensorSource  # noqa: E402
from sparknet_amd.engine import LocalSGDTrainer, fuse_relu  # noqa: E402

gpu = torch.device("cuda:0")
mean = [125.0, 123.0, 114.0]
x, y = _patterns(2000)
sp = models.solver_for("cifar10_quick", train_batch=100, test_batch=100)
if "lr" in args:
    sp.base_lr = float(args["lr"])
solver = Solver(sp, device=gpu, seed=int(args.get("seed", "5")),
                build_test_nets=False)
net = solver.net
fuse_relu(net)
feeder = DeviceFeeder(TensorSource(x, y, 100), net.blob_by_name("data"), net.blob_by_name("label"), crop=32,
                      mean=mean, mirror=False, train=True, rng_state=net.ctx.rng_state, device=gpu)
trainer = LocalSGDTrainer(solver, None, tau=50, feeder=feeder, use_graph=sys.argv[1] == "graph")
losses = [float(trainer.local_step()) for _ in range(300)]
torch.cuda.synchronize()
print(" ".join(sys.argv[1:]), "losses", " ".join(f"{losses[i]:.3f}" for i in range(0, 300, 25)),
      "max after 100:", f"{max(losses[100:]):.3f}", f"final {losses[-1]:.3f}",
      "OK" if losses[-1] < 0.5 * losses[0] else "FAIL", flush=True)
