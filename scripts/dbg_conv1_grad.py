"""Diagnose the conv1 update mismatch of tests/test_bench_fidelity_gpu.py at the bench config:
one step on the fp32 CPU engine vs the GPU engine with / without the fused augment + fold,
per-layer update errors, the augmented input blob, and conv1's weight gradient at other
split-K factors."""
import os
import sys

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), ".."))
sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "tests"))
import torch  # noqa: E402

import test_bench_fidelity_gpu as T  # noqa: E402
from sparknet_amd.core.solver import Solver  # noqa: E402
from sparknet_amd.data.prefetch import DeviceFeeder, TensorSource  # noqa: E402
from sparknet_amd.engine import LocalSGDTrainer, fuse_fc_updates, fuse_input_fold, fuse_relu  # noqa: E402


def run(dev, w0, x, y, fold=True, fuse=True, dtype=None):
    solver = Solver(T._solver_param(), device=dev, seed=1701, build_test_nets=False, dtype=dtype)
    net = solver.net
    net.flat_data.copy_(w0.to(net.flat_data.device))
    net.sync_compute()
    cuda = dev.type == "cuda"
    if cuda and fuse:
        fuse_relu(net)
    feeder = DeviceFeeder(TensorSource(x, y, T.B, pin=cuda), net.blob_by_name("data"), net.blob_by_name("label"),
                          crop=227, mean=T.MEAN, mirror=True, train=True, rng_state=net.ctx.rng_state, device=dev,
                          group=2 if cuda else 1)
    if cuda and fold:
        assert fuse_input_fold(net, feeder)
    tr = LocalSGDTrainer(solver, None, tau=1000, feeder=feeder, use_graph=False)
    if cuda and fuse:
        fuse_fc_updates(solver)
    loss = float(tr.local_step())
    if cuda:
        torch.cuda.synchronize()
    data = net.blob_by_name("data").nchw().float().cpu().clone()
    return loss, T._updates(solver, w0), data


x, y = T._data()
w0 = T._initial_weights()
lc, uc, dc = run(torch.device("cpu"), w0, x, y)
print("cpu loss", lc, flush=True)
lb, ub, db_ = run(torch.device("cpu"), w0, x, y, dtype=torch.bfloat16)
errs = sorted(((float((ub[k] - v).abs().max() / (v.abs().max() + 1e-12)), k) for k, v in uc.items()), reverse=True)
print("cpu bf16 vs cpu fp32: loss", lb, "worst:", [(k, round(e, 4)) for e, k in errs[:6]], flush=True)
gpu = torch.device("cuda:0")
for name, kw in [("fold+fuse", {}), ("no fold", {"fold": False}), ("no fold, no fusion", {"fold": False, "fuse": False})]:
    lg, ug, dg = run(gpu, w0, x, y, **kw)
    errs = sorted(((float((ug[k] - v).abs().max() / (v.abs().max() + 1e-12)), k) for k, v in ub.items()),
                  reverse=True)
    print(f"{name:22s} vs cpu bf16 worst:", [(k, round(e, 4)) for e, k in errs[:5]], flush=True)
    errs = sorted(((float((ug[k] - v).abs().max() / (v.abs().max() + 1e-12)), k) for k, v in uc.items()), reverse=True)
    derr = float((dg - dc).abs().max()) if not kw.get("fold", True) or True else -1
    print(f"{name:22s} loss {lg:.4f}  data max|d| {derr:.3f}  worst:", [(k, round(e, 4)) for e, k in errs[:5]],
          flush=True)
    k = "conv1/0"
    d = (ug[k] - uc[k]).reshape(96, -1)
    print("   conv1/0 per-filter max err / global max:", [round(float(v), 3) for v in
                                                          (d.abs().max(1).values / uc[k].abs().max())[:12]], flush=True)
