"""fp8 training fidelity over a whole convergence: VGG-16 trained to
convergence on the production path (GraphStep hipGraph, fused ReLU, e4m3 forward, data-gradient
AND weight-gradient products with amax-history delayed scaling, engine.enable_fp8(wgrad=True))
against the bf16 run with the same seeds and the same data stream, at lr 0.002 and at 0.005.

Round 6: kernel selection is reproducible (first-call autotuning off; shapes outside the
committed database take the cost-model tile), so both trajectories are deterministic and the
round-5 "bf16alt" chaos floor (bf16 with every GEMM forced onto the 128x128 tile) is identical
to bf16 on these shapes.  The run is long enough for bf16 to converge: on the 10-template task
the smoothed loss leaves the ln(10) plateau after ~240 (lr 0.002) / ~440 (lr 0.005) steps and
ends near 0.002 (profiles/r6_fp8_trajectories.txt).  Gates, per learning rate:

* bf16 converges (some 20-step window below 0.5; the last 100 steps below 0.05);
* fp8 ends within 10 % of bf16: its last-100-step loss is within 0.1 x bf16's loss drop of
  bf16's (fp8 achieves >= 90 % of the drop); and it leaves the plateau within 2x bf16's steps
  (fp8 with e4m3 gradients escapes the plateau later at lr 0.002: 420 vs 240 steps, on time at
  0.005: 460 vs 440).

The data is a learnable synthetic task (no datasets on the box): 10 fixed random class
templates plus Gaussian noise (scripts/fp8_trajectory.py).  The reference trains in fp32 only
(libccaffe/ccaffe.h:3); parity with it is unpinned — the bf16 run is the yardstick, and the
per-parameter one-step gate against the fp32 CPU engine is tests/test_fp8_update_gate_gpu.py."""
import os

import pytest
import torch

pytestmark = pytest.mark.gpu

STEPS, BATCH, CROP, CLASSES, NOISE, WINDOW = 1000, 64, 64, 10, 0.8, 20
# learning rates under test; SN_FP8_FID_LR overrides (e.g. "0.001")
LRS = [float(v) for v in os.environ.get("SN_FP8_FID_LR", "0.002,0.005").split(",")]


def _trajectory(mode, dev, lr):
    from sparknet_amd import models
    from sparknet_amd.core.solver import Solver
    from sparknet_amd.engine import GraphStep, enable_fp8, fuse_relu
    g0 = torch.Generator().manual_seed(11)
    templates = torch.randn(CLASSES, 3, CROP, CROP, generator=g0)
    net_p = models.vgg16(train_batch=BATCH, test_batch=BATCH, crop=CROP, classes=CLASSES)
    sp = models.zoo.vgg16_solver(net_p)
    sp.base_lr = lr
    solver = Solver(sp, device=dev, seed=5, build_test_nets=False)
    fuse_relu(solver.net)
    n8 = enable_fp8(solver.net, 0.0, dgrad=True, wgrad=True) if mode == "fp8" else 0
    g = torch.Generator().manual_seed(12)

    def pre():
        y = torch.randint(0, CLASSES, (BATCH,), generator=g)
        x = templates[y] + NOISE * torch.randn(BATCH, 3, CROP, CROP, generator=g)
        solver.net.blob_by_name("data").set_nchw(x)
        solver.net.blob_by_name("label").set_nchw(y.float().view(-1, 1))
    st = GraphStep(solver, warmup=2, pre=pre, overlap=False)
    losses = [float(st.step()) for _ in range(STEPS)]
    return losses, n8


def _smooth(v):
    return [sum(v[i:i + WINDOW]) / WINDOW for i in range(0, len(v) - WINDOW + 1, WINDOW)]


def _first_below(sm, v):
    return next((i for i, x in enumerate(sm) if x < v), None)


@pytest.mark.timeout(900)
@pytest.mark.parametrize("lr", LRS)
def test_fp8_vgg16_converges_like_bf16(gpu, monkeypatch, lr):
    from sparknet_amd.ops import gemm as G
    monkeypatch.setattr(G, "_AUTOTUNE", False)  # deterministic kernel selection
    bf, _ = _trajectory("bf16", gpu, lr)
    f8, n8 = _trajectory("fp8", gpu, lr)
    assert n8 >= 30, n8  # forward, data-gradient and weight-gradient products run fp8
    assert all(v == v for v in f8), "fp8 loss went non-finite"
    sb, s8 = _smooth(bf), _smooth(f8)
    end_b, end_8 = sum(bf[-100:]) / 100, sum(f8[-100:]) / 100
    cb, c8 = _first_below(sb, 0.5), _first_below(s8, 0.5)
    print(f"lr {lr}\nbf16 ", [round(v, 4) for v in sb], "\nfp8  ", [round(v, 4) for v in s8],
          f"\nplateau left at step bf16 {None if cb is None else cb * WINDOW} fp8 {None if c8 is None else c8 * WINDOW}"
          f"; last-100 loss bf16 {end_b:.4f} fp8 {end_8:.4f}")
    assert cb is not None and end_b < 0.05, (sb, end_b)  # the yardstick converges
    drop = sb[0] - end_b
    assert end_8 <= end_b + 0.1 * drop, (end_8, end_b, drop)
    assert c8 is not None and c8 <= 2 * max(cb, 1), (c8, cb)
