"""fp8 training fidelity pinned: >= 200 VGG-16 steps at lr 0.005 on the
production path (GraphStep hipGraph, fused ReLU, e4m3 forward + e4m3 data-gradient
products with amax-history delayed scaling, engine.enable_fp8) against the bf16 run with
the same seeds and the same data stream.  Every 20-step smoothed fp8 loss must stay within
0.15 of bf16's and the run must end below its starting loss.

The data is a learnable synthetic task (no datasets on the box): 10 fixed random class
templates plus Gaussian noise (scripts/fp8_trajectory.py), so the loss falls from ln(10).
The reference trains in fp32 only (libccaffe/ccaffe.h:3); parity with it is unpinned —
the bf16 run is the yardstick."""
import pytest
import torch

pytestmark = pytest.mark.gpu

STEPS, BATCH, CROP, CLASSES, LR, NOISE, WINDOW = 200, 64, 64, 10, 0.005, 0.8, 20


def _trajectory(mode, dev):
    from sparknet_amd import models
    from sparknet_amd.core.solver import Solver
    from sparknet_amd.engine import GraphStep, enable_fp8, fuse_relu
    g0 = torch.Generator().manual_seed(11)
    templates = torch.randn(CLASSES, 3, CROP, CROP, generator=g0)
    net_p = models.vgg16(train_batch=BATCH, test_batch=BATCH, crop=CROP, classes=CLASSES)
    sp = models.zoo.vgg16_solver(net_p)
    sp.base_lr = LR
    solver = Solver(sp, device=dev, seed=5, build_test_nets=False)
    fuse_relu(solver.net)
    n8 = enable_fp8(solver.net, 0.0, dgrad=True) if mode == "fp8" else 0
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


@pytest.mark.timeout(600)
def test_fp8_vgg16_200_steps_tracks_bf16(gpu):
    bf, _ = _trajectory("bf16", gpu)
    f8, n8 = _trajectory("fp8", gpu)
    assert n8 >= 20, n8  # forward + data-gradient products actually run e4m3
    sb, s8 = _smooth(bf), _smooth(f8)
    dev = [abs(a - b) for a, b in zip(sb, s8)]
    print("bf16", [round(v, 3) for v in sb], "\nfp8 ", [round(v, 3) for v in s8], "\nmax dev", max(dev))
    assert all(v == v for v in f8), "fp8 loss went non-finite"
    assert max(dev) <= 0.15, (max(dev), sb, s8)
    assert s8[-1] < s8[0], (s8[0], s8[-1])
