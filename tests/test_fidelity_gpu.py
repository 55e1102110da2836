"""Multi-step fidelity of the HEADLINE training path (bench.py's CaffeNet step).

The GPU run is the production path: LocalSGDTrainer with the whole iteration in one
hipGraph, the grouped H2D feeder with the fused augment + space-to-depth fold of conv1
(engine.fuse_input_fold), fused ReLU epilogues, Dropout ON inside the fc6 / fc7 GEMM
epilogues (Philox), and the InnerProduct SGD update inside the weight-gradient GEMM
(EPI_SGD).  The reference is the fp32 CPU engine fed the same uint8 batches, cropped /
mirrored by the same Philox draw (ops.ref.augment_params) and dropping the same units
(ops.ref dropout shares the Philox stream).

* 60 steps at batch 32 with the full-width fc6 / fc7 (4096): the production tiles, the
  split-K weight gradients and the 4096-wide EPI_SGD update tiles are the ones exercised.
  The bf16 GPU loss trajectory stays within 4 % (relative, per 10-step window mean) of the
  fp32 CPU one, and both decrease.
* 10 steps: graph replay and the eager GPU step (same kernels, EPI_SGD included, launched
  one by one) end at the same weights to 1e-5 (relative to the largest weight).

Reference: caffe/src/caffe/layers/dropout_layer.cu:10-45 (train-time mask), the
ImageNetApp crop / mirror / mean transform (src/main/scala/apps/ImageNetApp.scala), and
the CifarSpec-style learning check (src/test/scala/libs/CifarSpec.scala:92).
"""
import math

import pytest
import torch

from sparknet_amd import models

pytestmark = pytest.mark.gpu

B, CLASSES, SRC = 32, 10, 256
MEAN = [104.0, 117.0, 123.0]


def _data(n=256, seed=0):
    """Learnable uint8 256x256 images: class colour + oriented stripes + noise."""
    g = torch.Generator().manual_seed(seed)
    y = torch.randint(0, CLASSES, (n,), generator=g)
    yy, xx = torch.meshgrid(torch.arange(float(SRC)), torch.arange(float(SRC)), indexing="ij")
    imgs = torch.empty(n, 3, SRC, SRC)
    for c in range(CLASSES):
        idx = (y == c).nonzero().flatten()
        th = math.pi * c / CLASSES
        stripes = 50.0 * torch.sin(2 * math.pi * 6 * (xx * math.cos(th) + yy * math.sin(th)) / SRC)
        for ch in range(3):
            imgs[idx, ch] = 128 + 60 * math.cos(2 * math.pi * c / CLASSES + 2.1 * ch) + stripes
    imgs += torch.randn(imgs.shape, generator=g) * 12
    return imgs.clamp(0, 255).to(torch.uint8), y.int()


def _net():
    return models.caffenet(train_batch=B, test_batch=B, crop=227, classes=CLASSES)  # fc6 / fc7: 4096 wide


def _trainer(dev, w0, x, y, graph):
    from sparknet_amd.core.solver import Solver
    from sparknet_amd.data.prefetch import DeviceFeeder, TensorSource
    from sparknet_amd.engine import LocalSGDTrainer, fuse_input_fold, fuse_relu
    sp = models.zoo.caffenet_solver(_net())
    sp.base_lr = 0.005
    solver = Solver(sp, device=dev, seed=21, build_test_nets=False)
    net = solver.net
    net.flat_data.copy_(w0.to(net.flat_data.device))
    net.sync_compute()
    fold = False
    if dev.type == "cuda":
        fuse_relu(net)
    feeder = DeviceFeeder(TensorSource(x, y, B, pin=dev.type == "cuda"), net.blob_by_name("data"),
                          net.blob_by_name("label"), crop=227, mean=MEAN, mirror=True, train=True,
                          rng_state=net.ctx.rng_state, device=dev, group=2 if dev.type == "cuda" else 1)
    if dev.type == "cuda":
        fold = fuse_input_fold(net, feeder)
    tr = LocalSGDTrainer(solver, None, tau=1000, feeder=feeder, use_graph=graph)
    if dev.type == "cuda" and not graph:
        from sparknet_amd.engine import fuse_fc_updates
        fuse_fc_updates(solver)  # the eager GPU step runs the same EPI_SGD kernels as the graph
    return tr, solver, fold


def _initial_weights():
    from sparknet_amd.core.solver import Solver
    s = Solver(models.zoo.caffenet_solver(_net()), device=torch.device("cpu"), seed=21, build_test_nets=False)
    return s.net.flat_data.detach().clone()


@pytest.mark.timeout(900)
def test_caffenet_production_path_tracks_fp32_cpu(gpu):
    x, y = _data()
    w0 = _initial_weights()
    tr, solver, fold = _trainer(torch.device(gpu), w0, x, y, graph=True)
    assert fold and tr.step_fn is not None
    gl = [float(tr.local_step()) for _ in range(20)]  # the first call captures (3 iterations)
    steps = solver.iter
    while solver.iter < 60:
        gl.append(float(tr.local_step()))
    steps = solver.iter
    torch.cuda.synchronize()
    # per-iteration GPU losses: the capture call covered iterations 0..2 (its loss = the replay's)
    trc, sc, _ = _trainer(torch.device("cpu"), w0, x, y, graph=False)
    cl = []
    for _ in range(steps):
        cl.append(float(trc.local_step()))
    cl_aligned = [cl[2]] + cl[3:]  # GPU list: [iter 2 (capture call), iter 3, ...]
    assert len(cl_aligned) == len(gl)
    for w in range(0, len(gl) - 9, 10):
        a = sum(cl_aligned[w:w + 10]) / 10
        b = sum(gl[w:w + 10]) / 10
        assert abs(a - b) <= 0.04 * max(1.0, abs(a)), (w, a, b, cl_aligned, gl)
    assert sum(gl[-10:]) < sum(gl[:10]) and sum(cl_aligned[-10:]) < sum(cl_aligned[:10]), (cl_aligned, gl)


@pytest.mark.timeout(300)
def test_caffenet_graph_replay_matches_eager_gpu(gpu):
    x, y = _data()
    w0 = _initial_weights()
    out = []
    for graph in (True, False):
        tr, solver, _ = _trainer(torch.device(gpu), w0, x, y, graph=graph)
        while solver.iter < 10:
            tr.local_step()
        torch.cuda.synchronize()
        out.append(solver.net.flat_data.detach().clone())
    scale = out[1].abs().max().item()
    assert (out[0] - out[1]).abs().max().item() <= 1e-5 * scale
