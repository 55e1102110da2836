"""Correctness gate at the HEADLINE bench's exact configuration.

bench.py's CaffeNet step: the packaged prototxt at per-GPU batch 256, crop 227, 1000 outputs,
fused ReLU epilogues, the augment kernel writing conv1's space-to-depth-folded input, the
InnerProduct SGD updates inside the weight-gradient GEMMs (EPI_SGD), Dropout inside the fc6 /
fc7 epilogues, and the tuned GEMM database's tiles / split-K factors (e.g. fc6 forward split 8,
conv1's folded weight gradient split 109) — fed a learnable uint8 set instead of noise so the
loss moves.  The reference is the fp32 CPU engine from the same initial weights, fed the same
batches, cropped / mirrored / dropped by the same Philox draws.

* one iteration: every layer's weight and bias UPDATE (w1 - w0, i.e. -lr x gradient at zero
  momentum history) against the fp32 engine's, as the largest deviation relative to the
  layer's largest fp32 update AND as the relative L2 norm of the deviation, each within
  max(2 %, 1.5 x the bf16 floor of that layer).  The floor is measured in the fixture: the
  CPU engine run with bf16 storage (the GPU's activation / gradient / weight-copy rounding
  points, on the fp32 CPU kernels) against the fp32 engine.  At this initialisation the
  input layers' gradients are sums of nearly cancelling terms, so bf16 storage alone moves
  conv1's update by ~15 % (max) / ~11 % (L2) and conv2's by ~7 %; the fc layers' L2 floors
  are < 1 %, so there the 2 % bound applies;
* the production hipGraph path for 20 steps: its per-iteration losses track the fp32 engine
  within 4 % over the iterations both ran, and the loss falls;
* the gate has teeth: with conv1's weight-gradient product made to drop half its reduction
  (a simulated split-K bug) the update check fails on conv1 and only there.

Reference: caffe/src/caffe/test/test_gradient_based_solver.cpp:225-320 (update of one
iteration vs a reference computed independently)."""
import math

import pytest
import torch

from sparknet_amd import models

pytestmark = pytest.mark.gpu

B, SRC, CLASSES = 256, 256, 10
MEAN = [104.0, 117.0, 123.0]


def _data(n=2 * B, seed=0):
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


def _solver_param():
    return models.solver_for("caffenet", train_batch=B, test_batch=50, crop=227)  # bench.py's config


def _trainer(dev, w0, x, y, graph, dtype=None):
    from sparknet_amd.core.solver import Solver
    from sparknet_amd.data.prefetch import DeviceFeeder, TensorSource
    from sparknet_amd.engine import LocalSGDTrainer, fuse_fc_updates, fuse_input_fold, fuse_relu
    solver = Solver(_solver_param(), device=dev, seed=1701, build_test_nets=False, dtype=dtype)
    net = solver.net
    net.flat_data.copy_(w0.to(net.flat_data.device))
    net.sync_compute()
    cuda = dev.type == "cuda"
    if cuda:
        fuse_relu(net)
    feeder = DeviceFeeder(TensorSource(x, y, B, pin=cuda), net.blob_by_name("data"), net.blob_by_name("label"),
                          crop=227, mean=MEAN, mirror=True, train=True, rng_state=net.ctx.rng_state, device=dev,
                          group=2 if cuda else 1)
    if cuda:
        assert fuse_input_fold(net, feeder)
    tr = LocalSGDTrainer(solver, None, tau=1000, feeder=feeder, use_graph=graph)
    if cuda and not graph:
        assert fuse_fc_updates(solver) > 0  # the eager step runs the graph's EPI_SGD kernels
    return tr, solver


def _initial_weights():
    from sparknet_amd.core.solver import Solver
    return Solver(_solver_param(), device=torch.device("cpu"), seed=1701,
                  build_test_nets=False).net.flat_data.detach().clone()


def _updates(solver, w0):
    """{layer/param: w1 - w0} of every learnable parameter after the iterations run."""
    w1 = solver.net.flat_data.detach().float().cpu()
    out = {}
    for li, layer in enumerate(solver.net.layers):
        for pi, p in enumerate(layer.params):
            if p.owner is None and p.count:
                out[f"{layer.name}/{pi}"] = (w1[p.offset:p.offset + p.count] - w0[p.offset:p.offset + p.count])
    return out


def _one_step_updates(dev, w0, x, y, dtype=None):
    tr, solver = _trainer(dev, w0, x, y, graph=False, dtype=dtype)
    tr.local_step()
    if dev.type == "cuda":
        torch.cuda.synchronize()
    return _updates(solver, w0)


def _errs(u, uc):
    """{param: (max deviation / max |fp32 update|, ||deviation|| / ||fp32 update||)}"""
    return {k: (float((u[k] - c).abs().max() / (c.abs().max() + 1e-12)),
                float((u[k] - c).norm() / (c.norm() + 1e-12))) for k, c in uc.items()}


def _violations(ug, uc, floor):
    """Parameters whose GPU deviation exceeds max(2 %, 1.5 x the bf16 floor), per metric."""
    bad = []
    for k, (emax, el2) in _errs(ug, uc).items():
        fmax, fl2 = floor[k]
        if emax > max(0.02, 1.5 * fmax) or el2 > max(0.02, 1.5 * fl2):
            bad.append((k, round(emax, 4), round(el2, 4), round(fmax, 4), round(fl2, 4)))
    return bad


@pytest.fixture(scope="module")
def fixture_data():
    x, y = _data()
    w0 = _initial_weights()
    uc = _one_step_updates(torch.device("cpu"), w0, x, y)
    floor = _errs(_one_step_updates(torch.device("cpu"), w0, x, y, dtype=torch.bfloat16), uc)
    return x, y, w0, uc, floor


@pytest.mark.timeout(900)
def test_bench_config_one_step_updates_match_fp32(gpu, fixture_data):
    x, y, w0, uc, floor = fixture_data
    ug = _one_step_updates(torch.device(gpu), w0, x, y)
    assert ug.keys() == uc.keys() and len(uc) == 16  # 8 learnable layers x (weight, bias)
    print("per-parameter (max, L2) deviation vs fp32 / bf16 floor:",
          {k: (round(a, 4), round(b, 4), round(floor[k][0], 4), round(floor[k][1], 4))
           for k, (a, b) in _errs(ug, uc).items()})
    assert not _violations(ug, uc, floor)


@pytest.mark.timeout(900)
def test_bench_config_gate_catches_a_broken_wgrad(gpu, fixture_data, monkeypatch):
    """Half of conv1's weight-gradient reduction dropped (split-K chunks past the middle
    skipped) must fail the update gate."""
    from sparknet_amd.ops import gemm as G
    x, y, w0, uc, floor = fixture_data
    orig = G._launch

    def broken(M, N, K, *a, **k):
        if M == 96 and K >= 500000:  # conv1's folded weight gradient: 96 x 433 x 774400
            K = K // 2
        return orig(M, N, K, *a, **k)
    monkeypatch.setattr(G, "_launch", broken)
    ug = _one_step_updates(torch.device(gpu), w0, x, y)
    bad = _violations(ug, uc, floor)
    assert bad and all(b[0].startswith("conv1/") for b in bad), bad


@pytest.mark.timeout(900)
def test_bench_config_graph_losses_track_fp32(gpu, fixture_data):
    x, y, w0, _, _ = fixture_data
    tr, solver = _trainer(torch.device(gpu), w0, x, y, graph=True)
    assert tr.step_fn is not None
    gl = [float(tr.local_step())]  # capture call: iterations 0..2, the loss of iteration 2
    while solver.iter < 20:
        gl.append(float(tr.local_step()))
    torch.cuda.synchronize()
    trc, sc = _trainer(torch.device("cpu"), w0, x, y, graph=False)
    cl = [float(trc.local_step()) for _ in range(8)]
    for i, c in enumerate(cl[2:]):  # GPU list index 0 = iteration 2
        assert abs(gl[i] - c) <= 0.04 * max(1.0, abs(c)), (i + 2, gl[i], c, gl, cl)
    assert sum(gl[-5:]) < sum(gl[:5]), gl
