"""Multi-step bf16 training fidelity on the MI355X.

* cifar10_quick trained through the production path (captured hipGraph, device feeder:
  pinned H2D + on-device mean subtraction, fused ReLU / FC updates) on a learnable
  synthetic set reaches >= 90 % train accuracy in 300 steps, with the loss bounded after
  step 100, under two fp32 summation orders of conv1's weight gradient (the tuned split-K,
  and 229-way split-K on the 64-row tile 22).  Reference analogue: the CifarApp accuracy
  check (src/test/scala/libs/CifarSpec.scala:92 brackets the accuracy of an untrained net
  around chance; a trained one must leave that bracket).
  The solver runs at base_lr 0.0005, half the reference cifar10_quick rate: on this
  trivially separable set the loss collapses to ~0 and training at lr 0.001 spikes (to
  5-17) under EVERY summation order — the fp32 CPU engine too (scripts/
  cifar_quick_cpu_traj.py) — so whether step 300 lands inside a spike was a coin flip on
  the split count (round-4 'thin tile' report; profiles/r5_cifar_stability.txt).
  Learning parity at the reference rate (base_lr 0.001) is therefore UNPINNED by this
  test; what it pins is learning at half that rate under both summation orders.
* A 20-step loss trajectory of a small CaffeNet (dropout 0) on the bf16 GPU engine stays
  within 5 % (relative) of the fp32 CPU engine from identical initial weights, and both
  decrease.
"""
import math

import pytest
import torch

from sparknet_amd import models

pytestmark = pytest.mark.gpu


def _patterns(n, classes=10, seed=0):
    """Class-dependent colour + oriented stripe texture + noise, uint8 NCHW 3x32x32."""
    g = torch.Generator().manual_seed(seed)
    y = torch.randint(0, classes, (n,), generator=g)
    yy, xx = torch.meshgrid(torch.arange(32.0), torch.arange(32.0), indexing="ij")
    imgs = torch.empty(n, 3, 32, 32)
    for c in range(classes):
        idx = (y == c).nonzero().flatten()
        th = math.pi * c / classes
        stripes = 40.0 * torch.sin(2 * math.pi * 3 * (xx * math.cos(th) + yy * math.sin(th)) / 32)
        for ch in range(3):
            base = 128 + 60 * math.cos(2 * math.pi * c / classes + 2.1 * ch)
            imgs[idx, ch] = base + stripes
    imgs += torch.randn(imgs.shape, generator=g) * 15
    return imgs.clamp(0, 255).to(torch.uint8), y.int()


@pytest.mark.parametrize("order", ["tuned", "thin229"])
def test_cifar10_quick_learns_synthetic_patterns(gpu, order, monkeypatch):
    """cifar10_quick learns the synthetic patterns through the captured-graph local-SGD path,
    with the tuned kernels and with conv1's weight gradient forced onto the 64-row tile at 229
    splits.  It trains at base_lr 0.0005, HALF the reference solver's 0.001: on this synthetic
    set the reference rate is chaotic under every summation order, the fp32 CPU engine's
    included (profiles/r5_cifar_stability.txt), so parity at the reference rate is unpinned
    here; tests/test_bench_fidelity_gpu.py pins the per-parameter update instead."""
    from sparknet_amd.core.solver import Solver
    from sparknet_amd.data.prefetch import DeviceFeeder, TensorSource
    from sparknet_amd.engine import LocalSGDTrainer, fuse_relu
    from sparknet_amd.ops import gemm as G
    if order == "thin229":
        raw = G._tuned_config_raw

        def forced(M, N, K, *a, **k):
            if (M, N, K) == (32, 201, 102400):  # conv1 dW + bias column over 100 x 32 x 32 pixels
                return (22, 229, 448)
            return raw(M, N, K, *a, **k)
        monkeypatch.setattr(G, "_tuned_config_raw", forced)
    mean = [125.0, 123.0, 114.0]
    x, y = _patterns(2000)
    sp = models.solver_for("cifar10_quick", train_batch=100, test_batch=100)
    sp.base_lr = 0.0005
    solver = Solver(sp, device=gpu, seed=5, build_test_nets=False)
    net = solver.net
    fuse_relu(net)
    feeder = DeviceFeeder(TensorSource(x, y, 100), net.blob_by_name("data"), net.blob_by_name("label"), crop=32,
                          mean=mean, mirror=False, train=True, rng_state=net.ctx.rng_state, device=gpu)
    trainer = LocalSGDTrainer(solver, None, tau=50, feeder=feeder, use_graph=True)
    assert trainer.step_fn is not None  # the captured-graph path
    losses = [float(trainer.local_step()) for _ in range(300)]
    torch.cuda.synchronize()
    assert losses[-1] < 0.5 * losses[0], (losses[0], losses[-1])
    assert max(losses[100:]) < 1.0, max(losses[100:])  # no divergence spike once learnt
    # train accuracy: eager forward of the trained net on 5 batches
    correct = total = 0
    m = torch.tensor(mean).view(1, 3, 1, 1)
    for b in range(5):
        xb, yb = x[b * 100:(b + 1) * 100].float() - m, y[b * 100:(b + 1) * 100]
        net.blob_by_name("data").set_nchw(xb)
        net.blob_by_name("label").set_nchw(yb.float().view(-1, 1))
        net.forward()
        logits = net.blob_by_name("ip2").nchw().float().cpu().reshape(100, -1)
        correct += int((logits.argmax(1) == yb.long()).sum())
        total += 100
    acc = correct / total
    assert acc >= 0.9, acc


def _tiny_caffenet():
    n = models.caffenet(train_batch=4, test_batch=4, crop=67, classes=7)
    for l in n.layer:
        if l.type == "Dropout":
            l.dropout_param.dropout_ratio = 0.0
        if l.type == "InnerProduct" and l.name in ("fc6", "fc7"):
            l.inner_product_param.num_output = 64
    return n


def test_caffenet_bf16_gpu_loss_trajectory_matches_fp32_cpu(gpu):
    from sparknet_amd.core.solver import Solver
    from sparknet_amd.engine import fuse_relu
    g = torch.Generator().manual_seed(4)
    batches = [(torch.randn(4, 3, 67, 67, generator=g) * 30, torch.randint(0, 7, (4, 1), generator=g).float())
               for _ in range(2)]
    traj = {}
    w0 = None
    for dev in ("cpu", gpu):
        solver = Solver(models.zoo.caffenet_solver(_tiny_caffenet()), device=torch.device(dev), seed=8,
                        build_test_nets=False)
        net = solver.net
        if w0 is None:
            w0 = net.flat_data.detach().float().cpu().clone()
        else:
            net.flat_data.copy_(w0.to(net.flat_data.device))
            net.sync_compute()
            fuse_relu(net)
        out = []
        for it in range(20):
            xb, yb = batches[it % 2]
            net.blob_by_name("data").set_nchw(xb)
            net.blob_by_name("label").set_nchw(yb)
            solver.stage_hyper()
            out.append(float(solver.iteration()))
            solver.iter += 1
        traj[str(dev)] = out
    lc, lg = traj["cpu"], traj[str(gpu)]
    for i, (a, b) in enumerate(zip(lc, lg)):
        assert abs(a - b) <= 0.05 * max(1.0, abs(a)), (i, a, b)
    assert min(lc[-4:]) < lc[0] and min(lg[-4:]) < lg[0], (lc, lg)


def test_grouped_feeder_stages_same_sequence(gpu):
    """DeviceFeeder(group=3) issues its H2D copies three minibatches at a time behind one
    fence pair; the staged data / labels must be the per-step feeder's, step for step."""
    from sparknet_amd.core.solver import Solver
    from sparknet_amd.data.prefetch import DeviceFeeder, TensorSource
    x, y = _patterns(160, seed=3)
    nets, feeders = [], []
    for group in (1, 3):
        solver = Solver(models.solver_for("cifar10_quick", train_batch=10, test_batch=10), device=gpu, seed=5,
                        build_test_nets=False)
        net = solver.net
        feeders.append(DeviceFeeder(TensorSource(x, y, 10), net.blob_by_name("data"), net.blob_by_name("label"),
                                    crop=32, mean=[120.0, 120.0, 120.0], mirror=False, train=False,
                                    rng_state=net.ctx.rng_state, device=gpu, group=group))
        nets.append(net)
    assert feeders[1].group == 3 and len(feeders[1].slots) == 6
    for step in range(11):
        outs = []
        for f, net in zip(feeders, nets):
            f.stage()
            f.prefetch()
            outs.append((net.blob_by_name("data").data.clone(), net.blob_by_name("label").data.clone()))
        torch.cuda.synchronize()
        assert torch.equal(outs[0][0], outs[1][0]), step
        assert torch.equal(outs[0][1], outs[1][1]), step
