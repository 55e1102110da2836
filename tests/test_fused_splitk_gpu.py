"""Convolution weight gradients consumed as split-K slabs by the solver update
(engine.fuse_splitk_updates): the captured CaffeNet step must give bitwise the same
weights as the same step with a splitk_reduce launch + flat-gradient update, and no
splitk_reduce may run after a fused conv wgrad.  Reference semantics: SGDSolver
ComputeUpdateValue + Blob::Update (caffe/src/caffe/solvers/sgd_solver.cpp:207-239,
caffe/src/caffe/blob.cpp:154-176) on the summed gradient."""
import pytest
import torch

from sparknet_amd import models

pytestmark = pytest.mark.gpu


def _solver(dev, batch=32):
    from sparknet_amd.core.solver import Solver
    from sparknet_amd.engine import fuse_relu
    n = models.caffenet(train_batch=batch, test_batch=batch, crop=227, classes=10)
    for l in n.layer:
        if l.type == "InnerProduct" and l.name in ("fc6", "fc7"):
            l.inner_product_param.num_output = 256
    sp = models.zoo.caffenet_solver(n)
    sp.base_lr = 1e-3
    solver = Solver(sp, device=dev, seed=5, build_test_nets=False)
    fuse_relu(solver.net)
    return solver


def _run(dev, fuse, monkeypatch, steps=4):
    from sparknet_amd.engine import GraphStep
    monkeypatch.setenv("SN_FEATURES", "fuse_splitk=1" if fuse else "fuse_splitk=0")  # opt-in path
    solver = _solver(dev)
    g = torch.Generator().manual_seed(3)
    batches = iter([(torch.randn(32, 3, 227, 227, generator=g) * 40, torch.randint(0, 10, (32, 1), generator=g).float())
                    for _ in range(steps + 4)])

    def pre():
        x, y = next(batches)
        solver.net.blob_by_name("data").set_nchw(x)
        solver.net.blob_by_name("label").set_nchw(y)
    step = GraphStep(solver, warmup=2, pre=pre, overlap=False, fuse_fc=True)
    for _ in range(steps):
        step.step()
    torch.cuda.synchronize()
    sinks = [getattr(l, "slab_grad", None) for l in solver.net.layers]
    sinks = [s for s in sinks if s is not None]
    return solver.net.flat_data.detach().clone(), sinks


def test_splitk_slabs_consumed_by_solver_bitwise(gpu, monkeypatch):
    ref, none = _run(gpu, False, monkeypatch)
    assert none == []
    got, sinks = _run(gpu, True, monkeypatch)
    assert len(sinks) >= 3  # conv2-conv5 (conv1 reads the space-to-depth folded input)
    assert sum(s.desc is not None for s in sinks) >= 2, "expected split-K conv weight gradients"
    assert torch.isfinite(got).all()
    assert torch.equal(got, ref)
