"""Analytic solver tests (pattern of caffe/src/caffe/test/test_gradient_based_solver.cpp:
least-squares net = DummyData + InnerProduct + EuclideanLoss, each solver's update
checked against a closed-form update computed independently here), LR policies,
iter_size accumulation, snapshot/restore equivalence."""
import math
import os

import pytest
import torch

from sparknet_amd import proto
from sparknet_amd.core.solver import Solver

N, D = 4, 3


def lsq_solver(typ="SGD", **kw):
    net = proto.parse_prototxt(f"""
      name: "lsq"
      layer {{ name: "data" type: "DummyData" top: "data" top: "targets"
        dummy_data_param {{ shape {{ dim: {N} dim: {D} }} shape {{ dim: {N} dim: 1 }}
          data_filler {{ type: "gaussian" std: 1.0 }} data_filler {{ type: "gaussian" std: 1.0 }} }} }}
      layer {{ name: "ip" type: "InnerProduct" bottom: "data" top: "ip"
        inner_product_param {{ num_output: 1 weight_filler {{ type: "gaussian" std: 1.0 }}
                               bias_filler {{ type: "gaussian" std: 1.0 }} }} }}
      layer {{ name: "loss" type: "EuclideanLoss" bottom: "ip" bottom: "targets" top: "loss" }}
    """)
    sp = proto.SolverParameter(type=typ, base_lr=kw.pop("base_lr", 0.1), lr_policy=kw.pop("lr_policy", "fixed"))
    sp.net_param.CopyFrom(net)
    for k, v in kw.items():
        setattr(sp, k, v)
    return Solver(sp, device="cpu", seed=7)


def _fixed_data(s):
    """Freeze the DummyData outputs (gaussian fillers refill every forward)."""
    layer = s.net.layer_by_name("data")
    g = torch.Generator().manual_seed(11)
    X = torch.randn(N, D, generator=g)
    Y = torch.randn(N, 1, generator=g)
    layer.refill = [False, False]
    layer._filled = True
    s.net.blob_by_name("data").data.copy_(X)
    s.net.blob_by_name("targets").data.copy_(Y)
    layer.forward = lambda b, t: None
    return X.double(), Y.double()


def _grad(w, b, X, Y):
    r = X @ w.t() + b - Y  # [N,1]
    return (r.t() @ X) / N, r.sum(0) / N


@pytest.mark.parametrize("typ", ["SGD", "Nesterov", "AdaGrad", "RMSProp", "AdaDelta", "Adam"])
@pytest.mark.parametrize("wd,reg", [(0.0, "L2"), (0.1, "L2"), (0.1, "L1")])
def test_least_squares_update(typ, wd, reg):
    mom = 0.9 if typ != "RMSProp" else 0.0
    kw = dict(momentum=mom, weight_decay=wd, regularization_type=reg, rms_decay=0.95, delta=1e-6)
    if typ == "AdaGrad":
        kw["momentum"] = 0.0
    s = lsq_solver(typ, **kw)
    X, Y = _fixed_data(s)
    ip = s.net.layer_by_name("ip")
    w = ip.params[0].data.double().clone()
    b = ip.params[1].data.double().clone()
    h = [torch.zeros_like(w), torch.zeros_like(b)]
    h2 = [torch.zeros_like(w), torch.zeros_like(b)]
    lr, m = 0.1, kw["momentum"]
    for it in range(3):
        gw, gb = _grad(w, b, X, Y)
        new = []
        for k, (p, g) in enumerate(((w, gw), (b, gb))):
            lr_mult = 1.0
            decay = wd * 1.0
            g = g + decay * (torch.sign(p) if reg == "L1" else p)
            rate = lr * lr_mult
            if typ == "SGD":
                h[k] = m * h[k] + rate * g
                u = h[k]
            elif typ == "Nesterov":
                prev = h[k].clone()
                h[k] = m * h[k] + rate * g
                u = (1 + m) * h[k] - m * prev
            elif typ == "AdaGrad":
                h[k] = h[k] + g * g
                u = rate * g / (h[k].sqrt() + 1e-6)
            elif typ == "RMSProp":
                h[k] = 0.95 * h[k] + 0.05 * g * g
                u = rate * g / (h[k].sqrt() + 1e-6)
            elif typ == "AdaDelta":
                h[k] = m * h[k] + (1 - m) * g * g
                uu = g * ((h2[k] + 1e-6) / (h[k] + 1e-6)).sqrt()
                h2[k] = m * h2[k] + (1 - m) * uu * uu
                u = rate * uu
            else:
                t = it + 1
                corr = math.sqrt(1 - 0.999 ** t) / (1 - m ** t)
                h[k] = m * h[k] + (1 - m) * g
                h2[k] = 0.999 * h2[k] + 0.001 * g * g
                u = rate * corr * h[k] / (h2[k].sqrt() + 1e-6)
            new.append(p - u)
        w, b = new
        s.step(1)
        assert torch.allclose(ip.params[0].data.double(), w, rtol=1e-4, atol=1e-5), (typ, it)
        assert torch.allclose(ip.params[1].data.double(), b, rtol=1e-4, atol=1e-5), (typ, it)


def test_lr_policies():
    def rate(policy, it, **kw):
        s = lsq_solver("SGD", base_lr=0.5, lr_policy=policy, **kw)
        s.iter = it
        return s.get_learning_rate()
    assert rate("fixed", 10) == pytest.approx(0.5)
    assert rate("step", 25, gamma=0.1, stepsize=10) == pytest.approx(0.5 * 0.01)
    assert rate("exp", 3, gamma=0.9) == pytest.approx(0.5 * 0.9 ** 3)
    assert rate("inv", 100, gamma=1e-4, power=0.75) == pytest.approx(0.5 * (1 + 1e-4 * 100) ** -0.75)
    assert rate("poly", 25, power=2.0, max_iter=100) == pytest.approx(0.5 * 0.75 ** 2)
    assert rate("sigmoid", 12, gamma=0.5, stepsize=10) == pytest.approx(0.5 / (1 + math.exp(-0.5 * 2)), rel=1e-6)
    s = lsq_solver("SGD", base_lr=1.0, lr_policy="multistep", gamma=0.5)
    s.param.stepvalue.extend([2, 4])
    rates = []
    for it in range(6):
        s.iter = it
        rates.append(s.get_learning_rate())
    assert rates == [1.0, 1.0, 0.5, 0.5, 0.25, 0.25]


def test_iter_size_accumulation_equals_large_batch():
    """iter_size=2 with the same data twice == one step with iter_size=1 (normalised)."""
    a = lsq_solver("SGD", momentum=0.9, iter_size=2)
    b = lsq_solver("SGD", momentum=0.9)
    _fixed_data(a)
    _fixed_data(b)
    a.step(2)
    b.step(2)
    assert torch.allclose(a.net.flat_data, b.net.flat_data, rtol=1e-5, atol=1e-6)


def test_clip_gradients():
    s = lsq_solver("SGD", momentum=0.0, clip_gradients=1e-3)
    X, Y = _fixed_data(s)
    ip = s.net.layer_by_name("ip")
    w0, b0 = ip.params[0].data.double().clone(), ip.params[1].data.double().clone()
    gw, gb = _grad(w0, b0, X, Y)
    norm = torch.sqrt((gw ** 2).sum() + (gb ** 2).sum())
    s.step(1)
    scale = 1e-3 / float(norm)
    assert torch.allclose(ip.params[0].data.double(), w0 - 0.1 * gw * scale, atol=1e-6)


def test_snapshot_restore_equivalence(tmp_path):
    a = lsq_solver("SGD", momentum=0.9, snapshot_prefix=str(tmp_path / "lsq"))
    _fixed_data(a)
    a.step(2)
    model, state = a.snapshot()
    assert os.path.exists(model) and os.path.exists(state)
    a.step(3)
    b = lsq_solver("SGD", momentum=0.9)
    _fixed_data(b)
    b.restore(state)
    assert b.iter == 2
    b.step(3)
    assert torch.allclose(a.net.flat_data, b.net.flat_data, atol=1e-6)
    assert torch.allclose(a.history[0], b.history[0], atol=1e-6)


def test_stop_request_ends_solve():
    """A 'stop' action request ends Solve() (solver.cpp:300-310): iter stops advancing
    and no final display / test pass runs."""
    s = lsq_solver(max_iter=100, display=1, test_interval=0)
    calls = []

    def req():
        calls.append(s.iter)
        return "stop" if s.iter >= 5 else "none"

    s.action_request = req
    s.solve()
    assert s.iter == 5
    assert s.requested_early_exit


def test_copy_trained_layers_rejects_same_count_other_shape():
    """Net::CopyTrainedLayersFrom compares shapes (Blob::ShapeEquals), not element counts:
    an InnerProduct weight of the same count but transposed shape must be refused, while
    a legacy 4-D blob with leading 1s is accepted."""
    a = lsq_solver()
    src = a.net.to_proto()
    w = a.net.layer_by_name("ip").params[0].to_caffe()   # [1, D]
    lp = [l for l in src.layer if l.name == "ip"][0]
    del lp.blobs[0].shape.dim[:]
    lp.blobs[0].shape.dim.extend([D, 1])                  # same count, transposed
    with pytest.raises(ValueError, match="shape mismatch"):
        lsq_solver().net.copy_trained_layers_from(src)
    src2 = a.net.to_proto()
    lp2 = [l for l in src2.layer if l.name == "ip"][0]
    del lp2.blobs[0].shape.dim[:]
    lp2.blobs[0].ClearField("shape")
    lp2.blobs[0].num, lp2.blobs[0].channels, lp2.blobs[0].height, lp2.blobs[0].width = 1, 1, 1, D
    b = lsq_solver()
    b.net.copy_trained_layers_from(src2)
    assert torch.equal(b.net.layer_by_name("ip").params[0].to_caffe(), w)
