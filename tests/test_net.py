"""Net construction semantics (caffe/src/caffe/test/test_net.cpp, test_split_layer.cpp)
and whole-net numerics against an independent fp64 NCHW PyTorch oracle."""
import pytest
import torch

from sparknet_amd import dsl, models, proto
from sparknet_amd.core.net import Net, filter_net, insert_splits

import torch_oracle


def _dummy(name, shapes, fillers=None):
    lp = proto.LayerParameter(name=name, type="DummyData")
    for i, s in enumerate(shapes):
        lp.top.append(name if i == 0 else f"{name}{i}")
        lp.dummy_data_param.shape.add().dim.extend(s)
    for f in fillers or []:
        lp.dummy_data_param.data_filler.add().CopyFrom(f)
    return lp


def test_filter_net_phase_level_stage():
    n = proto.parse_prototxt("""
      name: "f"
      layer { name: "a" type: "Silence" bottom: "x" include { phase: TRAIN } }
      layer { name: "b" type: "Silence" bottom: "x" include { phase: TEST } }
      layer { name: "c" type: "Silence" bottom: "x" include { min_level: 2 } }
      layer { name: "d" type: "Silence" bottom: "x" include { stage: "s1" } }
      layer { name: "e" type: "Silence" bottom: "x" exclude { not_stage: "s1" } }
    """)
    n.state.phase = proto.TRAIN
    assert [l.name for l in filter_net(n).layer] == ["a"]
    n.state.level = 3
    n.state.stage.append("s1")
    assert [l.name for l in filter_net(n).layer] == ["a", "c", "d", "e"]


def test_insert_splits_names_and_loss_weight():
    n = proto.parse_prototxt("""
      name: "s"
      layer { name: "data" type: "DummyData" top: "data" top: "label"
              dummy_data_param { shape { dim: 2 dim: 3 } shape { dim: 2 } } }
      layer { name: "ip" type: "InnerProduct" bottom: "data" top: "ip" inner_product_param { num_output: 4 } }
      layer { name: "acc" type: "Accuracy" bottom: "ip" bottom: "label" top: "acc" }
      layer { name: "loss" type: "SoftmaxWithLoss" bottom: "ip" bottom: "label" top: "loss" }
    """)
    s = insert_splits(n)
    names = [l.name for l in s.layer]
    assert "ip_ip_0_split" in names and "label_data_1_split" in names
    split = s.layer[names.index("ip_ip_0_split")]
    assert list(split.top) == ["ip_ip_0_split_0", "ip_ip_0_split_1"]
    assert s.layer[names.index("acc")].bottom[0] == "ip_ip_0_split_0"
    assert s.layer[names.index("loss")].bottom[0] == "ip_ip_0_split_1"


def test_need_backward_pruning_and_outputs():
    net = Net(models.lenet(train_batch=2, test_batch=2), phase=proto.TEST)
    nb = dict(zip(net.layer_names, net.layer_need_backward))
    assert nb["conv1"] and nb["ip2"]
    assert not nb["accuracy"]
    assert not any(net.bottom_need_backward[net.layer_names.index("conv1")])  # data needs no grad
    assert sorted(b.name for b in net.output_blobs) == ["accuracy", "loss"]


def test_param_sharing_by_name():
    n = proto.parse_prototxt("""
      name: "share"
      layer { name: "data" type: "DummyData" top: "data" dummy_data_param { shape { dim: 2 dim: 5 }
              data_filler { type: "gaussian" } } }
      layer { name: "ip1" type: "InnerProduct" bottom: "data" top: "ip1" param { name: "w" } param { name: "b" }
              inner_product_param { num_output: 5 weight_filler { type: "gaussian" } } }
      layer { name: "ip2" type: "InnerProduct" bottom: "ip1" top: "ip2" param { name: "w" } param { name: "b" }
              inner_product_param { num_output: 5 weight_filler { type: "gaussian" } } }
      layer { name: "loss" type: "EuclideanLoss" bottom: "ip2" bottom: "data" top: "loss" }
    """)
    net = Net(n, phase=proto.TRAIN)
    assert len(net.learnable_params) == 2
    w1, w2 = net.layer_by_name("ip1").params[0], net.layer_by_name("ip2").params[0]
    assert w1.data.data_ptr() == w2.data.data_ptr() and w1.diff.data_ptr() == w2.diff.data_ptr()
    net.clear_param_diffs()
    net.forward_backward()
    # gradient of the shared weight == sum of both uses (check vs oracle)
    wts = {"ip1": [p.to_caffe() for p in net.layer_by_name("ip1").params],
           "ip2": [p.to_caffe() for p in net.layer_by_name("ip2").params]}
    wts["ip2"] = wts["ip1"]
    x = net.blob_by_name("data").data.clone()
    # oracle with true sharing: the same leaf used twice
    lw = [t.double().clone().requires_grad_(True) for t in wts["ip1"]]
    h = x.double() @ lw[0].t() + lw[1]
    h = h @ lw[0].t() + lw[1]
    loss = ((h - x.double()) ** 2).sum() / 2 / 2
    loss.backward()
    assert torch.allclose(w1.diff.double(), lw[0].grad, rtol=1e-4, atol=1e-5)


def _oracle_compare(netparam, batch_inputs, tol=2e-4, wscale=0.1):
    net = Net(netparam, phase=proto.TRAIN)
    g = torch.Generator().manual_seed(3)
    for p in net.learnable_params:  # non-trivial weights for every param
        p.set_caffe(torch.randn(p.caffe_shape, generator=g) * wscale)
    for name, t in batch_inputs.items():
        net.blob_by_name(name).set_nchw(t)
    net.clear_param_diffs()
    loss = net.forward_backward()
    weights = {l.name: [p.to_caffe() for p in l.params] for l in net.layers if l.params}
    tot, outs, leaves = torch_oracle.run(netparam, proto.TRAIN, weights, batch_inputs)
    tot.backward()
    assert abs(float(loss) - float(tot)) < tol * max(1.0, abs(float(tot))), (float(loss), float(tot))
    for lname, ws in leaves.items():
        mine = net.layer_by_name(lname).params
        for p, w in zip(mine, ws):
            d = p.to_caffe(p.diff).double()
            err = (d - w.grad).abs().max().item()
            scale = w.grad.abs().max().item() + 1e-12
            assert err / scale < 1e-3, (lname, err, scale)


def test_cifar10_quick_matches_oracle():
    n = models.cifar10_quick(train_batch=3, test_batch=3)
    g = torch.Generator().manual_seed(0)
    _oracle_compare(n, {"data": torch.randn(3, 3, 32, 32, generator=g),
                        "label": torch.tensor([[1.0], [7.0], [3.0]])})


def test_cifar10_full_matches_oracle():
    n = models.cifar10_full(train_batch=2, test_batch=2)
    g = torch.Generator().manual_seed(1)
    # moderate logits: Caffe clamps p_label at FLT_MIN (loss <= 87.34), the oracle does not
    _oracle_compare(n, {"data": torch.randn(2, 3, 32, 32, generator=g) * 0.3,
                        "label": torch.tensor([[4.0], [9.0]])})


def test_caffenet_small_matches_oracle():
    """Grouped convs, cross-channel LRN, IP on a 4-D (NHWC) bottom with HWC->CHW weight
    permutation, dropout in TEST-like identity (ratio 0 here)."""
    n = models.caffenet(train_batch=2, test_batch=2, crop=99, classes=7)
    for l in n.layer:
        if l.type == "Dropout":
            l.dropout_param.dropout_ratio = 0.0
        if l.type == "InnerProduct" and l.name in ("fc6", "fc7"):
            l.inner_product_param.num_output = 16
    g = torch.Generator().manual_seed(2)
    _oracle_compare(n, {"data": torch.randn(2, 3, 99, 99, generator=g),
                        "label": torch.tensor([[1.0], [5.0]])})


def test_googlenet_small_matches_oracle():
    n = models.googlenet(train_batch=1, test_batch=1, crop=64, classes=5, aux=False)
    for l in n.layer:
        if l.type == "Dropout":
            l.dropout_param.dropout_ratio = 0.0
        if l.name == "pool5/7x7_s1":
            l.pooling_param.ClearField("kernel_h")
            l.pooling_param.ClearField("kernel_w")
            l.pooling_param.ClearField("stride_h")
            l.pooling_param.ClearField("stride_w")
            l.pooling_param.global_pooling = True
    g = torch.Generator().manual_seed(4)
    _oracle_compare(n, {"data": torch.randn(1, 3, 64, 64, generator=g), "label": torch.tensor([[3.0]])},
                    wscale=0.03)


def test_forward_reshape_and_blob_views():
    net = Net(models.cifar10_quick(train_batch=2, test_batch=2), phase=proto.TRAIN)
    b = net.blob_by_name("conv1")
    assert b.shape == (2, 32, 32, 32) and tuple(b.data.shape) == (2, 32, 32, 32)
    assert tuple(net.blob_by_name("pool1").nchw().shape) == (2, 32, 16, 16)


def test_loss_weight_scales_gradient():
    base = models.cifar10_quick(train_batch=2, test_batch=2)
    inputs = {"data": torch.randn(2, 3, 32, 32), "label": torch.tensor([[1.0], [2.0]])}
    grads = []
    for lw in (1.0, 2.5):
        n = proto.copy(base)
        for l in n.layer:
            if l.type == "SoftmaxWithLoss":
                l.loss_weight.append(lw)
        net = Net(n, phase=proto.TRAIN, seed=5)
        for k, v in inputs.items():
            net.blob_by_name(k).set_nchw(v)
        net.clear_param_diffs()
        net.forward_backward()
        grads.append(net.flat_diff.clone())
    scale = grads[0].abs().max()
    assert torch.allclose(grads[1], 2.5 * grads[0], rtol=1e-3, atol=1e-5 * float(scale))


def _caffenet_tiny(ratio=0.5):
    n = models.caffenet(train_batch=2, test_batch=2, crop=67, classes=7)
    for l in n.layer:
        if l.type == "Dropout":
            l.dropout_param.dropout_ratio = ratio
        if l.type == "InnerProduct" and l.name in ("fc6", "fc7"):
            l.inner_product_param.num_output = 16
    return n


def _grads_with_fusion(netparam, fuse, device="cpu"):
    from sparknet_amd.engine import fuse_relu
    net = Net(netparam, phase=proto.TRAIN, seed=11, device=device)
    counts = (0, 0)
    if fuse:
        nf = fuse_relu(net)  # also runs the backward (gate) fusion pass
        counts = (nf, sum(1 for l in net.layers if getattr(l, "bwd_fused", False)))
    g = torch.Generator().manual_seed(9)
    net.blob_by_name("data").set_nchw(torch.randn(2, 3, 67, 67, generator=g))
    net.blob_by_name("label").set_nchw(torch.tensor([[1.0], [5.0]]))
    net.clear_param_diffs()
    loss = net.forward_backward()
    return float(loss), net.flat_diff.detach().cpu().clone(), counts


def test_relu_forward_backward_fusion_matches_unfused():
    """ReLU folded into the producer's epilogue (forward) and into the consumer's backward
    (dgrad gate / max-pool mask / dropout gate) gives the unfused gradients."""
    n = _caffenet_tiny()
    l0, g0, _ = _grads_with_fusion(n, False)
    l1, g1, counts = _grads_with_fusion(n, True)
    assert counts == (7, 7), counts  # relu1..7 forward-fused; all 7 backward-fused
    assert abs(l0 - l1) < 1e-5 * max(1.0, abs(l0))
    assert torch.allclose(g0, g1, rtol=1e-5, atol=1e-6 * float(g0.abs().max()))


def _googlenet_tiny():
    n = models.googlenet(train_batch=2, test_batch=2, crop=67, classes=7, aux=False)
    for l in n.layer:
        if l.type == "Dropout":
            l.dropout_param.dropout_ratio = 0.0
        if l.name == "pool5/7x7_s1":
            for f in ("kernel_h", "kernel_w", "stride_h", "stride_w", "kernel_size", "stride"):
                l.pooling_param.ClearField(f)
            l.pooling_param.global_pooling = True
    return n


def test_concat_relu_backward_fusion_matches_unfused():
    """Inception branch ReLUs feeding a Concat: their backward masks are applied by the
    concat backward (relu_gate_parts) and the result equals the unfused gradients."""
    n = _googlenet_tiny()
    l0, g0, _ = _grads_with_fusion(n, False)
    l1, g1, counts = _grads_with_fusion(n, True)
    assert counts[1] >= 9 * 4, counts  # at least the four branch outputs of each inception module
    assert abs(l0 - l1) < 1e-5 * max(1.0, abs(l0))
    assert torch.allclose(g0, g1, rtol=1e-5, atol=1e-6 * float(g0.abs().max()))


def test_lazy_gradient_clear_matches_memset():
    """clear_param_diffs(lazy=True) + first-write overwrite == memset + accumulate, with
    garbage left in the buffer, two accumulated passes (iter_size), a frozen layer and a
    shared parameter."""
    n = models.cifar10_quick(train_batch=2, test_batch=2)
    for l in n.layer:
        if l.name == "conv2":
            l.param[0].lr_mult = 0.0  # frozen weight: its diff must come out zero
            l.param[1].lr_mult = 0.0
    g = torch.Generator().manual_seed(0)
    x = torch.randn(2, 3, 32, 32, generator=g)
    y = torch.tensor([[1.0], [7.0]])
    out = []
    for lazy in (False, True):
        net = Net(n, phase=proto.TRAIN, seed=5)
        net.blob_by_name("data").set_nchw(x)
        net.blob_by_name("label").set_nchw(y)
        net.flat_diff.normal_()  # stale garbage
        net.clear_param_diffs(lazy=lazy)
        for _ in range(2):
            net.forward_backward()
        net.finish_param_diffs()
        # compare the param segments (the alignment padding is never written by layers)
        out.append(torch.cat([p.diff.reshape(-1) for p in net.learnable_params]))
        frozen = net.layer_by_name("conv2").params
    assert torch.allclose(out[0], out[1], rtol=1e-6, atol=1e-7)
    assert all(float(p.diff.abs().max()) == 0.0 for p in frozen)


def test_random_init_gives_chance_accuracy():
    """CifarSpec (src/test/scala/libs/CifarSpec.scala:10-94): a random-init cifar10_full on
    CIFAR-shaped data scores chance — sum over 10 test batches of accuracy x 100 lies in
    [70, 130].  Synthetic images / labels stand in for the CIFAR test set."""
    net = Net(models.cifar10_full(train_batch=100, test_batch=100), phase=proto.TEST, seed=1)
    g = torch.Generator().manual_seed(4)
    total = 0.0
    for _ in range(10):
        x = torch.randint(0, 256, (100, 3, 32, 32), generator=g).float() - 120.0
        y = torch.randint(0, 10, (100, 1), generator=g).float()
        net.blob_by_name("data").set_nchw(x)
        net.blob_by_name("label").set_nchw(y)
        net.forward()
        total += float(net.blob_by_name("accuracy").data.reshape(-1)[0])
    assert 70 <= total * 100 <= 130, total * 100


def test_python_layer():
    """python_param user layer (pycaffe protocol) inside a net, forward and backward."""
    n = proto.parse_prototxt("""
      name: "py"
      force_backward: true
      layer { name: "x" type: "Input" top: "x" java_data_param { shape { dim: 2 dim: 3 } } }
      layer { name: "s" type: "Python" bottom: "x" top: "y"
              python_param { module: "pylayers.scale_layer" layer: "ScaleByParam" param_str: "2.5" } }
      layer { name: "loss" type: "EuclideanLoss" bottom: "y" bottom: "x" top: "loss" }
    """)
    net = Net(n, phase=proto.TRAIN)
    x = torch.randn(2, 3)
    net.blob_by_name("x").set_nchw(x)
    loss = net.forward_backward()
    assert torch.allclose(net.blob_by_name("y").data, 2.5 * x)
    assert abs(float(loss) - float(((1.5 * x) ** 2).sum() / 2 / 2)) < 1e-5


def test_stochastic_pooling_train_samples_proportionally():
    """StoPoolForwardTrain / StoPoolBackward (pooling_layer.cu:88-122, 270-300): an
    element is drawn with probability value / window sum; the diff goes to it.  TEST
    returns sum(x^2) / sum(x) (pooling_layer.cu:125-155)."""
    n = 4000
    txt = ('name: "s" force_backward: true layer { name: "in" type: "Input" top: "x" java_data_param { shape { '
           f'dim: {n} dim: 1 dim: 1 dim: 2 }} }} }} '
           'layer { name: "p" type: "Pooling" bottom: "x" top: "y" pooling_param { pool: STOCHASTIC '
           'kernel_h: 1 kernel_w: 2 stride: 1 } }')
    net = Net(proto.parse_prototxt(txt), phase=proto.TRAIN, seed=5)
    x = net.blobs[net.blob_names.index("x")]
    x.set_nchw(torch.tensor([1.0, 3.0]).repeat(n, 1, 1, 1))
    net.forward()
    y = net.blobs[net.blob_names.index("y")]
    vals = y.nchw().reshape(-1)
    assert set(vals.tolist()) <= {1.0, 3.0}
    frac = float((vals == 3.0).float().mean())
    assert abs(frac - 0.75) < 0.03
    y.set_nchw(torch.ones(n, 1, 1, 1), diff=True)
    net.backward()
    g = x.nchw(diff=True).reshape(n, 2)
    assert torch.equal(g[:, 1], (vals == 3.0).float()) and torch.equal(g.sum(1), torch.ones(n))
    test = Net(proto.parse_prototxt(txt), phase=proto.TEST)
    test.blobs[test.blob_names.index("x")].set_nchw(torch.tensor([1.0, 3.0]).repeat(n, 1, 1, 1))
    test.forward()
    assert torch.allclose(test.blobs[test.blob_names.index("y")].nchw(), torch.full((n, 1, 1, 1), 2.5))


@pytest.mark.parametrize("aux, n_streams, star", [(False, 4, False), (True, 3, True), (True, 4, True)])
def test_branch_stream_plan_respects_dependencies(aux, n_streams, star):
    """engine.BranchStreams: GoogLeNet's Inception towers are spread over several streams,
    and replaying the plan in stream order (each stream serial, cross-stream waits
    honoured) never runs a layer before the producers of what it reads or before the
    readers / writers of what it overwrites — also with the auxiliary loss heads, whose
    backward depends on nothing and is placed on the least recently used stream, and in
    the star topology (side streams wait on the main stream only)."""
    from sparknet_amd import models, proto
    from sparknet_amd.core.net import Net
    from sparknet_amd.engine import BranchStreams
    n = models.googlenet(train_batch=1, test_batch=1, crop=67 if not aux else 227, classes=7, aux=aux)
    for l in n.layer:
        if l.name == "pool5/7x7_s1":
            for f in ("kernel_h", "kernel_w", "stride_h", "stride_w", "kernel_size", "stride"):
                l.pooling_param.ClearField(f)
            l.pooling_param.global_pooling = True
    net = Net(n, phase=proto.TRAIN, seed=1, device="cpu")
    bs = BranchStreams(net, n_streams, star=star)
    assert bs.streams_used() == n_streams and bs.streams_used(backward=True) == n_streams
    if star:
        for plan in (bs.fwd_plan, bs.bwd_plan):
            sid_of = [sid for _, sid, _, _ in plan]
            for _, sid, waits, _ in plan:
                assert sid == 0 or all(sid_of[d] == 0 for d in waits)
    for plan in (bs.fwd_plan, bs.bwd_plan):
        # the earliest time each node may run when streams proceed in parallel (unit cost)
        finish, stream_t = {}, [0] * n_streams
        for pos, (li, sid, waits, _) in enumerate(plan):
            start = max([stream_t[sid]] + [finish[d] for d in waits])
            finish[pos] = start + 1
            stream_t[sid] = finish[pos]
        # a node's start >= finish of every earlier node it conflicts with
        order = [li for li, _, _, _ in plan]
        fwd = plan is bs.fwd_plan
        def rw(li):
            if fwd:
                return set(net.bottom_ids[li]), set(net.top_ids[li])
            r = {("v", b) for b in list(net.bottom_ids[li]) + list(net.top_ids[li])} | \
                {("d", b) for b in net.top_ids[li]}
            w = {("d", b) for b, need in zip(net.bottom_ids[li], net.bottom_need_backward[li]) if need}
            return r, w | {("p", p.offset) for p in net.layers[li].params}
        for j in range(len(order)):
            rj, wj = rw(order[j])
            for i in range(j):
                ri, wi = rw(order[i])
                if (wi & rj) or (wi & wj) or (ri & wj):
                    assert finish[j] - 1 >= finish[i], (order[i], order[j])
        assert max(finish.values()) < len(plan)  # some layers really overlap


def test_fp8_macs_per_input_cost_model():
    """engine.fp8_macs_per_input: forward MACs per input element that the fp8 layer
    selection (enable_fp8 min_macs_per_input) compares against the quantisation pass."""
    from sparknet_amd import models
    from sparknet_amd.core.solver import Solver
    from sparknet_amd.engine import fp8_macs_per_input
    solver = Solver(models.solver_for("caffenet", train_batch=2, test_batch=2), build_test_nets=False)
    net = solver.net
    got = {}
    for li, layer in enumerate(net.layers):
        if layer.type_name in ("Convolution", "InnerProduct"):
            got[layer.name] = fp8_macs_per_input(layer, net.bottom_vecs[li][0])
    assert got["conv1"] == 96 * 11 * 11 / 16.0  # 11x11 stride 4
    assert got["conv2"] == 128 * 5 * 5  # group 2: 128 outputs per input channel
    assert got["conv3"] == 384 * 9
    assert got["fc6"] == 4096 and got["fc8"] == 1000


def test_fp8_dgrad_cost_model_and_eligibility():
    """engine.fp8_dgrad_macs_per_grad (data-gradient MACs per output-gradient element, the
    work an fp8 data gradient halves per element of its dy quantisation pass) and the
    shapes ops.hip.fp8_dgrad_ok accepts: stride-1 implicit convs whose output channels per
    group fill 16-byte fp8 chunks (CaffeNet conv1 is strided, conv2 has 128 per group)."""
    from sparknet_amd import models
    from sparknet_amd.core.solver import Solver
    from sparknet_amd.engine import fp8_dgrad_macs_per_grad
    solver = Solver(models.solver_for("caffenet", train_batch=2, test_batch=2), build_test_nets=False)
    net = solver.net
    got, ok = {}, {}
    for li, layer in enumerate(net.layers):
        if layer.type_name == "Convolution":
            b = net.bottom_vecs[li][0]
            got[layer.name] = fp8_dgrad_macs_per_grad(layer, b)
            ok[layer.name] = layer.fp8_dgrad_eligible(b)
    assert got["conv2"] == 48 * 5 * 5 and got["conv3"] == 256 * 9 and got["conv4"] == 192 * 9
    assert not ok["conv1"]  # 11x11 stride 4: the data gradient is not a stride-1 forward conv
    assert ok["conv2"] and ok["conv3"] and ok["conv4"] and ok["conv5"]


def test_branch_sim_script_runs():
    """scripts/branch_sim.py (CPU schedule simulation of the branch-stream plans) runs and
    reports a span for 2 / 3 / 4 streams."""
    import os
    import subprocess
    import sys
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    r = subprocess.run([sys.executable, "scripts/branch_sim.py", "--batch", "8"], cwd=root, capture_output=True,
                       text=True, timeout=300)
    assert r.returncode == 0, r.stderr[-2000:]
    lines = [l for l in r.stdout.splitlines() if "streams:" in l]
    assert len(lines) == 3 and all("forward" in l and "backward" in l for l in lines)
