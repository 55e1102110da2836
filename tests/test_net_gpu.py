"""Whole-net numerics on the MI355X: the HIP engine (bf16 NHWC, fused epilogues) against
the fp32 CPU engine on the same weights and inputs, and fused-vs-unfused graph passes.
Reference analogue: Caffe's layer tests run every layer on CPU and GPU with the CPU as
oracle (caffe/src/caffe/test/test_*_layer.cpp); here the whole net is compared."""
import math

import pytest
import torch

from sparknet_amd import models, proto
from sparknet_amd.core.net import Net

pytestmark = pytest.mark.gpu


def _tiny_caffenet(ratio):
    n = models.caffenet(train_batch=2, test_batch=2, crop=67, classes=7)
    for l in n.layer:
        if l.type == "Dropout":
            l.dropout_param.dropout_ratio = ratio
        if l.type == "InnerProduct" and l.name in ("fc6", "fc7"):
            l.inner_product_param.num_output = 32
    return n


def _run(netparam, device, fuse, weights=None):
    from sparknet_amd.engine import fuse_relu
    net = Net(netparam, phase=proto.TRAIN, seed=11, device=device)
    if weights is not None:
        net.flat_data.copy_(weights.to(net.flat_data.device))
        net.sync_compute()
    if fuse:
        fuse_relu(net)
    g = torch.Generator().manual_seed(9)
    net.blob_by_name("data").set_nchw(torch.randn(2, 3, 67, 67, generator=g) * 20)
    net.blob_by_name("label").set_nchw(torch.tensor([[1.0], [5.0]]))
    net.clear_param_diffs()
    loss = net.forward_backward()
    return float(loss), net.flat_diff.detach().float().cpu().clone(), net


def test_relu_gate_fusion_on_gpu(gpu):
    n = _tiny_caffenet(0.5)
    l0, g0, _ = _run(n, gpu, False)
    l1, g1, net = _run(n, gpu, True)
    assert sum(1 for l in net.layers if getattr(l, "bwd_fused", False)) == 7
    assert abs(l0 - l1) <= 1e-3 * max(1.0, abs(l0))
    err = (g0 - g1).abs().max().item() / (g0.abs().max().item() + 1e-12)
    assert err < 1e-2, err


def test_googlenet_concat_gate_on_gpu(gpu):
    """GoogLeNet: zero-copy channel concat with the Inception ReLU masks applied by the
    concat outputs' readers, fused vs unfused on the GPU, and the fused GPU pass vs the
    fp32 CPU engine."""
    n = models.googlenet(train_batch=2, test_batch=2, crop=67, classes=7, aux=False)
    for l in n.layer:
        if l.type == "Dropout":
            l.dropout_param.dropout_ratio = 0.0
        if l.name == "pool5/7x7_s1":
            for f in ("kernel_h", "kernel_w", "stride_h", "stride_w", "kernel_size", "stride"):
                l.pooling_param.ClearField(f)
            l.pooling_param.global_pooling = True
    l0, g0, net0 = _run(n, gpu, False)
    l1, g1, net = _run(n, gpu, True, weights=net0.flat_data.detach().float().cpu())
    cats = [l for l in net.layers if l.type_name == "Concat"]
    # zero-copy concat (engine.fuse_concat): the parts' ReLU masks moved into the readers
    # of each concat output; otherwise they are applied in the concat backward
    assert all(c.zero_copy_bwd and not c.relu_gate_parts for c in cats) or \
        sum(len(c.relu_gate_parts) for c in cats) == 9 * 4
    assert abs(l0 - l1) <= 1e-3 * max(1.0, abs(l0))
    err = (g0 - g1).abs().max().item() / (g0.abs().max().item() + 1e-12)
    assert err < 1e-2, err
    lc, gc, _ = _run(n, "cpu", False, weights=net0.flat_data.detach().float().cpu())
    assert abs(lc - l1) <= 3e-2 * max(1.0, abs(lc))
    cos = torch.nn.functional.cosine_similarity(gc, g1, dim=0).item()
    assert cos > 0.99, cos


def test_caffenet_gpu_matches_cpu_engine(gpu):
    n = _tiny_caffenet(0.0)
    lc, gc, netc = _run(n, "cpu", False)
    lg, gg, _ = _run(n, gpu, True, weights=netc.flat_data.detach().clone())
    assert abs(lc - lg) < 3e-2 * max(1.0, abs(lc)), (lc, lg)
    err = (gc - gg).abs().max().item() / (gc.abs().max().item() + 1e-12)
    assert err < 5e-2, err


def _graph_solver(overlap, fuse_fc=False):
    from sparknet_amd.core.solver import Solver
    from sparknet_amd.engine import GraphStep, fuse_relu
    sp = models.zoo.caffenet_solver(_tiny_caffenet(0.5))
    solver = Solver(sp, device=torch.device("cuda:0"), seed=3, build_test_nets=False)
    fuse_relu(solver.net)
    g = torch.Generator().manual_seed(1)
    batches = [(torch.randn(2, 3, 67, 67, generator=g) * 20, torch.tensor([[1.0], [4.0]])) for _ in range(6)]
    it = iter(batches)

    def pre():
        x, y = next(it)
        solver.net.blob_by_name("data").set_nchw(x)
        solver.net.blob_by_name("label").set_nchw(y)
    step = GraphStep(solver, warmup=1, pre=pre, overlap=overlap, fuse_fc=fuse_fc)
    if step.overlap is not None:  # the tiny net's layers are below the production threshold
        from sparknet_amd.engine import OverlappedUpdate
        solver.net.backward_hooks.clear()
        step.overlap = OverlappedUpdate(solver, min_group=1)
        solver.net.backward_hooks.append(step.overlap.hook)
        assert len(step.overlap.tables) >= 8
    for _ in range(4):  # 1 warmup + capture-replay + 2 replays
        step.step()
    torch.cuda.synchronize()
    return solver, step


def test_overlapped_update_matches_serial(gpu):
    """Per-layer solver updates on a side stream during backward == one update after it."""
    s0, st0 = _graph_solver(False)
    s1, st1 = _graph_solver(True)
    assert st0.overlap is None and st1.overlap is not None
    assert s0.iter == s1.iter
    assert torch.equal(s0.net.flat_data, s1.net.flat_data)
    assert torch.equal(s0.history[0], s1.history[0])


def test_fused_fc_update_matches_solver_kernel(gpu):
    """InnerProduct weight updates applied in the wgrad GEMM epilogue == the same
    iterations with gradients stored and updated by the solver kernel."""
    s0, _ = _graph_solver(False, fuse_fc=False)
    s1, st1 = _graph_solver(False, fuse_fc=True)
    fused = [l for l in s1.net.layers if getattr(l, "fused_update", None) is not None]
    assert len(fused) == 2  # fc6, fc7 (fc8 has 7 outputs: not a multiple of 8)
    assert s0.iter == s1.iter
    for a, b in ((s0.net.flat_data, s1.net.flat_data), (s0.history[0], s1.history[0])):
        err = (a - b).abs().max().item() / (a.abs().max().item() + 1e-12)
        assert err < 1e-5, err
    assert torch.equal(s1.net.flat_compute, s1.net.flat_data.to(torch.bfloat16))


def test_training_is_bitwise_deterministic(gpu):
    """Fixed Philox seeds + atomics-free reductions (split-K slabs, colsum, solver): two
    identical graph-captured runs end with bitwise-identical weights and momentum."""
    a, _ = _graph_solver(False, fuse_fc=True)
    b, _ = _graph_solver(False, fuse_fc=True)
    assert torch.equal(a.net.flat_data, b.net.flat_data)
    assert torch.equal(a.history[0], b.history[0])


@pytest.mark.parametrize("dgrad", [False, True])
def test_fp8_forward_training(gpu, dgrad):
    """enable_fp8: e4m3 forward products (and, with dgrad, e4m3 data gradients of the
    stride-1 convs) with delayed scaling track the bf16 net and train."""
    from sparknet_amd.core.solver import Solver
    from sparknet_amd.engine import GraphStep, enable_fp8, fuse_relu
    net_p = models.vgg16(train_batch=4, test_batch=4, crop=32, classes=10)
    losses = {}
    for mode in ("bf16", "fp8"):
        sp = models.zoo.vgg16_solver(net_p)
        sp.base_lr = 0.002
        solver = Solver(sp, device=torch.device("cuda:0"), seed=5, build_test_nets=False)
        fuse_relu(solver.net)
        if mode == "fp8":
            n = enable_fp8(solver.net, 0.0, dgrad=dgrad)
            # 12 of 13 convs (not the RGB input) + 3 IPs; data gradients of the 12 convs
            # that need one (conv1_1's is never computed)
            assert n >= (14 + 12 if dgrad else 14), n
            if dgrad:
                assert sum(getattr(ly, "fp8_dgrad_slots", None) is not None for ly in solver.net.layers) >= 12
        g = torch.Generator().manual_seed(2)
        x = torch.randn(4, 3, 32, 32, generator=g) * 0.5
        y = torch.tensor([[1.0], [3.0], [5.0], [7.0]])

        def pre():
            solver.net.blob_by_name("data").set_nchw(x)
            solver.net.blob_by_name("label").set_nchw(y)
        st = GraphStep(solver, warmup=2, pre=pre, overlap=False)
        seq = [float(st.step()) for _ in range(12)]
        losses[mode] = seq
        assert all(math.isfinite(v) for v in seq), seq
    # same data every step: both must fit it; fp8 stays close to bf16
    assert losses["fp8"][-1] < losses["fp8"][0]
    assert abs(losses["fp8"][0] - losses["bf16"][0]) < 0.05 * abs(losses["bf16"][0]) + 0.05


def test_fp8_fused_quant_is_bitwise_equal(gpu, monkeypatch):
    """engine.fuse_fp8_quant: the producing conv GEMMs' epilogues store the consumers' fp8
    inputs and fp8 output gradients (ops.gemm.Fp8Side) instead of separate quantisation
    passes — same bytes, same amax — so graph-captured training is bitwise equal with and
    without the fusion, and the side outputs are really consumed."""
    from sparknet_amd.core.solver import Solver
    from sparknet_amd.engine import GraphStep, enable_fp8, fuse_relu
    from sparknet_amd.ops import gemm as G
    net_p = models.vgg16(train_batch=4, test_batch=4, crop=32, classes=10)
    res = {}
    for fused in ("1", "0"):
        monkeypatch.setenv("SN_FEATURES", f"fuse_fp8_quant={fused}")
        sp = models.zoo.vgg16_solver(net_p)
        sp.base_lr = 0.002
        solver = Solver(sp, device=torch.device("cuda:0"), seed=5, build_test_nets=False)
        fuse_relu(solver.net)
        enable_fp8(solver.net, 0.0, dgrad=True)
        pairs = sum(ly.fp8_out is not None for ly in solver.net.layers if ly.type_name == "Convolution")
        pairs_bwd = sum(ly.fp8_dx_out is not None for ly in solver.net.layers if ly.type_name == "Convolution")
        if fused == "1":
            assert pairs >= 7 and pairs_bwd >= 7, (pairs, pairs_bwd)  # conv1_2 .. conv5_3 chains
        else:
            assert pairs == 0 and pairs_bwd == 0
        g = torch.Generator().manual_seed(2)
        x = torch.randn(4, 3, 32, 32, generator=g) * 0.5
        y = torch.tensor([[1.0], [3.0], [5.0], [7.0]])

        def pre():
            solver.net.blob_by_name("data").set_nchw(x)
            solver.net.blob_by_name("label").set_nchw(y)
        G.SIDE_STATS.update(used=0, missed=0)
        st = GraphStep(solver, warmup=2, pre=pre, overlap=False)
        losses = [float(st.step()) for _ in range(6)]
        res[fused] = (losses, solver.net.flat_data.clone(), dict(G.SIDE_STATS))
    # tiny deep layers run split-K products (their reduce writes the bf16 output): those
    # consumers quantise themselves; the large early layers take the side outputs
    assert res["1"][2]["used"] >= 4, res["1"][2]
    assert res["0"][2]["used"] == 0
    assert res["1"][0] == res["0"][0], (res["1"][0], res["0"][0])
    assert torch.equal(res["1"][1], res["0"][1])


@pytest.mark.parametrize("fp8", [False, True])
def test_release_activations_before_capture_is_bitwise_equal(gpu, monkeypatch, fp8):
    """engine.release_activations (run before a capture when the warm-up holds most of the
    device, forced here with engine.GRAPH_RELEASE): the captured iteration re-creates every
    activation, gradient, workspace and fp8 side output it dropped, so training is bitwise equal
    to a capture that kept the warm-up's buffers."""
    from sparknet_amd.core.solver import Solver
    from sparknet_amd.engine import GraphStep, enable_fp8, fuse_relu
    net_p = models.vgg16(train_batch=4, test_batch=4, crop=32, classes=10)
    res = {}
    for rel in ("1", "0"):
        from sparknet_amd import engine as _engine
        monkeypatch.setattr(_engine, "GRAPH_RELEASE", rel == "1")
        sp = models.zoo.vgg16_solver(net_p)
        sp.base_lr = 0.002
        solver = Solver(sp, device=torch.device("cuda:0"), seed=5, build_test_nets=False)
        fuse_relu(solver.net)
        if fp8:
            enable_fp8(solver.net, 0.0, dgrad=True, wgrad=True)
        g = torch.Generator().manual_seed(2)
        x = torch.randn(4, 3, 32, 32, generator=g) * 0.5
        y = torch.tensor([[1.0], [3.0], [5.0], [7.0]])

        def pre():
            solver.net.blob_by_name("data").set_nchw(x)
            solver.net.blob_by_name("label").set_nchw(y)
        st = GraphStep(solver, warmup=2, pre=pre, overlap=False)
        losses = [float(st.step()) for _ in range(6)]
        res[rel] = (losses, solver.net.flat_data.clone())
    assert res["1"][0] == res["0"][0], (res["1"][0], res["0"][0])
    assert torch.equal(res["1"][1], res["0"][1])


def test_fused_fold_weight_gradient_with_image_chunks(gpu, monkeypatch):
    """A conv whose S2D-folded input comes from the fused augment (the data blob itself is
    never written) and whose batch is split into image chunks (VGG-16 conv1_1 at batch
    2048): the chunked weight gradient reads the folded chunks, equal to the unchunked one."""
    from sparknet_amd.ops import hip
    from sparknet_amd.ops.spec import ConvSpec
    s = ConvSpec(4, 32, 32, 3, 64, 3, 3, 1, 1, 1, 1, 1, 1, 1)
    plan = hip.s2d_plan(s)
    assert plan is not None
    g = torch.Generator(device=gpu).manual_seed(4)
    x = torch.randn(4, 32, 32, 3, device=gpu, generator=g).to(torch.bfloat16)
    w = (torch.randn(64, 3, 3, 3, device=gpu, generator=g) * 0.1).to(torch.bfloat16)
    dy = torch.randn(4, 32, 32, 64, device=gpu, generator=g).to(torch.bfloat16)
    folded = hip._s2d_input(x, s, plan)
    stale = torch.zeros_like(x)  # the data blob the fused augment never writes
    grads = []
    for max_pix in (1 << 24, 2 * 34 * 34):  # whole batch / 2-image chunks
        monkeypatch.setattr(hip, "_MAX_PIX", max_pix)
        ws = {}
        hip.conv_forward(stale, w, None, s, ws=ws, folded=folded)
        dw = torch.zeros(64, 3, 3, 3, device=gpu)
        hip.conv_backward(dy, stale, w, s, False, dw, None, ws=ws, dw_acc=True)
        grads.append(dw)
    assert hip._image_chunk(s) < s.N  # the second pass really chunked
    assert grads[0].abs().sum() > 0
    assert torch.allclose(grads[1], grads[0], rtol=1e-3, atol=1e-3), (grads[1] - grads[0]).abs().max()


def test_googlenet_branch_streams_bitwise(gpu):
    """engine.BranchStreams runs the Inception towers on 4 HIP streams (eager); loss and
    every parameter gradient are bitwise equal to the sequential schedule; the same holds
    for the 2-stream and the 4-stream star schedules captured into hipGraphs and replayed.
    (Captures with side-stream -> side-stream waits crash in hipStreamEndCapture, see
    engine.BranchStreams.)"""
    from sparknet_amd.engine import BranchStreams, fuse_relu
    n = models.googlenet(train_batch=4, test_batch=4, crop=67, classes=7, aux=True)
    for l in n.layer:
        if l.type == "Dropout":
            l.dropout_param.dropout_ratio = 0.0
        if l.name in ("pool5/7x7_s1", "loss1/ave_pool", "loss2/ave_pool"):
            for f in ("kernel_h", "kernel_w", "stride_h", "stride_w", "kernel_size", "stride"):
                l.pooling_param.ClearField(f)
            l.pooling_param.global_pooling = True
    net = Net(n, phase=proto.TRAIN, seed=3, device=gpu)
    fuse_relu(net)
    g = torch.Generator().manual_seed(5)
    net.blob_by_name("data").set_nchw(torch.randn(4, 3, 67, 67, generator=g) * 20)
    net.blob_by_name("label").set_nchw(torch.tensor([[1.0], [5.0], [0.0], [6.0]]))

    def once(fn):
        net.clear_param_diffs()
        loss = fn()
        torch.cuda.synchronize()
        return float(loss), net.flat_diff.detach().clone()

    l0, g0 = once(net.forward_backward)
    bs = BranchStreams(net, 4)
    assert bs.streams_used() == 4
    l1, g1 = once(bs.forward_backward)
    assert l0 == l1 and torch.equal(g0, g1)
    s = torch.cuda.Stream()  # the same schedule forked from a non-default stream
    s.wait_stream(torch.cuda.current_stream())
    with torch.cuda.stream(s):
        l2, g2 = once(bs.forward_backward)
    torch.cuda.current_stream().wait_stream(s)
    assert l0 == l2 and torch.equal(g0, g2)
    # captured into hipGraphs: 2 streams (the GraphStep default) and 4 streams in the star
    # topology (side streams wait only on the main stream)
    graphs = []
    for b2 in (BranchStreams(net, 2), BranchStreams(net, 4, star=True)):
        with torch.cuda.stream(s):
            once(b2.forward_backward)
        torch.cuda.current_stream().wait_stream(s)
        graph = torch.cuda.CUDAGraph()
        net.clear_param_diffs()
        with torch.cuda.graph(graph):
            loss = b2.forward_backward()
        graphs.append(graph)
        for _ in range(2):
            net.flat_diff.zero_()
            graph.replay()
            torch.cuda.synchronize()
            assert float(loss) == l0 and torch.equal(net.flat_diff, g0)


def test_fused_dropout_matches_standalone(gpu, monkeypatch):
    """Dropout applied in the fc6 / fc7 forward epilogues and its backward in the fc7 /
    fc8 dgrad epilogues (engine.fuse_dropout) == the standalone Philox dropout kernels:
    same masks (same element index, stream and counter), same loss and gradients."""
    n = _tiny_caffenet(0.5)
    l0, g0, net0 = _run(n, gpu, True)  # fused (default)
    fused = [l.name for l in net0.layers if getattr(l, "fused_dropout", None) is not None]
    assert fused == ["fc6", "fc7"], fused
    monkeypatch.setenv("SN_FEATURES", "fuse_dropout=0")
    l1, g1, net1 = _run(n, gpu, True, weights=net0.flat_data.detach().float().cpu())
    assert not any(getattr(l, "fused_dropout", None) for l in net1.layers)
    assert torch.equal(net0.blob_by_name("fc6").data, net1.blob_by_name("fc6").data)
    assert abs(l0 - l1) <= 1e-3 * max(1.0, abs(l0))
    err = (g0 - g1).abs().max().item() / (g0.abs().max().item() + 1e-12)
    assert err < 2e-2, err


def test_googlenet_zero_copy_concat_bitwise(gpu, monkeypatch):
    """engine.fuse_concat: the Inception towers' convolutions write into channel slices of
    the concat buffer, the ReLU gates move into the readers of the concat output and the
    parts' gradients are slice views read in place by the wgrad / dgrad GEMMs.  Loss and
    every parameter gradient are bitwise equal to the copying Concat (same GEMM tiles:
    autotuning off), and no concat copy kernel runs."""
    from sparknet_amd.engine import fuse_relu
    from sparknet_amd.ops import gemm as G
    monkeypatch.setattr(G, "_AUTOTUNE", False)
    monkeypatch.setattr(G, "_TUNED", {})  # no tile choices cached by earlier tests
    n = models.googlenet(train_batch=4, test_batch=4, crop=67, classes=7, aux=True)
    for l in n.layer:
        if l.type == "Dropout":
            l.dropout_param.dropout_ratio = 0.0
        if l.name in ("pool5/7x7_s1", "loss1/ave_pool", "loss2/ave_pool"):
            for f in ("kernel_h", "kernel_w", "stride_h", "stride_w", "kernel_size", "stride"):
                l.pooling_param.ClearField(f)
            l.pooling_param.global_pooling = True
    res = {}
    for mode in ("copy", "zero"):
        monkeypatch.setenv("SN_FEATURES", "zero_copy_concat=1" if mode == "zero" else "zero_copy_concat=0")
        net = Net(n, phase=proto.TRAIN, seed=3, device=gpu)
        fuse_relu(net)
        cats = [l for l in net.layers if l.type_name == "Concat"]
        if mode == "zero":
            assert cats and all(c.zero_copy is not None and c.zero_copy_bwd for c in cats)
        g = torch.Generator().manual_seed(5)
        net.blob_by_name("data").set_nchw(torch.randn(4, 3, 67, 67, generator=g) * 20)
        net.blob_by_name("label").set_nchw(torch.tensor([[1.0], [5.0], [0.0], [6.0]]))
        out = []
        for _ in range(2):
            net.clear_param_diffs()
            loss = net.forward_backward()
            torch.cuda.synchronize()
            out.append((float(loss), net.flat_diff.detach().clone()))
        res[mode] = out
    for (la, ga), (lb, gb) in zip(res["copy"], res["zero"]):
        assert la == lb
        assert torch.equal(ga, gb)


@pytest.mark.parametrize("direct", [True, False])
def test_fp8_layer_selection_threshold(gpu, direct, monkeypatch):
    """enable_fp8's default cost-model threshold keeps a 10-way fc8 in bf16 and everything
    else eligible in e4m3; VGG's conv1_2 (576 MACs per input element, below the threshold)
    is chosen only for the e4m3 direct kernel (SN_CONV_DIRECT_FP8, default on)."""
    from sparknet_amd.core.solver import Solver
    from sparknet_amd.engine import enable_fp8
    from sparknet_amd.ops import hip
    monkeypatch.setattr(hip, "_DIRECT_FP8", direct)
    net_p = models.vgg16(train_batch=2, test_batch=2, crop=32, classes=10)
    solver = Solver(models.zoo.vgg16_solver(net_p), device=torch.device("cuda:0"), seed=5, build_test_nets=False)
    assert enable_fp8(solver.net) == (14 if direct else 13)
    chosen = {layer.name for layer in solver.net.layers if getattr(layer, "fp8_slots", None) is not None}
    assert ("conv1_2" in chosen) == direct and "fc8" not in chosen and "conv2_1" in chosen and "fc6" in chosen


def test_fp8_pool_dx_only_is_bitwise_equal(gpu, monkeypatch):
    """engine.fuse_fp8_quant fp8_dx_only: where the conv below a max pooling reads its output
    gradient only as fp8 (e4m3 data and weight gradients, bias on the ones column), the
    pooling backward stores just the fp8 bytes, not the bf16 gradient — graph-captured
    training is bitwise equal to storing both, and no bf16 read of the skipped tensor happens
    (conv_backward raises on one)."""
    from sparknet_amd.core.solver import Solver
    from sparknet_amd.engine import GraphStep, enable_fp8, fuse_relu
    net_p = models.vgg16(train_batch=4, test_batch=4, crop=32, classes=10)
    res = {}
    for only in ("1", "0"):
        monkeypatch.setenv("SN_FEATURES", f"fp8_dx_only={only}")
        sp = models.zoo.vgg16_solver(net_p)
        sp.base_lr = 0.002
        solver = Solver(sp, device=torch.device("cuda:0"), seed=5, build_test_nets=False)
        fuse_relu(solver.net)
        enable_fp8(solver.net, 0.0, dgrad=True, wgrad=True)
        pools = [ly for ly in solver.net.layers if ly.type_name == "Pooling"]
        n_only = sum(bool(ly.fp8_dx_only) for ly in pools)
        if only == "1":
            assert n_only >= 3, [(ly.name, ly.fp8_dx_out is not None, ly.fp8_dx_only) for ly in pools]
        else:
            assert n_only == 0
        g = torch.Generator().manual_seed(2)
        x = torch.randn(4, 3, 32, 32, generator=g) * 0.5
        y = torch.tensor([[1.0], [3.0], [5.0], [7.0]])

        def pre():
            solver.net.blob_by_name("data").set_nchw(x)
            solver.net.blob_by_name("label").set_nchw(y)
        st = GraphStep(solver, warmup=2, pre=pre, overlap=False)
        losses = [float(st.step()) for _ in range(6)]
        res[only] = (losses, solver.net.flat_data.clone())
    assert res["1"][0] == res["0"][0], (res["1"][0], res["0"][0])
    assert torch.equal(res["1"][1], res["0"][1])
