"""Every non-hot layer family on the GPU (csrc/kernels/layers.hip, eltwise.hip) against the
fp32 CPU reference engine: the same one-layer net is built on both devices, fed the same
bottoms / params / top diffs, and the tops, bottom diffs and param diffs are compared.
Reference analogue: Caffe's per-layer tests run each layer on CPU and GPU
(caffe/src/caffe/test/test_*_layer.cpp, e.g. test_neuron_layer.cpp, test_eltwise_layer.cpp,
test_batch_norm_layer.cpp, test_embed_layer.cpp)."""
import pytest
import torch

from sparknet_amd import proto
from sparknet_amd.core.net import Net

pytestmark = pytest.mark.gpu


def _net(layer_txt, bottoms, device):
    inputs = "".join(
        f'layer {{ name: "in_{n}" type: "Input" top: "{n}" '
        f'java_data_param {{ shape {{ {" ".join(f"dim: {d}" for d in shp)} }} }} }}\n'
        for n, shp in bottoms.items())
    return Net(proto.parse_prototxt(f'name: "g" force_backward: true\n{inputs}{layer_txt}'), phase=proto.TRAIN,
               seed=3, device=device)


def _rel(a, b):
    a, b = a.detach().double().cpu(), b.detach().double().cpu()
    return (a - b).abs().max().item() / (b.abs().max().item() + 1e-6)


def run_both(layer_txt, bottoms, *, values=None, int_bottoms=(), check=None, tol=3e-2, positive=False, seed=0,
             scale=1.0, phase_train=True):
    """values: {bottom name: logical tensor} overrides the random fill."""
    g = torch.Generator().manual_seed(seed)
    logical = {}
    for name, shp in bottoms.items():
        if values and name in values:
            logical[name] = values[name].float()
        elif name in int_bottoms:
            logical[name] = torch.randint(0, 3, shp, generator=g).float()
        else:
            x = torch.randn(shp, generator=g) * scale
            logical[name] = (x.abs() + 0.2) if positive else x
    nets = {d: _net(layer_txt, bottoms, d) for d in ("cpu", "cuda")}
    outs = {}
    params0 = None
    for dev, net in nets.items():
        li = len(net.layers) - 1
        layer = net.layers[li]
        bvec, tvec = net.bottom_vecs[li], net.top_vecs[li]
        for b, name in zip(bvec, bottoms):
            b.set_nchw(logical[name])
        if params0 is None:
            params0 = [torch.randn(tuple(p.data.shape), generator=g) * 0.5 for p in layer.params]
        for p, v in zip(layer.params, params0):
            if layer.type_name == "BatchNorm":
                v = v.abs() + 0.5
            p.data.copy_(v.to(p.data.device))
            p.diff.zero_()
        layer.forward(bvec, tvec)
        gR = torch.Generator().manual_seed(99)
        R = [torch.randn(t.shape, generator=gR) for t in tvec]
        for t, r in zip(tvec, R):
            if t.shape == ():
                t.diff = torch.ones((), dtype=t.dtype, device=t.data.device)
            else:
                t.set_nchw(r, diff=True)
        which = check if check is not None else [n not in int_bottoms for n in bottoms]
        layer.backward(tvec, which, bvec)
        outs[dev] = dict(
            tops=[t.nchw().float().cpu().clone() for t in tvec],
            bdiff=[b.nchw(diff=True).float().cpu().clone() if w else None for b, w in zip(bvec, which)],
            pdiff=[p.diff.float().cpu().clone() for p in layer.params],
            pdata=[p.data.float().cpu().clone() for p in layer.params])
    c, gp = outs["cpu"], outs["cuda"]
    for a, b in zip(gp["tops"], c["tops"]):
        assert _rel(a, b) < tol, ("top", _rel(a, b))
    for a, b in zip(gp["bdiff"], c["bdiff"]):
        if a is not None:
            assert _rel(a, b) < tol, ("bottom diff", _rel(a, b))
    for a, b in zip(gp["pdiff"], c["pdiff"]):
        assert _rel(a, b) < tol, ("param diff", _rel(a, b))
    for a, b in zip(gp["pdata"], c["pdata"]):
        assert _rel(a, b) < tol, ("param data", _rel(a, b))
    return outs


B4 = {"x": (2, 3, 6, 5)}
B8 = {"x": (2, 8, 4, 4)}
XZ = {"x": (2, 3, 4, 4), "z": (2, 3, 4, 4)}

CASES = {
    "sigmoid": ('layer { name: "L" type: "Sigmoid" bottom: "x" top: "y" }', B4, {}),
    "sigmoid_inplace": ('layer { name: "L" type: "Sigmoid" bottom: "x" top: "x" }', B4, {}),
    "tanh": ('layer { name: "L" type: "TanH" bottom: "x" top: "y" }', B8, {}),
    "absval": ('layer { name: "L" type: "AbsVal" bottom: "x" top: "y" }', B4, {}),
    "absval_inplace": ('layer { name: "L" type: "AbsVal" bottom: "x" top: "x" }', B8, {}),
    "bnll": ('layer { name: "L" type: "BNLL" bottom: "x" top: "y" }', B4, {}),
    "exp": ('layer { name: "L" type: "Exp" bottom: "x" top: "y" exp_param { base: 2.0 scale: 0.5 shift: 0.1 } }',
            B4, {}),
    "log": ('layer { name: "L" type: "Log" bottom: "x" top: "y" log_param { scale: 0.7 shift: 0.2 } }', B4,
            {"positive": True}),
    "power": ('layer { name: "L" type: "Power" bottom: "x" top: "y" power_param { power: 2.0 scale: 0.5 '
              'shift: 0.3 } }', B4, {}),
    "power_frac": ('layer { name: "L" type: "Power" bottom: "x" top: "y" power_param { power: 0.5 scale: 1.5 '
                   'shift: 0.1 } }', B8, {"positive": True}),
    "threshold": ('layer { name: "L" type: "Threshold" bottom: "x" top: "y" threshold_param { threshold: 0.3 } }',
                  B4, {"check": [False]}),
    "prelu": ('layer { name: "L" type: "PReLU" bottom: "x" top: "y" }', B4, {}),
    "prelu_shared": ('layer { name: "L" type: "PReLU" bottom: "x" top: "y" prelu_param { channel_shared: true } }',
                     B8, {}),
    "prelu_2d": ('layer { name: "L" type: "PReLU" bottom: "x" top: "y" }', {"x": (5, 7)}, {}),
    "relu_odd": ('layer { name: "L" type: "ReLU" bottom: "x" top: "y" relu_param { negative_slope: 0.1 } }',
                 {"x": (3, 5, 1, 1)}, {}),
    "dropout_odd_test": ('layer { name: "L" type: "Dropout" bottom: "x" top: "y" dropout_param '
                         '{ dropout_ratio: 0.0 } }', {"x": (3, 5)}, {}),
    "eltwise_sum": ('layer { name: "L" type: "Eltwise" bottom: "x" bottom: "z" top: "y" eltwise_param '
                    '{ operation: SUM coeff: 0.5 coeff: -2.0 } }', XZ, {}),
    "eltwise_prod": ('layer { name: "L" type: "Eltwise" bottom: "x" bottom: "z" top: "y" eltwise_param '
                     '{ operation: PROD } }', XZ, {}),
    "eltwise_prod_unstable": ('layer { name: "L" type: "Eltwise" bottom: "x" bottom: "z" top: "y" eltwise_param '
                              '{ operation: PROD stable_prod_grad: false } }', XZ, {"positive": True}),
    "eltwise_max": ('layer { name: "L" type: "Eltwise" bottom: "x" bottom: "z" top: "y" eltwise_param '
                    '{ operation: MAX } }', XZ, {}),
    "concat_axis0": ('layer { name: "L" type: "Concat" bottom: "x" bottom: "z" top: "y" concat_param { axis: 0 } }',
                     {"x": (2, 3, 4, 4), "z": (1, 3, 4, 4)}, {}),
    "concat_odd_channels": ('layer { name: "L" type: "Concat" bottom: "x" bottom: "z" top: "y" }',
                            {"x": (2, 3, 4, 4), "z": (2, 2, 4, 4)}, {}),
    "concat_2d": ('layer { name: "L" type: "Concat" bottom: "x" bottom: "z" top: "y" }',
                  {"x": (4, 3), "z": (4, 5)}, {}),
    "slice": ('layer { name: "L" type: "Slice" bottom: "x" top: "y" top: "y2" slice_param { slice_point: 1 } }',
              B4, {}),
    "slice_axis2": ('layer { name: "L" type: "Slice" bottom: "x" top: "y" top: "y2" top: "y3" slice_param '
                    '{ axis: 2 slice_point: 2 slice_point: 3 } }', B4, {}),
    "split_3": ('layer { name: "L" type: "Split" bottom: "x" top: "a" top: "b" top: "c" }', {"x": (3, 5)}, {}),
    "flatten": ('layer { name: "L" type: "Flatten" bottom: "x" top: "y" }', B4, {}),
    "reshape_img": ('layer { name: "L" type: "Reshape" bottom: "x" top: "y" reshape_param { shape { dim: 0 '
                    'dim: 6 dim: 3 dim: -1 } } }', B4, {}),
    "reshape_to_img": ('layer { name: "L" type: "Reshape" bottom: "x" top: "y" reshape_param { shape { dim: 0 '
                       'dim: 3 dim: 2 dim: 5 } } }', {"x": (2, 30)}, {}),
    "tile": ('layer { name: "L" type: "Tile" bottom: "x" top: "y" tile_param { axis: 1 tiles: 3 } }', B4, {}),
    "tile_axis3": ('layer { name: "L" type: "Tile" bottom: "x" top: "y" tile_param { axis: 3 tiles: 2 } }', B4, {}),
    "reduction_sumsq": ('layer { name: "L" type: "Reduction" bottom: "x" top: "y" reduction_param '
                        '{ operation: SUMSQ axis: 1 } }', {"x": (3, 4, 2)}, {}),
    "reduction_mean_img": ('layer { name: "L" type: "Reduction" bottom: "x" top: "y" reduction_param '
                           '{ operation: MEAN axis: 2 coeff: 2.0 } }', B4, {}),
    "reduction_asum_all": ('layer { name: "L" type: "Reduction" bottom: "x" top: "y" reduction_param '
                           '{ operation: ASUM axis: 0 } }', B4, {}),
    "reduction_sum_ax1": ('layer { name: "L" type: "Reduction" bottom: "x" top: "y" reduction_param '
                          '{ operation: SUM axis: 1 } }', B4, {}),
    "batchnorm": ('layer { name: "L" type: "BatchNorm" bottom: "x" top: "y" batch_norm_param '
                  '{ use_global_stats: false } }', {"x": (4, 3, 2, 2)}, {}),
    "batchnorm_2d": ('layer { name: "L" type: "BatchNorm" bottom: "x" top: "y" batch_norm_param '
                     '{ use_global_stats: false } }', {"x": (16, 5)}, {}),
    "batchnorm_global": ('layer { name: "L" type: "BatchNorm" bottom: "x" top: "y" batch_norm_param '
                         '{ use_global_stats: true } }', {"x": (4, 3, 2, 2)}, {}),
    "mvn": ('layer { name: "L" type: "MVN" bottom: "x" top: "y" }', {"x": (2, 3, 3, 3)}, {}),
    "mvn_across": ('layer { name: "L" type: "MVN" bottom: "x" top: "y" mvn_param { across_channels: true } }',
                   {"x": (2, 3, 3, 3)}, {}),
    "mvn_2d_per_channel": ('layer { name: "L" type: "MVN" bottom: "x" top: "y" }', {"x": (3, 4)}, {}),
    "mvn_mean_only": ('layer { name: "L" type: "MVN" bottom: "x" top: "y" mvn_param { normalize_variance: false } }',
                      {"x": (2, 3, 3, 3)}, {}),
    "im2col": ('layer { name: "L" type: "Im2col" bottom: "x" top: "y" convolution_param { kernel_size: 2 '
               'stride: 1 } }', B4, {}),
    "im2col_pad_stride": ('layer { name: "L" type: "Im2col" bottom: "x" top: "y" convolution_param { kernel_size: 3 '
                          'stride: 2 pad: 1 } }', B4, {}),
    "euclidean": ('layer { name: "L" type: "EuclideanLoss" bottom: "x" bottom: "z" top: "y" }',
                  {"x": (3, 4), "z": (3, 4)}, {}),
    "sigmoid_xent": ('layer { name: "L" type: "SigmoidCrossEntropyLoss" bottom: "x" bottom: "z" top: "y" }',
                     {"x": (3, 4), "z": (3, 4)}, {"check": [True, False], "positive": True}),
    "hinge_l1": ('layer { name: "L" type: "HingeLoss" bottom: "x" bottom: "lab" top: "y" }',
                 {"x": (4, 3), "lab": (4,)}, {"int_bottoms": ("lab",)}),
    "hinge_l2": ('layer { name: "L" type: "HingeLoss" bottom: "x" bottom: "lab" top: "y" hinge_loss_param '
                 '{ norm: L2 } }', {"x": (4, 3), "lab": (4,)}, {"int_bottoms": ("lab",)}),
    "multinomial": ('layer { name: "L" type: "MultinomialLogisticLoss" bottom: "x" bottom: "lab" top: "y" }',
                    {"x": (4, 3), "lab": (4,)}, {"int_bottoms": ("lab",), "positive": True}),
    "infogain_bottom": ('layer { name: "L" type: "InfogainLoss" bottom: "x" bottom: "lab" bottom: "H" top: "y" }',
                        {"x": (4, 3), "lab": (4,), "H": (3, 3)},
                        {"int_bottoms": ("lab",), "positive": True, "check": [True, False, False]}),
    "contrastive": ('layer { name: "L" type: "ContrastiveLoss" bottom: "x" bottom: "z" bottom: "sim" top: "y" '
                    'contrastive_loss_param { margin: 2.0 } }', {"x": (4, 3), "z": (4, 3), "sim": (4,)},
                    {"int_bottoms": ("sim",), "check": [True, True, False]}),
    "contrastive_legacy": ('layer { name: "L" type: "ContrastiveLoss" bottom: "x" bottom: "z" bottom: "sim" top: "y" '
                           'contrastive_loss_param { margin: 2.0 legacy_version: true } }',
                           {"x": (4, 3), "z": (4, 3), "sim": (4,)},
                           {"int_bottoms": ("sim",), "check": [True, True, False]}),
    "softmax_axis1_3d": ('layer { name: "L" type: "Softmax" bottom: "x" top: "y" }', {"x": (2, 5, 3)}, {}),
    "spp": ('layer { name: "L" type: "SPP" bottom: "x" top: "y" spp_param { pyramid_height: 2 } }',
            {"x": (2, 8, 5, 6)}, {}),
    "batch_reindex": ('layer { name: "L" type: "BatchReindex" bottom: "x" bottom: "idx" top: "y" }',
                      {"x": (3, 8, 2, 2), "idx": (5,)}, {"values": {"idx": torch.tensor([2., 0., 2., 1., 0.])},
                                                        "check": [True, False]}),
    "filter": ('layer { name: "L" type: "Filter" bottom: "x" bottom: "sel" top: "y" }',
               {"x": (4, 8, 2, 2), "sel": (4,)}, {"values": {"sel": torch.tensor([1., 0., 1., 1.])},
                                                 "check": [True, False]}),
    "embed": ('layer { name: "L" type: "Embed" bottom: "x" top: "y" embed_param { num_output: 6 input_dim: 5 } }',
              {"x": (4, 3)}, {"values": {"x": torch.tensor([[0., 4., 2.], [2., 2., 1.], [3., 0., 0.], [4., 1., 3.]])},
                              "check": [False]}),
}


@pytest.mark.parametrize("name", sorted(CASES))
def test_layer_gpu_matches_cpu(gpu, name):
    txt, bottoms, kw = CASES[name]
    run_both(txt, bottoms, **kw)


def test_argmax_gpu_matches_cpu(gpu):
    for txt in ('argmax_param { top_k: 2 }', 'argmax_param { top_k: 2 out_max_val: true }',
                'argmax_param { top_k: 1 axis: 1 }', 'argmax_param { top_k: 2 axis: 3 out_max_val: true }'):
        layer = f'layer {{ name: "L" type: "ArgMax" bottom: "x" top: "y" {txt} }}'
        g = torch.Generator().manual_seed(5)
        x = torch.randperm(2 * 4 * 3 * 5, generator=g).float().reshape(2, 4, 3, 5)  # distinct values: no ties
        outs = []
        for dev in ("cpu", "cuda"):
            net = _net(layer, {"x": (2, 4, 3, 5)}, dev)
            net.blob_by_name("x").set_nchw(x)
            net.forward()
            outs.append(net.blob_by_name("y").nchw().float().cpu())
        assert torch.equal(outs[0], outs[1]), (txt, outs)


def test_stochastic_pooling_gpu(gpu):
    """Train: every output is an element of its window and the gradient lands on it;
    test: sum(x^2) / sum(x) equals the CPU reference."""
    layer = 'layer { name: "L" type: "Pooling" bottom: "x" top: "y" pooling_param { pool: STOCHASTIC ' \
            'kernel_size: 3 stride: 2 } }'
    g = torch.Generator().manual_seed(0)
    x = torch.rand(2, 8, 7, 7, generator=g) + 0.1
    net = _net(layer, {"x": (2, 8, 7, 7)}, "cuda")
    net.blob_by_name("x").set_nchw(x)
    net.forward()
    y = net.blob_by_name("y").nchw().float().cpu()
    xb = x.bfloat16().float()
    for n in range(2):
        for c in range(8):
            for p in range(3):
                for q in range(3):
                    win = xb[n, c, 2 * p:2 * p + 3, 2 * q:2 * q + 3].reshape(-1)
                    assert (win == y[n, c, p, q]).any()
    layer_blob = net.blob_by_name("y")
    layer_blob.set_nchw(torch.ones_like(y), diff=True)
    li = len(net.layers) - 1
    net.layers[li].backward(net.top_vecs[li], [True], net.bottom_vecs[li])
    dx = net.blob_by_name("x").nchw(diff=True).float().cpu()
    assert dx.sum().item() == pytest.approx(y.numel())
    for dev_phase in ("test",):
        del dev_phase
        outs = []
        for dev in ("cpu", "cuda"):
            n2 = Net(proto.parse_prototxt(
                f'name: "g"\nlayer {{ name: "in_x" type: "Input" top: "x" java_data_param {{ shape {{ dim: 2 dim: 8 '
                f'dim: 7 dim: 7 }} }} }}\n{layer}'), phase=proto.TEST, seed=3, device=dev)
            n2.blob_by_name("x").set_nchw(x)
            n2.forward()
            outs.append(n2.blob_by_name("y").nchw().float().cpu())
        assert _rel(outs[1], outs[0]) < 3e-2


def test_dropout_odd_count_train(gpu):
    """Dropout on an element count that is not a multiple of 8 (was refused in round 1)."""
    layer = 'layer { name: "L" type: "Dropout" bottom: "x" top: "y" dropout_param { dropout_ratio: 0.5 } }'
    net = _net(layer, {"x": (3, 7)}, "cuda")
    net.blob_by_name("x").set_nchw(torch.ones(3, 7))
    net.forward()
    y = net.blob_by_name("y").nchw().float().cpu()
    assert set(torch.unique(y).tolist()) <= {0.0, 2.0}


@pytest.mark.parametrize("layer", [
    'layer { name: "L" type: "BatchNorm" bottom: "x" top: "y" batch_norm_param { use_global_stats: false } }',
    'layer { name: "L" type: "MVN" bottom: "x" top: "y" mvn_param { across_channels: true } }'])
def test_norm_variance_large_mean(gpu, layer):
    """|mean| >> std (un-normalised pixels): the variance is the centred second moment
    E[(x - EX)^2] (batch_norm_layer.cu:50-59, mvn_layer.cu:31-36), not E[x^2] - EX^2,
    which cancels in fp32 and drives 1 / sqrt(var + eps) towards 1 / sqrt(eps)."""
    g = torch.Generator().manual_seed(11)
    shape = (64, 5) if "BatchNorm" in layer else (5, 64)
    x = 1000.0 + torch.randn(*shape, generator=g)
    outs = run_both(layer, {"x": shape}, values={"x": x})
    y = outs["cuda"]["tops"][0]
    # normalised output: unit variance per channel (BatchNorm) / per row (MVN)
    dim = 0 if "BatchNorm" in layer else 1
    assert abs(y.var(dim=dim, unbiased=False).mean().item() - 1.0) < 0.05
