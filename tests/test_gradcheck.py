"""Finite-difference gradient checks of the layer catalogue on the fp32 CPU engine.

Reference: Caffe's GradientChecker (caffe/include/caffe/test/test_gradient_check_util.hpp:
19-60), used by every layer test (e.g. test_convolution_layer.cpp:610-690,
test_lrn_layer.cpp:156-240): the objective is sum(top * R) for a fixed random R, the
analytic gradient comes from the layer's Backward with top diff = R, and the numeric one
from central differences of Forward.  Here a random subset of the bottom / parameter
elements is probed per layer (stepsize 1e-2, relative threshold 1e-2 like Caffe's
float tests)."""
import pytest
import torch

from sparknet_amd import proto
from sparknet_amd.core.net import Net

EPS = 1e-2
PROBES = 24


def _net(layer_txt: str, bottoms: dict) -> Net:
    inputs = "".join(
        f'layer {{ name: "in_{n}" type: "Input" top: "{n}" '
        f'java_data_param {{ shape {{ {" ".join(f"dim: {d}" for d in shp)} }} }} }}\n'
        for n, shp in bottoms.items())
    return Net(proto.parse_prototxt(f'name: "g" force_backward: true\n{inputs}{layer_txt}'), phase=proto.TRAIN,
               seed=3)


def _objective(layer, tops, R):
    return sum(float((t.data.double() * r).sum()) for t, r in zip(tops, R))


def check_layer(layer_txt, bottoms, *, check_bottoms=None, positive=False, seed=0, scale=1.0, thresh=1e-2,
                int_bottoms=()):
    g = torch.Generator().manual_seed(seed)
    net = _net(layer_txt, bottoms)
    li = len(net.layers) - 1
    layer = net.layers[li]
    bvec, tvec = net.bottom_vecs[li], net.top_vecs[li]
    for b, name in zip(bvec, bottoms):
        if name in int_bottoms:
            b.data.copy_(torch.randint(0, 3, tuple(b.data.shape), generator=g).to(b.data.dtype))
            continue
        x = torch.randn(tuple(b.data.shape), generator=g) * scale
        b.data.copy_((x.abs() + 0.1) if positive else x)
    for p in layer.params:
        p.data.copy_(torch.randn(tuple(p.data.shape), generator=g) * 0.5)
    layer.forward(bvec, tvec)
    R = [torch.randn(tuple(t.data.shape), generator=g).double() for t in tvec]
    for t, r in zip(tvec, R):
        t.diff.copy_(r.to(t.diff.dtype))
    for b in bvec:
        b.diff.zero_()
    for p in layer.params:
        p.diff.zero_()
    which = check_bottoms if check_bottoms is not None else [n not in int_bottoms for n in bottoms]
    layer.backward(tvec, which, bvec)
    targets = [(b.data, b.diff) for b, chk in zip(bvec, which) if chk]
    targets += [(p.data, p.diff) for p in layer.params]
    assert targets, "nothing to check"
    for data, diff in targets:
        analytic = diff.double().reshape(-1).clone()
        flat = data.view(-1)
        idx = torch.randperm(flat.numel(), generator=g)[:PROBES]
        for j in idx.tolist():
            orig = float(flat[j])
            flat[j] = orig + EPS
            layer.forward(bvec, tvec)
            fp = _objective(layer, tvec, R)
            flat[j] = orig - EPS
            layer.forward(bvec, tvec)
            fm = _objective(layer, tvec, R)
            flat[j] = orig
            numeric = (fp - fm) / (2 * EPS)
            a = float(analytic[j])
            scale_ = max(abs(a), abs(numeric), 1.0)
            assert abs(a - numeric) <= thresh * scale_, (layer.type_name, j, a, numeric)


B4 = {"x": (2, 3, 6, 5)}

CASES = {
    "conv": ('layer { name: "L" type: "Convolution" bottom: "x" top: "y" convolution_param { num_output: 4 '
             'kernel_size: 3 stride: 2 pad: 1 } }', B4, {}),
    "conv_group": ('layer { name: "L" type: "Convolution" bottom: "x" top: "y" convolution_param { num_output: 4 '
                   'kernel_h: 2 kernel_w: 3 group: 2 } }', {"x": (2, 4, 5, 5)}, {}),
    "deconv": ('layer { name: "L" type: "Deconvolution" bottom: "x" top: "y" convolution_param { num_output: 2 '
               'kernel_size: 3 stride: 2 } }', B4, {}),
    "ip": ('layer { name: "L" type: "InnerProduct" bottom: "x" top: "y" inner_product_param { num_output: 5 } }',
           B4, {}),
    "pool_max": ('layer { name: "L" type: "Pooling" bottom: "x" top: "y" pooling_param { pool: MAX kernel_size: 3 '
                 'stride: 2 } }', B4, {}),
    "pool_ave": ('layer { name: "L" type: "Pooling" bottom: "x" top: "y" pooling_param { pool: AVE kernel_size: 3 '
                 'stride: 2 pad: 1 } }', B4, {}),
    "lrn_across": ('layer { name: "L" type: "LRN" bottom: "x" top: "y" lrn_param { local_size: 3 alpha: 0.5 '
                   'beta: 0.75 } }', {"x": (2, 7, 3, 3)}, {}),
    "lrn_within": ('layer { name: "L" type: "LRN" bottom: "x" top: "y" lrn_param { local_size: 3 alpha: 0.5 '
                   'beta: 0.75 norm_region: WITHIN_CHANNEL } }', {"x": (2, 3, 5, 5)}, {}),
    "relu_leaky": ('layer { name: "L" type: "ReLU" bottom: "x" top: "y" relu_param { negative_slope: 0.1 } }', B4, {}),
    "sigmoid": ('layer { name: "L" type: "Sigmoid" bottom: "x" top: "y" }', B4, {}),
    "tanh": ('layer { name: "L" type: "TanH" bottom: "x" top: "y" }', B4, {}),
    "bnll": ('layer { name: "L" type: "BNLL" bottom: "x" top: "y" }', B4, {}),
    "exp": ('layer { name: "L" type: "Exp" bottom: "x" top: "y" exp_param { base: 2.0 scale: 0.5 } }', B4, {}),
    "log": ('layer { name: "L" type: "Log" bottom: "x" top: "y" log_param { scale: 0.7 shift: 0.2 } }', B4,
            {"positive": True}),
    "power": ('layer { name: "L" type: "Power" bottom: "x" top: "y" power_param { power: 2.0 scale: 0.5 '
              'shift: 0.3 } }', B4, {}),
    "prelu": ('layer { name: "L" type: "PReLU" bottom: "x" top: "y" }', B4, {}),
    "softmax": ('layer { name: "L" type: "Softmax" bottom: "x" top: "y" }', {"x": (3, 5)}, {}),
    "eltwise_sum": ('layer { name: "L" type: "Eltwise" bottom: "x" bottom: "z" top: "y" eltwise_param '
                    '{ operation: SUM coeff: 0.5 coeff: -2.0 } }', {"x": (2, 3, 4, 4), "z": (2, 3, 4, 4)}, {}),
    "eltwise_prod": ('layer { name: "L" type: "Eltwise" bottom: "x" bottom: "z" top: "y" eltwise_param '
                     '{ operation: PROD } }', {"x": (2, 3, 4, 4), "z": (2, 3, 4, 4)}, {}),
    "eltwise_max": ('layer { name: "L" type: "Eltwise" bottom: "x" bottom: "z" top: "y" eltwise_param '
                    '{ operation: MAX } }', {"x": (2, 3, 4, 4), "z": (2, 3, 4, 4)}, {}),
    "concat": ('layer { name: "L" type: "Concat" bottom: "x" bottom: "z" top: "y" }',
               {"x": (2, 3, 4, 4), "z": (2, 2, 4, 4)}, {}),
    "slice": ('layer { name: "L" type: "Slice" bottom: "x" top: "y" top: "y2" slice_param { slice_point: 1 } }',
              B4, {}),
    "euclidean": ('layer { name: "L" type: "EuclideanLoss" bottom: "x" bottom: "z" top: "y" }',
                  {"x": (3, 4), "z": (3, 4)}, {}),
    "sigmoid_xent": ('layer { name: "L" type: "SigmoidCrossEntropyLoss" bottom: "x" bottom: "z" top: "y" }',
                     {"x": (3, 4), "z": (3, 4)}, {"check_bottoms": [True, False]}),
    "softmax_loss": ('layer { name: "L" type: "SoftmaxWithLoss" bottom: "x" bottom: "lab" top: "y" }',
                     {"x": (4, 3), "lab": (4,)}, {"int_bottoms": ("lab",)}),
    "batchnorm": ('layer { name: "L" type: "BatchNorm" bottom: "x" top: "y" batch_norm_param '
                  '{ use_global_stats: false } }', {"x": (4, 3, 2, 2)}, {"thresh": 3e-2}),
    "mvn": ('layer { name: "L" type: "MVN" bottom: "x" top: "y" }', {"x": (2, 3, 3, 3)}, {"thresh": 3e-2}),
    "flatten": ('layer { name: "L" type: "Flatten" bottom: "x" top: "y" }', B4, {}),
    "tile": ('layer { name: "L" type: "Tile" bottom: "x" top: "y" tile_param { axis: 1 tiles: 2 } }', B4, {}),
    "reduction": ('layer { name: "L" type: "Reduction" bottom: "x" top: "y" reduction_param { operation: SUMSQ '
                  'axis: 1 } }', {"x": (3, 4, 2)}, {}),
    "im2col": ('layer { name: "L" type: "Im2col" bottom: "x" top: "y" convolution_param { kernel_size: 2 '
               'stride: 1 } }', B4, {}),
    "absval": ('layer { name: "L" type: "AbsVal" bottom: "x" top: "y" }', B4, {}),
}


@pytest.mark.parametrize("name", sorted(CASES))
def test_gradient(name):
    txt, bottoms, kw = CASES[name]
    check_layer(txt, bottoms, **kw)
