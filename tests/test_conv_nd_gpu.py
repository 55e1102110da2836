"""N-d Convolution / Deconvolution / Im2col and general-axis Softmax on the GPU (HIP N-d
im2col / col2im kernels + the MFMA GEMM, csrc/kernels/conv_nd.hip) against the fp32 CPU
engine from identical initial weights (tests/test_conv_nd.py holds the CPU-side ports of
test_convolution_layer.cpp:297,492,628)."""
import pytest
import torch

from test_conv_nd import _net

pytestmark = pytest.mark.gpu

CASES = [
    # 3-D, two bottoms sharing filters (TestSimple3DConvolution's geometry)
    ('layer { name: "c" type: "Convolution" bottom: "x" bottom: "x2" top: "y" top: "y2" convolution_param { '
     'num_output: 4 kernel_size: 3 stride: 2 weight_filler { type: "gaussian" } bias_filler { type: "gaussian" } } }',
     {"x": (2, 3, 5, 6, 4), "x2": (2, 3, 5, 6, 4)}),
    # grouped, padded, anisotropic 3-D
    ('layer { name: "c" type: "Convolution" bottom: "x" top: "y" convolution_param { num_output: 8 group: 2 '
     'kernel_size: 2 kernel_size: 3 kernel_size: 1 stride: 1 stride: 2 stride: 1 pad: 1 pad: 0 pad: 1 '
     'weight_filler { type: "gaussian" } } }', {"x": (3, 6, 4, 7, 5)}),
    # force_nd_im2col on a 4-D blob (TestNDAgainst2D's layer, smaller)
    ('layer { name: "c" type: "Convolution" bottom: "x" top: "y" convolution_param { num_output: 12 bias_term: false '
     'group: 6 kernel_h: 5 kernel_w: 3 force_nd_im2col: true weight_filler { type: "gaussian" } } }',
     {"x": (3, 18, 11, 9)}),
    # one spatial axis, channel axis 2 of a 4-D blob
    ('layer { name: "c" type: "Convolution" bottom: "x" top: "y" convolution_param { num_output: 5 kernel_size: 3 '
     'axis: 2 weight_filler { type: "gaussian" } } }', {"x": (2, 3, 8, 9)}),
    ('layer { name: "d" type: "Deconvolution" bottom: "x" top: "y" convolution_param { num_output: 6 group: 2 '
     'kernel_size: 3 stride: 2 pad: 1 weight_filler { type: "gaussian" } bias_filler { type: "gaussian" } } }',
     {"x": (2, 4, 3, 4, 3)}),
    ('layer { name: "i" type: "Im2col" bottom: "x" top: "y" convolution_param { kernel_size: 2 stride: 2 pad: 1 } }',
     {"x": (2, 3, 4, 5, 4)}),
    ('layer { name: "s" type: "Softmax" bottom: "x" top: "y" softmax_param { axis: 2 } }', {"x": (2, 3, 6, 5)}),
]


def _run(txt, shapes, device, xs, dys):
    net = _net(txt, shapes, seed=11, device=device)
    for (name, _), x in zip(shapes.items(), xs):
        net.blob_by_name(name).set_nchw(x)
    net.forward()
    layer = net.layers[-1]
    tops = [net.top_vecs[-1][i] for i in range(len(net.top_vecs[-1]))]
    outs = [t.nchw().float().cpu().clone() for t in tops]
    for t, dy in zip(tops, dys):
        t.set_nchw(dy, diff=True)
    for p in layer.params:
        p.diff.zero_()
    bottoms = net.bottom_vecs[-1]
    layer.backward(tops, [True] * len(bottoms), bottoms)
    grads = [b.nchw(diff=True).float().cpu().clone() for b in bottoms]
    grads += [p.diff.float().cpu().clone() for p in layer.params]
    return outs, grads, layer.type_name


def _close(a, b, tol):
    err = (a - b).abs().max().item() / (b.abs().max().item() + 1e-6)
    assert err < tol, err


@pytest.mark.parametrize("case", range(len(CASES)))
def test_nd_layers_gpu_vs_cpu(gpu, case):
    txt, shapes = CASES[case]
    g = torch.Generator().manual_seed(case)
    xs = [torch.randn(s, generator=g) for s in shapes.values()]
    probe = _net(txt, shapes, seed=11)
    dys = [torch.randn(t.shape, generator=g) for t in probe.top_vecs[-1]]
    out_c, grad_c, kind = _run(txt, shapes, "cpu", xs, dys)
    out_g, grad_g, kind_g = _run(txt, shapes, gpu, xs, dys)
    assert kind == kind_g
    for a, b in zip(out_g, out_c):
        _close(a, b, 2e-2)
    for a, b in zip(grad_g, grad_c):
        _close(a, b, 2e-2)
