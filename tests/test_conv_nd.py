"""N-d convolution / deconvolution / im2col and general-axis softmax on the fp32 CPU engine.

Ports of caffe/src/caffe/test/test_convolution_layer.cpp TestSimple3DConvolution (:297),
TestNDAgainst2D (:492) and TestGradient3D (:628), the 3-D Deconvolution / Im2col analogues,
and softmax over a non-channel axis of an image blob (softmax_layer.cpp:12-13 and
softmax_loss_layer.cpp:36-37 canonicalise any axis).  The GPU (HIP) twins of these run in
tests/test_conv_nd_gpu.py against this CPU engine."""
import itertools

import pytest
import torch
import torch.nn.functional as F

from sparknet_amd import proto
from sparknet_amd.core.net import Net

from test_gradcheck import check_layer


def _net(txt, shapes, seed=3, device="cpu"):
    inputs = "".join(
        f'layer {{ name: "in_{n}" type: "Input" top: "{n}" '
        f'java_data_param {{ shape {{ {" ".join(f"dim: {d}" for d in s)} }} }} }}\n' for n, s in shapes.items())
    return Net(proto.parse_prototxt(f'name: "nd" force_backward: true\n{inputs}{txt}'), phase=proto.TRAIN,
               seed=seed, device=torch.device(device))


def _fill(net, name, t):
    net.blob_by_name(name).set_nchw(t)


def test_simple_3d_convolution_two_bottoms():
    """TestSimple3DConvolution: 5-D bottoms (2, 3, 5, 6, 4), kernel 3, stride 2, 4 outputs,
    gaussian weights and bias, two bottom / top pairs sharing the filters."""
    shp = (2, 3, 5, 6, 4)
    net = _net('layer { name: "c" type: "Convolution" bottom: "x" bottom: "x2" top: "y" top: "y2" '
               'convolution_param { num_output: 4 kernel_size: 3 stride: 2 weight_filler { type: "gaussian" } '
               'bias_filler { type: "gaussian" } } }', {"x": shp, "x2": shp})
    layer = net.layers[-1]
    assert layer.type_name == "ConvolutionND" and tuple(layer.weight.shape) == (4, 3, 3, 3, 3)
    g = torch.Generator().manual_seed(0)
    xs = [torch.randn(shp, generator=g) for _ in range(2)]
    _fill(net, "x", xs[0])
    _fill(net, "x2", xs[1])
    net.forward()
    for x, top in zip(xs, ("y", "y2")):
        ref = F.conv3d(x, layer.weight.data, layer.bias.data, stride=2)
        assert net.blob_by_name(top).shape == tuple(ref.shape)
        torch.testing.assert_close(net.blob_by_name(top).data, ref, rtol=1e-4, atol=1e-4)


def _conv_pass(force_nd, x, w, dy):
    net = _net('layer { name: "c" type: "Convolution" bottom: "x" top: "y" convolution_param { num_output: 12 '
               f'bias_term: false group: 6 kernel_h: 11 kernel_w: 13 force_nd_im2col: {str(force_nd).lower()} '
               '} }', {"x": tuple(x.shape)})
    layer = net.layers[-1]
    assert layer.type_name == ("ConvolutionND" if force_nd else "Convolution")
    layer.weight.set_caffe(w)
    _fill(net, "x", x)
    net.forward()
    y = net.blob_by_name("y").nchw().clone()
    net.blob_by_name("y").set_nchw(dy, diff=True)
    layer.weight.diff.zero_()
    layer.backward([net.blob_by_name("y")], [True], [net.blob_by_name("x")])
    dw = layer.weight.diff.clone()
    return y, net.blob_by_name("x").nchw(diff=True).clone(), dw if force_nd else dw.permute(0, 3, 1, 2)


def test_nd_against_2d():
    """TestNDAgainst2D: force_nd_im2col (the N-d path) gives the 2-D path's forward, bottom
    diff and weight diff: bottom (15, 18, 22, 26), 12 outputs in 6 groups, kernel 11 x 13."""
    g = torch.Generator().manual_seed(1)
    x = torch.randn(15, 18, 22, 26, generator=g)
    w = torch.randn(12, 3, 11, 13, generator=g)
    dy = torch.randn(15, 12, 12, 14, generator=g)
    y2, dx2, dw2 = _conv_pass(False, x, w, dy)
    yn, dxn, dwn = _conv_pass(True, x, w, dy)
    torch.testing.assert_close(yn, y2, rtol=1e-4, atol=1e-3)
    torch.testing.assert_close(dxn, dx2, rtol=1e-4, atol=1e-3)
    torch.testing.assert_close(dwn, dw2, rtol=1e-4, atol=1e-2)


def test_gradient_3d():
    """TestGradient3D: finite-difference check of a 3-D convolution (kernel 3, stride 2)."""
    check_layer('layer { name: "c" type: "Convolution" bottom: "x" top: "y" convolution_param { num_output: 2 '
                'kernel_size: 3 stride: 2 } }', {"x": (2, 3, 5, 6, 4)})


def test_gradient_3d_grouped_padded_anisotropic():
    check_layer('layer { name: "c" type: "Convolution" bottom: "x" top: "y" convolution_param { num_output: 4 '
                'group: 2 kernel_size: 2 kernel_size: 3 kernel_size: 1 stride: 1 stride: 2 stride: 1 pad: 1 pad: 0 '
                'pad: 1 } }', {"x": (2, 4, 3, 5, 4)})


def test_conv_1d_and_4d_spatial():
    """One spatial axis (3-D blob) and four spatial axes (6-D blob) against explicit sums."""
    net = _net('layer { name: "c" type: "Convolution" bottom: "x" top: "y" convolution_param { num_output: 3 '
               'kernel_size: 3 stride: 2 pad: 1 } }', {"x": (2, 4, 9)})
    layer = net.layers[-1]
    x = torch.randn(2, 4, 9)
    _fill(net, "x", x)
    net.forward()
    torch.testing.assert_close(net.blob_by_name("y").data,
                               F.conv1d(x, layer.weight.data, layer.bias.data, stride=2, padding=1))
    shp = (1, 2, 3, 4, 3, 4)
    net = _net('layer { name: "c" type: "Convolution" bottom: "x" top: "y" convolution_param { num_output: 2 '
               'kernel_size: 2 } }', {"x": shp})
    layer = net.layers[-1]
    x = torch.randn(shp)
    _fill(net, "x", x)
    net.forward()
    w, b = layer.weight.data, layer.bias.data
    y = torch.zeros(1, 2, 2, 3, 2, 3) + b.view(1, 2, 1, 1, 1, 1)
    for taps in itertools.product(range(2), repeat=4):
        sl = tuple(slice(t, t + o) for t, o in zip(taps, (2, 3, 2, 3)))
        y += torch.einsum("kc,nc...->nk...", w[(slice(None), slice(None)) + taps], x[(slice(None), slice(None)) + sl])
    torch.testing.assert_close(net.blob_by_name("y").data, y, rtol=1e-4, atol=1e-4)


def test_conv_channel_axis_2():
    """axis: 2 on a 4-D blob: axes 0-1 are batch, axis 2 the channels, axis 3 spatial."""
    net = _net('layer { name: "c" type: "Convolution" bottom: "x" top: "y" convolution_param { num_output: 5 '
               'kernel_size: 3 axis: 2 } }', {"x": (2, 3, 4, 7)})
    layer = net.layers[-1]
    assert net.blob_by_name("y").shape == (2, 3, 5, 5)
    x = torch.randn(2, 3, 4, 7)
    _fill(net, "x", x)
    net.forward()
    ref = F.conv1d(x.reshape(6, 4, 7), layer.weight.data, layer.bias.data).reshape(2, 3, 5, 5)
    torch.testing.assert_close(net.blob_by_name("y").nchw(), ref, rtol=1e-4, atol=1e-4)
    check_layer('layer { name: "c" type: "Convolution" bottom: "x" top: "y" convolution_param { num_output: 2 '
                'kernel_size: 2 axis: 2 } }', {"x": (2, 3, 4, 5)})


def test_deconvolution_3d():
    shp = (2, 4, 3, 4, 3)
    net = _net('layer { name: "d" type: "Deconvolution" bottom: "x" top: "y" convolution_param { num_output: 6 '
               'group: 2 kernel_size: 3 stride: 2 pad: 1 bias_filler { type: "gaussian" } } }', {"x": shp})
    layer = net.layers[-1]
    assert layer.type_name == "DeconvolutionND" and tuple(layer.weight.shape) == (4, 3, 3, 3, 3)
    x = torch.randn(shp)
    layer.weight.data.copy_(torch.randn(4, 3, 3, 3, 3))
    _fill(net, "x", x)
    net.forward()
    ref = F.conv_transpose3d(x, layer.weight.data, layer.bias.data, stride=2, padding=1, groups=2)
    torch.testing.assert_close(net.blob_by_name("y").data, ref, rtol=1e-4, atol=1e-4)
    check_layer('layer { name: "d" type: "Deconvolution" bottom: "x" top: "y" convolution_param { num_output: 2 '
                'kernel_size: 2 stride: 2 } }', {"x": (2, 3, 2, 3, 2)})


def test_im2col_3d():
    shp = (2, 3, 4, 5, 4)
    net = _net('layer { name: "i" type: "Im2col" bottom: "x" top: "y" convolution_param { kernel_size: 2 '
               'stride: 2 pad: 1 } }', {"x": shp})
    assert net.layers[-1].type_name == "Im2colND" and net.blob_by_name("y").shape == (2, 24, 3, 3, 3)
    x = torch.randn(shp)
    _fill(net, "x", x)
    net.forward()
    y = net.blob_by_name("y").data
    xp = F.pad(x, (1, 1, 1, 1, 1, 1))
    for c, a, b, d in itertools.product(range(3), range(2), range(2), range(2)):
        exp = xp[:, c, a:a + 5:2, b:b + 5:2, d:d + 5:2]
        torch.testing.assert_close(y[:, c * 8 + a * 4 + b * 2 + d], exp)
    check_layer('layer { name: "i" type: "Im2col" bottom: "x" top: "y" convolution_param { kernel_size: 2 '
                'stride: 1 } }', {"x": (2, 2, 3, 3, 3)})


@pytest.mark.parametrize("axis", [2, 3, -1, 0])
def test_softmax_any_axis_image_blob(axis):
    net = _net(f'layer {{ name: "s" type: "Softmax" bottom: "x" top: "y" softmax_param {{ axis: {axis} }} }}',
               {"x": (2, 3, 4, 5)})
    x = torch.randn(2, 3, 4, 5)
    _fill(net, "x", x)
    net.forward()
    torch.testing.assert_close(net.blob_by_name("y").nchw(), torch.softmax(x, dim=axis), rtol=1e-5, atol=1e-6)
    check_layer(f'layer {{ name: "s" type: "Softmax" bottom: "x" top: "y" softmax_param {{ axis: {axis} }} }}',
                {"x": (2, 3, 3, 2)})


def test_softmax_loss_axis_2_image_blob():
    """SoftmaxWithLoss over axis 2 of (N, C, H, W): one prediction per (n, c, w) over H classes,
    labels of shape (N, C, W) in that order; loss, prob top and gradient vs torch."""
    shp = (2, 3, 4, 5)
    net = _net('layer { name: "s" type: "SoftmaxWithLoss" bottom: "x" bottom: "l" top: "loss" top: "prob" '
               'softmax_param { axis: 2 } }', {"x": shp, "l": (2, 3, 5)})
    x = torch.randn(shp)
    lab = torch.randint(0, 4, (2, 3, 5)).float()
    _fill(net, "x", x)
    net.blob_by_name("l").data.copy_(lab)
    net.forward()
    logp = torch.log_softmax(x, dim=2)
    ref = -logp.gather(2, lab.long().unsqueeze(2)).mean()
    assert abs(float(net.blob_by_name("loss").data) - float(ref)) < 1e-5
    torch.testing.assert_close(net.blob_by_name("prob").nchw(), logp.exp(), rtol=1e-5, atol=1e-6)
    xr = x.clone().requires_grad_(True)
    (-torch.log_softmax(xr, 2).gather(2, lab.long().unsqueeze(2)).mean()).backward()
    net.blob_by_name("loss").diff.fill_(1.0)
    layer = net.layers[-1]
    layer.backward([net.blob_by_name("loss"), net.blob_by_name("prob")], [True, False],
                   [net.blob_by_name("x"), net.blob_by_name("l")])
    torch.testing.assert_close(net.blob_by_name("x").nchw(diff=True), xr.grad, rtol=1e-5, atol=1e-6)
