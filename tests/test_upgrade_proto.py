"""Legacy proto upgrades (proto/upgrade.py vs caffe/src/caffe/util/upgrade_proto.cpp).

Mirrors the eight cases of caffe/src/caffe/test/test_upgrade_proto.cpp with inline
prototxt written for this repo — padding-layer folding (simple, a padding layer behind a
two-top data layer, a whole V0 CaffeNet), V0 -> V1 (simple, every parameter), the
V0 -> V1 -> V2 chain, every V1 layer type instantiable after upgrade, and the solver type
upgrade — plus the data-transformation upgrade (upgrade_proto.cpp:586-646) and a V0
caffemodel loaded through ``Net.copy_trained_layers_from``.  When the reference tree is
present, ``test_reference_fixtures`` additionally runs every string fixture of the
reference test file through the matching upgrade function and compares the result
(the fixtures are read as data; the reference code is not executed)."""
import os
import re

import pytest
import torch
from google.protobuf import text_format

from sparknet_amd import proto
from sparknet_amd.core.layer import create_layer, layer_types
from sparknet_amd.proto import upgrade


def _net(txt):
    return proto.parse_prototxt(txt)


def _same(a, b):
    assert text_format.MessageToString(a) == text_format.MessageToString(b)


V0_PADDED = """
name: 'tiny'
input: 'img'
layers { layer { name: 'pad1' type: 'padding' pad: 2 } bottom: 'img' top: 'img_pad' }
layers { layer { name: 'conv1' type: 'conv' num_output: 8 kernelsize: 5 stride: 1 } bottom: 'img_pad' top: 'c1' }
layers { layer { name: 'relu1' type: 'relu' } bottom: 'c1' top: 'c1' }
layers { layer { name: 'pad2' type: 'padding' pad: 1 } bottom: 'c1' top: 'c1_pad' }
layers { layer { name: 'pool1' type: 'pool' pool: MAX kernelsize: 3 stride: 2 } bottom: 'c1_pad' top: 'p1' }
"""
V0_FOLDED = """
name: 'tiny'
input: 'img'
layers { layer { name: 'conv1' type: 'conv' num_output: 8 kernelsize: 5 stride: 1 pad: 2 } bottom: 'img' top: 'c1' }
layers { layer { name: 'relu1' type: 'relu' } bottom: 'c1' top: 'c1' }
layers { layer { name: 'pool1' type: 'pool' pool: MAX kernelsize: 3 stride: 2 pad: 1 } bottom: 'c1' top: 'p1' }
"""


def test_padding_simple_and_idempotent():
    out = upgrade.upgrade_v0_padding_layers(_net(V0_PADDED))
    _same(out, _net(V0_FOLDED))
    _same(upgrade.upgrade_v0_padding_layers(out), out)  # idempotent


def test_padding_behind_two_top_data_layer():
    src = _net("""
      name: 'two'
      layers { layer { name: 'data' type: 'data' source: 's' batchsize: 4 } top: 'data' top: 'label' }
      layers { layer { name: 'pad' type: 'padding' pad: 3 } bottom: 'data' top: 'data_pad' }
      layers { layer { name: 'conv' type: 'conv' num_output: 4 kernelsize: 7 } bottom: 'data_pad' top: 'c' }
      layers { layer { name: 'loss' type: 'softmax_loss' } bottom: 'c' bottom: 'label' }""")
    out = upgrade.upgrade_v0_padding_layers(src)
    assert [l.layer.name for l in out.layers] == ["data", "conv", "loss"]
    conv = out.layers[1]
    assert list(conv.bottom) == ["data"] and conv.layer.pad == 3
    assert list(out.layers[2].bottom) == ["c", "label"]


def test_padding_into_non_conv_is_refused():
    src = _net("""input: 'x'
      layers { layer { name: 'pad' type: 'padding' pad: 1 } bottom: 'x' top: 'xp' }
      layers { layer { name: 'r' type: 'relu' } bottom: 'xp' top: 'y' }""")
    with pytest.raises(ValueError, match="non-convolutional"):
        upgrade.upgrade_v0_padding_layers(src)


def test_v0_to_v1_simple():
    out, ok = upgrade.upgrade_v0_net(_net(V0_PADDED))
    assert ok
    _same(out, _net("""
      name: 'tiny'
      input: 'img'
      layers { name: 'conv1' type: CONVOLUTION bottom: 'img' top: 'c1'
               convolution_param { num_output: 8 pad: 2 kernel_size: 5 stride: 1 } }
      layers { name: 'relu1' type: RELU bottom: 'c1' top: 'c1' }
      layers { name: 'pool1' type: POOLING bottom: 'c1' top: 'p1'
               pooling_param { pool: MAX kernel_size: 3 stride: 2 pad: 1 } }"""))


def test_v0_to_v1_all_params():
    src = _net("""
      name: 'all'
      input: 'in' input_dim: 1 input_dim: 3 input_dim: 8 input_dim: 8 force_backward: true
      layers { layer { name: 'd' type: 'data' source: '/db' meanfile: '/m' batchsize: 8 cropsize: 6 mirror: true
                       scale: 0.5 rand_skip: 3 } top: 'data' top: 'label' }
      layers { layer { name: 'img' type: 'images' source: '/list' batchsize: 2 shuffle_images: true
                       new_height: 10 new_width: 12 rand_skip: 1 } top: 'i' top: 'il' }
      layers { layer { name: 'win' type: 'window_data' source: '/w' batchsize: 3 det_fg_threshold: 0.6
                       det_bg_threshold: 0.4 det_fg_fraction: 0.3 det_context_pad: 4 det_crop_mode: 'square' }
               top: 'w' top: 'wl' }
      layers { layer { name: 'h5' type: 'hdf5_data' source: '/h5' batchsize: 5 } top: 'h' }
      layers { layer { name: 'c' type: 'conv' num_output: 4 biasterm: false kernelsize: 3 pad: 1 stride: 2 group: 2
                       weight_filler { type: 'gaussian' std: 0.01 } bias_filler { type: 'constant' value: 1 }
                       blobs_lr: 1 blobs_lr: 2 weight_decay: 1 weight_decay: 0 } bottom: 'data' top: 'c' }
      layers { layer { name: 'ip' type: 'innerproduct' num_output: 7 biasterm: true
                       weight_filler { type: 'xavier' } bias_filler { type: 'constant' } } bottom: 'c' top: 'ip' }
      layers { layer { name: 'n' type: 'lrn' local_size: 3 alpha: 0.1 beta: 0.5 k: 2 } bottom: 'ip' top: 'n' }
      layers { layer { name: 'dr' type: 'dropout' dropout_ratio: 0.3 } bottom: 'n' top: 'n' }
      layers { layer { name: 'p' type: 'pool' pool: STOCHASTIC kernelsize: 2 stride: 2 pad: 1 } bottom: 'c' top: 'p' }
      layers { layer { name: 'cat' type: 'concat' concat_dim: 0 } bottom: 'p' bottom: 'p' top: 'cat' }
      layers { layer { name: 'ig' type: 'infogain_loss' source: '/H' } bottom: 'ip' bottom: 'label' }
      layers { layer { name: 'o' type: 'hdf5_output' hdf5_output_param { file_name: '/o.h5' } } bottom: 'ip' }
      layers { layer { name: 'bad' type: 'relu' num_output: 3 } bottom: 'ip' top: 'bad' }""")
    out, ok = upgrade.upgrade_v0_net(src)
    assert not ok  # num_output has no home on a ReLU layer: dropped and reported
    _same(out, _net("""
      name: 'all'
      input: 'in' input_dim: 1 input_dim: 3 input_dim: 8 input_dim: 8 force_backward: true
      layers { name: 'd' type: DATA top: 'data' top: 'label'
               data_param { source: '/db' batch_size: 8 rand_skip: 3 }
               transform_param { scale: 0.5 mirror: true crop_size: 6 mean_file: '/m' } }
      layers { name: 'img' type: IMAGE_DATA top: 'i' top: 'il'
               image_data_param { source: '/list' batch_size: 2 rand_skip: 1 shuffle: true new_height: 10
                                  new_width: 12 } }
      layers { name: 'win' type: WINDOW_DATA top: 'w' top: 'wl'
               window_data_param { source: '/w' batch_size: 3 fg_threshold: 0.6 bg_threshold: 0.4 fg_fraction: 0.3
                                   context_pad: 4 crop_mode: 'square' } }
      layers { name: 'h5' type: HDF5_DATA top: 'h' hdf5_data_param { source: '/h5' batch_size: 5 } }
      layers { name: 'c' type: CONVOLUTION bottom: 'data' top: 'c' blobs_lr: 1 blobs_lr: 2 weight_decay: 1
               weight_decay: 0
               convolution_param { num_output: 4 bias_term: false pad: 1 kernel_size: 3 group: 2 stride: 2
                                   weight_filler { type: 'gaussian' std: 0.01 }
                                   bias_filler { type: 'constant' value: 1 } } }
      layers { name: 'ip' type: INNER_PRODUCT bottom: 'c' top: 'ip'
               inner_product_param { num_output: 7 bias_term: true weight_filler { type: 'xavier' }
                                     bias_filler { type: 'constant' } } }
      layers { name: 'n' type: LRN bottom: 'ip' top: 'n' lrn_param { local_size: 3 alpha: 0.1 beta: 0.5 k: 2 } }
      layers { name: 'dr' type: DROPOUT bottom: 'n' top: 'n' dropout_param { dropout_ratio: 0.3 } }
      layers { name: 'p' type: POOLING bottom: 'c' top: 'p'
               pooling_param { pool: STOCHASTIC kernel_size: 2 stride: 2 pad: 1 } }
      layers { name: 'cat' type: CONCAT bottom: 'p' bottom: 'p' top: 'cat' concat_param { concat_dim: 0 } }
      layers { name: 'ig' type: INFOGAIN_LOSS bottom: 'ip' bottom: 'label' infogain_loss_param { source: '/H' } }
      layers { name: 'o' type: HDF5_OUTPUT bottom: 'ip' hdf5_output_param { file_name: '/o.h5' } }
      layers { name: 'bad' type: RELU bottom: 'ip' top: 'bad' }"""))


def test_v0_to_v2_chain_and_caffemodel(tmp_path):
    """V0 CaffeNet-style net -> current format through upgrade_net, and a V0 binary
    caffemodel (with weights) loaded into a current net by layer name."""
    v0 = _net("""
      name: 'v0net'
      input: 'data' input_dim: 2 input_dim: 3 input_dim: 9 input_dim: 9
      layers { layer { name: 'pad1' type: 'padding' pad: 1 } bottom: 'data' top: 'data_pad' }
      layers { layer { name: 'conv1' type: 'conv' num_output: 4 kernelsize: 3 stride: 2
                       weight_filler { type: 'gaussian' std: 0.1 } blobs_lr: 1 blobs_lr: 2
                       weight_decay: 1 weight_decay: 0 } bottom: 'data_pad' top: 'conv1' }
      layers { layer { name: 'relu1' type: 'relu' } bottom: 'conv1' top: 'conv1' }
      layers { layer { name: 'fc' type: 'innerproduct' num_output: 5 weight_filler { type: 'xavier' } }
               bottom: 'conv1' top: 'fc' }""")
    n = proto.NetParameter()
    n.CopyFrom(v0)
    upgrade.upgrade_net(n, strict=True)
    assert len(n.layers) == 0 and [l.type for l in n.layer] == ["Convolution", "ReLU", "InnerProduct"]
    c = n.layer[0]
    assert list(c.bottom) == ["data"] and list(c.convolution_param.pad) == [1]
    assert [(p.lr_mult, p.decay_mult) for p in c.param] == [(1.0, 1.0), (2.0, 0.0)]
    # a V0 "caffemodel": the same layers with legacy 4-D blobs
    from sparknet_amd.core.net import Net
    net = Net(v0, phase=proto.TRAIN, device="cpu")
    w = torch.arange(4 * 3 * 3 * 3, dtype=torch.float32).reshape(4, 3, 3, 3) / 100
    model = proto.NetParameter()
    model.CopyFrom(v0)
    conv = model.layers[1].layer
    bw = conv.blobs.add()
    bw.num, bw.channels, bw.height, bw.width = 4, 3, 3, 3
    bw.data.extend(w.reshape(-1).tolist())
    bb = conv.blobs.add()
    bb.num, bb.channels, bb.height, bb.width = 1, 1, 1, 4
    bb.data.extend([0.5, -0.5, 1.0, 2.0])
    del model.layers[3]  # only conv1's weights in this model (fc keeps its initialisation)
    path = tmp_path / "v0.caffemodel"
    proto.write_binary(str(path), model)
    net.copy_trained_layers_from(str(path))
    got = net.layer_by_name("conv1").params[0].to_caffe()
    assert torch.allclose(got, w)
    assert torch.allclose(net.layer_by_name("conv1").params[1].to_caffe().reshape(-1), torch.tensor([0.5, -0.5, 1.0, 2.0]))


def test_data_transformation_upgrade():
    n = _net("""
      layers { name: 'd' type: DATA top: 'data' top: 'label'
               data_param { source: '/db' batch_size: 4 scale: 0.25 mean_file: '/mean' crop_size: 5 mirror: true } }
      layers { name: 'i' type: IMAGE_DATA top: 'x' top: 'y' image_data_param { source: '/l' crop_size: 3 } }
      layers { name: 'w' type: WINDOW_DATA top: 'a' top: 'b' window_data_param { source: '/w' mirror: false } }
      layers { name: 'c' type: CONVOLUTION bottom: 'data' top: 'c' convolution_param { num_output: 1 kernel_size: 1 } }""")
    assert upgrade.net_needs_data_upgrade(n)
    upgrade.upgrade_net(n)
    d, i, w = n.layer[0], n.layer[1], n.layer[2]
    assert not any(d.data_param.HasField(f) for f in ("scale", "mean_file", "crop_size", "mirror"))
    assert (d.transform_param.scale, d.transform_param.mean_file, d.transform_param.crop_size,
            d.transform_param.mirror) == (0.25, "/mean", 5, True)
    assert d.data_param.source == "/db" and d.data_param.batch_size == 4
    assert i.transform_param.crop_size == 3 and not i.image_data_param.HasField("crop_size")
    assert w.transform_param.HasField("mirror") and not w.window_data_param.HasField("mirror")


def test_every_v1_layer_type_upgrades_to_a_registered_layer():
    enum = proto.V1LayerParameter.DESCRIPTOR.enum_types_by_name["LayerType"]
    from sparknet_amd.core.net import NetContext
    known = set(layer_types())
    ctx = NetContext(device=torch.device("cpu"), dtype=torch.float32, phase=proto.TRAIN)
    for v in enum.values:
        name = upgrade.v1_type_name(v.number)
        if v.name == "NONE":
            assert name == ""
            continue
        assert name in known, (v.name, name)
        layer = create_layer(proto.LayerParameter(name="x", type=name), ctx)  # registry lookup + construction
        assert layer.type_name == name


@pytest.mark.parametrize("old,new", [("SGD", "SGD"), ("ADAGRAD", "AdaGrad"), ("NESTEROV", "Nesterov"),
                                     ("RMSPROP", "RMSProp"), ("ADADELTA", "AdaDelta"), ("ADAM", "Adam")])
def test_solver_type_upgrade(old, new):
    sp = proto.parse_prototxt(f"net: 'n.prototxt' base_lr: 0.01 momentum: 0.0 lr_policy: 'inv' gamma: 0.0001 "
                              f"power: 0.75 solver_mode: GPU solver_type: {old}", proto.SolverParameter)
    upgrade.upgrade_solver(sp)
    assert sp.type == new and not sp.HasField("solver_type")


def test_v1_upgrade_param_specs_and_share_mode():
    n = _net("""layers { name: 'ip' type: INNER_PRODUCT bottom: 'x' top: 'y' param: 'w' param: ''
                         blob_share_mode: PERMISSIVE blobs_lr: 1 blobs_lr: 2 weight_decay: 1 weight_decay: 0
                         inner_product_param { num_output: 2 } }""")
    upgrade.upgrade_net(n)
    ps = n.layer[0].param
    assert [p.name for p in ps] == ["w", ""] and ps[1].HasField("name")
    assert ps[0].share_mode == 1 and not ps[1].HasField("share_mode")
    assert [(p.lr_mult, p.decay_mult) for p in ps] == [(1.0, 1.0), (2.0, 0.0)]


REF_TEST = "/root/reference/caffe/src/caffe/test/test_upgrade_proto.cpp"


def _fixtures():
    """(runner, input text, expected text) for every RunPaddingUpgradeTest / RunV0UpgradeTest /
    RunV1UpgradeTest call of the reference test file (string literals read as data)."""
    src = open(REF_TEST).read()
    out = []
    for body in re.split(r"\nTEST_F\(", src)[1:]:
        strings = {}
        for m in re.finditer(r"const string& (\w+) =\s*((?:\"(?:[^\"\\]|\\.)*\"\s*)+);", body):
            strings[m.group(1)] = "".join(re.findall(r"\"((?:[^\"\\]|\\.)*)\"", m.group(2)))
        for m in re.finditer(r"this->(Run(?:Padding|V0|V1)UpgradeTest)\(\s*(\w+),\s*(\w+)\)", body):
            out.append((m.group(1), strings[m.group(2)], strings[m.group(3)]))
    return out


@pytest.mark.skipif(not os.path.exists(REF_TEST), reason="reference tree not present")
def test_reference_fixtures():
    fx = _fixtures()
    assert len(fx) == 8  # 3 padding, V0 simple / all params / ImageNet, V1 simple / ImageNet, and one more V1
    for runner, inp, exp in fx:
        src, want = _net(inp), _net(exp)
        if runner == "RunPaddingUpgradeTest":
            got = upgrade.upgrade_v0_padding_layers(src)
        elif runner == "RunV0UpgradeTest":
            got, _ = upgrade.upgrade_v0_net(src)
        else:
            got, _ = upgrade.upgrade_v1_net(src)
        _same(got, want)
