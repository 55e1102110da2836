"""pycaffe-compatible API (sparknet_amd.pycaffe) on the CPU engine, mirroring the
reference's python tests (caffe/python/caffe/test/test_net.py, test_net_spec.py,
test_solver.py, test_io.py, test_python_layer.py)."""
import os

import numpy as np
import pytest

from sparknet_amd import proto
from sparknet_amd import pycaffe as caffe
from sparknet_amd.pycaffe import layers as L
from sparknet_amd.pycaffe import params as P


def simple_net_file(tmp_path, num_output=13):
    p = tmp_path / "net.prototxt"
    p.write_text("""name: 'testnet' force_backward: true
    layer { type: 'DummyData' name: 'data' top: 'data' top: 'label'
      dummy_data_param { num: 5 channels: 2 height: 3 width: 4
        num: 5 channels: 1 height: 1 width: 1
        data_filler { type: 'gaussian' std: 1 }
        data_filler { type: 'constant' } } }
    layer { type: 'Convolution' name: 'conv' bottom: 'data' top: 'conv'
      convolution_param { num_output: 11 kernel_size: 2 pad: 3
        weight_filler { type: 'gaussian' std: 1 }
        bias_filler { type: 'constant' value: 2 } }
        param { decay_mult: 1 } param { decay_mult: 0 } }
    layer { type: 'InnerProduct' name: 'ip' bottom: 'conv' top: 'ip'
      inner_product_param { num_output: %d
        weight_filler { type: 'gaussian' std: 2.5 }
        bias_filler { type: 'constant' value: -3 } } }
    layer { type: 'SoftmaxWithLoss' name: 'loss' bottom: 'ip' bottom: 'label' top: 'loss' }""" % num_output)
    return str(p)


def test_net_forward_backward_inputs_outputs(tmp_path):
    caffe.set_mode_cpu()
    net = caffe.Net(simple_net_file(tmp_path), caffe.TRAIN)
    assert net.inputs == [] and net.outputs == ["loss"]
    assert list(net.params) == ["conv", "ip"] and net.params["conv"][0].data.shape == (11, 2, 2, 2)
    out = net.forward()
    assert np.isfinite(out["loss"]).all()
    net.backward()
    assert np.abs(net.params["ip"][0].diff).sum() > 0
    assert net.blobs["conv"].data.shape == (5, 11, 8, 9)


def test_net_save_and_read(tmp_path):
    net = caffe.Net(simple_net_file(tmp_path), caffe.TRAIN)
    f = str(tmp_path / "w.caffemodel")
    net.save(f)
    net2 = caffe.Net(simple_net_file(tmp_path), f, caffe.TRAIN)
    for name in net.params:
        for a, b in zip(net.params[name], net2.params[name]):
            assert np.abs(a.data - b.data).sum() == 0


def test_param_write_back_and_blob_views(tmp_path):
    net = caffe.Net(simple_net_file(tmp_path), caffe.TRAIN)
    w = net.params["ip"][0]
    w.data[...] = 0.5
    assert np.all(net.params["ip"][0].data == 0.5)
    d = net.blobs["data"].data
    d[...] = 1.0  # CPU fp32 blobs are live views of the engine storage
    assert float(net._net.blob_by_name("data").data.sum()) == d.size


def lenet(batch):
    n = caffe.NetSpec()
    n.data, n.label = L.DummyData(shape=[dict(dim=[batch, 1, 28, 28]), dict(dim=[batch, 1, 1, 1])],
                                  transform_param=dict(scale=1. / 255), ntop=2)
    n.conv1 = L.Convolution(n.data, kernel_size=5, num_output=20, weight_filler=dict(type="xavier"))
    n.pool1 = L.Pooling(n.conv1, kernel_size=2, stride=2, pool=P.Pooling.MAX)
    n.conv2 = L.Convolution(n.pool1, kernel_size=5, num_output=50, weight_filler=dict(type="xavier"))
    n.pool2 = L.Pooling(n.conv2, kernel_size=2, stride=2, pool=P.Pooling.MAX)
    n.ip1 = L.InnerProduct(n.pool2, num_output=500, weight_filler=dict(type="xavier"))
    n.relu1 = L.ReLU(n.ip1, in_place=True)
    n.ip2 = L.InnerProduct(n.relu1, num_output=10, weight_filler=dict(type="xavier"))
    n.loss = L.SoftmaxWithLoss(n.ip2, n.label)
    return n.to_proto()


def anon_lenet(batch):
    data, label = L.DummyData(shape=[dict(dim=[batch, 1, 28, 28]), dict(dim=[batch, 1, 1, 1])], ntop=2)
    conv1 = L.Convolution(data, kernel_size=5, num_output=20, weight_filler=dict(type="xavier"))
    pool1 = L.Pooling(conv1, kernel_size=2, stride=2, pool=P.Pooling.MAX)
    ip1 = L.InnerProduct(pool1, num_output=500, weight_filler=dict(type="xavier"))
    relu1 = L.ReLU(ip1, in_place=True)
    ip2 = L.InnerProduct(relu1, num_output=10, weight_filler=dict(type="xavier"))
    return L.SoftmaxWithLoss(ip2, label).to_proto()


def test_net_spec_lenet(tmp_path):
    np_ = lenet(8)
    assert list(np_.layer[6].bottom) == list(np_.layer[6].top)  # in-place ReLU
    assert np_.layer[2].pooling_param.pool == 0 and np_.layer[1].convolution_param.num_output == 20
    assert list(np_.layer[1].convolution_param.kernel_size) == [5]
    p = tmp_path / "lenet.prototxt"
    p.write_text(proto.to_prototxt(np_))
    net = caffe.Net(str(p), caffe.TEST)
    assert len(net.layers) == 9
    anon = anon_lenet(8)
    assert [l.name for l in anon.layer][:2] == ["DummyData1", "Convolution1"]
    assert list(anon.layer[4].bottom) == list(anon.layer[4].top)


def test_net_spec_zero_tops(tmp_path):
    n = caffe.NetSpec()
    n.data, n.data2 = L.DummyData(shape=dict(dim=[3]), ntop=2)
    n.silence_data = L.Silence(n.data, ntop=0)
    n.silence_data2 = L.Silence(n.data2, ntop=0)
    p = tmp_path / "silent.prototxt"
    p.write_text(proto.to_prototxt(n.to_proto()))
    net = caffe.Net(str(p), caffe.TEST)
    assert len(net.forward()) == 0


def test_solver_solve_and_snapshot(tmp_path, monkeypatch):
    monkeypatch.chdir(tmp_path)
    net_f = simple_net_file(tmp_path)
    sf = tmp_path / "solver.prototxt"
    sf.write_text(f"""net: '{net_f}' test_iter: 2 test_interval: 10 base_lr: 0.01 momentum: 0.9
        weight_decay: 0.0005 lr_policy: 'inv' gamma: 0.0001 power: 0.75 display: 100 max_iter: 20
        snapshot_after_train: false snapshot_prefix: "model" """)
    solver = caffe.SGDSolver(str(sf))
    assert isinstance(caffe.get_solver(str(sf)), caffe.SGDSolver)
    assert len(solver.test_nets) == 1
    assert solver.iter == 0
    solver.solve()
    assert solver.iter == 20
    solver.snapshot()
    assert os.path.isfile("model_iter_20.caffemodel") and os.path.isfile("model_iter_20.solverstate")


def test_io_blobproto_and_datum():
    a = np.arange(24, dtype=np.float32).reshape(2, 3, 4)
    bp = caffe.io.array_to_blobproto(a)
    assert np.array_equal(caffe.io.blobproto_to_array(bp), a)
    old = proto.BlobProto(num=1, channels=2, height=3, width=4)
    old.data.extend(range(24))
    assert caffe.io.blobproto_to_array(old).shape == (1, 2, 3, 4)
    s = caffe.io.arraylist_to_blobprotovector_str([a, a * 2])
    back = caffe.io.blobprotovector_str_to_arraylist(s)
    assert np.array_equal(back[1], a * 2)
    u8 = (np.arange(24) % 251).astype(np.uint8).reshape(2, 3, 4)
    d = caffe.io.array_to_datum(u8, label=7)
    assert d.label == 7 and np.array_equal(caffe.io.datum_to_array(d), u8)


def test_io_transformer_roundtrip_and_oversample():
    t = caffe.io.Transformer({"data": (1, 3, 8, 10)})
    t.set_transpose("data", (2, 0, 1))
    t.set_channel_swap("data", (2, 1, 0))
    t.set_raw_scale("data", 255.0)
    t.set_mean("data", np.array([10.0, 20.0, 30.0]))
    t.set_input_scale("data", 0.5)
    img = np.random.default_rng(0).random((8, 10, 3)).astype(np.float32)
    x = t.preprocess("data", img)
    assert x.shape == (3, 8, 10)
    assert np.allclose(x[0], (img[:, :, 2] * 255 - 10) * 0.5, atol=1e-4)
    assert np.allclose(t.deprocess("data", x), img, atol=1e-5)
    crops = caffe.io.oversample([img, img], (4, 6))
    assert crops.shape == (20, 4, 6, 3)
    assert np.array_equal(crops[5], crops[0][:, ::-1, :])
    r = caffe.io.resize_image(img, (16, 20))
    assert r.shape == (16, 20, 3) and abs(float(r.mean()) - float(img.mean())) < 0.05


def test_classifier_predicts_probabilities(tmp_path):
    deploy = tmp_path / "deploy.prototxt"
    deploy.write_text("""name: 'tiny' input: 'data' input_shape { dim: 10 dim: 3 dim: 8 dim: 8 }
      layer { name: 'ip' type: 'InnerProduct' bottom: 'data' top: 'ip'
        inner_product_param { num_output: 4 weight_filler { type: 'gaussian' std: 0.1 } } }
      layer { name: 'prob' type: 'Softmax' bottom: 'ip' top: 'prob' }""")
    net = caffe.Net(str(deploy), caffe.TEST)
    w = str(tmp_path / "tiny.caffemodel")
    net.save(w)
    clf = caffe.Classifier(str(deploy), w, image_dims=(10, 10), raw_scale=255.0)
    imgs = [np.random.default_rng(i).random((12, 12, 3)).astype(np.float32) for i in range(3)]
    pr = clf.predict(imgs)
    assert pr.shape == (3, 4) and np.allclose(pr.sum(1), 1.0, atol=1e-4)
    pc = clf.predict(imgs, oversample=False)
    assert pc.shape == (3, 4)


def test_draw_dot_and_layer_types():
    dot = caffe.draw.get_graph_dot(lenet(4))
    assert dot.startswith('digraph') and "conv1" in dot and "kernel size: 5" in dot
    types = caffe.layer_type_list()
    assert "Convolution" in types and "Python" in types


class _DoubleLayer(caffe.Layer):
    def reshape(self, bottom, top):
        top[0].reshape(bottom[0].shape)

    def forward(self, bottom, top):
        top[0].data = bottom[0].data * 2

    def backward(self, top, propagate_down, bottom):
        bottom[0].diff = top[0].diff * 2


def test_python_layer_through_pycaffe(tmp_path, monkeypatch):
    import sys
    import types
    mod = types.ModuleType("pylayer_double")
    mod.DoubleLayer = _DoubleLayer
    monkeypatch.setitem(sys.modules, "pylayer_double", mod)
    p = tmp_path / "py.prototxt"
    p.write_text("""name: 'py' force_backward: true input: 'data' input_shape { dim: 2 dim: 3 }
      layer { type: 'Python' name: 'one' bottom: 'data' top: 'one'
        python_param { module: 'pylayer_double' layer: 'DoubleLayer' } }
      layer { type: 'Python' name: 'two' bottom: 'one' top: 'two'
        python_param { module: 'pylayer_double' layer: 'DoubleLayer' } }""")
    net = caffe.Net(str(p), caffe.TRAIN)
    x = np.arange(6, dtype=np.float32).reshape(2, 3)
    out = net.forward(data=x)
    assert np.allclose(out["two"], 4 * x)
    g = net.backward(two=np.ones((2, 3), np.float32))
    assert np.allclose(g["data"], 4.0)


@pytest.mark.parametrize("cls", ["NesterovSolver", "AdamSolver"])
def test_solver_types(tmp_path, cls):
    net_f = simple_net_file(tmp_path)
    sf = tmp_path / "s.prototxt"
    sf.write_text(f"net: '{net_f}' base_lr: 0.001 lr_policy: 'fixed' momentum: 0.9 max_iter: 3")
    s = getattr(caffe, cls)(str(sf))
    s.step(3)
    assert s.iter == 3 and s._s.type == cls[:-len("Solver")]


def test_detector_windows_and_context_crop(tmp_path):
    """detector.py: detect_windows warps every window through the net; context padding
    grows the box and fills the out-of-image part with the raw-space mean."""
    from PIL import Image
    deploy = tmp_path / "det.prototxt"
    deploy.write_text("""name: 'det' input: 'data' input_shape { dim: 4 dim: 3 dim: 8 dim: 8 }
      layer { name: 'ip' type: 'InnerProduct' bottom: 'data' top: 'ip'
        inner_product_param { num_output: 5 weight_filler { type: 'gaussian' std: 0.1 } } }
      layer { name: 'prob' type: 'Softmax' bottom: 'ip' top: 'prob' }""")
    net = caffe.Net(str(deploy), caffe.TEST)
    w = str(tmp_path / "det.caffemodel")
    net.save(w)
    img = tmp_path / "im.png"
    Image.fromarray(np.random.default_rng(0).integers(0, 256, (20, 24, 3), dtype=np.uint8)).save(img)
    det = caffe.Detector(str(deploy), w, raw_scale=255.0)
    wins = [np.array([0, 0, 10, 12]), np.array([5, 6, 19, 23]), np.array([2, 2, 8, 8])]
    out = det.detect_windows([(str(img), wins)])
    assert len(out) == 3 and out[1]["filename"] == str(img)
    assert all(d["prediction"].shape == (5,) and abs(d["prediction"].sum() - 1) < 1e-4 for d in out)
    mean = np.array([10.0, 20.0, 30.0])
    det = caffe.Detector(str(deploy), w, mean=mean, raw_scale=255.0, context_pad=2)
    im = caffe.io.load_image(str(img))
    c = det.crop(im, np.array([0, 0, 19, 23]))  # whole image: the border is context
    assert c.shape == (8, 8, 3)
    assert np.allclose(c[0, 0], mean / 255.0) and np.allclose(c[-1, -1], mean / 255.0)
    assert 0.0 <= c[4, 4].min() and c[4, 4].max() <= 1.0
