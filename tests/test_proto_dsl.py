"""Prototxt / binary codecs, V1 upgrade, the SparkNet DSL and ProtoLoader helpers.

Mirrors src/test/scala/libs/LayerSpec.scala (DSL LeNet + CaffeNet prototxt with
replaceDataLayers + solver construction)."""
import os

import pytest
import torch

from sparknet_amd import dsl, proto
from sparknet_amd.core.net import Net

REF = "/root/reference/caffe"
have_ref = pytest.mark.skipif(not os.path.isdir(REF), reason="reference tree not mounted")


def dsl_lenet(batch=4):
    D = dsl
    return D.NetParam("LeNet",
                      D.RDDLayer("data", shape=[batch, 1, 28, 28]),
                      D.RDDLayer("label", shape=[batch, 1]),
                      D.ConvolutionLayer("conv1", ["data"], kernel=(5, 5), numOutput=20),
                      D.PoolingLayer("pool1", ["conv1"], pooling=D.Pooling.Max, kernel=(2, 2), stride=(2, 2)),
                      D.ConvolutionLayer("conv2", ["pool1"], kernel=(5, 5), numOutput=50),
                      D.PoolingLayer("pool2", ["conv2"], pooling=D.Pooling.Max, kernel=(2, 2), stride=(2, 2)),
                      D.InnerProductLayer("ip1", ["pool2"], numOutput=500),
                      D.ReLULayer("relu1", ["ip1"]),
                      D.InnerProductLayer("ip2", ["relu1"], numOutput=10),
                      D.SoftmaxWithLoss("loss", ["ip2", "label"]))


def test_dsl_lenet_structure_and_roundtrip():
    n = dsl_lenet()
    assert [l.type for l in n.layer] == ["JavaData", "JavaData", "Convolution", "Pooling", "Convolution",
                                         "Pooling", "InnerProduct", "ReLU", "InnerProduct", "SoftmaxWithLoss"]
    assert n.layer[2].convolution_param.kernel_h == 5 and n.layer[2].convolution_param.num_output == 20
    assert list(n.layer[0].java_data_param.shape.dim) == [4, 1, 28, 28]
    b = n.SerializeToString()
    n2 = proto.NetParameter()
    n2.ParseFromString(b)
    assert n2 == n
    assert proto.parse_prototxt(proto.to_prototxt(n)) == n
    # DSL nets set no fillers: Caffe's default constant-0 init
    net = Net(n, phase=proto.TRAIN)
    assert all(float(p.data.abs().sum()) == 0 for p in net.learnable_params)
    assert net.blob_by_name("pool2").shape == (4, 50, 4, 4)
    assert net.blob_by_name("ip2").shape == (4, 10)


@have_ref
@pytest.mark.parametrize("path", ["examples/cifar10/cifar10_quick_train_test.prototxt",
                                  "examples/cifar10/cifar10_full_train_test.prototxt",
                                  "models/bvlc_reference_caffenet/train_val.prototxt",
                                  "models/bvlc_googlenet/train_val.prototxt",
                                  "examples/mnist/lenet_train_test.prototxt"])
def test_reference_prototxt_roundtrip(path):
    n = proto.read_prototxt(os.path.join(REF, path))
    assert proto.parse_prototxt(proto.to_prototxt(n)) == n
    b = proto.NetParameter()
    b.ParseFromString(n.SerializeToString())
    assert b == n


@have_ref
def test_replace_data_layers_caffenet_and_solver():
    n = dsl.load_net_prototxt(os.path.join(REF, "models/bvlc_reference_caffenet/train_val.prototxt"))
    n = dsl.replace_data_layers(n, 4, 2, 3, 227, 227)
    assert [l.type for l in n.layer[:4]] == ["JavaData"] * 4
    assert n.layer[0].include[0].phase == proto.TEST and n.layer[2].include[0].phase == proto.TRAIN
    s = dsl.load_solver_prototxt_with_net(os.path.join(REF, "models/bvlc_reference_caffenet/solver.prototxt"), n)
    assert not s.HasField("net") and not s.HasField("snapshot") and s.net_param.layer[0].type == "JavaData"
    train = Net(n, phase=proto.TRAIN)
    test = Net(n, phase=proto.TEST)
    assert train.blob_by_name("data").shape == (4, 3, 227, 227)
    assert test.blob_by_name("data").shape == (2, 3, 227, 227)
    assert "accuracy" not in train.layer_names and "accuracy" in test.layer_names
    assert sum(p.caffe_count for p in train.learnable_params) == 60965224


@have_ref
def test_zoo_matches_reference_prototxt_shapes():
    """DSL-built zoo models have exactly the reference models' parameter blobs."""
    from sparknet_amd import models
    for name, path in [("cifar10_quick", "examples/cifar10/cifar10_quick_train_test.prototxt"),
                       ("cifar10_full", "examples/cifar10/cifar10_full_train_test.prototxt"),
                       ("lenet", "examples/mnist/lenet_train_test.prototxt"),
                       ("caffenet", "models/bvlc_reference_caffenet/train_val.prototxt"),
                       ("alexnet", "models/bvlc_alexnet/train_val.prototxt"),
                       ("googlenet", "models/bvlc_googlenet/train_val.prototxt")]:
        ref = proto.read_prototxt(os.path.join(REF, path))
        mine = models.build(name)
        ref_layers = {l.name: l for l in ref.layer if l.type not in ("Data",)}
        for l in mine.layer:
            if l.type == "JavaData":
                continue
            r = ref_layers.get(l.name)
            assert r is not None, (name, l.name)
            assert r.type == l.type, (name, l.name)
            if l.type == "Convolution":
                a, b = l.convolution_param, r.convolution_param
                assert a.num_output == b.num_output and a.group == b.group, (name, l.name)
                kr = list(b.kernel_size)[0]
                assert (a.kernel_h, a.kernel_w) == (kr, kr), (name, l.name)
            if l.type == "InnerProduct":
                assert l.inner_product_param.num_output == r.inner_product_param.num_output
            if l.type in ("Convolution", "InnerProduct"):
                assert [(p.lr_mult, p.decay_mult) for p in l.param] == [(p.lr_mult, p.decay_mult) for p in r.param], \
                    (name, l.name)


def test_v1_upgrade():
    n = proto.NetParameter(name="old")
    v1 = n.layers.add(name="ip", type=14)  # INNER_PRODUCT
    v1.bottom.append("data")
    v1.top.append("ip")
    v1.blobs_lr.extend([1.0, 2.0])
    v1.weight_decay.extend([1.0, 0.0])
    v1.inner_product_param.num_output = 3
    from sparknet_amd.proto.upgrade import upgrade_net
    upgrade_net(n)
    assert len(n.layers) == 0 and n.layer[0].type == "InnerProduct"
    assert [(p.lr_mult, p.decay_mult) for p in n.layer[0].param] == [(1.0, 1.0), (2.0, 0.0)]


def test_solver_prototxt_defaults():
    s = proto.parse_prototxt('base_lr: 0.01 lr_policy: "step" stepsize: 10 gamma: 0.5', proto.SolverParameter)
    assert s.type == "SGD" and s.iter_size == 1 and s.clip_gradients == -1 and s.regularization_type == "L2"
    assert s.delta == pytest.approx(1e-8) and s.momentum2 == pytest.approx(0.999)
    assert torch.tensor(1.0) == 1.0
