"""Model zoo built with the DSL — the architectures SparkNet trains or BASELINE.json names:

* ``lenet``          — caffe/examples/mnist/lenet_train_test.prototxt
* ``cifar10_quick``  — caffe/examples/cifar10/cifar10_quick_train_test.prototxt
* ``cifar10_full``   — caffe/examples/cifar10/cifar10_full_train_test.prototxt (CifarApp)
* ``caffenet``       — caffe/models/bvlc_reference_caffenet/train_val.prototxt (ImageNetApp)
* ``alexnet``        — caffe/models/bvlc_alexnet/train_val.prototxt (LRN before pooling)
* ``googlenet``      — caffe/models/bvlc_googlenet/train_val.prototxt (aux heads 0.3)
* ``vgg16``          — not in the reference; authored here (BASELINE config #5)

Each builder returns a NetParameter whose data entry points are SparkNet ``JavaData``
layers (TRAIN and TEST variants, like ProtoLoader.replaceDataLayers), and each has a
matching ``*_solver`` with the reference hyper-parameters.
"""
from __future__ import annotations

from .. import proto
from ..dsl import (AccuracyLayer, ConcatLayer, ConvolutionLayer, DropoutLayer, Include, InnerProductLayer,
                   LRNLayer, NetParam, Pooling, PoolingLayer, RDDLayer, ReLULayer, SoftmaxWithLoss)

WB = [(1.0, 1.0), (2.0, 0.0)]   # weight / bias lr & decay mults used by the ImageNet models
W12 = [{"lr_mult": 1.0}, {"lr_mult": 2.0}]


def _g(std):
    return {"type": "gaussian", "std": std}


def _c(v=0.0):
    return {"type": "constant", "value": v}


XAV = {"type": "xavier"}


def data_layers(train_batch, test_batch, c, h, w):
    return [RDDLayer("data", [train_batch, c, h, w], Include.Train),
            RDDLayer("label", [train_batch, 1], Include.Train),
            RDDLayer("data", [test_batch, c, h, w], Include.Test),
            RDDLayer("label", [test_batch, 1], Include.Test)]


def _conv(name, bottom, k, n, stride=1, pad=0, group=1, wf=None, bf=None, param=WB):
    return ConvolutionLayer(name, [bottom], (k, k), n, stride=stride if stride != 1 else None,
                            pad=pad if pad else None, group=group, weight_filler=wf, bias_filler=bf, param=param)


def _relu(name, blob):
    return ReLULayer(name, [blob], in_place=True)


def _pool(name, bottom, k, s, ave=False, pad=0):
    return PoolingLayer(name, [bottom], Pooling.Ave if ave else Pooling.Max, (k, k), (s, s), pad=pad or None)


def _ip(name, bottom, n, wf, bf, param=WB):
    return InnerProductLayer(name, [bottom], n, weight_filler=wf, bias_filler=bf, param=param)


def _head(logits, top5=False, prefix=""):
    out = [AccuracyLayer(prefix + "accuracy", [logits, "label"])]
    if top5:
        out.append(AccuracyLayer(prefix + "accuracy_top5", [logits, "label"], top_k=5))
    out.append(SoftmaxWithLoss(prefix + "loss", [logits, "label"]))
    return out


# --------------------------------------------------------------------------------------

def lenet(train_batch=64, test_batch=100):
    return NetParam("LeNet", *data_layers(train_batch, test_batch, 1, 28, 28),
                    _conv("conv1", "data", 5, 20, wf=XAV, bf=_c(), param=W12),
                    _pool("pool1", "conv1", 2, 2),
                    _conv("conv2", "pool1", 5, 50, wf=XAV, bf=_c(), param=W12),
                    _pool("pool2", "conv2", 2, 2),
                    _ip("ip1", "pool2", 500, XAV, _c(), W12),
                    _relu("relu1", "ip1"),
                    _ip("ip2", "ip1", 10, XAV, _c(), W12),
                    *_head("ip2"))


def cifar10_quick(train_batch=100, test_batch=100):
    return NetParam("CIFAR10_quick", *data_layers(train_batch, test_batch, 3, 32, 32),
                    _conv("conv1", "data", 5, 32, pad=2, wf=_g(1e-4), bf=_c(), param=W12),
                    _pool("pool1", "conv1", 3, 2),
                    _relu("relu1", "pool1"),
                    _conv("conv2", "pool1", 5, 32, pad=2, wf=_g(0.01), bf=_c(), param=W12),
                    _relu("relu2", "conv2"),
                    _pool("pool2", "conv2", 3, 2, ave=True),
                    _conv("conv3", "pool2", 5, 64, pad=2, wf=_g(0.01), bf=_c(), param=W12),
                    _relu("relu3", "conv3"),
                    _pool("pool3", "conv3", 3, 2, ave=True),
                    _ip("ip1", "pool3", 64, _g(0.1), _c(), W12),
                    _ip("ip2", "ip1", 10, _g(0.1), _c(), W12),
                    *_head("ip2"))


def cifar10_full(train_batch=100, test_batch=100):
    return NetParam("CIFAR10_full", *data_layers(train_batch, test_batch, 3, 32, 32),
                    _conv("conv1", "data", 5, 32, pad=2, wf=_g(1e-4), bf=_c(), param=W12),
                    _pool("pool1", "conv1", 3, 2),
                    _relu("relu1", "pool1"),
                    LRNLayer("norm1", ["pool1"], 3, 5e-5, 0.75, within=True),
                    _conv("conv2", "norm1", 5, 32, pad=2, wf=_g(0.01), bf=_c(), param=W12),
                    _relu("relu2", "conv2"),
                    _pool("pool2", "conv2", 3, 2, ave=True),
                    LRNLayer("norm2", ["pool2"], 3, 5e-5, 0.75, within=True),
                    _conv("conv3", "norm2", 5, 64, pad=2, wf=_g(0.01), bf=_c(), param=None),
                    _relu("relu3", "conv3"),
                    _pool("pool3", "conv3", 3, 2, ave=True),
                    _ip("ip1", "pool3", 10, _g(0.01), _c(), [(1.0, 250.0), (2.0, 0.0)]),
                    *_head("ip1"))


def _fc_tail(bottom, drop=0.5, classes=1000):
    return [_ip("fc6", bottom, 4096, _g(0.005), _c(1.0)), _relu("relu6", "fc6"), DropoutLayer("drop6", ["fc6"], drop),
            _ip("fc7", "fc6", 4096, _g(0.005), _c(1.0)), _relu("relu7", "fc7"), DropoutLayer("drop7", ["fc7"], drop),
            _ip("fc8", "fc7", classes, _g(0.01), _c(0.0))]


def caffenet(train_batch=256, test_batch=50, crop=227, classes=1000):
    """bvlc_reference_caffenet: conv -> relu -> pool -> LRN ordering (ImageNetApp model)."""
    return NetParam("CaffeNet", *data_layers(train_batch, test_batch, 3, crop, crop),
                    _conv("conv1", "data", 11, 96, stride=4, wf=_g(0.01), bf=_c(0.0)),
                    _relu("relu1", "conv1"), _pool("pool1", "conv1", 3, 2),
                    LRNLayer("norm1", ["pool1"], 5, 1e-4, 0.75),
                    _conv("conv2", "norm1", 5, 256, pad=2, group=2, wf=_g(0.01), bf=_c(1.0)),
                    _relu("relu2", "conv2"), _pool("pool2", "conv2", 3, 2),
                    LRNLayer("norm2", ["pool2"], 5, 1e-4, 0.75),
                    _conv("conv3", "norm2", 3, 384, pad=1, wf=_g(0.01), bf=_c(0.0)), _relu("relu3", "conv3"),
                    _conv("conv4", "conv3", 3, 384, pad=1, group=2, wf=_g(0.01), bf=_c(1.0)), _relu("relu4", "conv4"),
                    _conv("conv5", "conv4", 3, 256, pad=1, group=2, wf=_g(0.01), bf=_c(1.0)), _relu("relu5", "conv5"),
                    _pool("pool5", "conv5", 3, 2),
                    *_fc_tail("pool5", classes=classes), *_head("fc8"))


def alexnet(train_batch=256, test_batch=50, crop=227, classes=1000):
    """bvlc_alexnet: conv -> relu -> LRN -> pool ordering."""
    return NetParam("AlexNet", *data_layers(train_batch, test_batch, 3, crop, crop),
                    _conv("conv1", "data", 11, 96, stride=4, wf=_g(0.01), bf=_c(0.0)),
                    _relu("relu1", "conv1"), LRNLayer("norm1", ["conv1"], 5, 1e-4, 0.75),
                    _pool("pool1", "norm1", 3, 2),
                    _conv("conv2", "pool1", 5, 256, pad=2, group=2, wf=_g(0.01), bf=_c(0.1)),
                    _relu("relu2", "conv2"), LRNLayer("norm2", ["conv2"], 5, 1e-4, 0.75),
                    _pool("pool2", "norm2", 3, 2),
                    _conv("conv3", "pool2", 3, 384, pad=1, wf=_g(0.01), bf=_c(0.0)), _relu("relu3", "conv3"),
                    _conv("conv4", "conv3", 3, 384, pad=1, group=2, wf=_g(0.01), bf=_c(0.1)), _relu("relu4", "conv4"),
                    _conv("conv5", "conv4", 3, 256, pad=1, group=2, wf=_g(0.01), bf=_c(0.1)), _relu("relu5", "conv5"),
                    _pool("pool5", "conv5", 3, 2),
                    *_fc_tail("pool5", classes=classes), *_head("fc8"))


INCEPTION = {  # name: (1x1, 3x3_reduce, 3x3, 5x5_reduce, 5x5, pool_proj)
    "3a": (64, 96, 128, 16, 32, 32), "3b": (128, 128, 192, 32, 96, 64),
    "4a": (192, 96, 208, 16, 48, 64), "4b": (160, 112, 224, 24, 64, 64),
    "4c": (128, 128, 256, 24, 64, 64), "4d": (112, 144, 288, 32, 64, 64),
    "4e": (256, 160, 320, 32, 128, 128), "5a": (256, 160, 320, 32, 128, 128),
    "5b": (384, 192, 384, 48, 128, 128),
}
B02 = _c(0.2)


def _inception(name, bottom):
    n1, r3, n3, r5, n5, pp = INCEPTION[name]
    p = f"inception_{name}/"
    L = []
    for suffix, k, n, src, pad in (("1x1", 1, n1, bottom, 0), ("3x3_reduce", 1, r3, bottom, 0),
                                   ("3x3", 3, n3, p + "3x3_reduce", 1), ("5x5_reduce", 1, r5, bottom, 0),
                                   ("5x5", 5, n5, p + "5x5_reduce", 2)):
        L += [_conv(p + suffix, src, k, n, pad=pad, wf=XAV, bf=B02), _relu(p + "relu_" + suffix, p + suffix)]
    L += [_pool(p + "pool", bottom, 3, 1, pad=1),
          _conv(p + "pool_proj", p + "pool", 1, pp, wf=XAV, bf=B02), _relu(p + "relu_pool_proj", p + "pool_proj"),
          ConcatLayer(p + "output", [p + "1x1", p + "3x3", p + "5x5", p + "pool_proj"])]
    return L, p + "output"


def _aux(idx, bottom, classes):
    p = f"loss{idx}/"
    return [_pool(p + "ave_pool", bottom, 5, 3, ave=True),
            _conv(p + "conv", p + "ave_pool", 1, 128, wf=XAV, bf=B02), _relu(p + "relu_conv", p + "conv"),
            _ip(p + "fc", p + "conv", 1024, XAV, B02), _relu(p + "relu_fc", p + "fc"),
            DropoutLayer(p + "drop_fc", [p + "fc"], 0.7),
            _ip(p + "classifier", p + "fc", classes, XAV, _c(0.0)),
            SoftmaxWithLoss(p + "loss", [p + "classifier", "label"], loss_weight=0.3, top=[p + f"loss{idx}"]),
            AccuracyLayer(p + "top-1", [p + "classifier", "label"]),
            AccuracyLayer(p + "top-5", [p + "classifier", "label"], top_k=5)]


def googlenet(train_batch=32, test_batch=50, crop=224, classes=1000, aux=True):
    L = list(data_layers(train_batch, test_batch, 3, crop, crop))
    L += [_conv("conv1/7x7_s2", "data", 7, 64, stride=2, pad=3, wf=XAV, bf=B02), _relu("conv1/relu_7x7", "conv1/7x7_s2"),
          _pool("pool1/3x3_s2", "conv1/7x7_s2", 3, 2), LRNLayer("pool1/norm1", ["pool1/3x3_s2"], 5, 1e-4, 0.75),
          _conv("conv2/3x3_reduce", "pool1/norm1", 1, 64, wf=XAV, bf=B02),
          _relu("conv2/relu_3x3_reduce", "conv2/3x3_reduce"),
          _conv("conv2/3x3", "conv2/3x3_reduce", 3, 192, pad=1, wf=XAV, bf=B02), _relu("conv2/relu_3x3", "conv2/3x3"),
          LRNLayer("conv2/norm2", ["conv2/3x3"], 5, 1e-4, 0.75), _pool("pool2/3x3_s2", "conv2/norm2", 3, 2)]
    x = "pool2/3x3_s2"
    for name in ("3a", "3b"):
        m, x = _inception(name, x)
        L += m
    L.append(_pool("pool3/3x3_s2", x, 3, 2))
    x = "pool3/3x3_s2"
    for name in ("4a", "4b", "4c", "4d", "4e"):
        m, x = _inception(name, x)
        L += m
        if aux and name == "4a":
            L += _aux(1, x, classes)
        if aux and name == "4d":
            L += _aux(2, x, classes)
    L.append(_pool("pool4/3x3_s2", x, 3, 2))
    x = "pool4/3x3_s2"
    for name in ("5a", "5b"):
        m, x = _inception(name, x)
        L += m
    L += [_pool("pool5/7x7_s1", x, 7, 1, ave=True), DropoutLayer("pool5/drop_7x7_s1", ["pool5/7x7_s1"], 0.4),
          _ip("loss3/classifier", "pool5/7x7_s1", classes, XAV, _c(0.0)),
          SoftmaxWithLoss("loss3/loss3", ["loss3/classifier", "label"], loss_weight=1.0),
          AccuracyLayer("loss3/top-1", ["loss3/classifier", "label"]),
          AccuracyLayer("loss3/top-5", ["loss3/classifier", "label"], top_k=5)]
    return NetParam("GoogleNet", *L)


def vgg16(train_batch=64, test_batch=50, crop=224, classes=1000):
    L = list(data_layers(train_batch, test_batch, 3, crop, crop))
    x = "data"
    cfg = [(64, 2), (128, 2), (256, 3), (512, 3), (512, 3)]
    for stage, (n, reps) in enumerate(cfg, 1):
        for r in range(1, reps + 1):
            name = f"conv{stage}_{r}"
            L += [_conv(name, x, 3, n, pad=1, wf={"type": "msra"}, bf=_c(0.0)), _relu(f"relu{stage}_{r}", name)]
            x = name
        L.append(_pool(f"pool{stage}", x, 2, 2))
        x = f"pool{stage}"
    L += [_ip("fc6", x, 4096, _g(0.005), _c(0.1)), _relu("relu6", "fc6"), DropoutLayer("drop6", ["fc6"], 0.5),
          _ip("fc7", "fc6", 4096, _g(0.005), _c(0.1)), _relu("relu7", "fc7"), DropoutLayer("drop7", ["fc7"], 0.5),
          _ip("fc8", "fc7", classes, _g(0.01), _c(0.0)), *_head("fc8", top5=True)]
    return NetParam("VGG_ILSVRC_16_layers", *L)


# --- solvers ------------------------------------------------------------------------------

def _solver(net, **kw):
    s = proto.SolverParameter()
    s.net_param.CopyFrom(net)
    for k, v in kw.items():
        if isinstance(v, list):
            getattr(s, k).extend(v)
        else:
            setattr(s, k, v)
    return s


def lenet_solver(net=None):
    return _solver(net or lenet(), test_iter=[100], test_interval=500, base_lr=0.01, momentum=0.9,
                   weight_decay=5e-4, lr_policy="inv", gamma=1e-4, power=0.75, display=100, max_iter=10000)


def cifar10_quick_solver(net=None):
    return _solver(net or cifar10_quick(), test_iter=[100], test_interval=500, base_lr=0.001, momentum=0.9,
                   weight_decay=0.004, lr_policy="fixed", display=100, max_iter=4000)


def cifar10_full_solver(net=None):
    return _solver(net or cifar10_full(), test_iter=[100], test_interval=1000, base_lr=0.001, momentum=0.9,
                   weight_decay=0.004, lr_policy="fixed", display=200, max_iter=60000)


def caffenet_solver(net=None):
    return _solver(net or caffenet(), test_iter=[1000], test_interval=1000, base_lr=0.01, lr_policy="step",
                   gamma=0.1, stepsize=100000, display=20, max_iter=450000, momentum=0.9, weight_decay=5e-4)


def alexnet_solver(net=None):
    return caffenet_solver(net or alexnet())


def googlenet_solver(net=None):
    return _solver(net or googlenet(), test_iter=[1000], test_interval=4000, test_initialization=False, display=40,
                   average_loss=40, base_lr=0.01, lr_policy="step", stepsize=320000, gamma=0.96,
                   max_iter=10000000, momentum=0.9, weight_decay=2e-4)


def vgg16_solver(net=None):
    return _solver(net or vgg16(), test_iter=[1000], test_interval=10000, base_lr=0.01, lr_policy="step",
                   gamma=0.1, stepsize=100000, display=20, max_iter=370000, momentum=0.9, weight_decay=5e-4)


MODELS = {
    "lenet": (lenet, lenet_solver), "cifar10_quick": (cifar10_quick, cifar10_quick_solver),
    "cifar10_full": (cifar10_full, cifar10_full_solver), "caffenet": (caffenet, caffenet_solver),
    "alexnet": (alexnet, alexnet_solver), "googlenet": (googlenet, googlenet_solver),
    "vgg16": (vgg16, vgg16_solver),
}


def build(name: str, **kw):
    return MODELS[name][0](**kw)


def solver_for(name: str, **net_kw):
    net_fn, solver_fn = MODELS[name]
    return solver_fn(net_fn(**net_kw))
