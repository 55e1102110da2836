"""Programmatic NetParameter construction — SparkNet's Scala DSL
(src/main/scala/libs/Layers.scala:11-137) and ProtoLoader helpers
(src/main/scala/libs/ProtoLoader.scala:9-57), in Python.

The SparkNet functions keep their names and semantics (``RDDLayer``,
``ConvolutionLayer``, ``PoolingLayer``, ``InnerProductLayer``, ``ReLULayer``,
``SoftmaxWithLoss``, ``NetParam``; no fillers set => Caffe's default ``constant 0``),
so a DSL-built LeNet serialises to the same NetParameter bytes as the Scala DSL.
Optional keyword arguments (stride, pad, group, fillers, lr/decay mults) extend them for
the model zoo in :mod:`sparknet_amd.models`.
"""
from __future__ import annotations

import enum

from . import proto


class Include(enum.Enum):
    Train = 0
    Test = 1


class Pooling(enum.Enum):
    Max = 0
    Ave = 1


def _filler(spec):
    if spec is None:
        return None
    if isinstance(spec, proto.FillerParameter):
        return spec
    if isinstance(spec, dict):
        f = proto.FillerParameter()
        for k, v in spec.items():
            setattr(f, k, v)
        return f
    raise TypeError(spec)


def _params(lp, mults):
    for m in mults or ():
        ps = lp.param.add()
        if isinstance(m, dict):
            for k, v in m.items():
                setattr(ps, k, v)
        else:
            ps.lr_mult, ps.decay_mult = m


def _include(lp, include):
    if include is None:
        return
    rule = lp.include.add()
    rule.phase = proto.TRAIN if include in (Include.Train, "train", proto.TRAIN) else proto.TEST


def _base(type_, name, bottom=(), top=None, include=None):
    lp = proto.LayerParameter(name=name, type=type_)
    lp.bottom.extend(list(bottom))
    lp.top.extend([name] if top is None else list(top))
    _include(lp, include)
    return lp


def RDDLayer(name, shape, include=None):
    """JavaData layer fed from outside the net (Layers.scala:18-40)."""
    lp = _base("JavaData", name, include=include)
    lp.java_data_param.shape.dim.extend(int(s) for s in shape)
    return lp


def ConvolutionLayer(name, bottom, kernel, numOutput, *, stride=None, pad=None, group=1, top=None,
                     weight_filler=None, bias_filler=None, param=None, bias_term=True):
    lp = _base("Convolution", name, bottom, top)
    cp = lp.convolution_param
    cp.kernel_h, cp.kernel_w = kernel
    cp.num_output = numOutput
    if stride is not None:
        cp.stride_h, cp.stride_w = (stride, stride) if isinstance(stride, int) else stride
    if pad is not None:
        cp.pad_h, cp.pad_w = (pad, pad) if isinstance(pad, int) else pad
    if group != 1:
        cp.group = group
    if not bias_term:
        cp.bias_term = False
    if weight_filler is not None:
        cp.weight_filler.CopyFrom(_filler(weight_filler))
    if bias_filler is not None:
        cp.bias_filler.CopyFrom(_filler(bias_filler))
    _params(lp, param)
    return lp


def PoolingLayer(name, bottom, pooling=Pooling.Max, kernel=(2, 2), stride=(1, 1), *, pad=None, top=None,
                 global_pooling=False):
    lp = _base("Pooling", name, bottom, top)
    pp = lp.pooling_param
    if global_pooling:
        pp.global_pooling = True
    else:
        pp.kernel_h, pp.kernel_w = kernel
        pp.stride_h, pp.stride_w = stride
    if pad is not None:
        pp.pad_h, pp.pad_w = (pad, pad) if isinstance(pad, int) else pad
    pp.pool = 1 if pooling in (Pooling.Ave, "ave", "AVE") else 0
    return lp


def InnerProductLayer(name, bottom, numOutput, *, top=None, weight_filler=None, bias_filler=None, param=None):
    lp = _base("InnerProduct", name, bottom, top)
    lp.inner_product_param.num_output = numOutput
    if weight_filler is not None:
        lp.inner_product_param.weight_filler.CopyFrom(_filler(weight_filler))
    if bias_filler is not None:
        lp.inner_product_param.bias_filler.CopyFrom(_filler(bias_filler))
    _params(lp, param)
    return lp


def ReLULayer(name, bottom, *, top=None, in_place=False):
    lp = _base("ReLU", name, bottom, list(bottom) if in_place else top)
    lp.relu_param.SetInParent()
    return lp


def SoftmaxWithLoss(name, bottom, *, loss_weight=None, top=None):
    lp = _base("SoftmaxWithLoss", name, bottom, top)
    lp.loss_param.SetInParent()
    lp.softmax_param.SetInParent()
    if loss_weight is not None:
        lp.loss_weight.append(loss_weight)
    return lp


def LRNLayer(name, bottom, local_size=5, alpha=1e-4, beta=0.75, *, within=False, k=None, top=None):
    lp = _base("LRN", name, bottom, top)
    p = lp.lrn_param
    p.local_size, p.alpha, p.beta = local_size, alpha, beta
    if within:
        p.norm_region = 1
    if k is not None:
        p.k = k
    return lp


def DropoutLayer(name, bottom, ratio=0.5, *, in_place=True):
    lp = _base("Dropout", name, bottom, list(bottom) if in_place else None)
    lp.dropout_param.dropout_ratio = ratio
    return lp


def AccuracyLayer(name, bottom, top_k=1, include=Include.Test, top=None):
    lp = _base("Accuracy", name, bottom, top, include)
    if top_k != 1:
        lp.accuracy_param.top_k = top_k
    return lp


def ConcatLayer(name, bottom, axis=1, top=None):
    lp = _base("Concat", name, bottom, top)
    if axis != 1:
        lp.concat_param.axis = axis
    return lp


def NetParam(name, *layers):
    net = proto.NetParameter(name=name)
    for lp in layers:
        net.layer.add().CopyFrom(lp)
    return net


# --- ProtoLoader (ProtoLoader.scala) ---------------------------------------------------

def load_net_prototxt(path):
    return proto.read_prototxt(path, proto.NetParameter)


def load_solver_prototxt(path):
    return proto.read_prototxt(path, proto.SolverParameter)


def load_solver_prototxt_with_net(solver_path, net_param, snapshot_path=None):
    s = load_solver_prototxt(solver_path) if isinstance(solver_path, str) else proto.copy(solver_path)
    if snapshot_path is None:
        s.ClearField("snapshot")
        s.ClearField("snapshot_prefix")
    else:
        s.snapshot_prefix = snapshot_path
    s.ClearField("net")
    s.net_param.CopyFrom(net_param)
    return s


def load_solver_with_net_prototxt(solver_path, net_path, snapshot_path=None):
    return load_solver_prototxt_with_net(solver_path, load_net_prototxt(net_path), snapshot_path)


def replace_data_layers(net, train_batch, test_batch, channels, height, width):
    """Replace layers 0-1 (file-backed data/label) by TRAIN JavaData layers and insert
    TEST ones at 0-1 (ProtoLoader.replaceDataLayers)."""
    out = proto.copy(net)
    layers = list(out.layer)
    layers[0] = RDDLayer("data", [train_batch, channels, height, width], Include.Train)
    layers[1] = RDDLayer("label", [train_batch, 1], Include.Train)
    layers = [RDDLayer("data", [test_batch, channels, height, width], Include.Test),
              RDDLayer("label", [test_batch, 1], Include.Test)] + layers
    del out.layer[:]
    for lp in layers:
        out.layer.add().CopyFrom(lp)
    return out


# snake_case aliases
rdd_layer = RDDLayer
convolution_layer = ConvolutionLayer
pooling_layer = PoolingLayer
inner_product_layer = InnerProductLayer
relu_layer = ReLULayer
softmax_with_loss = SoftmaxWithLoss
net_param = NetParam
