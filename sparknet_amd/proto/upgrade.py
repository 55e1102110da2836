"""V1 -> current NetParameter upgrade (subset of caffe/src/caffe/util/upgrade_proto.cpp).

Old nets/caffemodels store layers in the ``layers`` field (V1LayerParameter, enum
types, ``blobs_lr``/``weight_decay`` instead of ParamSpec).  This converts them to
``layer`` entries so the rest of the engine only ever sees the current format.
"""
from __future__ import annotations

from . import schema

_V1_TYPE_NAMES = {
    "ABSVAL": "AbsVal", "ACCURACY": "Accuracy", "ARGMAX": "ArgMax", "BNLL": "BNLL", "CONCAT": "Concat",
    "CONTRASTIVE_LOSS": "ContrastiveLoss", "CONVOLUTION": "Convolution", "DATA": "Data",
    "DECONVOLUTION": "Deconvolution", "DROPOUT": "Dropout", "DUMMY_DATA": "DummyData",
    "EUCLIDEAN_LOSS": "EuclideanLoss", "ELTWISE": "Eltwise", "EXP": "Exp", "FLATTEN": "Flatten",
    "HDF5_DATA": "HDF5Data", "HDF5_OUTPUT": "HDF5Output", "HINGE_LOSS": "HingeLoss", "IM2COL": "Im2col",
    "IMAGE_DATA": "ImageData", "INFOGAIN_LOSS": "InfogainLoss", "INNER_PRODUCT": "InnerProduct",
    "LRN": "LRN", "MEMORY_DATA": "MemoryData", "MULTINOMIAL_LOGISTIC_LOSS": "MultinomialLogisticLoss",
    "MVN": "MVN", "POOLING": "Pooling", "POWER": "Power", "RELU": "ReLU", "SIGMOID": "Sigmoid",
    "SIGMOID_CROSS_ENTROPY_LOSS": "SigmoidCrossEntropyLoss", "SILENCE": "Silence", "SOFTMAX": "Softmax",
    "SOFTMAX_LOSS": "SoftmaxWithLoss", "SPLIT": "Split", "SLICE": "Slice", "TANH": "TanH",
    "WINDOW_DATA": "WindowData", "THRESHOLD": "Threshold",
}

_COPY_FIELDS = [
    "accuracy_param", "argmax_param", "concat_param", "contrastive_loss_param", "convolution_param",
    "data_param", "dropout_param", "dummy_data_param", "eltwise_param", "exp_param", "hdf5_data_param",
    "hdf5_output_param", "hinge_loss_param", "image_data_param", "infogain_loss_param",
    "inner_product_param", "lrn_param", "memory_data_param", "mvn_param", "pooling_param",
    "power_param", "relu_param", "sigmoid_param", "softmax_param", "slice_param", "tanh_param",
    "threshold_param", "window_data_param", "transform_param", "loss_param",
]


def upgrade_v1_layer(v1, layer) -> None:
    enum = schema.message_class("V1LayerParameter").DESCRIPTOR.enum_types_by_name["LayerType"]
    layer.name = v1.name
    layer.type = _V1_TYPE_NAMES.get(enum.values_by_number[v1.type].name, "")
    layer.bottom.extend(v1.bottom)
    layer.top.extend(v1.top)
    for rule in v1.include:
        layer.include.add().CopyFrom(rule)
    for rule in v1.exclude:
        layer.exclude.add().CopyFrom(rule)
    layer.loss_weight.extend(v1.loss_weight)
    for b in v1.blobs:
        layer.blobs.add().CopyFrom(b)
    n = max(len(v1.param), len(v1.blobs_lr), len(v1.weight_decay))
    for i in range(n):
        ps = layer.param.add()
        if i < len(v1.param) and v1.param[i]:
            ps.name = v1.param[i]
        if i < len(v1.blobs_lr):
            ps.lr_mult = v1.blobs_lr[i]
        if i < len(v1.weight_decay):
            ps.decay_mult = v1.weight_decay[i]
    for f in _COPY_FIELDS:
        if v1.HasField(f):
            getattr(layer, f).CopyFrom(getattr(v1, f))


_SOLVER_TYPE_NAMES = {0: "SGD", 1: "Nesterov", 2: "AdaGrad", 3: "RMSProp", 4: "AdaDelta", 5: "Adam"}


def solver_needs_upgrade(sp) -> bool:
    return sp.HasField("solver_type")


def upgrade_solver(sp):
    """UpgradeSolverType (caffe/src/caffe/util/upgrade_proto.cpp:948-980): the legacy
    ``solver_type`` enum becomes the ``type`` string."""
    if sp.HasField("solver_type"):
        if sp.HasField("type"):
            raise ValueError("Failed to upgrade solver: old solver_type field (enum) and new type field "
                             "(string) cannot be both specified")
        t = int(sp.solver_type)
        if t not in _SOLVER_TYPE_NAMES:
            raise ValueError(f"Unknown SolverParameter solver_type: {t}")
        sp.type = _SOLVER_TYPE_NAMES[t]
        sp.ClearField("solver_type")
    return sp


def net_needs_upgrade(net) -> bool:
    return len(net.layers) > 0


def upgrade_net(net):
    if len(net.layers) == 0:
        return net
    if len(net.layer) != 0:
        raise ValueError("net has both 'layer' and legacy 'layers' fields")
    for v1 in net.layers:
        upgrade_v1_layer(v1, net.layer.add())
    del net.layers[:]
    return net
