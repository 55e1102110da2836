"""Legacy NetParameter / SolverParameter upgrades (caffe/src/caffe/util/upgrade_proto.cpp).

Three generations of net definitions exist in the wild and every reader of nets and
caffemodels goes through :func:`upgrade_net` (``UpgradeNetAsNeeded``,
upgrade_proto.cpp:19-64, which ``Net::CopyTrainedLayersFrom`` runs through
``ReadNetParamsFromBinaryFileOrDie``, net.cpp:853-858):

1. **V0** (``layers { layer { type: 'conv' kernelsize: 11 ... } }``, upgrade_proto.cpp:80-530):
   a free-form lower-case ``type`` string with every hyper-parameter flattened into the
   one V0LayerParameter, and explicit ``padding`` layers in front of convolutions /
   poolings.  :func:`upgrade_v0_padding_layers` folds each padding layer into its
   consumer's ``pad``; :func:`upgrade_v0_layer` routes every V0 field to the typed
   sub-message of the V1 layer (``num_output`` -> ``convolution_param`` or
   ``inner_product_param`` by type, ``cropsize`` / ``meanfile`` / ``mirror`` / ``scale`` ->
   ``transform_param`` ...).
2. **data transformation** (upgrade_proto.cpp:586-646): V1 data layers that still carry
   ``scale`` / ``mean_file`` / ``crop_size`` / ``mirror`` in their ``data_param`` /
   ``image_data_param`` / ``window_data_param`` move them to ``transform_param``.
3. **V1** (``layers { type: CONVOLUTION blobs_lr: 1 ... }``, upgrade_proto.cpp:648-946): enum
   types become type strings, ``param`` / ``blob_share_mode`` / ``blobs_lr`` /
   ``weight_decay`` become ParamSpecs.

Each step reports whether the input was fully representable (the reference's
``is_fully_compatible``: an unknown field for a layer type is logged and dropped).
"""
from __future__ import annotations

import logging

from . import schema

log = logging.getLogger("sparknet_amd.proto.upgrade")

# -- V1 enum -> V2 type string (UpgradeV1LayerType, upgrade_proto.cpp:858-946) -------------
_V1_TYPE_NAMES = {
    "NONE": "", "ABSVAL": "AbsVal", "ACCURACY": "Accuracy", "ARGMAX": "ArgMax", "BNLL": "BNLL",
    "CONCAT": "Concat", "CONTRASTIVE_LOSS": "ContrastiveLoss", "CONVOLUTION": "Convolution", "DATA": "Data",
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

# typed sub-messages carried over verbatim from V1 to V2 (upgrade_proto.cpp:719-843)
_COPY_FIELDS = [
    "accuracy_param", "argmax_param", "concat_param", "contrastive_loss_param", "convolution_param",
    "data_param", "dropout_param", "dummy_data_param", "eltwise_param", "exp_param", "hdf5_data_param",
    "hdf5_output_param", "hinge_loss_param", "image_data_param", "infogain_loss_param",
    "inner_product_param", "lrn_param", "memory_data_param", "mvn_param", "pooling_param",
    "power_param", "relu_param", "sigmoid_param", "softmax_param", "slice_param", "tanh_param",
    "threshold_param", "window_data_param", "transform_param", "loss_param",
]

# -- V0 type string -> V1 enum name (UpgradeV0LayerType, upgrade_proto.cpp:532-584) ---------
_V0_TYPES = {
    "accuracy": "ACCURACY", "bnll": "BNLL", "concat": "CONCAT", "conv": "CONVOLUTION", "data": "DATA",
    "dropout": "DROPOUT", "euclidean_loss": "EUCLIDEAN_LOSS", "flatten": "FLATTEN", "hdf5_data": "HDF5_DATA",
    "hdf5_output": "HDF5_OUTPUT", "im2col": "IM2COL", "images": "IMAGE_DATA", "infogain_loss": "INFOGAIN_LOSS",
    "innerproduct": "INNER_PRODUCT", "lrn": "LRN", "multinomial_logistic_loss": "MULTINOMIAL_LOGISTIC_LOSS",
    "pool": "POOLING", "relu": "RELU", "sigmoid": "SIGMOID", "softmax": "SOFTMAX", "softmax_loss": "SOFTMAX_LOSS",
    "split": "SPLIT", "tanh": "TANH", "window_data": "WINDOW_DATA",
}

# V0 field -> {V0 type: (V1 sub-message, field)} ; "*" = every type.  Fields whose type is
# not listed are dropped with an error (is_fully_compatible = false), as the reference does.
_DATA_SRC = {"data": "data_param", "hdf5_data": "hdf5_data_param", "images": "image_data_param",
             "window_data": "window_data_param"}
_V0_ROUTES = {
    "num_output": {"conv": ("convolution_param", "num_output"), "innerproduct": ("inner_product_param", "num_output")},
    "biasterm": {"conv": ("convolution_param", "bias_term"), "innerproduct": ("inner_product_param", "bias_term")},
    "weight_filler": {"conv": ("convolution_param", "weight_filler"),
                      "innerproduct": ("inner_product_param", "weight_filler")},
    "bias_filler": {"conv": ("convolution_param", "bias_filler"), "innerproduct": ("inner_product_param", "bias_filler")},
    "pad": {"conv": ("convolution_param", "pad"), "pool": ("pooling_param", "pad")},
    "kernelsize": {"conv": ("convolution_param", "kernel_size"), "pool": ("pooling_param", "kernel_size")},
    "group": {"conv": ("convolution_param", "group")},
    "stride": {"conv": ("convolution_param", "stride"), "pool": ("pooling_param", "stride")},
    "pool": {"pool": ("pooling_param", "pool")},
    "dropout_ratio": {"dropout": ("dropout_param", "dropout_ratio")},
    "local_size": {"lrn": ("lrn_param", "local_size")},
    "alpha": {"lrn": ("lrn_param", "alpha")},
    "beta": {"lrn": ("lrn_param", "beta")},
    "k": {"lrn": ("lrn_param", "k")},
    "source": dict({t: (m, "source") for t, m in _DATA_SRC.items()},
                   infogain_loss=("infogain_loss_param", "source")),
    "scale": {"*": ("transform_param", "scale")},
    "meanfile": {"*": ("transform_param", "mean_file")},
    "batchsize": {t: (m, "batch_size") for t, m in _DATA_SRC.items()},
    "cropsize": {"*": ("transform_param", "crop_size")},
    "mirror": {"*": ("transform_param", "mirror")},
    "rand_skip": {"data": ("data_param", "rand_skip"), "images": ("image_data_param", "rand_skip")},
    "shuffle_images": {"images": ("image_data_param", "shuffle")},
    "new_height": {"images": ("image_data_param", "new_height")},
    "new_width": {"images": ("image_data_param", "new_width")},
    "concat_dim": {"concat": ("concat_param", "concat_dim")},
    "det_fg_threshold": {"window_data": ("window_data_param", "fg_threshold")},
    "det_bg_threshold": {"window_data": ("window_data_param", "bg_threshold")},
    "det_fg_fraction": {"window_data": ("window_data_param", "fg_fraction")},
    "det_context_pad": {"window_data": ("window_data_param", "context_pad")},
    "det_crop_mode": {"window_data": ("window_data_param", "crop_mode")},
    "hdf5_output_param": {"hdf5_output": ("hdf5_output_param", None)},
}
# V1 data layer -> the parameter message that may still hold transformation fields
_DATA_TRANSFORM = {"DATA": "data_param", "IMAGE_DATA": "image_data_param", "WINDOW_DATA": "window_data_param"}
_TRANSFORM_FIELDS = ("scale", "mean_file", "crop_size", "mirror")


def _v1_enum():
    return schema.message_class("V1LayerParameter").DESCRIPTOR.enum_types_by_name["LayerType"]


def v1_type_name(v1_type: int) -> str:
    """``UpgradeV1LayerType``: V1 enum value -> V2 type string ('' for NONE)."""
    return _V1_TYPE_NAMES[_v1_enum().values_by_number[int(v1_type)].name]


# -- V0 -> V1 -------------------------------------------------------------------------------

def net_needs_v0_upgrade(net) -> bool:
    return any(l.HasField("layer") for l in net.layers)


def upgrade_v0_padding_layers(net):
    """``UpgradeV0PaddingLayers`` (upgrade_proto.cpp:118-178): drop V0 ``padding`` layers and
    give their pad to the single-input conv / pool layer that consumes their output, which
    then reads the padding layer's own input.  Returns a new NetParameter."""
    out = type(net)()
    out.CopyFrom(net)
    del out.layers[:]
    producer = {b: -1 for b in net.input}  # blob -> index of the last layer that wrote it
    for i, conn in enumerate(net.layers):
        v0 = conn.layer
        if v0.type != "padding":
            out.layers.add().CopyFrom(conn)
        for j, b in enumerate(conn.bottom):
            if b not in producer:
                raise ValueError(f"Unknown blob input {b} to layer {j}")
            src = producer[b]
            if src == -1 or net.layers[src].layer.type != "padding":
                continue
            pad = net.layers[src]
            if v0.type not in ("conv", "pool"):
                raise ValueError(f"Padding layer input to non-convolutional / non-pooling layer type {v0.type}")
            if len(conn.bottom) != 1 or len(pad.bottom) != 1 or len(pad.top) != 1:
                raise ValueError("padding upgrade needs single-input / single-output layers")
            tgt = out.layers[len(out.layers) - 1]
            tgt.layer.pad = pad.layer.pad
            tgt.bottom[j] = pad.bottom[0]
        for b in conn.top:
            producer[b] = i
    return out


def upgrade_v0_layer(conn, v1) -> bool:
    """``UpgradeV0LayerParameter`` (upgrade_proto.cpp:179-530): one V0 layer (wrapped in its
    V1 connection) into the V1 layer ``v1``.  Returns False when a field had no home."""
    v1.Clear()
    v1.bottom.extend(conn.bottom)
    v1.top.extend(conn.top)
    if not conn.HasField("layer"):
        return True
    v0 = conn.layer
    ok = True
    if v0.HasField("name"):
        v1.name = v0.name
    typ = v0.type
    if v0.HasField("type"):
        if typ not in _V0_TYPES:
            raise ValueError(f"Unknown layer name: {typ}")
        v1.type = _v1_enum().values_by_name[_V0_TYPES[typ]].number
    for b in v0.blobs:
        v1.blobs.add().CopyFrom(b)
    v1.blobs_lr.extend(v0.blobs_lr)
    v1.weight_decay.extend(v0.weight_decay)
    for field, routes in _V0_ROUTES.items():
        if not v0.HasField(field):
            continue
        route = routes.get(typ) or routes.get("*")
        if route is None:
            log.error("Unknown parameter %s for layer type %s", field, typ)
            ok = False
            continue
        msg_name, sub = route
        msg = getattr(v1, msg_name)
        val = getattr(v0, field)
        if sub is None:
            msg.CopyFrom(val)
        elif hasattr(getattr(msg, sub), "append"):
            getattr(msg, sub).append(val)  # conv pad / kernel_size / stride are repeated in V1+
        elif msg.DESCRIPTOR.fields_by_name[sub].message_type is not None:
            getattr(msg, sub).CopyFrom(val)
        else:
            setattr(msg, sub, val)  # PoolMethod enums share numbering (MAX/AVE/STOCHASTIC)
    return ok


def upgrade_v0_net(net):
    """``UpgradeV0Net`` (upgrade_proto.cpp:93-116): padding fold, then every layer; only name,
    inputs, input_dim and force_backward survive from the V0 net header.  Returns
    (new NetParameter, fully compatible)."""
    padded = upgrade_v0_padding_layers(net)
    out = type(net)()
    ok = True
    if padded.HasField("name"):
        out.name = padded.name
    for conn in padded.layers:
        ok &= upgrade_v0_layer(conn, out.layers.add())
    out.input.extend(padded.input)
    out.input_dim.extend(padded.input_dim)
    if padded.HasField("force_backward"):
        out.force_backward = padded.force_backward
    return out, ok


# -- data transformation --------------------------------------------------------------------

def net_needs_data_upgrade(net) -> bool:
    enum = _v1_enum()
    for l in net.layers:
        pname = _DATA_TRANSFORM.get(enum.values_by_number[l.type].name) if l.HasField("type") else None
        if pname and any(getattr(l, pname).HasField(f) for f in _TRANSFORM_FIELDS):
            return True
    return False


def upgrade_net_data_transformation(net) -> None:
    """``UpgradeNetDataTransformation`` (upgrade_proto.cpp:615-646), in place."""
    enum = _v1_enum()
    for l in net.layers:
        pname = _DATA_TRANSFORM.get(enum.values_by_number[l.type].name) if l.HasField("type") else None
        if not pname:
            continue
        p = getattr(l, pname)
        for f in _TRANSFORM_FIELDS:
            if p.HasField(f):
                setattr(l.transform_param, f, getattr(p, f))
                p.ClearField(f)


# -- V1 -> V2 -------------------------------------------------------------------------------

def net_needs_v1_upgrade(net) -> bool:
    return len(net.layers) > 0


def upgrade_v1_layer(v1, layer) -> bool:
    """``UpgradeV1LayerParameter`` (upgrade_proto.cpp:666-856)."""
    layer.Clear()
    layer.bottom.extend(v1.bottom)
    layer.top.extend(v1.top)
    if v1.HasField("name"):
        layer.name = v1.name
    for rule in v1.include:
        layer.include.add().CopyFrom(rule)
    for rule in v1.exclude:
        layer.exclude.add().CopyFrom(rule)
    if v1.HasField("type"):
        layer.type = v1_type_name(v1.type)
    for b in v1.blobs:
        layer.blobs.add().CopyFrom(b)

    def spec(i):
        while len(layer.param) <= i:
            layer.param.add()
        return layer.param[i]

    for i, name in enumerate(v1.param):
        spec(i).name = name
    for i, mode in enumerate(v1.blob_share_mode):
        spec(i).share_mode = mode  # STRICT / PERMISSIVE share numbering with ParamSpec
    for i, lr in enumerate(v1.blobs_lr):
        spec(i).lr_mult = lr
    for i, wd in enumerate(v1.weight_decay):
        spec(i).decay_mult = wd
    layer.loss_weight.extend(v1.loss_weight)
    for f in _COPY_FIELDS:
        if v1.HasField(f):
            getattr(layer, f).CopyFrom(getattr(v1, f))
    if v1.HasField("layer"):
        log.error("Input NetParameter has V0 layer -- ignoring.")
        return False
    return True


def upgrade_v1_net(net):
    """``UpgradeV1Net`` (upgrade_proto.cpp:648-664): returns (new NetParameter, fully
    compatible); pre-existing ``layer`` entries are dropped, as in the reference."""
    out = type(net)()
    out.CopyFrom(net)
    del out.layers[:]
    del out.layer[:]
    ok = len(net.layer) == 0
    if not ok:
        log.error("Input NetParameter to be upgraded already specifies 'layer' fields; these will be ignored.")
    for i, v1 in enumerate(net.layers):
        if not upgrade_v1_layer(v1, out.layer.add()):
            log.error("Upgrade of input layer %d failed.", i)
            ok = False
    return out, ok


# -- entry points ---------------------------------------------------------------------------

def net_needs_upgrade(net) -> bool:
    return net_needs_v0_upgrade(net) or net_needs_data_upgrade(net) or net_needs_v1_upgrade(net)


def upgrade_net(net, strict: bool = False):
    """``UpgradeNetAsNeeded`` in place: V0 -> V1, data transformation, V1 -> V2.  Returns the
    same message (upgraded).  ``strict`` raises instead of logging when a field is lost."""
    ok = True
    if net_needs_v0_upgrade(net):
        up, good = upgrade_v0_net(net)
        net.CopyFrom(up)
        ok &= good
    if net_needs_data_upgrade(net):
        upgrade_net_data_transformation(net)
    if net_needs_v1_upgrade(net):
        up, good = upgrade_v1_net(net)
        net.CopyFrom(up)
        ok &= good
    if strict and not ok:
        raise ValueError("net upgrade lost fields (see log)")
    return net


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
