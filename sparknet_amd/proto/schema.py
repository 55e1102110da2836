"""Caffe protobuf schema, built at import time as dynamic protobuf descriptors.

Wire- and text-format compatible with the reference's ``caffe.proto`` (package
``caffe``; field numbers from caffe/src/caffe/proto/caffe.proto:6-1239), so reference
``.prototxt`` files parse unchanged and ``.caffemodel`` / ``.solverstate`` /
``.binaryproto`` files round-trip bit-exactly.  There is no protoc in the toolchain, so
the schema is declared as Python tables and turned into a ``FileDescriptorProto``; the
generated classes are real protobuf messages (text_format, SerializeToString, ...).

The legacy layer messages are modelled too — ``V1LayerParameter`` (``layers`` field of
NetParameter) and the V0 ``V0LayerParameter`` nested in it as ``layer`` (caffe.proto:1134-1230)
— so V0- and V1-era nets and caffemodels parse and are upgraded by ``proto.upgrade``.
"""
from __future__ import annotations

from google.protobuf import descriptor_pb2, descriptor_pool, message_factory

_FD = descriptor_pb2.FieldDescriptorProto
_SCALARS = {
    "double": _FD.TYPE_DOUBLE, "float": _FD.TYPE_FLOAT, "int64": _FD.TYPE_INT64,
    "uint64": _FD.TYPE_UINT64, "int32": _FD.TYPE_INT32, "uint32": _FD.TYPE_UINT32,
    "bool": _FD.TYPE_BOOL, "string": _FD.TYPE_STRING, "bytes": _FD.TYPE_BYTES,
}

ENGINE = [("DEFAULT", 0), ("CAFFE", 1), ("CUDNN", 2)]
POOL3 = [("MAX", 0), ("AVE", 1), ("STOCHASTIC", 2)]

# Top-level enums.
ENUMS = {"Phase": [("TRAIN", 0), ("TEST", 1)]}


def o(name, num, typ, default=None):  # optional
    return (name, num, "opt", typ, default, False)


def r(name, num, typ, packed=False):  # repeated
    return (name, num, "rep", typ, None, packed)


# message -> (nested enums, fields).  Nested enum types are referenced as "Msg.Enum".
MESSAGES: dict[str, tuple[dict, list]] = {
    "BlobShape": ({}, [r("dim", 1, "int64", packed=True)]),
    "BlobProto": ({}, [
        o("shape", 7, "BlobShape"), r("data", 5, "float", True), r("diff", 6, "float", True),
        r("double_data", 8, "double", True), r("double_diff", 9, "double", True),
        o("num", 1, "int32", 0), o("channels", 2, "int32", 0), o("height", 3, "int32", 0),
        o("width", 4, "int32", 0)]),
    "BlobProtoVector": ({}, [r("blobs", 1, "BlobProto")]),
    "Datum": ({}, [
        o("channels", 1, "int32"), o("height", 2, "int32"), o("width", 3, "int32"),
        o("data", 4, "bytes"), o("label", 5, "int32"), r("float_data", 6, "float"),
        o("encoded", 7, "bool", False)]),
    "FillerParameter": ({"VarianceNorm": [("FAN_IN", 0), ("FAN_OUT", 1), ("AVERAGE", 2)]}, [
        o("type", 1, "string", "constant"), o("value", 2, "float", 0), o("min", 3, "float", 0),
        o("max", 4, "float", 1), o("mean", 5, "float", 0), o("std", 6, "float", 1),
        o("sparse", 7, "int32", -1), o("variance_norm", 8, "FillerParameter.VarianceNorm", "FAN_IN")]),
    "NetParameter": ({}, [
        o("name", 1, "string"), r("input", 3, "string"), r("input_shape", 8, "BlobShape"),
        r("input_dim", 4, "int32"), o("force_backward", 5, "bool", False), o("state", 6, "NetState"),
        o("debug_info", 7, "bool", False), r("layer", 100, "LayerParameter"),
        r("layers", 2, "V1LayerParameter")]),
    "SolverParameter": ({
        "SnapshotFormat": [("HDF5", 0), ("BINARYPROTO", 1)],
        "SolverMode": [("CPU", 0), ("GPU", 1)],
        "SolverType": [("SGD", 0), ("NESTEROV", 1), ("ADAGRAD", 2), ("RMSPROP", 3), ("ADADELTA", 4),
                       ("ADAM", 5)]}, [
        o("net", 24, "string"), o("net_param", 25, "NetParameter"), o("train_net", 1, "string"),
        r("test_net", 2, "string"), o("train_net_param", 21, "NetParameter"),
        r("test_net_param", 22, "NetParameter"), o("train_state", 26, "NetState"),
        r("test_state", 27, "NetState"), r("test_iter", 3, "int32"), o("test_interval", 4, "int32", 0),
        o("test_compute_loss", 19, "bool", False), o("test_initialization", 32, "bool", True),
        o("base_lr", 5, "float"), o("display", 6, "int32"), o("average_loss", 33, "int32", 1),
        o("max_iter", 7, "int32"), o("iter_size", 36, "int32", 1), o("lr_policy", 8, "string"),
        o("gamma", 9, "float"), o("power", 10, "float"), o("momentum", 11, "float"),
        o("weight_decay", 12, "float"), o("regularization_type", 29, "string", "L2"),
        o("stepsize", 13, "int32"), r("stepvalue", 34, "int32"), o("clip_gradients", 35, "float", -1),
        o("snapshot", 14, "int32", 0), o("snapshot_prefix", 15, "string"),
        o("snapshot_diff", 16, "bool", False),
        o("snapshot_format", 37, "SolverParameter.SnapshotFormat", "BINARYPROTO"),
        o("solver_mode", 17, "SolverParameter.SolverMode", "GPU"), o("device_id", 18, "int32", 0),
        o("random_seed", 20, "int64", -1), o("type", 40, "string", "SGD"), o("delta", 31, "float", 1e-8),
        o("momentum2", 39, "float", 0.999), o("rms_decay", 38, "float"),
        o("debug_info", 23, "bool", False), o("snapshot_after_train", 28, "bool", True),
        o("solver_type", 30, "SolverParameter.SolverType", "SGD")]),
    "SolverState": ({}, [
        o("iter", 1, "int32"), o("learned_net", 2, "string"), r("history", 3, "BlobProto"),
        o("current_step", 4, "int32", 0)]),
    "NetState": ({}, [o("phase", 1, "Phase", "TEST"), o("level", 2, "int32", 0), r("stage", 3, "string")]),
    "NetStateRule": ({}, [
        o("phase", 1, "Phase"), o("min_level", 2, "int32"), o("max_level", 3, "int32"),
        r("stage", 4, "string"), r("not_stage", 5, "string")]),
    "ParamSpec": ({"DimCheckMode": [("STRICT", 0), ("PERMISSIVE", 1)]}, [
        o("name", 1, "string"), o("share_mode", 2, "ParamSpec.DimCheckMode"),
        o("lr_mult", 3, "float", 1.0), o("decay_mult", 4, "float", 1.0)]),
    "LayerParameter": ({}, [
        o("name", 1, "string"), o("type", 2, "string"), r("bottom", 3, "string"), r("top", 4, "string"),
        o("phase", 10, "Phase"), r("loss_weight", 5, "float"), r("param", 6, "ParamSpec"),
        r("blobs", 7, "BlobProto"), r("propagate_down", 11, "bool"), r("include", 8, "NetStateRule"),
        r("exclude", 9, "NetStateRule"),
        o("transform_param", 100, "TransformationParameter"), o("loss_param", 101, "LossParameter"),
        o("accuracy_param", 102, "AccuracyParameter"), o("argmax_param", 103, "ArgMaxParameter"),
        o("batch_norm_param", 139, "BatchNormParameter"), o("concat_param", 104, "ConcatParameter"),
        o("contrastive_loss_param", 105, "ContrastiveLossParameter"),
        o("convolution_param", 106, "ConvolutionParameter"), o("data_param", 107, "DataParameter"),
        o("dropout_param", 108, "DropoutParameter"), o("dummy_data_param", 109, "DummyDataParameter"),
        o("eltwise_param", 110, "EltwiseParameter"), o("embed_param", 137, "EmbedParameter"),
        o("exp_param", 111, "ExpParameter"), o("flatten_param", 135, "FlattenParameter"),
        o("hdf5_data_param", 112, "HDF5DataParameter"), o("hdf5_output_param", 113, "HDF5OutputParameter"),
        o("hinge_loss_param", 114, "HingeLossParameter"), o("image_data_param", 115, "ImageDataParameter"),
        o("infogain_loss_param", 116, "InfogainLossParameter"),
        o("inner_product_param", 117, "InnerProductParameter"), o("log_param", 134, "LogParameter"),
        o("lrn_param", 118, "LRNParameter"), o("memory_data_param", 119, "MemoryDataParameter"),
        o("mvn_param", 120, "MVNParameter"), o("pooling_param", 121, "PoolingParameter"),
        o("power_param", 122, "PowerParameter"), o("prelu_param", 131, "PReLUParameter"),
        o("python_param", 130, "PythonParameter"), o("reduction_param", 136, "ReductionParameter"),
        o("relu_param", 123, "ReLUParameter"), o("reshape_param", 133, "ReshapeParameter"),
        o("sigmoid_param", 124, "SigmoidParameter"), o("softmax_param", 125, "SoftmaxParameter"),
        o("spp_param", 132, "SPPParameter"), o("slice_param", 126, "SliceParameter"),
        o("tanh_param", 127, "TanHParameter"), o("threshold_param", 128, "ThresholdParameter"),
        o("tile_param", 138, "TileParameter"), o("java_data_param", 149, "JavaDataParameter"),
        o("window_data_param", 129, "WindowDataParameter")]),
    "TransformationParameter": ({}, [
        o("scale", 1, "float", 1), o("mirror", 2, "bool", False), o("crop_size", 3, "uint32", 0),
        o("mean_file", 4, "string"), r("mean_value", 5, "float"), o("force_color", 6, "bool", False),
        o("force_gray", 7, "bool", False)]),
    "LossParameter": ({}, [o("ignore_label", 1, "int32"), o("normalize", 2, "bool", True)]),
    "AccuracyParameter": ({}, [o("top_k", 1, "uint32", 1), o("axis", 2, "int32", 1),
                               o("ignore_label", 3, "int32")]),
    "ArgMaxParameter": ({}, [o("out_max_val", 1, "bool", False), o("top_k", 2, "uint32", 1),
                             o("axis", 3, "int32")]),
    "ConcatParameter": ({}, [o("axis", 2, "int32", 1), o("concat_dim", 1, "uint32", 1)]),
    "BatchNormParameter": ({}, [o("use_global_stats", 1, "bool"),
                                o("moving_average_fraction", 2, "float", 0.999), o("eps", 3, "float", 1e-5)]),
    "ContrastiveLossParameter": ({}, [o("margin", 1, "float", 1.0), o("legacy_version", 2, "bool", False)]),
    "ConvolutionParameter": ({"Engine": ENGINE}, [
        o("num_output", 1, "uint32"), o("bias_term", 2, "bool", True), r("pad", 3, "uint32"),
        r("kernel_size", 4, "uint32"), r("stride", 6, "uint32"), o("pad_h", 9, "uint32", 0),
        o("pad_w", 10, "uint32", 0), o("kernel_h", 11, "uint32"), o("kernel_w", 12, "uint32"),
        o("stride_h", 13, "uint32"), o("stride_w", 14, "uint32"), o("group", 5, "uint32", 1),
        o("weight_filler", 7, "FillerParameter"), o("bias_filler", 8, "FillerParameter"),
        o("engine", 15, "ConvolutionParameter.Engine", "DEFAULT"), o("axis", 16, "int32", 1),
        o("force_nd_im2col", 17, "bool", False)]),
    "DataParameter": ({"DB": [("LEVELDB", 0), ("LMDB", 1)]}, [
        o("source", 1, "string"), o("batch_size", 4, "uint32"), o("rand_skip", 7, "uint32", 0),
        o("backend", 8, "DataParameter.DB", "LEVELDB"), o("scale", 2, "float", 1),
        o("mean_file", 3, "string"), o("crop_size", 5, "uint32", 0), o("mirror", 6, "bool", False),
        o("force_encoded_color", 9, "bool", False), o("prefetch", 10, "uint32", 4)]),
    "DropoutParameter": ({}, [o("dropout_ratio", 1, "float", 0.5)]),
    "DummyDataParameter": ({}, [
        r("data_filler", 1, "FillerParameter"), r("shape", 6, "BlobShape"), r("num", 2, "uint32"),
        r("channels", 3, "uint32"), r("height", 4, "uint32"), r("width", 5, "uint32")]),
    "EltwiseParameter": ({"EltwiseOp": [("PROD", 0), ("SUM", 1), ("MAX", 2)]}, [
        o("operation", 1, "EltwiseParameter.EltwiseOp", "SUM"), r("coeff", 2, "float"),
        o("stable_prod_grad", 3, "bool", True)]),
    "EmbedParameter": ({}, [
        o("num_output", 1, "uint32"), o("input_dim", 2, "uint32"), o("bias_term", 3, "bool", True),
        o("weight_filler", 4, "FillerParameter"), o("bias_filler", 5, "FillerParameter")]),
    "ExpParameter": ({}, [o("base", 1, "float", -1.0), o("scale", 2, "float", 1.0), o("shift", 3, "float", 0.0)]),
    "FlattenParameter": ({}, [o("axis", 1, "int32", 1), o("end_axis", 2, "int32", -1)]),
    "HDF5DataParameter": ({}, [o("source", 1, "string"), o("batch_size", 2, "uint32"),
                               o("shuffle", 3, "bool", False)]),
    "HDF5OutputParameter": ({}, [o("file_name", 1, "string")]),
    "HingeLossParameter": ({"Norm": [("L1", 1), ("L2", 2)]}, [o("norm", 1, "HingeLossParameter.Norm", "L1")]),
    "ImageDataParameter": ({}, [
        o("source", 1, "string"), o("batch_size", 4, "uint32", 1), o("rand_skip", 7, "uint32", 0),
        o("shuffle", 8, "bool", False), o("new_height", 9, "uint32", 0), o("new_width", 10, "uint32", 0),
        o("is_color", 11, "bool", True), o("scale", 2, "float", 1), o("mean_file", 3, "string"),
        o("crop_size", 5, "uint32", 0), o("mirror", 6, "bool", False), o("root_folder", 12, "string", "")]),
    "InfogainLossParameter": ({}, [o("source", 1, "string")]),
    "InnerProductParameter": ({}, [
        o("num_output", 1, "uint32"), o("bias_term", 2, "bool", True),
        o("weight_filler", 3, "FillerParameter"), o("bias_filler", 4, "FillerParameter"),
        o("axis", 5, "int32", 1)]),
    "LogParameter": ({}, [o("base", 1, "float", -1.0), o("scale", 2, "float", 1.0), o("shift", 3, "float", 0.0)]),
    "LRNParameter": ({"NormRegion": [("ACROSS_CHANNELS", 0), ("WITHIN_CHANNEL", 1)], "Engine": ENGINE}, [
        o("local_size", 1, "uint32", 5), o("alpha", 2, "float", 1.0), o("beta", 3, "float", 0.75),
        o("norm_region", 4, "LRNParameter.NormRegion", "ACROSS_CHANNELS"), o("k", 5, "float", 1.0),
        o("engine", 6, "LRNParameter.Engine", "DEFAULT")]),
    "MemoryDataParameter": ({}, [o("batch_size", 1, "uint32"), o("channels", 2, "uint32"),
                                 o("height", 3, "uint32"), o("width", 4, "uint32")]),
    "MVNParameter": ({}, [o("normalize_variance", 1, "bool", True), o("across_channels", 2, "bool", False),
                          o("eps", 3, "float", 1e-9)]),
    "PoolingParameter": ({"PoolMethod": POOL3, "Engine": ENGINE}, [
        o("pool", 1, "PoolingParameter.PoolMethod", "MAX"), o("pad", 4, "uint32", 0),
        o("pad_h", 9, "uint32", 0), o("pad_w", 10, "uint32", 0), o("kernel_size", 2, "uint32"),
        o("kernel_h", 5, "uint32"), o("kernel_w", 6, "uint32"), o("stride", 3, "uint32", 1),
        o("stride_h", 7, "uint32"), o("stride_w", 8, "uint32"),
        o("engine", 11, "PoolingParameter.Engine", "DEFAULT"), o("global_pooling", 12, "bool", False)]),
    "PowerParameter": ({}, [o("power", 1, "float", 1.0), o("scale", 2, "float", 1.0), o("shift", 3, "float", 0.0)]),
    "PythonParameter": ({}, [o("module", 1, "string"), o("layer", 2, "string"), o("param_str", 3, "string", ""),
                             o("share_in_parallel", 4, "bool", False)]),
    "ReductionParameter": ({"ReductionOp": [("SUM", 1), ("ASUM", 2), ("SUMSQ", 3), ("MEAN", 4)]}, [
        o("operation", 1, "ReductionParameter.ReductionOp", "SUM"), o("axis", 2, "int32", 0),
        o("coeff", 3, "float", 1.0)]),
    "ReLUParameter": ({"Engine": ENGINE}, [o("negative_slope", 1, "float", 0),
                                           o("engine", 2, "ReLUParameter.Engine", "DEFAULT")]),
    "ReshapeParameter": ({}, [o("shape", 1, "BlobShape"), o("axis", 2, "int32", 0), o("num_axes", 3, "int32", -1)]),
    "SigmoidParameter": ({"Engine": ENGINE}, [o("engine", 1, "SigmoidParameter.Engine", "DEFAULT")]),
    "SliceParameter": ({}, [o("axis", 3, "int32", 1), r("slice_point", 2, "uint32"), o("slice_dim", 1, "uint32", 1)]),
    "SoftmaxParameter": ({"Engine": ENGINE}, [o("engine", 1, "SoftmaxParameter.Engine", "DEFAULT"),
                                              o("axis", 2, "int32", 1)]),
    "TanHParameter": ({"Engine": ENGINE}, [o("engine", 1, "TanHParameter.Engine", "DEFAULT")]),
    "TileParameter": ({}, [o("axis", 1, "int32", 1), o("tiles", 2, "int32")]),
    "ThresholdParameter": ({}, [o("threshold", 1, "float", 0)]),
    "JavaDataParameter": ({}, [o("shape", 1, "BlobShape")]),
    "WindowDataParameter": ({}, [
        o("source", 1, "string"), o("scale", 2, "float", 1), o("mean_file", 3, "string"),
        o("batch_size", 4, "uint32"), o("crop_size", 5, "uint32", 0), o("mirror", 6, "bool", False),
        o("fg_threshold", 7, "float", 0.5), o("bg_threshold", 8, "float", 0.5),
        o("fg_fraction", 9, "float", 0.25), o("context_pad", 10, "uint32", 0),
        o("crop_mode", 11, "string", "warp"), o("cache_images", 12, "bool", False),
        o("root_folder", 13, "string", "")]),
    "SPPParameter": ({"PoolMethod": POOL3, "Engine": ENGINE}, [
        o("pyramid_height", 1, "uint32"), o("pool", 2, "SPPParameter.PoolMethod", "MAX"),
        o("engine", 6, "SPPParameter.Engine", "DEFAULT")]),
    "PReLUParameter": ({}, [o("filler", 1, "FillerParameter"), o("channel_shared", 2, "bool", False)]),
    "V1LayerParameter": ({
        "LayerType": [
            ("NONE", 0), ("ABSVAL", 35), ("ACCURACY", 1), ("ARGMAX", 30), ("BNLL", 2), ("CONCAT", 3),
            ("CONTRASTIVE_LOSS", 37), ("CONVOLUTION", 4), ("DATA", 5), ("DECONVOLUTION", 39),
            ("DROPOUT", 6), ("DUMMY_DATA", 32), ("EUCLIDEAN_LOSS", 7), ("ELTWISE", 25), ("EXP", 38),
            ("FLATTEN", 8), ("HDF5_DATA", 9), ("HDF5_OUTPUT", 10), ("HINGE_LOSS", 28), ("IM2COL", 11),
            ("IMAGE_DATA", 12), ("INFOGAIN_LOSS", 13), ("INNER_PRODUCT", 14), ("LRN", 15),
            ("MEMORY_DATA", 29), ("MULTINOMIAL_LOGISTIC_LOSS", 16), ("MVN", 34), ("POOLING", 17),
            ("POWER", 26), ("RELU", 18), ("SIGMOID", 19), ("SIGMOID_CROSS_ENTROPY_LOSS", 27),
            ("SILENCE", 36), ("SOFTMAX", 20), ("SOFTMAX_LOSS", 21), ("SPLIT", 22), ("SLICE", 33),
            ("TANH", 23), ("WINDOW_DATA", 24), ("THRESHOLD", 31)],
        "DimCheckMode": [("STRICT", 0), ("PERMISSIVE", 1)]}, [
        r("bottom", 2, "string"), r("top", 3, "string"), o("name", 4, "string"),
        r("include", 32, "NetStateRule"), r("exclude", 33, "NetStateRule"),
        o("type", 5, "V1LayerParameter.LayerType"), r("blobs", 6, "BlobProto"), r("param", 1001, "string"),
        r("blob_share_mode", 1002, "V1LayerParameter.DimCheckMode"), r("blobs_lr", 7, "float"),
        r("weight_decay", 8, "float"), r("loss_weight", 35, "float"),
        o("accuracy_param", 27, "AccuracyParameter"), o("argmax_param", 23, "ArgMaxParameter"),
        o("concat_param", 9, "ConcatParameter"), o("contrastive_loss_param", 40, "ContrastiveLossParameter"),
        o("convolution_param", 10, "ConvolutionParameter"), o("data_param", 11, "DataParameter"),
        o("dropout_param", 12, "DropoutParameter"), o("dummy_data_param", 26, "DummyDataParameter"),
        o("eltwise_param", 24, "EltwiseParameter"), o("exp_param", 41, "ExpParameter"),
        o("hdf5_data_param", 13, "HDF5DataParameter"), o("hdf5_output_param", 14, "HDF5OutputParameter"),
        o("hinge_loss_param", 29, "HingeLossParameter"), o("image_data_param", 15, "ImageDataParameter"),
        o("infogain_loss_param", 16, "InfogainLossParameter"),
        o("inner_product_param", 17, "InnerProductParameter"), o("lrn_param", 18, "LRNParameter"),
        o("memory_data_param", 22, "MemoryDataParameter"), o("mvn_param", 34, "MVNParameter"),
        o("pooling_param", 19, "PoolingParameter"), o("power_param", 21, "PowerParameter"),
        o("relu_param", 30, "ReLUParameter"), o("sigmoid_param", 38, "SigmoidParameter"),
        o("softmax_param", 39, "SoftmaxParameter"), o("slice_param", 31, "SliceParameter"),
        o("tanh_param", 37, "TanHParameter"), o("threshold_param", 25, "ThresholdParameter"),
        o("window_data_param", 20, "WindowDataParameter"),
        o("transform_param", 36, "TransformationParameter"), o("loss_param", 42, "LossParameter"),
        o("layer", 1, "V0LayerParameter")]),
    "V0LayerParameter": ({"PoolMethod": POOL3}, [
        o("name", 1, "string"), o("type", 2, "string"), o("num_output", 3, "uint32"),
        o("biasterm", 4, "bool", True), o("weight_filler", 5, "FillerParameter"),
        o("bias_filler", 6, "FillerParameter"), o("pad", 7, "uint32", 0), o("kernelsize", 8, "uint32"),
        o("group", 9, "uint32", 1), o("stride", 10, "uint32", 1),
        o("pool", 11, "V0LayerParameter.PoolMethod", "MAX"), o("dropout_ratio", 12, "float", 0.5),
        o("local_size", 13, "uint32", 5), o("alpha", 14, "float", 1.0), o("beta", 15, "float", 0.75),
        o("k", 22, "float", 1.0), o("source", 16, "string"), o("scale", 17, "float", 1),
        o("meanfile", 18, "string"), o("batchsize", 19, "uint32"), o("cropsize", 20, "uint32", 0),
        o("mirror", 21, "bool", False), r("blobs", 50, "BlobProto"), r("blobs_lr", 51, "float"),
        r("weight_decay", 52, "float"), o("rand_skip", 53, "uint32", 0),
        o("det_fg_threshold", 54, "float", 0.5), o("det_bg_threshold", 55, "float", 0.5),
        o("det_fg_fraction", 56, "float", 0.25), o("det_context_pad", 58, "uint32", 0),
        o("det_crop_mode", 59, "string", "warp"), o("new_num", 60, "int32", 0),
        o("new_channels", 61, "int32", 0), o("new_height", 62, "int32", 0), o("new_width", 63, "int32", 0),
        o("shuffle_images", 64, "bool", False), o("concat_dim", 65, "uint32", 1),
        o("hdf5_output_param", 1001, "HDF5OutputParameter")]),
}


def _default_str(typ: str, v) -> str:
    if isinstance(v, bool):
        return "true" if v else "false"
    if isinstance(v, float):
        return repr(v)
    return str(v)


def _build_file() -> descriptor_pb2.FileDescriptorProto:
    fdp = descriptor_pb2.FileDescriptorProto(name="sparknet_amd/caffe.proto", package="caffe",
                                             syntax="proto2")
    for en, vals in ENUMS.items():
        e = fdp.enum_type.add(name=en)
        for vn, vv in vals:
            e.value.add(name=vn, number=vv)
    enum_names = set(ENUMS)
    for mname, (enums, _) in MESSAGES.items():
        enum_names.update(f"{mname}.{e}" for e in enums)
    for mname, (enums, fields) in MESSAGES.items():
        m = fdp.message_type.add(name=mname)
        for en, vals in enums.items():
            e = m.enum_type.add(name=en)
            for vn, vv in vals:
                e.value.add(name=vn, number=vv)
        for (fname, num, label, typ, default, packed) in fields:
            f = m.field.add(name=fname, number=num)
            f.label = _FD.LABEL_REPEATED if label == "rep" else _FD.LABEL_OPTIONAL
            if typ in _SCALARS:
                f.type = _SCALARS[typ]
            elif typ in enum_names:
                f.type = _FD.TYPE_ENUM
                f.type_name = ".caffe." + typ
            else:
                assert typ in MESSAGES, typ
                f.type = _FD.TYPE_MESSAGE
                f.type_name = ".caffe." + typ
            if default is not None:
                f.default_value = _default_str(typ, default)
            if packed:
                f.options.packed = True
    return fdp


FILE_DESCRIPTOR = _build_file()
_POOL = descriptor_pool.DescriptorPool()
_CLASSES = message_factory.GetMessages([FILE_DESCRIPTOR], pool=_POOL)


def message_class(name: str):
    return _CLASSES["caffe." + name]


def phase_value(name: str) -> int:
    return dict(ENUMS["Phase"])[name]
