"""Caffe-compatible configuration and checkpoint formats.

Mirrors the reference's IO surface:
* ``read_prototxt`` / ``parse_prototxt``  <- ``ReadProtoFromTextFile``
  (caffe/src/caffe/util/io.cpp:34) and ``parse_{net,solver}_prototxt``
  (libccaffe/ccaffe.cpp:275-296, ProtoLoader.scala:9-29)
* ``read_binary`` / ``write_binary``       <- ``ReadProtoFromBinaryFile`` /
  ``WriteProtoToBinaryFile`` (io.cpp:52-67) used for .caffemodel / .solverstate /
  mean .binaryproto files
* ``to_prototxt``                           <- text_format printing
"""
from __future__ import annotations

from pathlib import Path

from google.protobuf import text_format

from .schema import message_class, phase_value

BlobShape = message_class("BlobShape")
BlobProto = message_class("BlobProto")
BlobProtoVector = message_class("BlobProtoVector")
Datum = message_class("Datum")
FillerParameter = message_class("FillerParameter")
NetParameter = message_class("NetParameter")
SolverParameter = message_class("SolverParameter")
SolverState = message_class("SolverState")
NetState = message_class("NetState")
NetStateRule = message_class("NetStateRule")
ParamSpec = message_class("ParamSpec")
LayerParameter = message_class("LayerParameter")
V1LayerParameter = message_class("V1LayerParameter")

TRAIN = phase_value("TRAIN")
TEST = phase_value("TEST")

__all__ = [
    "BlobShape", "BlobProto", "BlobProtoVector", "Datum", "FillerParameter", "NetParameter",
    "SolverParameter", "SolverState", "NetState", "NetStateRule", "ParamSpec", "LayerParameter",
    "V1LayerParameter", "TRAIN", "TEST", "parse_prototxt", "read_prototxt", "to_prototxt",
    "read_binary", "write_binary", "read_net", "read_solver", "copy",
]


def parse_prototxt(text: str, cls=NetParameter):
    msg = cls()
    text_format.Parse(text, msg)
    return msg


def read_prototxt(path, cls=NetParameter):
    return parse_prototxt(Path(path).read_text(), cls)


def to_prototxt(msg) -> str:
    return text_format.MessageToString(msg)


def write_prototxt(path, msg) -> None:
    Path(path).write_text(to_prototxt(msg))


def read_binary(path, cls=NetParameter):
    msg = cls()
    msg.ParseFromString(Path(path).read_bytes())
    return msg


def write_binary(path, msg) -> None:
    Path(path).write_bytes(msg.SerializeToString())


def read_net(path):
    """Read a NetParameter from .prototxt (text) or .caffemodel (binary), upgrading V1."""
    p = Path(path)
    if p.suffix in (".prototxt", ".pbtxt", ".txt"):
        net = read_prototxt(p, NetParameter)
    else:
        net = read_binary(p, NetParameter)
    from .upgrade import upgrade_net
    return upgrade_net(net)


def read_solver(path):
    return read_prototxt(path, SolverParameter)


def copy(msg):
    out = type(msg)()
    out.CopyFrom(msg)
    return out
