"""pycaffe-compatible Python API (caffe/python/caffe/__init__.py) over the sparknet_amd
engine, so scripts written against ``import caffe`` port by changing the import:

    from sparknet_amd import pycaffe as caffe
    caffe.set_mode_gpu()
    net = caffe.Net("deploy.prototxt", "weights.caffemodel", caffe.TEST)
    net.blobs["data"].data[...] = batch
    out = net.forward()
    solver = caffe.get_solver("solver.prototxt"); solver.step(100)

Provided: ``Net``, ``SGDSolver`` / ``NesterovSolver`` / ``AdaGradSolver`` /
``RMSPropSolver`` / ``AdaDeltaSolver`` / ``AdamSolver``, ``get_solver``, ``set_mode_cpu`` /
``set_mode_gpu`` / ``set_device``, ``TRAIN`` / ``TEST``, ``layer_type_list``, the NetSpec
builder (``layers``, ``params``, ``NetSpec``, ``to_proto``), ``io`` (Transformer,
BlobProto / Datum conversion, image IO, oversampling), ``Classifier``, ``draw`` and the
``Layer`` base class for Python layers.
"""
from __future__ import annotations

from .. import proto as _proto
from . import draw, io  # noqa: F401
from .classifier import Classifier  # noqa: F401
from .detector import Detector  # noqa: F401
from .net import (AdaDeltaSolver, AdaGradSolver, AdamSolver, Net, NesterovSolver, RMSPropSolver,  # noqa: F401
                  SGDSolver, get_solver, set_device, set_mode_cpu, set_mode_gpu)
from .net_spec import NetSpec, layers, params, to_proto  # noqa: F401

TRAIN = _proto.TRAIN
TEST = _proto.TEST


def layer_type_list() -> list[str]:
    """Registered layer type strings (LayerRegistry::LayerTypeList)."""
    from ..core.layer import layer_types
    return sorted(layer_types())


class Layer:
    """Base class for ``type: "Python"`` layers (caffe/include/caffe/python_layer.hpp):
    override setup / reshape / forward / backward; ``self.param_str`` holds
    python_param.param_str and ``self.phase`` the net phase."""

    param_str = ""
    phase = TRAIN

    def setup(self, bottom, top):
        pass

    def reshape(self, bottom, top):
        pass

    def forward(self, bottom, top):
        raise NotImplementedError

    def backward(self, top, propagate_down, bottom):
        pass
