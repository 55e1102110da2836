"""pycaffe's ``caffe.Net`` / solver classes (caffe/python/caffe/_caffe.cpp:215-331 and
pycaffe.py) over this framework's :class:`~sparknet_amd.core.net.Net` and
:class:`~sparknet_amd.core.solver.Solver`.

Blob and param contents are numpy arrays in Caffe's logical layout (N x C x H x W blobs,
Caffe-shaped weights).  On a CPU fp32 net a blob's ``.data`` is a live strided view of the
engine's NHWC storage; on the GPU (or for parameters, whose internal layout differs) it
is a host copy whose top-level item assignment (``blob.data[...] = x``, ``blob.data[i] =
x``) writes back to the device.
"""
from __future__ import annotations

from collections import OrderedDict
from itertools import zip_longest

import numpy as np
import torch

from .. import proto
from ..core.net import Net as _CoreNet
from ..core.solver import Solver as _CoreSolver

_STATE = {"device": "cpu"}


def set_mode_cpu() -> None:
    _STATE["device"] = "cpu"


def set_mode_gpu() -> None:
    idx = int(_STATE["device"].split(":")[1]) if ":" in _STATE["device"] else 0
    _STATE["device"] = f"cuda:{idx}"


def set_device(device_id: int) -> None:
    _STATE["device"] = f"cuda:{int(device_id)}"


def current_device() -> str:
    return _STATE["device"]


class _SyncedArray(np.ndarray):
    """Host copy of device (or re-laid-out) data; top-level item assignment writes back."""

    def __new__(cls, arr, setter):
        obj = np.array(arr, dtype=np.float32).view(cls)
        obj._setter = setter
        return obj

    def __array_finalize__(self, obj):
        self._setter = None  # views / results of operations do not write back

    def __setitem__(self, key, value):
        super().__setitem__(key, value)
        if self._setter is not None:
            self._setter(np.asarray(self).view(np.ndarray))


class Blob:
    """pycaffe Blob: ``data`` / ``diff`` arrays in logical (NCHW) layout."""

    def __init__(self, blob):
        self._b = blob

    def _get(self, diff: bool):
        b = self._b
        t = b.nchw(diff)
        if t.device.type == "cpu" and t.dtype == torch.float32:
            return t.numpy()  # live view (writable, strided for image blobs)
        return _SyncedArray(t.detach().float().cpu().numpy(),
                            lambda a, b=b, diff=diff: b.set_nchw(torch.from_numpy(np.ascontiguousarray(a)), diff))

    @property
    def data(self):
        return self._get(False)

    @property
    def diff(self):
        return self._get(True)

    @property
    def shape(self):
        return tuple(self._b.shape)

    @property
    def count(self):
        return self._b.count

    @property
    def num(self):
        return self._b.shape[0] if self._b.shape else 1

    @property
    def channels(self):
        return self._b.shape[1] if len(self._b.shape) > 1 else 1

    @property
    def height(self):
        return self._b.shape[2] if len(self._b.shape) > 2 else 1

    @property
    def width(self):
        return self._b.shape[3] if len(self._b.shape) > 3 else 1

    def reshape(self, *shape):
        self._b.reshape(tuple(int(s) for s in shape))


class ParamBlob:
    """A learnable parameter in Caffe layout (``net.params[layer][i]``)."""

    def __init__(self, param, net):
        self._p, self._net = param, net

    @property
    def data(self):
        p, net = self._p, self._net

        def setter(a):
            p.set_caffe(torch.from_numpy(np.ascontiguousarray(a)))
            net.sync_compute()
        return _SyncedArray(p.to_caffe().cpu().numpy(), setter)

    @property
    def diff(self):
        p = self._p

        def setter(a):
            p.diff.copy_(p.from_caffe(torch.from_numpy(np.ascontiguousarray(a)).to(p.diff.device)))
        return _SyncedArray(p.to_caffe(p.diff).cpu().numpy(), setter)

    @property
    def shape(self):
        return tuple(self._p.caffe_shape)

    @property
    def count(self):
        return self._p.caffe_count

    @property
    def num(self):
        return self._p.caffe_shape[0]


class _LayerView:
    def __init__(self, layer, net):
        self._l = layer
        self.type = layer.type_name
        self.blobs = [ParamBlob(p, net) for p in layer.params]

    def __repr__(self):
        return f"<Layer {self._l.name!r} type={self.type}>"


def _read_net(path_or_param):
    if not isinstance(path_or_param, str):
        return proto.copy(path_or_param)
    with open(path_or_param, "rb") as f:
        raw = f.read()
    try:
        return proto.parse_prototxt(raw.decode("utf-8"))
    except Exception:  # binary NetParameter
        return proto.read_binary(path_or_param)


class Net:
    """``Net(prototxt, phase)``, ``Net(prototxt, weights, phase)`` or
    ``Net(prototxt, phase, weights=...)`` (caffe/python/caffe/_caffe.cpp:215-253)."""

    def __init__(self, network_file, *args, weights: str | None = None, phase: int | None = None,
                 level: int | None = None, stages=None):
        for a in args:
            if isinstance(a, str):
                weights = a
            else:
                phase = a
        if phase is None:
            raise ValueError("Net needs a phase (TRAIN or TEST)")
        self._net = _CoreNet(_read_net(network_file), phase=phase, level=level, stages=stages,
                             device=current_device())
        if weights:
            self._net.copy_trained_layers_from(weights)
            self._net.sync_compute()

    @classmethod
    def _wrap(cls, core_net) -> "Net":
        obj = cls.__new__(cls)
        obj._net = core_net
        return obj

    # -- introspection ----------------------------------------------------------------
    @property
    def _blob_names(self):
        return list(self._net.blob_names)

    @property
    def _layer_names(self):
        return list(self._net.layer_names)

    @property
    def blobs(self):
        return OrderedDict((n, Blob(b)) for n, b in zip(self._net.blob_names, self._net.blobs))

    @property
    def blob_loss_weights(self):
        w = {id(t): lw for t, lw in self._net._loss_tops}
        return OrderedDict((n, float(w.get(id(b), 0.0))) for n, b in zip(self._net.blob_names, self._net.blobs))

    @property
    def params(self):
        return OrderedDict((n, [ParamBlob(p, self._net) for p in layer.params])
                           for n, layer in zip(self._net.layer_names, self._net.layers) if layer.params)

    @property
    def layers(self):
        return [_LayerView(layer, self._net) for layer in self._net.layers]

    @property
    def inputs(self):
        """Net inputs: declared ``input`` blobs, else the tops of externally fed data layers."""
        net = self._net
        if net.input_blob_ids:
            return [net.blob_names[i] for i in net.input_blob_ids]
        return [net.blob_names[t] for li, layer in enumerate(net.layers)
                if layer.type_name in ("JavaData", "RDD", "Input", "MemoryData") for t in net.top_ids[li]]

    @property
    def outputs(self):
        return [self._net.blob_names[i] for i in self._net.output_blob_ids]

    # -- execution --------------------------------------------------------------------
    def _set(self, name, arr, diff=False):
        b = self._net.blob_by_name(name)
        arr = np.asarray(arr, dtype=np.float32)
        if arr.shape[0] != (b.shape[0] if b.shape else 1):
            raise ValueError(("Diff" if diff else "Input") + " is not batch sized")
        b.set_nchw(torch.from_numpy(np.ascontiguousarray(arr)).reshape(b.shape), diff)

    def forward(self, blobs=None, start=None, end=None, **kwargs):
        """Forward from layer ``start`` to ``end`` (names, inclusive); kwargs set input
        blobs.  Returns {blob name: array} for the outputs (or ``end``) plus ``blobs``."""
        blobs = list(blobs or [])
        s = self._net.layer_names_index[start] if start is not None else 0
        e = self._net.layer_names_index[end] if end is not None else len(self._net.layers) - 1
        outputs = set(([end] if end is not None else self.outputs) + blobs)
        for name, arr in kwargs.items():
            self._set(name, arr)
        self._net.forward_from_to(s, e)
        got = self.blobs
        return {o: got[o].data for o in outputs if o in got}

    def backward(self, diffs=None, start=None, end=None, **kwargs):
        diffs = list(diffs or [])
        s = self._net.layer_names_index[start] if start is not None else len(self._net.layers) - 1
        e = self._net.layer_names_index[end] if end is not None else 0
        outputs = set(([end] if end is not None else self.inputs) + diffs)
        for name, arr in kwargs.items():
            self._set(name, arr, diff=True)
        self._net.backward_from_to(s, e)
        got = self.blobs
        return {o: got[o].diff for o in outputs if o in got}

    def _batch(self, arrays: dict):
        n = len(next(iter(arrays.values())))
        bs = self._net.blobs[self._net.blob_names_index[next(iter(arrays))]].shape[0]
        for i in range(0, n - n % bs, bs):
            yield {k: v[i:i + bs] for k, v in arrays.items()}
        if n % bs:
            rem = n % bs
            yield {k: np.concatenate([v[-rem:], np.zeros((bs - rem,) + np.asarray(v).shape[1:], np.float32)])
                   for k, v in arrays.items()}

    def forward_all(self, blobs=None, **kwargs):
        """Forward over arbitrarily many inputs in batch-size pieces (last one zero-padded)."""
        outs = {o: [] for o in set(self.outputs + list(blobs or []))}
        for batch in self._batch(kwargs):
            for k, v in self.forward(blobs=blobs, **batch).items():
                outs[k].extend(np.array(v, copy=True))
        n = len(next(iter(kwargs.values())))
        return {k: np.asarray(v)[:n] for k, v in outs.items()}

    def forward_backward_all(self, blobs=None, diffs=None, **kwargs):
        outs = {o: [] for o in set(self.outputs + list(blobs or []))}
        grads = {d: [] for d in set(self.inputs + list(diffs or []))}
        fwd = {k: v for k, v in kwargs.items() if k in self.inputs}
        bwd = {k: v for k, v in kwargs.items() if k in self.outputs}
        for fb, bb in zip_longest(self._batch(fwd) if fwd else [], self._batch(bwd) if bwd else [], fillvalue={}):
            for k, v in self.forward(blobs=blobs, **fb).items():
                outs[k].extend(np.array(v, copy=True))
            for k, v in self.backward(diffs=diffs, **bb).items():
                grads[k].extend(np.array(v, copy=True))
        n = len(next(iter(kwargs.values()))) if kwargs else None
        return ({k: np.asarray(v)[:n] for k, v in outs.items()}, {k: np.asarray(v)[:n] for k, v in grads.items()})

    def set_input_arrays(self, data, labels):
        """Feed the MemoryData layer (pycaffe.py:235-243)."""
        for layer in self._net.layers:
            if layer.type_name == "MemoryData":
                layer.reset(torch.as_tensor(np.asarray(data, np.float32)),
                            torch.as_tensor(np.asarray(labels, np.float32).reshape(-1)))
                return
        raise RuntimeError("set_input_arrays needs a MemoryData layer")

    def reshape(self):
        self._net.reshape()

    def copy_from(self, weights: str):
        self._net.copy_trained_layers_from(weights)
        self._net.sync_compute()

    def share_with(self, other: "Net"):
        self._net.share_trained_layers_with(other._net)

    def save(self, filename: str):
        proto.write_binary(filename, self._net.to_proto())

    def save_hdf5(self, filename: str):
        self._net.to_hdf5(filename)


class _Solver:
    TYPE = "SGD"

    def __init__(self, solver_file):
        sp = proto.read_solver(solver_file) if isinstance(solver_file, str) else proto.copy(solver_file)
        sp.type = self.TYPE
        self._s = _CoreSolver(sp, device=current_device())
        self.net = Net._wrap(self._s.net)
        self.test_nets = [Net._wrap(n) for n in self._s.test_nets]

    @property
    def iter(self) -> int:
        return self._s.iter

    @property
    def param(self):
        return self._s.param

    def step(self, iters: int) -> None:
        self._s.step(iters)

    def solve(self, resume_file: str | None = None) -> None:
        self._s.solve(resume_file)

    def snapshot(self):
        return self._s.snapshot()

    def restore(self, state_file: str) -> None:
        self._s.restore(state_file)

    def test(self, test_net_id: int = 0):
        return self._s.test(test_net_id)


class SGDSolver(_Solver):
    TYPE = "SGD"


class NesterovSolver(_Solver):
    TYPE = "Nesterov"


class AdaGradSolver(_Solver):
    TYPE = "AdaGrad"


class RMSPropSolver(_Solver):
    TYPE = "RMSProp"


class AdaDeltaSolver(_Solver):
    TYPE = "AdaDelta"


class AdamSolver(_Solver):
    TYPE = "Adam"


_SOLVERS = {c.TYPE: c for c in (SGDSolver, NesterovSolver, AdaGradSolver, RMSPropSolver, AdaDeltaSolver, AdamSolver)}


def get_solver(solver_file):
    """The solver class named by the file's ``type`` (legacy ``solver_type`` honoured)."""
    sp = proto.read_solver(solver_file) if isinstance(solver_file, str) else solver_file
    legacy = {0: "SGD", 1: "Nesterov", 2: "AdaGrad", 3: "RMSProp", 4: "AdaDelta", 5: "Adam"}
    t = sp.type if sp.HasField("type") else legacy.get(int(sp.solver_type), "SGD")
    return _SOLVERS[t](solver_file)
