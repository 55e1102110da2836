"""Python side of ``libsn_core.so`` — the C ABI that replaces SparkNet's ``libccaffe``
(libccaffe/ccaffe.cpp:22-296, called from the JVM through JNA, CaffeLibrary.java:8-76).

The native library (csrc/core/sn_core.cpp) owns the C entry points, GIL handling and
handle lifetime; every verb lands in one function here operating on a
:class:`CoreState`.  Data stays device-resident: weights are exchanged as one flat fp32
buffer (the reference copied them float by float through JNA, Net.scala:132-172), and the
JavaData layers are fed through a C callback ``cb(float* buf, int batch, int ndims,
const int* shape, void* user)`` with the same contract as ``java_callback_t``
(CaffeLibrary.java:12-14), invoked once per forward with a host staging buffer that is
then copied to the device.
"""
from __future__ import annotations

import ctypes as C
import os

import numpy as np
import torch

from . import proto
from .core.net import Net
from .core.solver import Solver

CALLBACK = C.CFUNCTYPE(None, C.c_void_p, C.c_int, C.c_int, C.POINTER(C.c_int), C.c_void_p)


class CoreState:
    """caffenet_state (ccaffe.cpp:22-31): a solver with its train net, a test net, the
    device, callbacks and the last test scores."""

    def __init__(self):
        self.device = torch.device("cpu")
        self.solver: Solver | None = None
        self.net: Net | None = None        # net used by forward/backward (solver's train net)
        self.test_net: Net | None = None
        self.scores: list[float] = []
        self._callbacks = {}                # (phase, layer index) -> (ctypes fn, user) kept alive

    # -- construction -------------------------------------------------------------------
    def set_device(self, device: int) -> None:
        if device >= 0 and torch.cuda.is_available():
            torch.cuda.set_device(device)
            from .ops import _lib
            _lib.kernels()
            self.device = torch.device("cuda", device)
        else:
            self.device = torch.device("cpu")

    def load_solver(self, data: bytes) -> None:
        """load_solver_from_protobuf (ccaffe.cpp:128-134): SolverParameter bytes with an
        embedded net; the solver's first test net becomes the test net."""
        sp = proto.SolverParameter()
        sp.ParseFromString(data)
        self.solver = Solver(sp, device=self.device)
        if self.device.type == "cuda":
            from .engine import fuse_relu
            fuse_relu(self.solver.net)
            for tn in self.solver.test_nets:
                fuse_relu(tn)
        self.net = self.solver.net
        self.test_net = self.solver.test_nets[0] if self.solver.test_nets else None

    def load_net(self, data: bytes) -> None:
        """load_net_from_protobuf (ccaffe.cpp:136-140): a stand-alone TEST-phase net."""
        npm = proto.NetParameter()
        npm.ParseFromString(data)
        self.test_net = Net(npm, phase=proto.TEST, device=self.device)
        if self.net is None:
            self.net = self.test_net

    # -- data feed ----------------------------------------------------------------------------
    def set_data_callback(self, test: bool, layer_index: int, fn_addr: int, user: int) -> None:
        """set_train_data_callback / set_test_data_callback (ccaffe.cpp:197-216)."""
        net = self.test_net if test else self.net
        layer = net.layers[layer_index]
        fn = CALLBACK(fn_addr)

        def source(lay, tops, _fn=fn, _user=user):
            t = tops[0]
            shape = tuple(t.shape)
            host = np.empty(shape, dtype=np.float32)
            dims = (C.c_int * len(shape))(*shape)
            _fn(host.ctypes.data, shape[0], len(shape), dims, _user)
            t.set_nchw(torch.from_numpy(host))
        layer.set_source(source)
        self._callbacks[(test, layer_index)] = (fn, user)

    # -- execution ------------------------------------------------------------------------------
    def forward(self) -> float:
        return float(self.net.forward())

    def backward(self) -> None:
        self.net.backward()

    def step(self, n: int) -> None:
        self.solver.step(n)

    def test(self, n: int) -> int:
        """solver_test -> TestAndStoreResult (solver.cpp:413-444): sum of every output
        blob over n forwards; returns the number of scores."""
        net = self.test_net
        sums = None
        for _ in range(n):
            net.forward()
            v = [float(b.data.float().sum()) for b in net.output_blobs]
            sums = v if sums is None else [a + b for a, b in zip(sums, v)]
        self.scores = sums or []
        return len(self.scores)

    # -- weights --------------------------------------------------------------------------------
    def num_params(self) -> int:
        return int(self.net.num_param_elems)

    def get_weights(self, addr: int, n: int) -> None:
        dst = np.ctypeslib.as_array(C.cast(addr, C.POINTER(C.c_float)), shape=(n,))
        dst[:] = self.net.flat_data[:n].detach().cpu().numpy()

    def set_weights(self, addr: int, n: int) -> None:
        src = np.ctypeslib.as_array(C.cast(addr, C.POINTER(C.c_float)), shape=(n,))
        self.net.flat_data[:n].copy_(torch.from_numpy(src.copy()))
        self.net.sync_compute()

    def weights_device_ptr(self) -> int:
        """Zero-copy access for device-side callers (RCCL, custom kernels)."""
        return int(self.net.flat_data.data_ptr())

    def save_weights(self, path: str) -> None:
        from .utils.checkpoint import save_caffemodel
        save_caffemodel(self.net, path)

    def load_weights(self, path: str) -> None:
        self.net.copy_trained_layers_from(path)

    def restore_solver(self, path: str) -> None:
        self.solver.restore(path)

    def layer_names(self) -> list[str]:
        return list(self.net.layer_names)

    # -- databases (ccaffe.cpp:51-81) ---------------------------------------------------------
    def create_db(self, name: str, db_type: str) -> None:
        import shutil
        from .data.db import DatumWriter
        if os.path.isdir(name):
            shutil.rmtree(name)
        self._db = DatumWriter(name, commit_every=1 << 62, backend=db_type)

    def write_to_db(self, image: bytes, label: int, c: int, h: int, w: int, key: str) -> None:
        d = proto.Datum(channels=c, height=h, width=w, data=image, label=label, encoded=False)
        self._db.put(d, key or None)

    def commit_db_txn(self) -> None:
        self._db.commit()

    def close_db(self) -> None:
        self._db.close()
        self._db = None

    # -- blobs (ccaffe.cpp:142-195) -----------------------------------------------------------
    def num_layer_weights(self, layer: int) -> int:
        return len(self.net.layers[layer].params)

    def num_data_blobs(self) -> int:
        return len(self.net.blobs)

    def data_blob_name(self, index: int) -> str:
        return self.net.blob_names[index]

    def num_output_blobs(self) -> int:
        return len(self.net.output_blobs)

    def num_test_scores(self) -> int:
        return len(self.scores)

    def _blob(self, layer: int, index: int):
        if layer < 0:
            return self.net.blobs[index], None
        return None, self.net.layers[layer].params[index]

    def blob_shape(self, layer: int, index: int) -> tuple:
        blob, prm = self._blob(layer, index)
        return tuple(blob.shape) if blob is not None else tuple(prm.caffe_shape)

    def blob_num_axes(self, layer: int, index: int) -> int:
        return len(self.blob_shape(layer, index))

    def blob_axis_shape(self, layer: int, index: int, axis: int) -> int:
        return int(self.blob_shape(layer, index)[axis])

    def blob_get(self, layer: int, index: int, diff: int, addr: int, n: int) -> None:
        blob, prm = self._blob(layer, index)
        if blob is not None:
            t = blob.nchw(diff=bool(diff))
        else:
            t = prm.to_caffe(prm.diff if diff else None)
        src = t.detach().float().cpu().reshape(-1).numpy()
        if n < src.size:
            raise ValueError(f"buffer holds {n} floats, blob has {src.size}")
        dst = np.ctypeslib.as_array(C.cast(addr, C.POINTER(C.c_float)), shape=(src.size,))
        dst[:] = src

    def blob_set(self, layer: int, index: int, diff: int, addr: int, n: int) -> None:
        blob, prm = self._blob(layer, index)
        shape = self.blob_shape(layer, index)
        count = int(np.prod(shape)) if shape else 1
        if n < count:
            raise ValueError(f"buffer holds {n} floats, blob has {count}")
        src = torch.from_numpy(np.ctypeslib.as_array(C.cast(addr, C.POINTER(C.c_float)), shape=(count,)).copy())
        src = src.reshape(shape)
        if blob is not None:
            blob.set_nchw(src, diff=bool(diff))
        elif diff:
            prm.diff.copy_(prm.from_caffe(src).to(prm.diff.device))
        else:
            prm.set_caffe(src)
            self.net.sync_compute()


def init_logging(log_filename: str, verbosity: int) -> None:
    """init_logging (ccaffe.cpp:33-37): log records to a file, stderr from ``verbosity``."""
    import logging
    root = logging.getLogger("sparknet_amd")
    root.setLevel(logging.INFO)
    fh = logging.FileHandler(log_filename)
    fh.setFormatter(logging.Formatter("%(asctime)s %(levelname)s %(name)s] %(message)s"))
    root.addHandler(fh)
    sh = logging.StreamHandler()
    sh.setLevel([logging.INFO, logging.WARNING, logging.ERROR, logging.CRITICAL][max(0, min(verbosity, 3))])
    root.addHandler(sh)


def set_basepath(path: str) -> None:
    """set_basepath (ccaffe.cpp:39-41): relative paths in prototxts resolve from here."""
    os.chdir(path)


def save_mean_image(addr: int, c: int, h: int, w: int, filename: str) -> None:
    """save_mean_image (ccaffe.cpp:83-97)."""
    from .data.loaders import write_mean_binaryproto
    mean = np.ctypeslib.as_array(C.cast(addr, C.POINTER(C.c_float)), shape=(c * h * w,)).copy()
    write_mean_binaryproto(mean.reshape(c, h, w), filename)


def parse_net_prototxt(path: str) -> bytes:
    return proto.read_net(path).SerializeToString()


def parse_solver_prototxt(path: str) -> bytes:
    return proto.read_solver(path).SerializeToString()
