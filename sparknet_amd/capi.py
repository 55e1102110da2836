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
import math
import os

import numpy as np
import torch

from . import proto
from .core.net import Net
from .core.solver import Solver

CALLBACK = C.CFUNCTYPE(None, C.c_void_p, C.c_int, C.c_int, C.POINTER(C.c_int), C.c_void_p)


class _plain_backward:
    """The net's backward as Caffe's Net::Backward: gradients into the parameter diffs, no
    solver work.  The native step path (engine.GraphStep) fuses the InnerProduct SGD update
    into the weight-gradient GEMM (engine.fuse_fc_updates) and may route conv weight
    gradients to split-K slabs the solver consumes (engine.fuse_splitk_updates); both are
    switched off for an sn_backward / backward-plan capture and restored afterwards."""

    def __init__(self, net):
        self.net = net

    def __enter__(self):
        self.saved = []
        for layer in self.net.layers:
            for attr in ("fused_update", "slab_grad"):
                if getattr(layer, attr, None) is not None:
                    self.saved.append((layer, attr, getattr(layer, attr)))
                    setattr(layer, attr, None)
        return self

    def __exit__(self, *exc):
        for layer, attr, val in self.saved:
            setattr(layer, attr, val)
        return False


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
        self.native_ran = 0                 # iterations a failed native_plan capture had run

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
        with _plain_backward(self.net):
            self.net.backward()

    def step(self, n: int) -> None:
        self.solver.step(n)

    # -- native step executor (csrc/core/sn_core.cpp NativeStep) ---------------------------
    # On the GPU, sn_solver_step runs training iterations without Python: this method
    # captures ONE full iteration (forward, backward, fused solver update — every kernel a
    # HIP kernel of libsn_kernels) into a hipGraph through engine.GraphStep, running
    # `warmup` eager iterations plus the capture's replay as real iterations fed by the
    # Python path, and hands the C++ executor the graph-exec handle, the stream, the device
    # buffers it stages callback data / hyper-parameters into and the solver schedule.
    # Per iteration the C++ loop then calls the C data callbacks, copies the minibatches
    # into the data blobs (sn_stage_nchw_f32_bf16 for images), stages the learning rate and
    # launches the graph; Python is re-entered only at display / snapshot iterations.
    NATIVE_WARMUP = 2

    def native_eligible(self) -> bool:
        return self.device.type == "cuda" and self.solver is not None and self.net is self.solver.net

    def _c_feeds(self, net, test: bool) -> list:
        """(layer, source, feed dict) for every data layer of ``net``: each must be an
        ExternalDataLayer fed by a C callback registered for that phase.  The feed dict is
        what the native loops stage per iteration: device blob pointer, kind (1: 4-D bf16
        NHWC image blob staged by sn_stage_nchw_f32_bf16, 0: fp32 blob copied as is),
        logical shape, callback and user pointer."""
        from .layers.data import ExternalDataLayer
        feeds = []
        for li, layer in enumerate(net.layers):
            if not getattr(layer, "is_data", False):
                continue
            if isinstance(layer, ExternalDataLayer) and layer.source is None:
                continue  # blobs set once by the host (sn_blob_set) stay as they are
            if not isinstance(layer, ExternalDataLayer) or (test, li) not in self._callbacks:
                raise RuntimeError(f"data layer {layer.name!r} is not fed by a C callback")
            fn, user = self._callbacks[(test, li)]
            top = net.top_vecs[li][0]
            t = top.data
            if len(top.shape) == 4:
                if t.dtype != torch.bfloat16 or not t.is_contiguous():
                    raise RuntimeError(f"data blob of {layer.name!r} is not a bf16 NHWC image blob")
                kind = 1
            else:
                if t.dtype != torch.float32 or not t.is_contiguous():
                    raise RuntimeError(f"data blob of {layer.name!r} is not fp32")
                kind = 0
            feeds.append((layer, layer.source, {"dev": t.data_ptr(), "kind": kind, "shape": tuple(top.shape),
                                                "cb": C.cast(fn, C.c_void_p).value, "user": user or 0}))
        return feeds

    def native_plan(self) -> tuple:
        """-> (iterations already run, plan dict of ints / floats) or raises if the
        state cannot run natively (CPU device, solver features the graph cannot hold)."""
        from .engine import GraphStep
        self.native_ran = 0
        s = self.solver
        if self.device.type != "cuda" or s is None:
            raise RuntimeError("native stepping needs a GPU solver")
        p = s.param
        if p.iter_size > 1 or p.clip_gradients > 0 or s.callbacks or s.action_request is not None:
            raise RuntimeError("native stepping: iter_size / clip_gradients / callbacks / action requests "
                               "stay on the Python path")
        net = self.net
        feeds = self._c_feeds(net, False)
        for layer, _, _ in feeds:
            layer.set_source(None)  # inside the graph the blobs are already staged (restored below)

        def pre():
            for layer, src, _ in feeds:
                src(layer, net.top_vecs[net.layers.index(layer)])

        it0 = s.iter
        self._graph_step = GraphStep(s, warmup=self.NATIVE_WARMUP, pre=pre, overlap=False)
        s.stage_hyper()
        try:
            loss = self._graph_step.step()  # warmup iterations + capture + one replay
        except BaseException:
            # iterations already run count against the caller's request (sn_core.cpp
            # subtracts native_ran before falling back to the Python solver)
            self.native_ran = s.iter - it0
            raise
        finally:
            for layer, src, _ in feeds:  # the Python verbs (sn_forward, ...) keep their feeds
                layer.set_source(src)
        torch.cuda.synchronize(self.device)
        pol = ["fixed", "step", "exp", "inv", "multistep", "poly", "sigmoid"].index(p.lr_policy)
        hyper = s.hyper_values(s.get_learning_rate())
        plan = {
            "exec": int(self._graph_step.graph.raw_cuda_graph_exec()),
            "stream": int(torch.cuda.current_stream(self.device).cuda_stream),
            "hyper_dev": int(s.hyper.data_ptr()), "hyper": [float(v) for v in hyper],
            "loss_dev": int(loss.data_ptr()), "iter": int(s.iter),
            "policy": pol, "base_lr": float(p.base_lr), "gamma": float(p.gamma), "power": float(p.power),
            "stepsize": int(p.stepsize), "max_iter": int(p.max_iter), "stepvalues": [int(v) for v in p.stepvalue],
            "adam": int(s.type == "Adam"), "momentum": float(p.momentum), "momentum2": float(p.momentum2),
            "display": int(p.display), "snapshot": int(p.snapshot), "average_loss": max(1, int(p.average_loss)),
            "feeds": [f for _, _, f in feeds],
        }
        return s.iter - it0, plan

    def native_event(self, it: int, smoothed_loss: float, snapshot: int) -> None:
        """Display / snapshot iteration reached by the native loop (Solver.step's logging
        and snapshot, solver.cpp:227-262)."""
        s = self.solver
        s.iter = it
        if smoothed_loss == smoothed_loss and smoothed_loss >= 0:
            import logging
            s.smoothed_loss = smoothed_loss
            logging.getLogger("sparknet_amd.solver").info("Iteration %d, loss = %g", it - 1, smoothed_loss)
        if snapshot:
            s.snapshot()

    def native_done(self, it: int) -> None:
        self.solver.iter = it

    # -- native forward / test (csrc/core/sn_core.cpp NativeForward) ------------------------
    # sn_forward and sn_solver_test on a GPU state replay a captured forward-only graph of
    # the train net / the test net (ccaffe.cpp:181-187 forward, 218-228 solver_test ->
    # TestAndStoreResult).  The test graph also adds every element of every output blob
    # into a device accumulator (one score per element, solver.cpp:427-440), so n test
    # iterations are n graph launches and ONE host read at the end.
    #
    # Capturing rebinds the Python-visible blobs and saved layer buffers (masks, folds,
    # loss state) to the graph's own memory, which the capture itself never writes: the
    # plan therefore replays the graph once on the same staged batch, so the net is left
    # in the state of that replay (sn_backward, blob reads), and the caller reports the
    # replay's loss.  Any later Python forward of the same net rebinds the blobs again,
    # so sn_core.cpp drops the plan whenever one can run (invalidate(P_FWD_*)).
    @staticmethod
    def _stateful_params(net) -> list:
        """Parameter blobs a forward pass writes: train-phase BatchNorm running statistics
        (batch_norm_layer.cpp:104-121 updates them inside Forward)."""
        out = []
        for layer in net.layers:
            if layer.type_name == "BatchNorm" and not getattr(layer, "use_global", True):
                out += [p for p in layer.params if p.data is not None]
        return out

    def forward_plan(self, test: bool) -> dict:
        """Capture one forward pass and replay it once; called right after the Python
        verb ran the same forward eagerly, so every GEMM is already autotuned."""
        net = self.test_net if test else self.net
        if self.device.type != "cuda" or net is None:
            raise RuntimeError("native forward needs a GPU net")
        feeds = self._c_feeds(net, test)
        dev = self.device
        torch.cuda.synchronize(dev)
        for layer, _, _ in feeds:
            layer.set_source(None)
        outs = net.output_blobs if test else []
        n_out = sum(int(b.count) for b in outs)
        acc = torch.zeros(max(1, n_out), dtype=torch.float32, device=dev)
        loss_buf = torch.zeros(1, dtype=torch.float32, device=dev)
        graph = torch.cuda.CUDAGraph()
        try:
            with torch.cuda.graph(graph):
                loss = net.forward()
                if torch.is_tensor(loss):
                    loss_buf.copy_(loss.reshape(1).float())
                if outs:
                    acc.add_(torch.cat([b.nchw().float().reshape(-1) for b in outs]))
        finally:
            for layer, src, _ in feeds:
                layer.set_source(src)
        # The eager forward of this call already updated the stateful layers (train-phase
        # BatchNorm running mean / variance / factor, Caffe updates them once per Forward):
        # the replay below must not update them a second time, so their parameter blobs are
        # saved and put back around it.
        saved = [(p.data, p.data.clone()) for p in self._stateful_params(net)]
        graph.replay()  # the blobs now hold a real forward of the staged batch (see above)
        for dst, src in saved:
            dst.copy_(src)
        torch.cuda.synchronize(dev)
        acc.zero_()
        self.__dict__.setdefault("_fwd_graphs", {})[bool(test)] = (graph, acc, loss_buf)
        if not test:
            self.__dict__.pop("_bwd_graph", None)  # it read the blobs this capture rebound
        return {"exec": int(graph.raw_cuda_graph_exec()),
                "stream": int(torch.cuda.current_stream(dev).cuda_stream),
                "loss_dev": int(loss_buf.data_ptr()), "acc_dev": int(acc.data_ptr()), "n_out": n_out,
                "feeds": [f for _, _, f in feeds], "blobs": [] if test else self.blob_table()}

    # -- native backward and activation blobs (sn_core.cpp NativeBackward, BlobDesc) -------------
    # sn_backward replays a captured backward of the train net: built right after the Python
    # verb ran a backward (on the blobs the train forward plan left bound to its graph
    # memory), replayed once (so the blob gradients hold a real backward of the staged batch)
    # with the flat gradient buffer restored afterwards (the eager call already accumulated
    # this pass: Caffe's Backward adds into the parameter diffs once per call).  The blob
    # table gives the native sn_blob_* verbs on activation blobs (layer < 0) each blob's
    # device data / gradient pointer, dtype and layout, read with hipMemcpy.
    def backward_plan(self) -> dict:
        net = self.net
        if self.device.type != "cuda" or False not in self.__dict__.get("_fwd_graphs", {}):
            raise RuntimeError("native backward needs the train forward plan")
        if net.ctx.stale_diffs:
            net.finish_param_diffs()
        dev = self.device
        torch.cuda.synchronize(dev)
        saved = net.flat_diff.clone()
        graph = torch.cuda.CUDAGraph()
        with _plain_backward(net):
            with torch.cuda.graph(graph):
                net.backward()
        graph.replay()
        net.flat_diff.copy_(saved)
        torch.cuda.synchronize(dev)
        self.__dict__["_bwd_graph"] = graph
        return {"exec": int(graph.raw_cuda_graph_exec()),
                "stream": int(torch.cuda.current_stream(dev).cuda_stream), "blobs": self.blob_table()}

    def blob_table(self) -> list:
        """(data ptr, diff ptr or 0, dtype (0 bf16, 1 fp32), NHWC image, ndim, dims[6]) per
        net blob, in blob order; blobs whose storage is not a plain contiguous bf16 / fp32
        device tensor get a null data pointer (they stay on the Python path)."""
        rows = []
        for b in self.net.blobs:
            d = b._data
            g = b._diff
            ok = d is not None and d.is_cuda and d.is_contiguous() and d.dtype in (torch.bfloat16, torch.float32)
            gok = ok and g is not None and g.is_cuda and g.is_contiguous() and g.dtype == d.dtype
            shape = tuple(int(x) for x in b.shape)
            rows.append((int(d.data_ptr()) if ok and len(shape) <= 6 else 0, int(g.data_ptr()) if gok else 0,
                         int(d.dtype == torch.float32) if ok else 0, int(b.is_image), len(shape))
                        + shape + (1,) * (6 - len(shape)))
        return rows

    def meta_plan(self) -> dict:
        """Names and counts the metadata verbs return (read once per loaded net)."""
        net = self.net
        return {"layers": list(net.layer_names), "weights": [len(l.params) for l in net.layers],
                "blobs": list(net.blob_names), "outputs": len(net.output_blobs)}

    def weights_plan(self) -> dict:
        """Flat fp32 master buffer (device or host memory) and its compute shadow for the
        native sn_get_weights / sn_set_weights (a hipMemcpy plus, on the GPU, the
        sn_cast_f32_bf16 refresh of the bf16 shadow that Net.sync_compute does)."""
        net = self.net
        data, comp = net.flat_data, net.flat_compute
        if data is None:
            raise RuntimeError("net has no parameters")
        shadow = comp is not None and comp is not data
        if shadow and (not data.is_cuda or comp.dtype != torch.bfloat16):
            raise RuntimeError("host nets with a separate compute copy stay on the Python path")
        return {"data": int(data.data_ptr()), "count": int(net.num_param_elems), "cuda": int(data.is_cuda),
                "compute": int(comp.data_ptr()) if shadow else 0, "compute_count": int(comp.numel()) if shadow else 0,
                "stream": int(torch.cuda.current_stream(self.device).cuda_stream) if data.is_cuda else 0,
                "diff": int(net.flat_diff.data_ptr()), "params": self._param_table(),
                "net_name": str(net.name or ""),
                "layers": [(str(l.name), str(l.type_name), len(l.params)) for l in net.layers]}

    def _param_table(self) -> list:
        """Per-parameter rows for the native sn_blob_* verbs on layer parameters:
        (layer, index, flat offset, count, layout, caffe ndim, caffe dims[6], internal dims[4]);
        layout 0 = the internal order is Caffe's, 1 = internal [K][R][S][C] holding Caffe's
        [K][C][R][S] (convolution weights).  Params with any other layout are left out and
        stay on the Python path."""
        net = self.net
        base = net.flat_data.data_ptr()
        rows = []
        for li, layer in enumerate(net.layers):
            for pi, prm in enumerate(layer.params):
                off = getattr(prm, "offset", None)
                cs = tuple(prm.caffe_shape)
                if off is None or len(cs) > 6 or prm.data is None or prm.data.data_ptr() != base + 4 * off:
                    continue
                layout = 0
                ishape = tuple(prm.shape) + (1,) * (4 - len(prm.shape)) if len(prm.shape) <= 4 else None
                if prm._to_caffe is not None:
                    # a 4-D [K][R][S][C] view of the internal tensor: the conv weight itself,
                    # or an InnerProduct weight over an NHWC image bottom (layer.perm = (C, H, W))
                    view = tuple(prm.shape) if len(prm.shape) == 4 else None
                    perm = getattr(layer, "perm", None)
                    if view is None and pi == 0 and perm is not None and len(prm.shape) == 2:
                        view = (prm.shape[0], perm[1], perm[2], perm[0])
                    if view is None or math.prod(view) != prm.count:
                        continue
                    probe = torch.arange(prm.count, dtype=torch.float64).reshape(prm.shape)
                    expect = probe.reshape(view).permute(0, 3, 1, 2).reshape(cs)
                    if not torch.equal(prm._to_caffe(probe).reshape(cs), expect):
                        continue
                    layout, ishape = 1, view
                if ishape is None:
                    continue
                rows.append((li, pi, int(off), int(prm.count), layout, len(cs)) + tuple(int(d) for d in cs)
                            + (1,) * (6 - len(cs)) + tuple(int(d) for d in ishape))
        return rows

    def set_scores(self, scores: list) -> None:
        """Scores of a native sn_solver_test, handed over at the next Python entry."""
        self.scores = [float(v) for v in scores]

    def test(self, n: int) -> int:
        """solver_test -> TestAndStoreResult (solver.cpp:413-444): one score per ELEMENT
        of every output blob (Caffe's NCHW element order), summed over n forwards;
        returns the number of scores."""
        net = self.test_net
        sums = None
        for _ in range(n):
            net.forward()
            v = torch.cat([b.nchw().float().reshape(-1) for b in net.output_blobs]) if net.output_blobs else None
            if v is not None:
                sums = v.clone() if sums is None else sums + v
        self.scores = [float(x) for x in sums.cpu()] if sums is not None else []
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
