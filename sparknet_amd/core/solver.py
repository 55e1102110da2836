"""Solvers: SGD (+ Nesterov, AdaGrad, RMSProp, AdaDelta, Adam) with Caffe semantics.

References: ``Solver`` (caffe/src/caffe/solver.cpp — Init :44-190, Step :193-282,
Test :338-411, TestAndStoreResult :413-444 (SparkNet-added), Snapshot :447-499,
Restore :510-519), ``SGDSolver`` (caffe/src/caffe/solvers/sgd_solver.cpp — GetLearningRate
:27-63, ClipGradients :81-99, ApplyUpdate :102-116, Normalize :119-142, Regularize
:145-204, ComputeUpdateValue :207-239, snapshot/restore :242-343) and the other solvers
in caffe/src/caffe/solvers/*.cpp.  The reference SparkNet shim always constructed an
SGDSolver (libccaffe/ccaffe.cpp:131); here the ``type`` field is honoured.

MI355X-first: the whole update — global-norm clip, 1/iter_size, L1/L2 decay with
per-param decay_mult, per-param lr_mult, momentum / adaptive history, the master write
and the bf16 shadow write — is ONE fused HIP kernel over the flat parameter buffer
(``csrc/kernels/solver.hip``).  Hyper-parameters live in a small device tensor so the
update can be replayed inside a captured hipGraph.
"""
from __future__ import annotations

import logging
import math
import os
import time
from typing import Callable

import numpy as np
import torch

from .. import proto
from .net import Net, blob_proto_to_tensor

log = logging.getLogger("sparknet_amd.solver")

SOLVER_KINDS = {"SGD": 0, "Nesterov": 1, "AdaGrad": 2, "RMSProp": 3, "AdaDelta": 4, "Adam": 5}
_LEGACY_TYPES = {0: "SGD", 1: "Nesterov", 2: "AdaGrad", 3: "RMSProp", 4: "AdaDelta", 5: "Adam"}
N_HISTORY = {"SGD": 1, "Nesterov": 1, "AdaGrad": 1, "RMSProp": 1, "AdaDelta": 2, "Adam": 2}

# hyper tensor layout (device, fp32)
H_LR, H_MOM, H_WD, H_CLIP, H_NORM, H_DELTA, H_MOM2, H_RMS, H_CORR, H_T = range(10)
N_HYPER = 16


class Solver:
    def __init__(self, param, *, device="cpu", dtype=None, seed: int | None = None,
                 train_net: Net | None = None, build_test_nets: bool = True):
        if isinstance(param, str):
            param = proto.read_solver(param)
        self.param = proto.copy(param)
        p = self.param
        self.type = p.type if p.HasField("type") else (
            _LEGACY_TYPES[int(p.solver_type)] if p.HasField("solver_type") else "SGD")
        if self.type not in SOLVER_KINDS:
            raise ValueError(f"Unknown solver type {self.type!r}")
        self.device = torch.device(device)
        if seed is None:
            seed = int(p.random_seed) if p.random_seed >= 0 else 1701
        self.seed = seed
        self.iter = 0
        self.current_step = 0
        self.callbacks: list = []
        self.action_request: Callable[[], str] | None = None
        self.requested_early_exit = False
        self.losses: list[torch.Tensor] = []
        self.smoothed_loss = 0.0
        self.net = train_net if train_net is not None else self._init_train_net(dtype)
        self.test_nets: list[Net] = []
        if build_test_nets:
            self._init_test_nets(dtype)
        self.history: list[torch.Tensor] = []
        self._init_state()

    # -- construction (Solver::InitTrainNet / InitTestNets) ------------------------------
    def _net_param_source(self):
        p = self.param
        n = int(p.HasField("train_net_param")) + int(p.HasField("train_net")) + \
            int(p.HasField("net_param")) + int(p.HasField("net"))
        if n != 1:
            raise ValueError("SolverParameter must specify exactly one of train_net_param, train_net, "
                             "net_param, net")
        if p.HasField("train_net_param"):
            return proto.copy(p.train_net_param)
        if p.HasField("train_net"):
            return proto.read_net(p.train_net)
        if p.HasField("net_param"):
            return proto.copy(p.net_param)
        return proto.read_net(p.net)

    def _init_train_net(self, dtype) -> Net:
        netp = self._net_param_source()
        state = proto.NetState(phase=proto.TRAIN)
        state.MergeFrom(netp.state)
        state.MergeFrom(self.param.train_state)
        netp.state.CopyFrom(state)
        return Net(netp, device=self.device, dtype=dtype, seed=self.seed)

    def _init_test_nets(self, dtype) -> None:
        p = self.param
        sources = []
        for tp in p.test_net_param:
            sources.append(proto.copy(tp))
        for tf in p.test_net:
            sources.append(proto.read_net(tf))
        remaining = len(p.test_iter) - len(sources)
        if remaining > 0:
            if p.HasField("net_param"):
                sources += [proto.copy(p.net_param)] * remaining
            elif p.HasField("net"):
                base = proto.read_net(p.net)
                sources += [base] * remaining
        if len(p.test_state) and len(p.test_state) != len(sources):
            raise ValueError("test_state must be unspecified or specified once per test net")
        for i, netp in enumerate(sources):
            netp = proto.copy(netp)
            state = proto.NetState(phase=proto.TEST)
            state.MergeFrom(netp.state)
            if len(p.test_state):
                state.MergeFrom(p.test_state[i])
            netp.state.CopyFrom(state)
            tn = Net(netp, device=self.device, dtype=self.net.dtype, seed=self.seed, allocate=True)
            tn.share_trained_layers_with(self.net)
            self.test_nets.append(tn)

    def _init_state(self) -> None:
        n = self.net.num_param_elems
        self.history = [torch.zeros(max(n, 1), dtype=torch.float32, device=self.device)
                        for _ in range(N_HISTORY[self.type])]
        self.hyper = torch.zeros(N_HYPER, dtype=torch.float32, device=self.device)
        self._hyper_staged: list | None = None
        self._build_tables()

    def _build_tables(self) -> None:
        """Chunk table for the fused update kernel: (start, count, lr_mult, decay_mult).
        Params updated inside their layer's backward (set_fused_update) are left out."""
        from .. import ops
        segs = self.net.param_segments()
        self.segments = segs
        fused = set(getattr(self, "fused_offsets", set()))
        for sink in getattr(self, "slab_sinks", ()):
            if sink.desc is not None:  # updated in backward from its split-K slabs
                fused.update(p.offset for p in sink.params())
        self._tables = ops.solver_tables([s for s in segs if s[0] not in fused], self.net.num_param_elems,
                                         self.device)
        self.slab_tables_dirty = False

    def set_slab_sinks(self, sinks) -> None:
        """Convolution weight gradients left as split-K slabs (engine.fuse_splitk_updates):
        the update tables are rebuilt whenever a layer's slab layout changes (first pass,
        a re-tuned split factor) — always before a graph capture."""
        self.slab_sinks = list(sinks)
        self.slab_tables_dirty = True
        if not getattr(self, "fused_offsets", None):
            self.fused_offsets = set()  # stage hyper-parameters before backward (Solver.iteration)

    def set_fused_update(self, offsets) -> None:
        """Declare params whose solver update runs in their layer's weight-gradient GEMM
        epilogue (engine.fuse_fc_updates); hyper-parameters are then staged before the
        forward pass, since that update reads them during backward."""
        self.fused_offsets = set(offsets)
        self._build_tables()

    # -- learning rate (SGDSolver::GetLearningRate) ------------------------------------
    def get_learning_rate(self) -> float:
        p = self.param
        pol = p.lr_policy
        it = self.iter
        if pol == "fixed":
            return p.base_lr
        if pol == "step":
            self.current_step = it // p.stepsize
            return p.base_lr * math.pow(p.gamma, self.current_step)
        if pol == "exp":
            return p.base_lr * math.pow(p.gamma, it)
        if pol == "inv":
            return p.base_lr * math.pow(1.0 + p.gamma * it, -p.power)
        if pol == "multistep":
            if self.current_step < len(p.stepvalue) and it >= p.stepvalue[self.current_step]:
                self.current_step += 1
            return p.base_lr * math.pow(p.gamma, self.current_step)
        if pol == "poly":
            return p.base_lr * math.pow(1.0 - float(it) / float(p.max_iter), p.power)
        if pol == "sigmoid":
            return p.base_lr * (1.0 / (1.0 + math.exp(-p.gamma * (float(it) - float(p.stepsize)))))
        raise ValueError(f"Unknown learning rate policy: {pol!r}")

    def hyper_values(self, rate: float) -> list[float]:
        p = self.param
        h = [0.0] * N_HYPER
        h[H_LR] = rate
        h[H_MOM] = p.momentum
        h[H_WD] = p.weight_decay
        h[H_CLIP] = p.clip_gradients
        h[H_NORM] = 1.0 / max(1, p.iter_size)
        h[H_DELTA] = p.delta
        h[H_MOM2] = p.momentum2
        h[H_RMS] = p.rms_decay
        t = self.iter + 1
        if self.type == "Adam":
            h[H_CORR] = math.sqrt(1.0 - math.pow(p.momentum2, t)) / (1.0 - math.pow(p.momentum, t))
        h[H_T] = float(t)
        return h

    def stage_hyper(self, rate: float | None = None) -> float:
        """Write this iteration's hyper-parameters into the device tensor (async H2D)."""
        rate = self.get_learning_rate() if rate is None else rate
        vals = self.hyper_values(rate)
        vals[H_T] = 0.0  # host-side only (Adam's correction is folded into H_CORR)
        if vals == self._hyper_staged:  # unchanged (fixed / step policies): no copy at all
            return rate
        self._hyper_staged = vals
        # a fresh pinned buffer per change: a host write never races an H2D still queued
        host = torch.tensor(vals, dtype=torch.float32)
        if self.device.type == "cuda":
            host = host.pin_memory()
        self.hyper.copy_(host, non_blocking=True)
        return rate

    # -- update (ApplyUpdate) -------------------------------------------------------------
    def apply_update(self) -> float:
        rate = self.stage_hyper()
        if self.param.display and self.iter % self.param.display == 0:
            log.info("Iteration %d, lr = %g", self.iter, rate)
        self.update_params()
        return rate

    # -- overlapped update (graph path) ---------------------------------------------------
    def overlap_eligible(self) -> bool:
        """Per-layer updates may run while backward continues only when every update is
        local to its own parameters: no gradient clipping (global norm), no gradient
        accumulation over iter_size passes, no gradient callbacks (sync-SGD all-reduce)."""
        return (self.device.type == "cuda" and self.param.clip_gradients <= 0 and self.param.iter_size <= 1
                and not self.callbacks)

    def overlap_plan(self, min_group: int = 1) -> tuple[dict, list]:
        """({layer index: [segments]}, late segments): a param's segment joins the group of
        the LAST layer (in backward order) that writes its gradient; params whose gradient
        is not written by backward (frozen / pruned) are updated after the pass."""
        net = self.net
        seg_of = {seg[0]: seg for seg in self.segments}
        final, late = {}, set()
        for li, layer in enumerate(net.layers):
            for i, p in enumerate(layer.params):
                if p.offset not in seg_of:
                    continue
                if not net.layer_need_backward[li] or not layer.param_grads_needed(i):
                    late.add(p.offset)
                final[p.offset] = min(final.get(p.offset, li), li)
        groups: dict = {}
        for off, li in final.items():
            if off not in late:
                groups.setdefault(li, []).append(seg_of[off])
        # only large groups are worth a fork/join on the side stream (each costs ~10 us of
        # graph synchronisation); the rest are updated after the backward pass
        big = {li: segs for li, segs in groups.items() if sum(sg[1] for sg in segs) >= min_group}
        rest = [seg_of[o] for o in seg_of if not any(o == sg[0] for segs in big.values() for sg in segs)]
        return big, rest

    def update_params_segments(self, tables, grid_limit: int = 0) -> None:
        from .. import ops
        net = self.net
        ops.solver_update(SOLVER_KINDS[self.type], net.flat_data, net.flat_diff, self.history,
                          net.flat_compute if net.flat_compute is not net.flat_data else None,
                          tables, self.hyper, self.param.regularization_type == "L1", False, grid_limit)

    def update_params(self) -> None:
        from .. import ops
        l1 = self.param.regularization_type == "L1"
        if self.param.regularization_type not in ("L1", "L2"):
            raise ValueError(f"Unknown regularization type: {self.param.regularization_type}")
        net = self.net
        if getattr(self, "slab_tables_dirty", False):
            assert not torch.cuda.is_current_stream_capturing(), "split-K slab layout changed during capture"
            self._build_tables()
        ops.solver_update(SOLVER_KINDS[self.type], net.flat_data, net.flat_diff, self.history,
                          net.flat_compute if net.flat_compute is not net.flat_data else None,
                          self._tables, self.hyper, l1, self.param.clip_gradients > 0)

    # -- main loop (Solver::Step) -----------------------------------------------------------
    def iteration(self):
        """One training iteration minus bookkeeping: returns the device loss."""
        net = self.net
        if getattr(self, "fused_offsets", None) or getattr(self, "slab_sinks", None):
            self.stage_hyper()  # the in-backward (fused) updates read this iteration's rate
        net.clear_param_diffs(lazy=True)
        for cb in self.callbacks:
            getattr(cb, "on_start", lambda: None)()
        loss = None
        for _ in range(max(1, self.param.iter_size)):
            l = net.forward_backward()
            loss = l if loss is None else loss + l
            from .. import ops
            ops.advance_rng(net.ctx.rng_state)
        net.finish_param_diffs()
        if getattr(net.ctx, "fp8", None) is not None:
            net.ctx.fp8.update()
        if self.param.iter_size > 1:
            loss = loss / self.param.iter_size
        for cb in self.callbacks:
            getattr(cb, "on_gradients_ready", lambda: None)()
        self.apply_update()
        return loss

    def step(self, iters: int) -> None:
        start_iter = self.iter
        stop_iter = self.iter + iters
        avg = max(1, self.param.average_loss)
        while self.iter < stop_iter:
            loss = self.iteration()
            self.losses.append(loss.detach())
            if len(self.losses) > avg:
                self.losses.pop(0)
            display = self.param.display and self.iter % self.param.display == 0
            self.iter += 1
            if display:
                self.smoothed_loss = float(torch.stack(self.losses).mean())
                log.info("Iteration %d, loss = %g", self.iter - 1, self.smoothed_loss)
            if self.param.snapshot and self.iter % self.param.snapshot == 0:
                self.snapshot()
            req = self.action_request() if self.action_request else "none"
            if req == "snapshot":
                self.snapshot()
            elif req == "stop":
                self.requested_early_exit = True
                break
        del start_iter

    def solve(self, resume_file: str | None = None) -> None:
        """Solver::Solve: run to max_iter with periodic testing."""
        if resume_file:
            self.restore(resume_file)
        p = self.param
        self.requested_early_exit = False
        while self.iter < p.max_iter and not self.requested_early_exit:
            if p.test_interval and self.iter % p.test_interval == 0 and (self.iter > 0 or p.test_initialization):
                self.test_all()
            n = p.max_iter - self.iter
            if p.test_interval:
                n = min(n, p.test_interval - self.iter % p.test_interval)
            self.step(n)
        if p.snapshot_after_train and (not p.snapshot or self.iter % p.snapshot != 0):
            self.snapshot()
        if self.requested_early_exit:  # solver.cpp:300-310: no final pass after a stop request
            log.info("Optimization stopped early.")
            return
        # solver.cpp:317-324: final forward-only loss display, then test on test_interval
        if p.display and self.iter % p.display == 0:
            loss = self.net.forward()
            log.info("Iteration %d, loss = %g", self.iter, float(loss))
        if p.test_interval and self.iter % p.test_interval == 0:
            self.test_all()

    # -- testing ------------------------------------------------------------------------------
    def test(self, test_net_id: int = 0, iters: int | None = None) -> list[float]:
        """Solver::Test — mean of every output blob over ``test_iter`` batches."""
        scores = self.test_and_store_result(test_net_id, iters)
        n = iters if iters is not None else self.param.test_iter[test_net_id]
        res = [s / max(n, 1) for s in scores]
        tn = self.test_nets[test_net_id]
        names = [b.name for b in tn.output_blobs]
        for name, v in zip(names, res):
            log.info("    Test net output #%s: %s = %g", test_net_id, name, v)
        return res

    def test_and_store_result(self, test_net_id: int = 0, iters: int | None = None) -> list[float]:
        """SparkNet's Solver::TestAndStoreResult (solver.cpp:413-444): per-output SUM over
        ``iters`` forward passes of the test net (weights shared with the train net)."""
        tn = self.test_nets[test_net_id]
        n = iters if iters is not None else self.param.test_iter[test_net_id]
        acc = None
        for _ in range(n):
            tn.forward()
            vals = torch.stack([b.data.float().sum() for b in tn.output_blobs])
            acc = vals if acc is None else acc + vals
        return [] if acc is None else acc.cpu().tolist()

    def test_all(self) -> list[list[float]]:
        return [self.test(i) for i in range(len(self.test_nets))]

    # -- snapshot / restore -----------------------------------------------------------------
    def _prefix(self) -> str:
        return self.param.snapshot_prefix or "snapshot"

    def snapshot(self, prefix: str | None = None) -> tuple[str, str]:
        """Solver::Snapshot (solver.cpp:447-500): binaryproto pair by default, or
        ``.caffemodel.h5`` / ``.solverstate.h5`` with ``snapshot_format: HDF5``."""
        prefix = prefix or self._prefix()
        h5 = self.param.HasField("snapshot_format") and self.param.snapshot_format == 0
        ext = ".h5" if h5 else ""
        model = f"{prefix}_iter_{self.iter}.caffemodel{ext}"
        state = f"{prefix}_iter_{self.iter}.solverstate{ext}"
        d = os.path.dirname(model)
        if d:
            os.makedirs(d, exist_ok=True)
        if h5:
            self.net.to_hdf5(model, write_diff=self.param.snapshot_diff)
            self._state_to_hdf5(state, model)
        else:
            from ..utils.checkpoint import save_caffemodel
            save_caffemodel(self.net, model, write_diff=self.param.snapshot_diff)
            proto.write_binary(state, self.solver_state(model))
        log.info("Snapshotting to %s / %s", model, state)
        return model, state

    def _history_blobs(self):
        """history_ in Caffe order and layout: one blob per (history slot, param)."""
        for h in self.history:
            for prm in self.net.learnable_params:
                yield prm, h[prm.offset:prm.offset + prm.count].view(prm.shape)

    def _state_to_hdf5(self, path: str, learned_net: str) -> None:
        """SGDSolver::SnapshotSolverStateToHDF5 (sgd_solver.cpp:277-298)."""
        from ..utils import hdf5
        hist = {str(i): prm.to_caffe(seg).float().cpu().numpy()
                for i, (prm, seg) in enumerate(self._history_blobs())}
        hdf5.write(path, {"iter": np.array([self.iter], np.int32), "learned_net": learned_net,
                          "current_step": np.array([self.current_step], np.int32), "history": hist})

    def solver_state(self, learned_net: str = ""):
        st = proto.SolverState(iter=self.iter, learned_net=learned_net, current_step=self.current_step)
        for prm, seg in self._history_blobs():
            bp = st.history.add()
            bp.shape.dim.extend(prm.caffe_shape)
            bp.data.extend(prm.to_caffe(seg).cpu().reshape(-1).tolist())
        return st

    def restore(self, state_file: str) -> None:
        """Solver::Restore (solver.cpp:509-518): ``.h5`` selects the HDF5 reader."""
        if state_file.endswith(".h5"):
            from ..utils import hdf5
            f = hdf5.File(state_file)
            self.iter = hdf5.read_int(f["iter"])
            learned = hdf5.read_string(f["learned_net"]) if "learned_net" in f else ""
            self.current_step = hdf5.read_int(f["current_step"])
            hist = f["history"]
            blobs = [torch.from_numpy(hist[str(i)].read().astype(np.float32)) for i in range(len(hist))]
        else:
            st = proto.read_binary(state_file, proto.SolverState)
            self.iter, self.current_step, learned = st.iter, st.current_step, st.learned_net
            blobs = [blob_proto_to_tensor(b) for b in st.history]
        if learned:
            self.net.copy_trained_layers_from(learned)
        slots = list(self._history_blobs())
        if len(blobs) != len(slots):
            raise ValueError("Incorrect length of history blobs.")
        for (prm, seg), t in zip(slots, blobs):
            seg.copy_(prm.from_caffe(t).to(seg.device))
        log.info("Restored solver state from %s (iter %d)", state_file, self.iter)

    # -- SparkNet-facing helpers --------------------------------------------------------------
    def add_callback(self, cb) -> None:
        self.callbacks.append(cb)


def create_solver(param, **kw) -> Solver:
    """SolverRegistry::CreateSolver (solver_factory.hpp): one class, kind from ``type``."""
    return Solver(param, **kw)


def timed(fn):
    def wrap(*a, **k):
        t = time.perf_counter()
        r = fn(*a, **k)
        return r, time.perf_counter() - t
    return wrap
