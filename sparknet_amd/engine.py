"""Execution engine: graph-captured solver iterations and SparkNet's round structure.

* :class:`GraphStep` captures ONE full training iteration (gradient memset, forward,
  backward, Philox advance, fused solver update) into a hipGraph via
  ``torch.cuda.CUDAGraph`` and replays it; per-iteration hyper-parameters (learning
  rate, Adam correction) are staged into a device tensor with one async H2D copy before
  each replay.  This removes the Python/launch overhead of ~100 kernels per iteration
  (the reference instead paid a host sync for every loss scalar).
* :class:`LocalSGDTrainer` runs SparkNet's algorithm (src/main/scala/apps/CifarApp.scala:
  95-136, ImageNetApp.scala:106-189) on one process per GPU: every rank runs tau local
  solver steps on its own data shard, then the flat fp32 weights are averaged with an
  RCCL all-reduce (:mod:`sparknet_amd.parallel.comm`) — the Spark driver's
  broadcast / collect / reduce / divide loop collapsed into one collective.
"""
from __future__ import annotations

import gc
import logging
import os
import time

import torch

from . import ops
from .core.solver import Solver
from .utils import features
from .utils.trace import trace_range

from .ops.spec import ConvSpec

log = logging.getLogger("sparknet_amd.engine")


def fuse_relu(net) -> int:
    """Fold in-place ReLU (slope 0) into the producing Convolution / InnerProduct
    epilogue.  Returns the number of fused pairs.  The ReLU layer keeps its backward.
    fp32 nets on the GPU (the fp32 device mode, ops.f32dev) run the plain layer graph."""
    if net.device.type == "cuda" and net.dtype == torch.float32:
        return 0
    n = 0
    for li in range(1, len(net.layers)):
        relu = net.layers[li]
        prod = net.layers[li - 1]
        if relu.type_name != "ReLU" or getattr(relu, "slope", 1.0) != 0.0:
            continue
        if net.bottom_ids[li] != net.top_ids[li]:
            continue
        if prod.type_name not in ("Convolution", "InnerProduct") or len(net.top_ids[li - 1]) != 1:
            continue
        if net.top_ids[li - 1][0] != net.bottom_ids[li][0]:
            continue
        prod.fuse_relu = True
        relu.fused = True
        n += 1
    fuse_relu_backward(net)
    fuse_dropout(net)
    fuse_concat(net)
    fuse_pool_lrn(net)
    fuse_lrn_pool_backward(net)
    batch_weight_flips(net)
    return n


def fuse_pool_lrn(net) -> int:
    """Run a cross-channel LRN that reads a 3x3 / stride-2 max pooling's output inside the
    pooling layer's kernels (csrc/kernels/pool_lrn.hip): CaffeNet's pool1 -> norm1 and
    pool2 -> norm2, GoogLeNet's pool1 -> norm1.  Caffe runs them as two layers with two
    passes each way (pooling_layer.cu:11-47,217-260, lrn_layer.cu:9-177); fused, the LRN
    normalises the pooled tile out of LDS, and in backward the pooled gradient is built in
    LDS and gathered straight into the pooling input gradient.  Requires the pooled blob to
    be read by the LRN alone (not a net output, no in-place LRN).  Returns the count."""
    from .ops import hip
    if net.device.type != "cuda" or net.debug_info or not features.enabled("fuse_pool_lrn"):
        return 0
    outputs = set(getattr(net, "output_blob_ids", ()))
    n = 0
    for li, pool in enumerate(net.layers):
        if pool.type_name != "Pooling" or len(net.top_ids[li]) != 1 or pool.global_pooling:
            continue
        blob = net.top_ids[li][0]
        readers = [lj for lj in range(li + 1, len(net.layers)) if blob in net.bottom_ids[lj]]
        if blob in outputs or len(readers) != 1:
            continue
        lj = readers[0]
        lrn = net.layers[lj]
        if lrn.type_name != "LRN" or lrn.relu_gate or net.top_ids[lj][0] == blob:
            continue
        if net.layer_need_backward[li] != net.layer_need_backward[lj]:
            continue
        s = pool.spec(net.bottom_vecs[li][0])
        if not hip.pool_lrn_eligible(s, lrn.size, lrn.within):
            continue
        lrn.pool_fused = True
        lrn.top = net.top_vecs[lj][0]
        pool.fused_lrn = lrn
        n += 1
    return n


def fuse_lrn_pool_backward(net) -> int:
    """The other order: a cross-channel LRN whose output only a 3x3 / stride-2 max pooling
    reads (AlexNet's norm1 -> pool1 and norm2 -> pool2, GoogLeNet's conv2/norm2 -> pool2).
    Backward only: the pooling layer's backward computes the LRN INPUT gradient in one launch
    (csrc/kernels/pool_lrn.hip: pool_lrn_bwd_rev, bitwise equal to the two kernels) and the
    LRN layer's backward is skipped.  Caffe runs the two backwards as separate passes
    (pooling_layer.cu:217-260, lrn_layer.cu:121-177).  The forward stays two launches.
    Returns the count."""
    from .ops import hip
    if net.device.type != "cuda" or net.debug_info or not features.enabled("fuse_lrn_pool_bwd"):
        return 0
    outputs = set(getattr(net, "output_blob_ids", ()))
    n = 0
    for lj, lrn in enumerate(net.layers):
        if lrn.type_name != "LRN" or lrn.pool_fused or lrn.within or len(net.top_ids[lj]) != 1:
            continue
        blob = net.top_ids[lj][0]
        if blob in outputs or blob == net.bottom_ids[lj][0]:
            continue
        readers = [li for li in range(lj + 1, len(net.layers)) if blob in net.bottom_ids[li]]
        if len(readers) != 1:
            continue
        li = readers[0]
        pool = net.layers[li]
        if (pool.type_name != "Pooling" or len(net.top_ids[li]) != 1 or pool.global_pooling
                or pool.fused_lrn is not None or pool.relu_gate or net.top_ids[li][0] == blob):
            continue
        if not (net.layer_need_backward[li] and net.layer_need_backward[lj] and net.bottom_need_backward[li][0]
                and net.bottom_need_backward[lj][0]):
            continue
        s = pool.spec(net.bottom_vecs[li][0])
        if not hip.pool_lrn_rev_eligible(s, lrn.size, lrn.within):
            continue
        pool.bwd_lrn = lrn
        lrn.bottom = net.bottom_vecs[lj][0]
        # BranchStreams: the pooling backward now reads the LRN input and writes its gradient
        bid = net.bottom_ids[lj][0]
        ex = dict(getattr(pool, "sched_extra", None) or {})
        ex["bwd_r"] = set(ex.get("bwd_r", ())) | {("v", bid)}
        ex["bwd_w"] = set(ex.get("bwd_w", ())) | {("d", bid)}
        pool.sched_extra = ex
        n += 1
    return n


def _gating_consumers(net, blob: int, after: int):
    """Layers that would gate the gradient of ``blob`` with its own data if the ReLU
    backward of ``blob`` were moved into them — every reader after layer ``after``,
    following Split fan-outs — or None if some reader cannot (in-place readers, layers
    without a fused gate, net outputs)."""
    if blob in getattr(net, "output_blob_ids", ()):
        return None
    out = []
    for lj in range(after + 1, len(net.layers)):
        if blob not in net.bottom_ids[lj]:
            continue
        lay = net.layers[lj]
        if blob in net.top_ids[lj] or not net.layer_need_backward[lj]:
            return None
        if lay.type_name == "Split":
            for t in net.top_ids[lj]:
                sub = _gating_consumers(net, t, lj)
                if sub is None:
                    return None
                out += sub
            continue
        if lay.type_name not in _GATE_CONSUMERS or len(net.bottom_ids[lj]) != 1 or getattr(lay, "relu_gate", False):
            return None
        if lay.type_name == "Pooling" and (lay.method not in (0, 1) or len(net.top_ids[lj]) != 1):
            return None
        if lay.type_name in ("InnerProduct", "Dropout"):
            return None  # their gate doubles as the fused-dropout channel (fuse_dropout)
        out.append(lj)
    return out


def fuse_concat(net) -> int:
    """Zero-copy channel Concat (GoogLeNet Inception outputs).  Caffe copies every part
    into the output (concat_layer.cu:9-25) and back out in backward.  Here, when every
    part is produced by an ungrouped implicit-GEMM Convolution whose only other reader is
    its fused in-place ReLU, the convolutions write their GEMM output straight into the
    part's channel slice of one NHWC buffer (ldc = the concat width) and the Concat
    forward is free.  If, in addition, every reader of the concat output (through Split
    fan-outs: the next module's convolutions and max-pool, the stage pools, the loss-branch
    average pools) can apply a ReLU gate, the parts' ReLU backward moves into them (each
    part is a ReLU output, so the concat output is its own gate) and the Concat backward
    hands each part a channel-slice view of the output gradient, which the producing
    convolution's wgrad / dgrad GEMMs read in place.  GPU only; returns the count."""
    if net.device.type != "cuda" or not features.enabled("zero_copy_concat"):
        return 0
    from .layers.common import ConcatSlots
    from .ops import hip
    n = 0
    outputs = set(getattr(net, "output_blob_ids", ()))
    for lc, cat in enumerate(net.layers):
        if cat.type_name != "Concat" or len(net.bottom_ids[lc]) < 2 or cat.zero_copy is not None:
            continue
        bots = net.bottom_ids[lc]
        if len(set(bots)) != len(bots) or len(net.bottom_vecs[lc][0].shape) != 4:
            continue
        if cat.axis != 1:
            continue
        prods = []
        for bid in bots:
            writers = [lj for lj in range(lc) if bid in net.top_ids[lj]]
            readers = [lj for lj in range(len(net.layers)) if bid in net.bottom_ids[lj] and lj != lc]
            if not writers or bid in outputs:
                break
            prod = net.layers[writers[0]]
            inplace_ok = all(net.layers[lj].type_name == "ReLU" and getattr(net.layers[lj], "fused", False)
                             and net.top_ids[lj] == [bid] and net.bottom_ids[lj] == [bid] for lj in readers)
            if (not inplace_ok or set(writers[1:]) != set(readers) or prod.type_name != "Convolution"
                    or len(net.top_ids[writers[0]]) != 1 or prod.concat_slot is not None
                    or prod.fp8_slots is not None or prod.folded_input is not None):
                break
            s = prod.spec(net.bottom_vecs[writers[0]][0])
            if not hip._slice_ok(s) or hip._s2d_plan(s) is not None:
                break
            prods.append((prod, s.K))
        if len(prods) != len(bots):
            continue
        slots = ConcatSlots([k for _, k in prods])
        for part, (prod, _) in enumerate(prods):
            prod.concat_slot = (slots, part)
        cat.zero_copy = slots
        gated = _gating_consumers(net, net.top_ids[lc][0], lc)
        if gated is not None and cat.relu_gate_parts == frozenset(range(len(bots))):
            for lj in gated:
                net.layers[lj].relu_gate = True
            cat.relu_gate_parts = frozenset()
            cat.zero_copy_bwd = True
        n += 1
    return n


def fuse_dropout(net) -> int:
    """Apply an in-place TRAIN-phase Dropout inside the producing InnerProduct's epilogue
    (after its fused bias + ReLU: CaffeNet fc6 -> relu6 -> drop6, fc7 -> relu7 -> drop7),
    and its backward inside the consumer InnerProduct's dgrad epilogue: with the ReLU
    backward already folded into the dropout (fuse_relu_backward), d(pre-activation) =
    dy / (1-p) where the dropout output is > 0, else 0 — exactly Caffe's ReLU-after-in-place-
    dropout gate (relu_layer.cu reads the overwritten bottom) times dropout_layer.cu's
    mask * scale.  Both standalone dropout passes disappear.  GPU only; returns the count."""
    if net.device.type != "cuda" or not features.enabled("fuse_dropout"):
        return 0
    n = 0
    for li in range(1, len(net.layers)):
        d = net.layers[li]
        if d.type_name != "Dropout" or d.phase != 0 or not (d.ratio > 0) or d.fused_into is not None:
            continue
        if net.bottom_ids[li] != net.top_ids[li] or not getattr(d, "relu_gate", False):
            continue
        blob = net.top_ids[li][0]
        # the producer: the InnerProduct whose fused-ReLU output this is (the ReLU in between is fused)
        prods = [lj for lj in range(li) if blob in net.top_ids[lj]]
        lp = next((lj for lj in reversed(prods) if net.layers[lj].type_name == "InnerProduct"), None)
        if lp is None or not getattr(net.layers[lp], "fuse_relu", False):
            continue
        between = [net.layers[lj] for lj in prods if lj > lp]
        if any(not (l.type_name == "ReLU" and getattr(l, "fused", False)) for l in between):
            continue
        consumers = [lj for lj in range(li + 1, len(net.layers)) if blob in net.bottom_ids[lj]]
        if len(consumers) != 1 or blob in getattr(net, "output_blob_ids", ()):
            continue
        lc = consumers[0]
        cons = net.layers[lc]
        if cons.type_name != "InnerProduct" or len(net.bottom_ids[lc]) != 1 or blob in net.top_ids[lc]:
            continue
        prod = net.layers[lp]
        if prod.fused_dropout is not None:
            continue
        prod.fused_dropout = d
        d.fused_into = prod
        cons.relu_gate = True
        cons.gate_scale = 1.0 / (1.0 - d.ratio)
        n += 1
    return n


def batch_weight_flips(net) -> int:
    """Flip-transpose the dgrad weights of every stride-1 convolution in ONE launch at
    the start of backward (ops.hip.FlipBatch) instead of one flip launch per layer inside
    its backward.  GPU only; idempotent; returns the number of layers covered."""
    if net.device.type != "cuda" or getattr(net, "_flip_batch", None) is not None:
        return 0
    from .ops import hip
    items = []
    for li, layer in enumerate(net.layers):
        if layer.type_name != "Convolution" or not net.layer_need_backward[li]:
            continue
        if not any(net.bottom_need_backward[li]):
            continue
        specs = [layer.spec(b) for b in net.bottom_vecs[li]]
        if not all(hip.dgrad_uses_flip(s) for s in specs):
            continue
        s = specs[0]
        wt = torch.empty((s.groups, s.Cg, s.R, s.S, s.Kg), dtype=torch.bfloat16, device=net.device)
        items.append((layer.weight.compute, wt, s.groups, s.Kg, s.R, s.S, s.Cg))
        layer.flipped_weights = wt
    if not items:
        return 0
    net._flip_batch = hip.FlipBatch(items, net.device)
    net.pre_backward_hooks.append(net._flip_batch.run)
    return len(items)


_GATE_CONSUMERS = ("Convolution", "InnerProduct", "Dropout", "Pooling", "LRN")


def fuse_relu_backward(net) -> int:
    """Fold the backward of every in-place slope-0 ReLU into the backward of the single
    layer that consumes its output (Caffe's ReLU backward is a separate pass over the
    gradient, relu_layer.cu:24-41): conv / inner-product dgrad epilogues, the dropout
    kernel, the max-pool argmax mask, the LRN backward and the channel-concat backward (Inception outputs)
    then zero the gradient where the ReLU output is not positive, and the ReLU layer's
    own backward becomes a no-op.  Returns the count."""
    n = 0
    for li, relu in enumerate(net.layers):
        if relu.type_name != "ReLU" or getattr(relu, "slope", 1.0) != 0.0:
            continue
        if net.bottom_ids[li] != net.top_ids[li]:
            continue
        blob = net.top_ids[li][0]
        consumers = [lj for lj in range(li + 1, len(net.layers)) if blob in net.bottom_ids[lj]]
        if not consumers:
            continue
        lc = consumers[0]
        # later readers are fine only behind an in-place consumer (e.g. relu6 -> drop6 ->
        # fc7 all on blob "fc6"): they read the consumer's output, not the ReLU's
        if len(consumers) > 1 and blob not in net.top_ids[lc]:
            continue
        cons = net.layers[lc]
        if cons.type_name == "Concat" and len(net.bottom_ids[lc]) > 1 and blob not in net.top_ids[lc] \
                and blob not in getattr(net, "output_blob_ids", ()):
            # concat backward slices the gradient per bottom: the mask is applied while slicing
            pos = {i for i, b in enumerate(net.bottom_ids[lc]) if b == blob}
            cons.relu_gate_parts = frozenset(cons.relu_gate_parts | pos)
            relu.bwd_fused = True
            n += 1
            continue
        if cons.type_name not in _GATE_CONSUMERS or len(net.bottom_ids[lc]) != 1:
            continue
        if cons.type_name == "Pooling" and (cons.method != 0 or len(net.top_ids[lc]) != 1):
            continue
        if blob in getattr(net, "output_blob_ids", ()):
            continue
        cons.relu_gate = True
        relu.bwd_fused = True
        n += 1
    return n


class _FusedFCUpdate:
    """The solver state an InnerProduct layer needs to apply its weight update in the
    wgrad GEMM epilogue (resolved at call time, so re-allocated buffers are followed)."""

    def __init__(self, solver, param, flags: int):
        self.solver, self.p, self.flags = solver, param, flags

    def sgd(self) -> dict:
        p = self.p
        h = self.solver.history[0][p.offset:p.offset + p.count].view(p.data.shape)
        return {"w": p.data, "h": h, "shadow": p.compute, "hyper": self.solver.hyper, "lr_mult": p.lr_mult,
                "decay_mult": p.decay_mult, "flags": self.flags}


def fuse_fc_updates(solver) -> int:
    """Apply the SGD / Nesterov update of InnerProduct weights inside their weight-gradient
    GEMM (EPI_SGD epilogue): the gradient is consumed where it is produced instead of
    being written to the flat gradient buffer and read back by the solver kernel
    (CaffeNet: 58.6 M of 61 M parameters, 8 B/param of HBM traffic saved).  Caffe applies
    the update after the whole backward pass (solver.cpp:237-240); per parameter the
    arithmetic is identical.  Requires what OverlappedUpdate requires (no clipping, no
    iter_size accumulation, no gradient callbacks) plus unshared weights with channel
    counts % 8 == 0.  Returns the number of fused layers."""
    net = solver.net
    if net.device.type != "cuda" or not solver.overlap_eligible() or solver.type not in ("SGD", "Nesterov"):
        return 0
    if net.flat_compute is net.flat_data or solver.param.regularization_type not in ("L1", "L2"):
        return 0
    users: dict = {}
    for layer in net.layers:
        for p in layer.params:
            users[p.offset] = users.get(p.offset, 0) + 1
    flags = (1 if solver.type == "Nesterov" else 0) | (2 if solver.param.regularization_type == "L1" else 0)
    offsets = []
    for li, layer in enumerate(net.layers):
        if layer.type_name != "InnerProduct" or not net.layer_need_backward[li] or not layer.param_grads_needed(0):
            continue
        p = layer.weight
        if p.owner is not None or users.get(p.offset, 0) != 1 or layer.N % 8 or layer.Kdim % 8:
            continue
        layer.fused_update = _FusedFCUpdate(solver, p, flags)
        offsets.append(p.offset)
    if offsets:
        solver.set_fused_update(offsets)
    return len(offsets)


class _SlabGrad:
    """Split-K slabs of one Convolution's weight gradient (and its bias column) left for
    the solver: the update kernel sums them in split order per parameter (solver.hip
    chunk_grad) instead of a splitk_reduce launch writing the flat gradient buffer and the
    solver reading it back.  The slab buffer is persistent (allocated on the first pass,
    before any graph capture) so the captured update reads the slabs at a fixed address."""

    def __init__(self, solver, layer):
        self.solver, self.layer = solver, layer
        self.buf = None
        self.desc = None
        self.key = None
        self.got = False
        self.table = None

    # gemm.defer_reduce protocol
    def begin(self):
        self.got = False

    def end(self):
        if not self.got:
            self._set(None)

    def accepts(self, out, bias_grad) -> bool:
        ok = out.data_ptr() == self.layer.weight.diff.data_ptr()
        if ok and bias_grad is not None:
            ok = self.layer.bias is not None and bias_grad.data_ptr() == self.layer.bias.diff.data_ptr()
        return ok

    def slab(self, numel: int, device):
        if self.buf is None or self.buf.numel() < numel:
            assert not torch.cuda.is_current_stream_capturing(), "split-K slab buffer grown during capture"
            self.buf = torch.empty(numel, dtype=torch.float32, device=device)
        return self.buf[:numel]

    def record(self, d):
        self.got = True
        self._set(d)

    def _set(self, d):
        key = None if d is None else (d["ws"].data_ptr(), d["splits"], d["M"], d["N"], d["ldw"], d["groups"],
                                      d["ones"], d["ldc"], d["c_gstride"])
        if key != self.key:
            assert not torch.cuda.is_current_stream_capturing(), "split-K slab layout changed during capture"
            self.key, self.desc = key, d
            self.solver.slab_tables_dirty = True
            self.table = None
            if d is not None:
                from . import ops
                mine = {p.offset for p in self.params()}
                segs = [sg for sg in self.solver.net.param_segments() if sg[0] in mine]
                self.table = ops.solver_tables(segs, self.solver.net.num_param_elems, self.solver.device,
                                               self.chunks())

    def params(self):
        return [self.layer.weight] + ([self.layer.bias] if self.layer.bias is not None else [])

    def apply(self) -> None:
        """The layer's solver update, right after its backward (its data gradient has read
        the old weights): on the layer's own stream, so Inception towers overlap it."""
        if self.table is not None:
            self.solver.update_params_segments(self.table)

    def chunks(self) -> dict:
        """{param offset: [(flat start, count, slab address, slab stride, splits, element
        stride)]}: one chunk per weight row (g, m) — contiguous (tap, channel) columns of
        slab row m of group g — and one strided chunk per group for the bias column."""
        d = self.desc
        if d is None:
            return {}
        M, N, ldw, G, S = d["M"], d["N"], d["ldw"], d["groups"], d["splits"]
        assert d["ldc"] == N and d["c_gstride"] == M * N, "weight gradient must be the dense [K][RS*Cg] layout"
        base, ss, gs = d["ws"].data_ptr(), M * ldw, S * M * ldw
        wp = self.layer.weight
        out = {wp.offset: [(wp.offset + (g * M + m) * N, N, base + 4 * (g * gs + m * ldw), ss, S, 1)
                           for g in range(G) for m in range(M)]}
        bp = self.layer.bias
        if d["ones"] >= 0 and bp is not None:
            out[bp.offset] = [(bp.offset + g * M, M, base + 4 * (g * gs + d["ones"]), ss, S, ldw) for g in range(G)]
        return out


def fuse_splitk_updates(solver) -> int:
    """Let the solver update consume Convolution weight-gradient split-K slabs directly
    (see :class:`_SlabGrad`): removes every splitk_reduce launch after a conv wgrad product
    and the flat-gradient round trip of those parameters; the update of such a layer runs
    right after its backward (like the fused InnerProduct update), on the layer's stream.
    Same eligibility as the fused InnerProduct update (no clipping / iter_size
    accumulation / gradient callbacks / debug info) plus a single-bottom, unshared, unfolded (no space-to-depth input), unchunked
    convolution.  The per-parameter arithmetic and the split summation order are those
    of the reduce kernel + solver update; the flat gradient of fused params is not
    written.  Returns the number of layers.

    Opt-in (SN_FEATURES=fuse_splitk=1): measured on one MI355X, same box, alternating runs, it is
    2 % slower on CaffeNet and 5 % slower on GoogLeNet than the wide split-K reduce kernel
    it replaces (docs/PERF_NOTES.md, "split-K slabs consumed by the solver")."""
    net = solver.net
    if (net.device.type != "cuda" or not solver.overlap_eligible() or net.debug_info
            or not features.enabled("fuse_splitk")):
        return 0
    from .ops import hip
    users: dict = {}
    for layer in net.layers:
        for p in layer.params:
            users[p.offset] = users.get(p.offset, 0) + 1
    sinks = []
    for li, layer in enumerate(net.layers):
        if layer.type_name != "Convolution" or not net.layer_need_backward[li] or not layer.param_grads_needed(0):
            continue
        if len(net.bottom_vecs[li]) != 1 or getattr(layer, "folded_input", None) is not None:
            continue
        ps = [layer.weight] + ([layer.bias] if layer.bias is not None else [])
        if any(p.owner is not None or users.get(p.offset, 0) != 1 for p in ps):
            continue
        s = layer.spec(net.bottom_vecs[li][0])
        if hip.s2d_plan(s) is not None or hip._image_chunk(s) < s.N or not hip._implicit_ok(s) or s.Kg % 8:
            continue
        layer.slab_grad = _SlabGrad(solver, layer)
        sinks.append(layer.slab_grad)
    if sinks:
        solver.set_slab_sinks(sinks)
    return len(sinks)


def fuse_input_fold(net, feeder) -> bool:
    """If the feeder's data blob is consumed only by a strided low-channel convolution on
    the space-to-depth path (AlexNet/CaffeNet conv1), make the feeder write the folded
    tensor directly (one fused augment + fold kernel) and the convolution read it.  The
    NHWC data blob is then no longer written during training steps.  GPU only."""
    if feeder is None or feeder.device.type != "cuda" or net.dtype == torch.float32:
        return False
    from .ops import hip
    try:
        bid = net.blob_names.index(feeder.data_blob.name)
    except (AttributeError, ValueError):
        return False
    consumers = [li for li, b in enumerate(net.bottom_ids) if bid in b]
    if len(consumers) != 1:
        return False
    conv = net.layers[consumers[0]]
    if conv.type_name != "Convolution" or net.bottom_ids[consumers[0]].index(bid) != 0:
        return False
    spec = conv.spec(feeder.data_blob)
    plan = hip.s2d_plan(spec)
    if plan is None or spec.H != feeder.crop or spec.C != feeder.shape[1]:
        return False
    s2 = plan[4]
    x2 = torch.empty((spec.N, s2.H, s2.W, s2.C), dtype=torch.bfloat16, device=feeder.device)
    feeder.fold = (x2, plan, spec)
    conv.folded_input = x2
    return True


def fp8_macs_per_input(layer, bottom) -> float:
    """Forward multiply-adds per input element of a Convolution / InnerProduct layer: the
    MFMA work the e4m3 path halves, per element of the bf16 -> e4m3 input quantisation
    pass it costs (a 3-byte-per-element HBM pass)."""
    if layer.type_name == "Convolution":
        s = layer.spec(bottom)
        return (s.K // s.groups) * s.R * s.S / float(s.sh * s.sw)
    return float(layer.N)


def fp8_dgrad_macs_per_grad(layer, bottom) -> float:
    """Data-gradient multiply-adds per output-gradient element of a stride-1 Convolution
    (the work the e4m3 data gradient halves per element of its dy quantisation pass)."""
    s = layer.spec(bottom)
    return float(s.Cg * s.R * s.S)


def enable_fp8(net, min_macs_per_input: float = 1000.0, dgrad: bool = False, dgrad_format: str = "e4m3",
               wgrad: bool = False) -> int:
    """Run the forward products of eligible Convolution / InnerProduct layers in OCP e4m3
    (v_mfma_scale_f32_16x16x128_f8f6f4, fp32 accumulation) with per-tensor delayed
    scaling: each layer quantises its input and weights with the scale derived from the
    previous iteration's amax (ops.hip.Fp8Scales; updated once per iteration by
    :func:`fp8_step`).  Gradients, masters and checkpoints stay bf16 / fp32.  Layers whose
    channels are not multiples of 16 (e.g. an RGB input conv) stay bf16, and so do layers
    with fewer than ``min_macs_per_input`` forward MACs per input element (where the
    quantisation pass over a large activation costs more than the faster product saves),
    except 64 -> 64 3x3 convs (VGG's conv1_2), which run the e4m3 direct kernel
    (ops.hip.direct_fp8_ok; SN_FEATURES=conv_direct_fp8=0 returns them to bf16).

    ``dgrad``: also run the data gradients of stride-1 Convolutions in e4m3 (the output
    gradient and the flip-transposed weights quantised per tensor; weight gradients stay
    bf16), for layers with at least ``min_macs_per_input`` data-gradient MACs per output-
    gradient element (:func:`fp8_dgrad_macs_per_grad`); ``dgrad_format`` "e5m2" quantises
    the output gradients to e5m2 (2 mantissa bits, 2^32 of range) instead of e4m3.

    ``wgrad`` (with ``dgrad``): the weight gradients of the layers that run BOTH an fp8
    forward and an fp8 data gradient become fp8 products as well (reduction over pixels:
    the output gradient's fp8 copy, shared with the data gradient, against the forward's
    e4m3 input kept for the backward; ops.hip._conv_wgrad_fp8).  GPU only; returns the
    number of fp8 products (forward + data gradient + weight gradient)."""
    if net.device.type != "cuda":
        return 0
    from .ops import hip
    chosen, chosen_dg = [], []
    for li, layer in enumerate(net.layers):
        if layer.type_name in ("Convolution", "InnerProduct") and len(net.bottom_vecs[li]) == 1:
            b = net.bottom_vecs[li][0]
            # 64 -> 64 3x3 convs run the e4m3 direct kernel (no idle MFMA columns), worth it below
            # the MAC threshold too
            direct = layer.type_name == "Convolution" and hip.direct_fp8_ok(layer.spec(b))
            if layer.fp8_eligible(b) and (direct or fp8_macs_per_input(layer, b) >= min_macs_per_input):
                chosen.append(layer)
            if (dgrad and layer.type_name == "Convolution" and layer.fp8_dgrad_eligible(b)
                    and net.bottom_need_backward[li][0]
                    and ((direct and dgrad_format == "e4m3")
                         or fp8_dgrad_macs_per_grad(layer, b) >= min_macs_per_input)):
                chosen_dg.append(layer)
    sc = hip.Fp8Scales(2 * (len(chosen) + len(chosen_dg)), net.device)
    for i, layer in enumerate(chosen):
        layer.fp8_slots = (2 * i, 2 * i + 1)
    assert dgrad_format in ("e4m3", "e5m2"), dgrad_format
    for i, layer in enumerate(chosen_dg, start=len(chosen)):
        layer.fp8_dgrad_slots = (2 * i, 2 * i + 1)
        if dgrad_format == "e5m2":
            sc.set_e5m2(2 * i)
    n_wg = 0
    if wgrad:
        both = set(map(id, chosen)) & set(map(id, chosen_dg))
        for li, layer in enumerate(net.layers):
            if id(layer) in both and hip.fp8_wgrad_ok(layer.spec(net.bottom_vecs[li][0])):
                layer.fp8_wgrad = True
                n_wg += 1
    net.ctx.fp8 = sc if (chosen or chosen_dg) else None
    fuse_fp8_quant(net)
    return len(chosen) + len(chosen_dg) + n_wg


def fuse_fp8_quant(net) -> int:
    """Pair each fp8 product with the conv GEMM that produces its bf16 operand, so that GEMM's
    epilogue also stores the fp8 bytes (ops.gemm.Fp8Side) and the separate bf16 -> fp8 pass
    (3 bytes of HBM traffic per element) becomes a 1-byte side store:
      forward:  conv P (ReLU fused) -> conv Q with an e4m3 forward: P's output GEMM stores Q's
                e4m3 input (Q's x slot);
      backward: the same pair with an fp8 data gradient on P: Q's data-gradient GEMM (ReLU
                gate of P's output fused) stores P's fp8 output gradient (P's dy slot).
    P's output must be read by Q alone (VGG-16's conv2_2 .. conv5_3 chains; the inputs that
    come out of pooling layers keep their quantisation pass).  The slots use delayed
    scaling, so the side stores start once the first fp8_update_scales has initialised them
    (eager warm-up steps); the bytes equal the separate pass's.  Returns the pairs fused."""
    if getattr(net.ctx, "fp8", None) is None or not features.enabled("fuse_fp8_quant"):
        return 0
    from .ops import hip
    outputs = set(getattr(net, "output_blob_ids", ()))
    n = 0

    def sole_reader(pi):
        blob = net.top_ids[pi][0]
        readers = [lj for lj in range(pi + 1, len(net.layers))
                   if blob in net.bottom_ids[lj] and not getattr(net.layers[lj], "fused", False)]
        return readers[0] if (blob not in outputs and len(readers) == 1) else None

    # pooling in between: conv P (ReLU fused) -> max pool -> conv Q (VGG's block boundaries)
    for oi, pool in enumerate(net.layers):
        if (pool.type_name != "Pooling" or len(net.top_ids[oi]) != 1 or pool.fused_lrn is not None
                or pool.global_pooling):
            continue
        s = pool.spec(net.bottom_vecs[oi][0])
        lq = sole_reader(oi)
        if lq is not None and net.layers[lq].type_name == "Convolution" and net.layers[lq].fp8_slots is not None \
                and hip.pool_side_ok(s, False):
            cons = net.layers[lq]
            pool.fp8_out = (cons, cons.fp8_slots[0])
            n += 1
        bid = net.bottom_ids[oi][0]
        prods = [pj for pj in range(oi) if bid in net.top_ids[pj] and not getattr(net.layers[pj], "fused", False)]
        if prods and hip.pool_side_ok(s, True) and net.bottom_need_backward[oi][0]:
            prod = net.layers[prods[-1]]
            if (prod.type_name == "Convolution" and prod.fp8_dgrad_slots is not None
                    and net.bottom_need_backward[prods[-1]][0] and sole_reader(prods[-1]) == oi):
                pool.fp8_dx_out = (prod, prod.fp8_dgrad_slots[0])
                # the conv reads that gradient only as fp8 (e4m3 data and weight gradients, bias
                # on the ones column): the pooling stores the fp8 bytes alone, not the bf16
                # tensor too — VGG-16 b2048 writes 25 GB less per step
                pool.fp8_dx_only = (features.enabled("fp8_dx_only") and not net.debug_info  # debug_info prints diffs
                                    and hip.conv_dy_fp8_only_ok(prod, prod.spec(net.bottom_vecs[prods[-1]][0])))
                n += 1
    for pi, prod in enumerate(net.layers):
        if prod.type_name != "Convolution" or not prod.fuse_relu or len(net.top_ids[pi]) != 1:
            continue
        if prod.concat_slot is not None:
            continue
        blob = net.top_ids[pi][0]
        readers = [lj for lj in range(pi + 1, len(net.layers))
                   if blob in net.bottom_ids[lj] and not getattr(net.layers[lj], "fused", False)]
        if blob in outputs or len(readers) != 1:
            continue
        lq = readers[0]
        cons = net.layers[lq]
        if cons.type_name != "Convolution" or len(net.bottom_ids[lq]) != 1:
            continue
        if cons.fp8_slots is not None:
            prod.fp8_out = (cons, cons.fp8_slots[0])
            n += 1
        if prod.fp8_dgrad_slots is not None and net.bottom_need_backward[pi][0]:
            cons.fp8_dx_out = (prod, prod.fp8_dgrad_slots[0])  # (conv1_1's data gradient never runs)
            n += 1
    return n


def fp8_step(net) -> None:
    """Per-iteration amax -> scale update of an fp8-enabled net (one small launch)."""
    if getattr(net.ctx, "fp8", None) is not None:
        net.ctx.fp8.update()


_DEPFREE_LRU = features.enabled("branch_depfree")


class BranchStreams:
    """Run independent branches of a DAG net on parallel HIP streams.

    Caffe executes layers strictly in prototxt order on the default stream
    (net.cpp:565-581, :635-645).  On a 256-CU MI355X the late GoogLeNet Inception stages
    (7x7 / 14x14 maps, 4 parallel towers) launch GEMMs of 50-150 tiles each, so a
    sequential schedule leaves most CUs idle.  This scheduler derives the dependency DAG
    from blob reads / writes (forward: bottoms -> tops; backward: top diffs + blob data ->
    bottom diffs + param diffs; read-after-write, write-after-read and write-after-write
    hazards), assigns every layer to one of ``n_streams`` streams (a layer continues the
    stream of a producer it directly follows, otherwise — also when it depends on nothing,
    like an auxiliary loss head's backward — takes the least recently used stream) and
    joins streams with events.  ``scripts/branch_sim.py`` simulates the plans on the CPU.  Inside a hipGraph capture the events become
    graph edges, so the towers of one Inception module run concurrently with no host
    involvement.  Every blob and gradient keeps its single producer, so results are
    bitwise identical to the sequential order.  Nets with backward hooks keep a
    sequential backward.  Status on the MI355X: eager runs with 4 streams and hipGraph
    captures with 2 streams or with 4 streams in the ``star`` topology are verified
    bitwise (GoogLeNet 17.1k -> 19.4k / 19.5k img/s).  A capture in which one side stream
    waits on an event of another side stream segfaults in hipStreamEndCapture on ROCm 7,
    so ``star`` (side streams wait only on the main stream; a layer with inputs from
    several side streams runs on the main stream) is used whenever n_streams > 2."""

    def __init__(self, net, n_streams: int = 4, star: bool = False):
        self.net = net
        self.n = max(1, n_streams)
        self.star = star
        self.side = None  # created on first run (the plan itself is device-independent)
        L = len(net.layers)
        # layer.sched_extra: hazards a fusion pass adds that the blob lists do not show
        # ({"fwd_r", "fwd_w", "bwd_r", "bwd_w"} token sets)
        ex = [getattr(net.layers[li], "sched_extra", None) or {} for li in range(L)]
        fwd = [(li, {("v", b) for b in net.bottom_ids[li]} | set(ex[li].get("fwd_r", ())),
                {("v", b) for b in net.top_ids[li]} | set(ex[li].get("fwd_w", ()))) for li in range(L)]
        bwd = []
        for li in range(L - 1, -1, -1):
            if not net.layer_need_backward[li]:
                continue
            reads = {("v", b) for b in list(net.bottom_ids[li]) + list(net.top_ids[li])}
            reads |= {("d", b) for b in net.top_ids[li]}
            reads |= set(ex[li].get("bwd_r", ()))
            writes = {("d", b) for b, need in zip(net.bottom_ids[li], net.bottom_need_backward[li]) if need}
            writes |= {("p", p.offset) for p in net.layers[li].params}
            writes |= set(ex[li].get("bwd_w", ()))
            bwd.append((li, reads, writes))
        self.fwd_plan = self._plan(fwd)
        self.bwd_plan = self._plan(bwd)

    def _plan(self, nodes):
        last_w, readers = {}, {}
        tail = [-1] * self.n                           # last position placed on each stream
        seen = [[-1] * self.n for _ in range(self.n)]  # seen[s][x]: last pos of stream x that s waited on
        stream_of, plan = [], []
        for pos, (li, reads, writes) in enumerate(nodes):
            deps = {last_w[r] for r in reads if r in last_w}
            for w in writes:
                if w in last_w:
                    deps.add(last_w[w])
                deps |= readers.get(w, set())
            deps.discard(pos)
            follow = [stream_of[d] for d in sorted(deps, reverse=True) if tail[stream_of[d]] == d]
            if follow:
                sid = follow[0]
            elif not deps and (pos == 0 or not _DEPFREE_LRU):
                sid = 0
            else:
                # a node with no dependency (a loss head's backward: its
                # top diff is the constant loss weight) takes the least recently used stream
                # too, instead of queueing on the main stream behind the towers (GoogLeNet
                # 22.36-22.42 -> 22.46-22.56 k img/s, profiles/r5_branch_depfree.txt;
                # SN_FEATURES=branch_depfree=0: the main stream)
                sid = min(range(self.n), key=lambda s: tail[s])
            if self.star and sid != 0 and any(stream_of[d] not in (0, sid) for d in deps):
                sid = 0  # star topology: side streams only ever wait on the main stream
            waits = [d for d in sorted(deps) if stream_of[d] != sid and d > seen[sid][stream_of[d]]]
            for d in waits:
                seen[sid][stream_of[d]] = max(seen[sid][stream_of[d]], d)
            stream_of.append(sid)
            tail[sid] = pos
            plan.append([li, sid, waits, False])
            for r in reads:
                readers.setdefault(r, set()).add(pos)
            for w in writes:
                last_w[w] = pos
                readers[w] = set()
        for _, _, waits, _ in list(plan):
            for d in waits:
                plan[d][3] = True
        return plan

    def streams_used(self, backward: bool = False) -> int:
        return len({sid for _, sid, _, _ in (self.bwd_plan if backward else self.fwd_plan)})

    def _run(self, plan, fn) -> None:
        if self.side is None:
            self.side = [torch.cuda.Stream(self.net.device) for _ in range(self.n - 1)]
            self._events = {}
            self._fork_join = (torch.cuda.Event(), [torch.cuda.Event() for _ in self.side])
        main = torch.cuda.current_stream(self.net.device)
        streams = [main] + self.side
        # Events live as long as the executor: a captured hipGraph references the event
        # objects of its record / wait nodes, and HIP crashes at capture end if an event
        # recorded during the capture was destroyed before it.
        evs = self._events.setdefault(id(plan), {})
        fork, join = self._fork_join
        fork.record(main)
        for s in self.side:
            s.wait_event(fork)
        for pos, (li, sid, waits, record) in enumerate(plan):
            st = streams[sid]
            for d in waits:
                st.wait_event(evs[d])
            with torch.cuda.stream(st):
                fn(li)
            if record:
                if pos not in evs:
                    evs[pos] = torch.cuda.Event()
                evs[pos].record(st)
        for s, ev in zip(self.side, join):
            ev.record(s)
            main.wait_event(ev)

    def forward(self):
        net = self.net
        self._run(self.fwd_plan, lambda li: net.layers[li].forward(net.bottom_vecs[li], net.top_vecs[li]))
        return net.loss_value()

    def backward(self) -> None:
        net = self.net
        if net.backward_hooks:
            net.backward()
            return
        net.prefill_loss_diffs()
        for hook in net.pre_backward_hooks:
            hook()
        self._run(self.bwd_plan, lambda li: net.layers[li].backward(
            net.top_vecs[li], net.bottom_need_backward[li], net.bottom_vecs[li]))

    def forward_backward(self):
        loss = self.forward()
        self.backward()
        return loss


def branch_streams(net, n_streams: int = 4):
    """A :class:`BranchStreams` executor for ``net`` when its layer DAG has parallel
    branches (the plan puts work on more than one stream), else None."""
    if net.device.type != "cuda" or n_streams <= 1:
        return None
    bs = BranchStreams(net, n_streams, star=n_streams > 2)
    if bs.streams_used() <= 1 and bs.streams_used(backward=True) <= 1:
        return None
    return bs


class OverlappedUpdate:
    """Runs each layer's fused solver update on a side stream as soon as backward has
    produced that layer's final gradients, so the bandwidth-bound update (CaffeNet: 61 M
    params, ~1.3 GB of traffic, fc6-fc8 first) overlaps the compute-bound conv backward
    GEMMs.  Caffe applies the update only after the whole backward pass
    (solver.cpp:237-240 -> sgd_solver.cpp:102-116); the result is identical because each
    parameter's update reads only its own gradient and history."""

    MIN_GROUP = 1 << 22   # params: smaller layers are updated after the backward pass
    GRID = 128            # background update blocks (a slice of the 256 CUs)

    def __init__(self, solver: Solver, min_group: int | None = None):
        self.solver = solver
        groups, rest = solver.overlap_plan(self.MIN_GROUP if min_group is None else min_group)
        dev = solver.device
        self.tables = {li: ops.solver_tables(segs, solver.net.num_param_elems, dev) for li, segs in groups.items()}
        self.rest = ops.solver_tables(rest, solver.net.num_param_elems, dev) if rest else None
        self.side = torch.cuda.Stream(dev)
        self.active = False

    def hook(self, li: int) -> None:
        t = self.tables.get(li)
        if t is None or not self.active:
            return
        main = torch.cuda.current_stream(self.solver.device)
        self.side.wait_stream(main)
        with torch.cuda.stream(self.side):
            self.solver.update_params_segments(t, grid_limit=self.GRID)

    def begin(self) -> None:
        self.active = True

    def end(self) -> None:
        """After backward + finish_param_diffs: late params, then join the side stream."""
        self.active = False
        if self.rest is not None:
            self.solver.update_params_segments(self.rest)
        torch.cuda.current_stream(self.solver.device).wait_stream(self.side)


def release_activations(net) -> int:
    """Drop the net's references to its per-iteration tensors — the data / diff of every blob
    a layer with bottoms produces, and the layers' forward-to-backward workspaces — so the
    eager warm-up's buffers return to the caching allocator.  A graph capture allocates every
    activation afresh in its private pool; without this the warm-up's copies stay referenced
    until the capture overwrites them one layer at a time, and a net that fills most of the
    288 GB (VGG-16 at per-GPU batch 2048) holds both sets at once.  The tops of data layers
    (written in place by the feeders) and the parameters are kept.  Returns the blobs dropped."""
    keep = set()
    for li in range(len(net.layers)):
        if not net.bottom_ids[li]:
            keep.update(net.top_ids[li])
    n = 0
    for bi, blob in enumerate(net.blobs):
        if bi in keep:
            continue
        blob._data = None
        blob._diff = None
        n += 1
    for layer in net.layers:
        for d in getattr(layer, "_ws", None) or ():
            if isinstance(d, dict):
                d.clear()
    gc.collect()
    torch.cuda.empty_cache()
    return n


GRAPH_RELEASE = None  # None: decide by memory use; True / False force it (tests)


def _release_before_capture(dev) -> bool:
    """release_activations before a capture when the warm-up holds over 45 % of the device
    (engine.GRAPH_RELEASE = True / False forces it on / off)."""
    if GRAPH_RELEASE is not None:
        return bool(GRAPH_RELEASE)
    if dev.type != "cuda":
        return False
    total = torch.cuda.get_device_properties(dev).total_memory
    return torch.cuda.memory_reserved(dev) > 0.45 * total


class GraphStep:
    """One captured solver iteration (iter_size = 1)."""

    def __init__(self, solver: Solver, warmup: int = 2, pre=None, overlap: bool = True, fuse_fc: bool = True,
                 streams: int = 2, comm=None):
        self.solver = solver
        self.pre = pre  # callable run (eagerly) before each replay, e.g. feeder.stage
        self.comm = comm  # N > 1 ranks: adopt rank 0's GEMM choices before capture (gemm.sync_tuned)
        self.graph = None
        self.loss = None
        self.warmup = warmup
        self.overlap = None
        if overlap and solver.overlap_eligible():
            self.overlap = OverlappedUpdate(solver)
            solver.net.backward_hooks.append(self.overlap.hook)
        elif fuse_fc:
            fuse_fc_updates(solver)
            fuse_splitk_updates(solver)
        # parallel Inception towers etc.; built lazily, used from the 2nd warmup iteration
        # on (the first one autotunes GEMMs, timed on an otherwise idle GPU).  Two
        # streams by default; more use the star topology (see BranchStreams)
        self.n_streams = streams if not solver.net.debug_info else 1
        self.branches = None
        self._use_branches = False
        # (weight gradients on a side stream measured slower three times — L2 thrash between
        # concurrent GEMMs, docs/PERF_NOTES.md rounds 3 and 5 — and were removed in round 6)

    def _body(self):
        s = self.solver
        net = s.net
        net.clear_param_diffs(lazy=True)
        # solver callbacks (P2PSync-style sync SGD, parallel.comm.SyncSGDCallback): their
        # bucketed gradient all-reduces, launched from backward hooks, are captured with
        # the iteration (RCCL collectives on the capturing stream become graph nodes)
        for cb in s.callbacks:
            getattr(cb, "on_start", lambda: None)()
        if self.overlap is not None:
            self.overlap.begin()
        if self._use_branches and self.branches is None:
            self.branches = branch_streams(net, self.n_streams) or False
        loss = (self.branches.forward_backward() if self._use_branches and self.branches
                else net.forward_backward())
        net.finish_param_diffs()
        fp8_step(net)
        for cb in s.callbacks:
            getattr(cb, "on_gradients_ready", lambda: None)()
        ops.advance_rng(net.ctx.rng_state)
        if self.overlap is not None:
            self.overlap.end()
        else:
            s.update_params()
        return loss

    def capture(self) -> None:
        s = self.solver
        dev = s.device
        side = torch.cuda.Stream(dev)
        side.wait_stream(torch.cuda.current_stream(dev))
        with torch.cuda.stream(side):
            for w in range(self.warmup):
                self._use_branches = w > 0
                if self.pre:
                    self.pre()
                s.stage_hyper()
                self._body()
                s.iter += 1
        torch.cuda.current_stream(dev).wait_stream(side)
        torch.cuda.synchronize(dev)
        if self.comm is not None:
            from .ops import gemm as _gemm
            _gemm.sync_tuned(self.comm)  # every rank captures the same kernel for each product
        if _release_before_capture(dev):
            release_activations(s.net)
        self.graph = torch.cuda.CUDAGraph()
        self._use_branches = True
        if self.pre:
            self.pre()
        s.stage_hyper()
        with torch.cuda.graph(self.graph):
            self.loss = self._body()
        # the capture did not execute: replay it once as a real iteration
        self.graph.replay()
        s.iter += 1
        # The replay loop allocates almost nothing, but Python's cyclic collector still runs
        # full passes over every object built so far (net, captured graph, torch state):
        # a gen-2 pass stalls the host for ~30 ms while the GPU drains its queue (measured:
        # the first 100 CaffeNet steps after capture ran at 94k instead of 105k img/s).
        # Collect once now and move the surviving objects out of the collector's view.
        gc.collect()
        gc.freeze()

    # Host run-ahead bound (SN_MAX_AHEAD = D > 0): before issuing step k, wait until step k - D
    # has finished on the GPU, so at most D captured iterations (and their H2D minibatch
    # copies) are queued ahead of the device; 0 = unbounded.  Unbounded, the host queues
    # dozens of iterations and the first ~60 of a run execute at 84-95k instead of 107k
    # img/s on CaffeNet (the "slow phase" of docs/PERF_NOTES.md); with D = 2 the in-stream
    # rate is a flat 107k from the first step and the driver-shaped 20-step bench measures
    # 105.7-106.1k vs 89.2-102.8k unbounded on the same box (scripts/ahead_ab.sh).
    max_ahead = int(os.environ.get("SN_MAX_AHEAD", "2"))

    def step(self):
        s = self.solver
        if self.graph is None:
            self.capture()
            return self.loss
        d = self.max_ahead
        if d > 0:
            ring = self.__dict__.setdefault("_ahead", [None] * d)
            k = self.__dict__.get("_ahead_k", 0)
            if ring[k % d] is not None:
                ring[k % d].synchronize()
        if self.pre:
            self.pre()
        s.stage_hyper()
        self.graph.replay()
        s.iter += 1
        if d > 0:
            ev = ring[k % d] or torch.cuda.Event()
            ev.record()
            ring[k % d] = ev
            self._ahead_k = k + 1
        return self.loss


class LocalSGDTrainer:
    """tau local steps + weight averaging per round (SparkNet's model averaging)."""

    def __init__(self, solver: Solver, comm=None, tau: int = 50, feeder=None, use_graph: bool = True,
                 log_every: int = 0, overlap_update: bool = False, fuse_fc: bool = True, streams: int = 2):
        self.solver = solver
        self.comm = comm
        self.tau = tau
        self.feeder = feeder
        self.round = 0
        self.use_graph = use_graph and solver.device.type == "cuda"
        self.step_fn = (GraphStep(solver, pre=self._pre, overlap=overlap_update, fuse_fc=fuse_fc, streams=streams,
                                  comm=comm)
                        if self.use_graph else None)
        self.log_every = log_every
        self.times = {"compute": 0.0, "allreduce": 0.0}

    def _pre(self):
        if self.feeder is not None:
            with trace_range("data"):
                self.feeder.stage()
                self.feeder.prefetch()

    def broadcast_initial(self) -> None:
        """All ranks start from rank 0's initial weights (CifarApp.scala:92)."""
        if self.comm is not None and getattr(self.comm, "active", self.comm.world_size > 1):
            self.comm.broadcast_params(self.solver.net)

    def local_step(self):
        with trace_range("compute"):
            if self.use_graph:
                return self.step_fn.step()
            self._pre()
            loss = self.solver.iteration()
            self.solver.iter += 1
            return loss

    def average(self) -> None:
        if self.comm is not None and getattr(self.comm, "active", self.comm.world_size > 1):
            with trace_range("allreduce"):
                self.comm.average_params(self.solver.net)

    def run_round(self):
        loss = None
        for _ in range(self.tau):
            loss = self.local_step()
        self.average()
        self.round += 1
        return loss

    def train(self, rounds: int, on_round=None):
        for r in range(rounds):
            t = time.perf_counter()
            loss = self.run_round()
            if on_round:
                on_round(r, loss, time.perf_counter() - t)
        return self.round
