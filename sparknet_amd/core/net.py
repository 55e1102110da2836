"""Net: graph construction and execution with Caffe semantics.

Reference: ``Net<Dtype>`` (caffe/src/caffe/net.cpp) — ``Init`` (:40-284), ``FilterNet`` /
``StateMeetsRule`` (:287-380), ``AppendTop/Bottom/Param`` (:383-562), ``ForwardFromTo``
(:565-581), ``BackwardFromTo`` (:635-645), ``ShareTrainedLayersWith`` (:737-766),
``CopyTrainedLayersFrom`` (:805-858), ``ToProto`` (:911-923), ``ClearParamDiffs``
(:990-1008); ``InsertSplits`` (caffe/src/caffe/util/insert_splits.cpp:12-145).

MI355X-first differences:
* all learnable parameters live in ONE flat fp32 master buffer + ONE flat fp32 gradient
  buffer (+ ONE flat bf16 compute shadow on GPU).  Zeroing gradients is one memset,
  the solver update is one fused kernel per bucket, and model averaging / gradient
  all-reduce operate on the flat buffer directly (RCCL over xGMI).
* forward / backward never synchronise with the host: the loss is a device scalar.
"""
from __future__ import annotations

import logging
from dataclasses import dataclass, field

import torch

from .. import ops, proto
from .blob import Blob
from .filler import fill
from .layer import Layer, Param, create_layer

log = logging.getLogger("sparknet_amd.net")

PARAM_ALIGN = 64  # elements; keeps every param segment 256-B aligned in the flat buffers


@dataclass
class NetContext:
    device: torch.device
    dtype: torch.dtype
    phase: int
    seed: int = 1701
    gen: torch.Generator = field(default=None)
    # Philox state for in-kernel RNG (dropout): [seed, counter] on the net's device.
    rng_state: torch.Tensor = field(default=None)
    layer_counter: int = 0
    # flat offsets of params whose gradient buffer was NOT cleared (lazy clear): the first
    # backward contribution overwrites instead of accumulating (Layer.grad_overwrite)
    stale_diffs: set = field(default_factory=set)
    # fp8 forward products (engine.enable_fp8): ops.hip.Fp8Scales shared by the net's layers
    fp8: object = None

    def next_stream_id(self) -> int:
        self.layer_counter += 1
        return self.layer_counter


# ------------------------------------------------------------------------------------
# FilterNet / StateMeetsRule
# ------------------------------------------------------------------------------------

def state_meets_rule(state, rule) -> bool:
    if rule.HasField("phase") and rule.phase != state.phase:
        return False
    if rule.HasField("min_level") and state.level < rule.min_level:
        return False
    if rule.HasField("max_level") and state.level > rule.max_level:
        return False
    stages = set(state.stage)
    if any(s not in stages for s in rule.stage):
        return False
    if any(s in stages for s in rule.not_stage):
        return False
    return True


def filter_net(param, state=None):
    state = state if state is not None else param.state
    out = proto.copy(param)
    del out.layer[:]
    for lp in param.layer:
        if len(lp.include) and len(lp.exclude):
            raise ValueError(f"layer {lp.name!r}: specify either include or exclude rules, not both")
        included = len(lp.include) == 0
        for rule in lp.exclude:
            if state_meets_rule(state, rule):
                included = False
        for rule in lp.include:
            if not included and state_meets_rule(state, rule):
                included = True
        if included:
            out.layer.add().CopyFrom(lp)
    return out


# ------------------------------------------------------------------------------------
# InsertSplits
# ------------------------------------------------------------------------------------

def split_layer_name(layer_name, blob_name, blob_idx):
    return f"{blob_name}_{layer_name}_{blob_idx}_split"


def split_blob_name(layer_name, blob_name, blob_idx, split_idx):
    return f"{blob_name}_{layer_name}_{blob_idx}_split_{split_idx}"


def _configure_split(layer_name, blob_name, blob_idx, count, loss_weight, lp):
    lp.Clear()
    lp.bottom.append(blob_name)
    lp.name = split_layer_name(layer_name, blob_name, blob_idx)
    lp.type = "Split"
    for k in range(count):
        lp.top.append(split_blob_name(layer_name, blob_name, blob_idx, k))
        if loss_weight:
            lp.loss_weight.append(loss_weight if k == 0 else 0.0)


def insert_splits(param):
    out = proto.copy(param)
    del out.layer[:]
    last_top: dict[str, tuple[int, int]] = {}
    bottom_src: dict[tuple[int, int], tuple[int, int]] = {}
    count: dict[tuple[int, int], int] = {}
    loss_w: dict[tuple[int, int], float] = {}
    split_idx: dict[tuple[int, int], int] = {}
    lname = {-1: "input"}
    for i, name in enumerate(param.input):
        last_top[name] = (-1, i)
    for i, lp in enumerate(param.layer):
        lname[i] = lp.name
        for j, b in enumerate(lp.bottom):
            if b not in last_top:
                raise ValueError(f"Unknown bottom blob {b!r} (layer {lp.name!r}, bottom index {j})")
            src = last_top[b]
            bottom_src[(i, j)] = src
            count[src] = count.get(src, 0) + 1
        for j, t in enumerate(lp.top):
            last_top[t] = (i, j)
        for j in range(min(len(lp.loss_weight), len(lp.top))):
            src = last_top[lp.top[j]]
            loss_w[src] = lp.loss_weight[j]
            if loss_w[src]:
                count[src] = count.get(src, 0) + 1
    for i, name in enumerate(param.input):
        c = count.get((-1, i), 0)
        if c > 1:
            _configure_split(lname[-1], name, i, c, 0.0, out.layer.add())
    for i, src_lp in enumerate(param.layer):
        lp = out.layer.add()
        lp.CopyFrom(src_lp)
        for j in range(len(lp.bottom)):
            src = bottom_src[(i, j)]
            c = count.get(src, 0)
            if c > 1:
                k = split_idx.get(src, 0)
                lp.bottom[j] = split_blob_name(lname[src[0]], lp.bottom[j], src[1], k)
                split_idx[src] = k + 1
        for j in range(len(lp.top)):
            src = (i, j)
            c = count.get(src, 0)
            if c > 1:
                lw = loss_w.get(src, 0.0)
                _configure_split(lname[i], lp.top[j], j, c, lw, out.layer.add())
                if lw:
                    del lp.loss_weight[:]
                    split_idx[src] = split_idx.get(src, 0) + 1
    return out


# ------------------------------------------------------------------------------------
# Net
# ------------------------------------------------------------------------------------

class Net:
    def __init__(self, param, phase: int | None = None, *, level: int | None = None,
                 stages=None, device="cpu", dtype: torch.dtype | None = None, seed: int = 1701,
                 ctx: NetContext | None = None, allocate: bool = True):
        if isinstance(param, str):
            param = proto.read_net(param)
        param = proto.copy(param)
        from ..proto.upgrade import upgrade_net
        upgrade_net(param)
        if phase is not None:
            param.state.phase = phase
        if level is not None:
            param.state.level = level
        if stages is not None:
            del param.state.stage[:]
            param.state.stage.extend(stages)
        device = torch.device(device)
        if dtype is None:
            dtype = torch.bfloat16 if device.type == "cuda" else torch.float32
        self.phase = param.state.phase
        if ctx is None:
            gen = torch.Generator().manual_seed(seed)
            rng = torch.tensor([seed, 0], dtype=torch.int64, device=device)
            ctx = NetContext(device, dtype, self.phase, seed, gen, rng)
        self.ctx = ctx
        self.device = device
        self.dtype = dtype
        self.name = param.name
        self.debug_info = param.debug_info
        filtered = filter_net(param)
        self.param = insert_splits(filtered)
        self._build(self.param)
        self.flat_data = self.flat_diff = self.flat_compute = None
        if allocate:
            self.allocate_params()

    # -- construction ----------------------------------------------------------------
    def _build(self, param) -> None:
        self.blobs: list[Blob] = []
        self.blob_names: list[str] = []
        self.blob_need_backward: list[bool] = []
        self.layers: list[Layer] = []
        self.layer_names: list[str] = []
        self.bottom_vecs: list[list[Blob]] = []
        self.top_vecs: list[list[Blob]] = []
        self.backward_hooks: list = []  # callables(layer_index) run after each layer's backward
        self.pre_backward_hooks: list = []  # callables() run before the first layer's backward
        self.bottom_ids: list[list[int]] = []
        self.top_ids: list[list[int]] = []
        self.bottom_need_backward: list[list[bool]] = []
        self.layer_need_backward: list[bool] = []
        self.params: list[Param] = []
        self.param_owners: list[int] = []
        self.param_layer_indices: list[tuple[int, int]] = []
        self.param_names_index: dict[str, int] = {}
        self.learnable_params: list[Param] = []
        self.input_blob_ids: list[int] = []
        name_to_idx: dict[str, int] = {}
        available: set[str] = set()

        if len(param.input_dim) and len(param.input_shape):
            raise ValueError("specify either input_shape or deprecated input_dim, not both")
        for i, name in enumerate(param.input):
            if len(param.input_dim):
                shape = tuple(param.input_dim[4 * i:4 * i + 4])
            else:
                shape = tuple(param.input_shape[i].dim)
            bid = self._new_blob(name, shape, name_to_idx)
            self.input_blob_ids.append(bid)
            available.add(name)

        for li, lp in enumerate(param.layer):
            if not lp.HasField("phase"):
                lp.phase = self.phase
            if len(lp.propagate_down) and len(lp.propagate_down) != len(lp.bottom):
                raise ValueError(f"layer {lp.name!r}: propagate_down must be given 0 or bottom_size times")
            layer = create_layer(lp, self.ctx)
            self.layers.append(layer)
            self.layer_names.append(lp.name)
            bvec, bids, bneed = [], [], []
            need_backward = False
            for j, bname in enumerate(lp.bottom):
                if bname not in available:
                    raise ValueError(f"Unknown bottom blob {bname!r} (layer {lp.name!r}, bottom index {j})")
                bid = name_to_idx[bname]
                bvec.append(self.blobs[bid])
                bids.append(bid)
                available.discard(bname)
                pd = lp.propagate_down[j] if len(lp.propagate_down) else True
                nb = self.blob_need_backward[bid] and pd
                bneed.append(nb)
                need_backward |= self.blob_need_backward[bid]
            tvec, tids = [], []
            ntop = len(lp.top)
            for j, tname in enumerate(lp.top):
                if j < len(lp.bottom) and tname == lp.bottom[j]:
                    bid = name_to_idx[tname]  # in-place
                elif tname in name_to_idx:
                    raise ValueError(f"Top blob {tname!r} produced by multiple sources.")
                else:
                    bid = self._new_blob(tname, (), name_to_idx)
                tvec.append(self.blobs[bid])
                tids.append(bid)
                available.add(tname)
            if layer.auto_top_blobs:
                while ntop < layer.needed_tops():
                    bid = self._new_blob("(automatic)", (), None)
                    tvec.append(self.blobs[bid])
                    tids.append(bid)
                    ntop += 1
            self.bottom_vecs.append(bvec)
            self.bottom_ids.append(bids)
            self.bottom_need_backward.append(bneed)
            self.top_vecs.append(tvec)
            self.top_ids.append(tids)
            layer.setup(bvec, tvec)
            nparam = len(layer.params)
            if len(lp.param) > nparam:
                raise ValueError(f"Too many params specified for layer {lp.name!r}")
            layer.param_propagate_down = []
            for pid in range(nparam):
                spec = lp.param[pid] if pid < len(lp.param) else proto.ParamSpec()
                pneed = spec.lr_mult != 0
                need_backward |= pneed
                layer.param_propagate_down.append(pneed)
            for pid in range(nparam):
                self._append_param(li, pid)
            self.layer_need_backward.append(need_backward)
            if need_backward:
                for tid in tids:
                    self.blob_need_backward[tid] = True

        # Backward pruning: only layers whose tops reach a loss need backward.
        under_loss: set[str] = set()
        skip_bp: set[str] = set()
        for li in range(len(self.layers) - 1, -1, -1):
            layer = self.layers[li]
            contributes = False
            skip_pd = True
            for j, tid in enumerate(self.top_ids[li]):
                bname = self.blob_names[tid]
                if layer.loss(j) or bname in under_loss:
                    contributes = True
                if bname not in skip_bp:
                    skip_pd = False
                if contributes and not skip_pd:
                    break
            if self.layer_need_backward[li] and skip_pd:
                self.layer_need_backward[li] = False
                self.bottom_need_backward[li] = [False] * len(self.bottom_vecs[li])
            if not contributes:
                self.layer_need_backward[li] = False
            for j, bid in enumerate(self.bottom_ids[li]):
                if contributes:
                    under_loss.add(self.blob_names[bid])
                else:
                    self.bottom_need_backward[li][j] = False
                if not self.bottom_need_backward[li][j]:
                    skip_bp.add(self.blob_names[bid])
        if param.force_backward:
            for li, layer in enumerate(self.layers):
                self.layer_need_backward[li] = True
                for j, bid in enumerate(self.bottom_ids[li]):
                    v = self.bottom_need_backward[li][j] or layer.allow_force_backward(j)
                    self.bottom_need_backward[li][j] = v
                    self.blob_need_backward[bid] = self.blob_need_backward[bid] or v
                layer.param_propagate_down = [True] * len(layer.params)
        self.output_blob_ids = [name_to_idx[n] for n in sorted(available)]
        self.blob_names_index = {n: i for i, n in enumerate(self.blob_names)}
        self.layer_names_index = {n: i for i, n in enumerate(self.layer_names)}
        # Loss tops: top diff = loss weight (Layer::SetLossWeights)
        self._loss_tops: list[tuple[Blob, float]] = []
        for li, layer in enumerate(self.layers):
            for j, t in enumerate(self.top_vecs[li]):
                w = layer.loss(j)
                if w:
                    self._loss_tops.append((t, w))
        for li, layer in enumerate(self.layers):
            log.debug("%s needs backward: %s", layer.name, self.layer_need_backward[li])

    def _new_blob(self, name, shape, name_to_idx) -> int:
        b = Blob(name, shape, self.dtype, self.device)
        bid = len(self.blobs)
        self.blobs.append(b)
        self.blob_names.append(name)
        self.blob_need_backward.append(False)
        if name_to_idx is not None:
            name_to_idx[name] = bid
        return bid

    def _append_param(self, li: int, pid: int) -> None:
        layer = self.layers[li]
        lp = layer.lp
        spec = lp.param[pid] if pid < len(lp.param) else proto.ParamSpec()
        pname = spec.name if pid < len(lp.param) else ""
        net_pid = len(self.params)
        p = layer.params[pid]
        self.params.append(p)
        self.param_layer_indices.append((li, pid))
        if not pname or pname not in self.param_names_index:
            self.param_owners.append(-1)
            if pname:
                self.param_names_index[pname] = net_pid
            p.lr_mult = spec.lr_mult
            p.decay_mult = spec.decay_mult
            p._has_lr = spec.HasField("lr_mult")
            p._has_decay = spec.HasField("decay_mult")
            self.learnable_params.append(p)
        else:
            owner_id = self.param_names_index[pname]
            self.param_owners.append(owner_id)
            owner = self.params[owner_id]
            if spec.share_mode == 1:  # PERMISSIVE
                if owner.count != p.count:
                    raise ValueError(f"Cannot share param {pname!r}: count mismatch")
            elif owner.caffe_shape != p.caffe_shape:
                raise ValueError(f"Cannot share param {pname!r}: shape mismatch "
                                 f"{owner.caffe_shape} vs {p.caffe_shape}")
            root = owner.root()
            if spec.HasField("lr_mult"):
                if root._has_lr and root.lr_mult != spec.lr_mult:
                    raise ValueError(f"Shared param {pname!r} has mismatched lr_mult.")
                root._has_lr, root.lr_mult = True, spec.lr_mult
            if spec.HasField("decay_mult"):
                if root._has_decay and root.decay_mult != spec.decay_mult:
                    raise ValueError(f"Shared param {pname!r} has mismatched decay_mult.")
                root._has_decay, root.decay_mult = True, spec.decay_mult
            p.owner = root

    # -- flat parameter buffers ----------------------------------------------------------
    def allocate_params(self, init: bool = True) -> None:
        """Lay every learnable param out in the flat master / grad / compute buffers and
        run the fillers (or keep the values already present)."""
        offs = []
        total = 0
        for p in self.learnable_params:
            offs.append(total)
            total += -(-p.count // PARAM_ALIGN) * PARAM_ALIGN
        self.num_param_elems = total
        dev = self.device
        self.flat_data = torch.zeros(max(total, 1), dtype=torch.float32, device=dev)
        self.flat_diff = torch.zeros(max(total, 1), dtype=torch.float32, device=dev)
        if self.dtype == torch.float32:
            self.flat_compute = self.flat_data
        else:
            self.flat_compute = torch.zeros(max(total, 1), dtype=self.dtype, device=dev)
        gen = self.ctx.gen
        for p, off in zip(self.learnable_params, offs):
            prev = p.data
            p.offset = off
            p.data = self.flat_data[off:off + p.count].view(p.shape)
            p.diff = self.flat_diff[off:off + p.count].view(p.shape)
            p.compute = self.flat_compute[off:off + p.count].view(p.shape)
            if init and getattr(p, "_initialized", None) is None:
                vals = fill(p.filler, p.caffe_shape, gen)
                p.data.copy_(p.from_caffe(vals).to(dev))
            elif prev is not None and prev.numel() == p.count:
                p.data.copy_(prev.reshape(p.shape).to(dev))
        for p in self.params:
            if p.owner is not None:
                r = p.owner
                p.offset = r.offset
                p.data = r.data.view(p.shape)
                p.diff = r.diff.view(p.shape)
                p.compute = r.compute.view(p.shape)
        self.sync_compute()

    def sync_compute(self) -> None:
        """Refresh the bf16 compute shadow from the fp32 masters (after load / set)."""
        if self.flat_compute is not self.flat_data and self.flat_data is not None:
            from .. import ops
            ops.cast_f32_to_bf16(self.flat_data, self.flat_compute)

    def param_segments(self) -> list[tuple[int, int, float, float]]:
        """(offset, count, lr_mult, decay_mult) per learnable (owner) param."""
        return [(p.offset, p.count, p.lr_mult, p.decay_mult) for p in self.learnable_params]

    # -- execution ---------------------------------------------------------------------
    def forward_from_to(self, start: int, end: int):
        with ops.precision(self.dtype):  # fp32 nets on the GPU: the fp32 device mode (ops.f32dev)
            for li in range(start, end + 1):
                layer = self.layers[li]
                layer.forward(self.bottom_vecs[li], self.top_vecs[li])
                if self.debug_info:
                    self._debug_forward(li)
            return self.loss_value()

    def loss_value(self):
        """Weighted sum of the loss tops as a device scalar (no host sync)."""
        loss = None
        if len(self._loss_tops) == 1 and self._loss_tops[0][1] == 1.0:
            t = self._loss_tops[0][0].data
            if t.numel() == 1 and t.dtype == torch.float32:
                return t.reshape(())  # the usual single unit-weight loss: no extra kernel
        for t, w in self._loss_tops:
            v = t.data.float()
            v = v.sum() * w if v.numel() > 1 else v.reshape(()) * w
            loss = v if loss is None else loss + v
        return loss if loss is not None else torch.zeros((), device=self.device)

    def forward(self, bottom: list[torch.Tensor] | None = None):
        """Net::Forward — returns the (device) scalar loss; never syncs with the host."""
        if bottom is not None:
            for bid, t in zip(self.input_blob_ids, bottom):
                self.blobs[bid].set_nchw(t)
        return self.forward_from_to(0, len(self.layers) - 1)

    def prefill_loss_diffs(self) -> None:
        """Top diff of every loss blob = its loss weight (Layer::SetLossWeights).  The fill
        is skipped while the diff tensor still holds it (same tensor, no in-place write
        since), so a captured training step carries no fill kernel."""
        done = self.__dict__.setdefault("_loss_diff_filled", {})
        for t, w in self._loss_tops:
            d = t.diff
            key = (id(d), d.data_ptr(), d._version, w)
            if done.get(id(t)) != key:
                d.fill_(w)
                done[id(t)] = (id(d), d.data_ptr(), d._version, w)

    def backward_from_to(self, start: int, end: int) -> None:
        self.prefill_loss_diffs()
        for hook in self.pre_backward_hooks:  # e.g. batched dgrad weight flips
            hook()
        with ops.precision(self.dtype):
            for li in range(start, end - 1, -1):
                if self.layer_need_backward[li]:
                    self.layers[li].backward(self.top_vecs[li], self.bottom_need_backward[li],
                                             self.bottom_vecs[li])
                    if self.debug_info:
                        self._debug_backward(li)
                for hook in self.backward_hooks:  # e.g. overlapped per-layer solver update
                    hook(li)

    def backward(self) -> None:
        self.backward_from_to(len(self.layers) - 1, 0)

    def forward_backward(self):
        loss = self.forward()
        self.backward()
        return loss

    def reshape(self) -> None:
        for li, layer in enumerate(self.layers):
            layer.reshape(self.bottom_vecs[li], self.top_vecs[li])

    def clear_param_diffs(self, lazy: bool = False) -> None:
        """Net::ClearParamDiffs.  lazy=True skips the memset for params whose every user
        layer can overwrite its gradient on first write (Convolution / InnerProduct:
        their wgrad GEMM stores instead of read-modify-writes); the rest are zeroed.
        Pair with :meth:`finish_param_diffs` after the last backward."""
        if self.flat_diff is None:
            return
        st = self.ctx.stale_diffs
        st.clear()
        if not lazy:
            self.flat_diff.zero_()
            return
        ok = self._overwrite_ok()
        for off, cnt in self._zero_ranges(ok):
            self.flat_diff[off:off + cnt].zero_()
        st.update(o for o, good in ok.items() if good)

    def finish_param_diffs(self) -> None:
        """Zero the gradients of lazily-cleared params that no backward wrote (e.g. a
        layer whose backward was pruned this pass)."""
        st = self.ctx.stale_diffs
        if st:
            for p in self.learnable_params:
                if p.offset in st:
                    p.diff.zero_()
            st.clear()

    def _overwrite_ok(self) -> dict:
        if getattr(self, "_ow_cache", None) is None:
            ok = {p.offset: True for p in self.learnable_params}
            for layer in self.layers:
                good = getattr(layer, "supports_grad_overwrite", False)
                for p in layer.params:
                    if not good:
                        ok[p.offset] = False
            self._ow_cache = ok
        return self._ow_cache

    def _zero_ranges(self, ok: dict):
        """Contiguous flat ranges covering every param that must be zeroed eagerly."""
        ranges = []
        for p in sorted(self.learnable_params, key=lambda q: q.offset):
            if ok.get(p.offset, False):
                continue
            seg = -(-p.count // PARAM_ALIGN) * PARAM_ALIGN
            if ranges and ranges[-1][0] + ranges[-1][1] == p.offset:
                ranges[-1][1] += seg
            else:
                ranges.append([p.offset, seg])
        return ranges

    def update(self) -> None:
        """Net::Update: data -= diff for every owner param (plain Blob::Update)."""
        self.flat_data.sub_(self.flat_diff)
        self.sync_compute()

    # -- accessors ---------------------------------------------------------------------
    @property
    def input_blobs(self) -> list[Blob]:
        return [self.blobs[i] for i in self.input_blob_ids]

    @property
    def output_blobs(self) -> list[Blob]:
        return [self.blobs[i] for i in self.output_blob_ids]

    def has_blob(self, name: str) -> bool:
        return name in self.blob_names_index

    def blob_by_name(self, name: str) -> Blob:
        return self.blobs[self.blob_names_index[name]]

    def has_layer(self, name: str) -> bool:
        return name in self.layer_names_index

    def layer_by_name(self, name: str) -> Layer:
        return self.layers[self.layer_names_index[name]]

    # -- weight exchange (SparkNet Net.getWeights / setWeights, Net.scala:132-172) ------
    def get_weights(self) -> dict[str, list[torch.Tensor]]:
        """Caffe-layout fp32 copies of every layer's param blobs, keyed by layer name."""
        out = {}
        for layer in self.layers:
            if layer.params:
                out[layer.name] = [p.to_caffe().cpu().clone() for p in layer.params]
        return out

    def set_weights(self, weights: dict[str, list[torch.Tensor]]) -> None:
        for name, blobs in weights.items():
            layer = self.layer_by_name(name)
            if len(blobs) != len(layer.params):
                raise ValueError(f"layer {name!r}: expected {len(layer.params)} blobs, got {len(blobs)}")
            for p, t in zip(layer.params, blobs):
                t = torch.as_tensor(t)
                if tuple(t.shape) != p.caffe_shape and t.numel() != p.caffe_count:
                    raise ValueError(f"layer {name!r}: shape mismatch {tuple(t.shape)} vs {p.caffe_shape}")
                p.set_caffe(t)
        self.sync_compute()

    # -- checkpoints -------------------------------------------------------------------
    def to_proto(self, write_diff: bool = False):
        """Net::ToProto: the (split-free) net definition with Caffe-layout blobs."""
        net = proto.copy(self.param)
        del net.layer[:]
        for li, layer in enumerate(self.layers):
            if layer.type_name == "Split" and layer.lp.name.endswith("_split"):
                continue
            lp = net.layer.add()
            lp.CopyFrom(layer.lp)
            del lp.blobs[:]
            for p in layer.params:
                bp = lp.blobs.add()
                bp.shape.dim.extend(p.caffe_shape)
                bp.data.extend(p.to_caffe().cpu().reshape(-1).tolist())
                if write_diff:
                    bp.diff.extend(p.to_caffe(p.diff).cpu().reshape(-1).tolist())
        return net

    def to_hdf5(self, path: str, write_diff: bool = False) -> None:
        """Net::ToHDF5 (net.cpp:926-980): ``data/<layer>/<i>`` for params that own
        themselves, ``diff/<layer>/<i>`` for every param when ``write_diff``."""
        from ..utils import hdf5
        net_pid = {lj: i for i, lj in enumerate(self.param_layer_indices)}
        data, diff = {}, {}
        for li, layer in enumerate(self.layers):
            if layer.type_name == "Split" and layer.lp.name.endswith("_split"):
                continue
            ld, lg = {}, {}
            for j, p in enumerate(layer.params):
                if self.param_owners[net_pid[(li, j)]] == -1:
                    ld[str(j)] = p.to_caffe().float().cpu().numpy()
                if write_diff:
                    lg[str(j)] = p.to_caffe(p.diff).float().cpu().numpy()
            data[layer.name] = ld
            if write_diff:
                diff[layer.name] = lg
        tree = {"data": data}
        if write_diff:
            tree["diff"] = diff
        hdf5.write(path, tree)

    def copy_trained_layers_from_hdf5(self, path: str) -> None:
        """Net::CopyTrainedLayersFromHDF5 (net.cpp:861-908)."""
        from ..utils import hdf5
        f = hdf5.File(path)
        data = f["data"]
        for lname in data.keys():
            if lname not in self.layer_names_index:
                log.info("Ignoring source layer %s", lname)
                continue
            li = self.layer_names_index[lname]
            layer = self.layers[li]
            src = data[lname]
            if len(src) > len(layer.params):
                raise ValueError(f"Incompatible number of blobs for layer {lname!r}")
            for j, p in enumerate(layer.params):
                if str(j) not in src:
                    if p.owner is not None:        # weight-shared in the target: fine
                        continue
                    raise ValueError(f"Incompatible number of blobs for layer {lname!r}")
                t = torch.from_numpy(src[str(j)].read().astype("float32"))
                if tuple(t.shape) != tuple(p.caffe_shape):
                    raise ValueError(f"Cannot copy param of layer {lname!r}; shape mismatch. "
                                     f"Source {tuple(t.shape)}, target {p.caffe_shape}")
                p.set_caffe(t.reshape(p.caffe_shape))
        self.sync_compute()

    def copy_trained_layers_from(self, src) -> None:
        """Net::CopyTrainedLayersFrom: match by layer name, fail on shape mismatch; a
        ``.h5`` file name selects the HDF5 reader (net.cpp:842-858)."""
        if isinstance(src, str):
            if src.endswith(".h5"):
                self.copy_trained_layers_from_hdf5(src)
                return
            src = proto.read_net(src)  # upgrades V0 / V1 nets (net.cpp:853-858)
        elif len(src.layers):
            from ..proto.upgrade import upgrade_net
            up = proto.NetParameter()
            up.CopyFrom(src)
            src = upgrade_net(up)
        for slp in src.layer:
            if slp.name not in self.layer_names_index:
                continue
            layer = self.layer_by_name(slp.name)
            if len(slp.blobs) != len(layer.params):
                raise ValueError(f"Incompatible number of blobs for layer {slp.name!r}")
            for p, bp in zip(layer.params, slp.blobs):
                t = blob_proto_to_tensor(bp)
                if not blob_shape_equals(bp, p.caffe_shape):
                    raise ValueError(f"Cannot copy param of layer {slp.name!r}; shape mismatch. "
                                     f"Source {tuple(t.shape)}, target {p.caffe_shape}")
                p.set_caffe(t.reshape(p.caffe_shape))
        self.sync_compute()

    def share_trained_layers_with(self, other: "Net") -> None:
        """Net::ShareTrainedLayersWith: alias param storage of same-named layers."""
        for li, layer in enumerate(other.layers):
            if layer.name not in self.layer_names_index:
                continue
            mine = self.layer_by_name(layer.name)
            if len(mine.params) != len(layer.params):
                raise ValueError(f"Incompatible number of blobs for layer {layer.name!r}")
            for p, q in zip(mine.params, layer.params):
                if p.count != q.count:
                    raise ValueError(f"Cannot share param of layer {layer.name!r}; shape mismatch")
                p.data = q.data.view(p.shape)
                p.diff = q.diff.view(p.shape) if q.diff is not None else None
                p.compute = q.compute.view(p.shape)

    # -- debug info (net.cpp:648-734) -----------------------------------------------------
    def _debug_forward(self, li: int) -> None:
        for t in self.top_vecs[li]:
            log.info("    [Forward] Layer %s, top blob %s data: %g", self.layer_names[li], t.name,
                     float(t.data.float().abs().mean()))
        for p in self.layers[li].params:
            log.info("    [Forward] Layer %s, param blob %s data: %g", self.layer_names[li], p.name,
                     float(p.data.abs().mean()))

    def _debug_backward(self, li: int) -> None:
        for j, b in enumerate(self.bottom_vecs[li]):
            if self.bottom_need_backward[li][j] and b.has_diff():
                log.info("    [Backward] Layer %s, bottom blob %s diff: %g", self.layer_names[li], b.name,
                         float(b.diff.float().abs().mean()))
        for p in self.layers[li].params:
            if p.diff is not None:
                log.info("    [Backward] Layer %s, param blob %s diff: %g", self.layer_names[li], p.name,
                         float(p.diff.abs().mean()))

    def memory_used(self) -> int:
        return sum(b.count * b.data.element_size() for b in self.blobs if b.shape)

    def __repr__(self):
        return f"Net({self.name!r}, {len(self.layers)} layers, {self.num_param_elems if self.flat_data is not None else '?'} param elems)"


def blob_shape_equals(bp, shape) -> bool:
    """Blob::ShapeEquals (blob.cpp:474-490): a legacy (num, channels, height, width) proto
    matches a target of <= 4 axes padded with leading 1s; otherwise shapes match exactly."""
    shape = tuple(int(s) for s in shape)
    legacy = any(bp.HasField(f) for f in ("num", "channels", "height", "width"))
    if legacy:
        # legacy 4-D fields: unset ones read as their default 0, like Blob::LegacyShape
        if len(shape) > 4:
            return False
        return (1,) * (4 - len(shape)) + shape == (bp.num, bp.channels, bp.height, bp.width)
    return tuple(bp.shape.dim) == shape  # no shape either: only a 0-axis blob matches


def blob_proto_to_tensor(bp) -> torch.Tensor:
    """Blob::FromProto (blob.cpp:446-495): ``shape`` or legacy 4-D fields, float or double."""
    if bp.HasField("shape"):
        shape = tuple(bp.shape.dim)
    elif any(bp.HasField(f) for f in ("num", "channels", "height", "width")):
        shape = (bp.num, bp.channels, bp.height, bp.width)
    else:
        shape = (len(bp.data) or len(bp.double_data),)
    if len(bp.double_data):
        t = torch.tensor(list(bp.double_data), dtype=torch.float64).float()
    else:
        import numpy as np
        t = torch.from_numpy(np.asarray(bp.data, dtype=np.float32).copy())
    return t.reshape(shape)


def tensor_to_blob_proto(t: torch.Tensor, bp=None, legacy_4d: bool = False):
    bp = bp if bp is not None else proto.BlobProto()
    t = t.detach().float().cpu()
    if legacy_4d and t.dim() == 4:
        bp.num, bp.channels, bp.height, bp.width = (int(s) for s in t.shape)
    else:
        bp.shape.dim.extend(int(s) for s in t.shape)
    bp.data.extend(t.reshape(-1).numpy().tolist())
    return bp
