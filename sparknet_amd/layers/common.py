"""Structural layers: Split, Concat, Slice, Eltwise, Flatten, Reshape, Silence, Tile,
Reduction, ArgMax, BatchReindex, Filter, Embed, MVN, BatchNorm, SPP.

References: caffe/src/caffe/layers/{split,concat,slice,eltwise,flatten,reshape,silence,
tile,reduction,argmax,batch_reindex,filter,embed,mvn,batch_norm,spp}_layer.*.

Channel-axis operations on 4-D blobs (Concat/Slice along axis 1) act on the physical
last axis of the NHWC storage.  Flatten/Reshape keep Caffe's logical (C, H, W) order by
converting through the NCHW view.

On the GPU every layer here runs HIP kernels (csrc/kernels/eltwise.hip for the hot Split /
channel Concat, csrc/kernels/layers.hip for the rest, wrapped by ops.layers_hip); the
tensor-math bodies are the fp32 CPU reference path.
"""
from __future__ import annotations

import torch

from .. import ops
from ..core.layer import Layer, register


def _phys_axis(blob, axis):
    axis = blob.canonical_axis(axis)
    if blob.is_image:
        return {0: 0, 1: 3, 2: 1, 3: 2}[axis]
    return axis


def _oai(t: torch.Tensor, ax: int):
    """(outer, A, inner) of a contiguous tensor around physical axis ``ax``."""
    outer = 1
    for d in t.shape[:ax]:
        outer *= d
    inner = 1
    for d in t.shape[ax + 1:]:
        inner *= d
    return outer, t.shape[ax], inner


def _lh():
    from ..ops import layers_hip
    return layers_hip


def _to_logical(blob, diff=False):
    """Contiguous logical-order (NCHW for images) copy / view of a GPU blob."""
    t = blob.diff if diff else blob.data
    if blob.is_image:
        return _lh().nhwc_to_nchw(t)
    return t


def _from_logical(t, blob):
    """Physical-layout tensor for ``blob`` from a logical-order tensor of the same count."""
    if blob.is_image:
        N, C_, H, W = blob.shape
        return _lh().nchw_to_nhwc(t.reshape(N, C_, H * W), N, C_, H, W)
    return t.reshape(blob.data.shape)


@register("Split")
class SplitLayer(Layer):
    exact_bottoms = 1
    min_tops = 1

    def reshape(self, bottoms, tops):
        for t in tops:
            t.reshape(bottoms[0].shape, bottoms[0].dtype)

    def forward(self, bottoms, tops):
        for t in tops:
            t.data = bottoms[0].data  # ShareData: no copy

    def backward(self, tops, propagate_down, bottoms):
        if not propagate_down[0]:
            return
        if len(tops) == 1:
            bottoms[0].diff = tops[0].diff
            return
        diffs = [t.diff for t in tops]
        d0 = diffs[0]
        if d0.is_cuda and d0.dtype == torch.bfloat16 and d0.numel() % 8 == 0:
            # one fused fp32-accumulating pass over all top diffs (HIP sum_bf16)
            bottoms[0].diff = ops.sum_bf16(diffs)
            return
        if d0.is_cuda:
            bottoms[0].diff = _eltwise_sum_gpu(diffs)
            return
        acc = d0.float() if d0.dtype != torch.float32 else d0.clone()
        for d in diffs[1:]:
            acc = acc + d.float()
        bottoms[0].diff = acc.to(bottoms[0].dtype)


def _eltwise_sum_gpu(ts, coeffs=None):
    """Sum (with coefficients) of same-shape GPU tensors with the HIP eltwise kernel; more
    than 16 inputs are folded in chunks (the running sum is input 0 of the next chunk)."""
    lh = _lh()
    coeffs = list(coeffs) if coeffs is not None else [1.0] * len(ts)
    acc, _ = lh.eltwise_fwd(1, ts[:16], coeffs[:16])
    i = 16
    while i < len(ts):
        chunk = ts[i:i + 15]
        acc, _ = lh.eltwise_fwd(1, [acc] + chunk, [1.0] + coeffs[i:i + 15])
        i += 15
    return acc


@register("Concat")
class ConcatLayer(Layer):
    min_bottoms = 1
    exact_tops = 1

    def layer_setup(self, bottoms, tops):
        p = self.lp.concat_param
        self.axis = bottoms[0].canonical_axis(p.axis if p.HasField("axis") or not p.HasField("concat_dim")
                                              else p.concat_dim)

    def reshape(self, bottoms, tops):
        shape = list(bottoms[0].shape)
        for b in bottoms[1:]:
            if len(b.shape) != len(shape):
                raise ValueError("Concat: all bottoms need the same number of axes")
            for d in range(len(shape)):
                if d != self.axis and b.shape[d] != shape[d]:
                    raise ValueError("Concat: bottoms differ outside the concat axis")
            shape[self.axis] += b.shape[self.axis]
        tops[0].reshape(tuple(shape), bottoms[0].dtype)

    relu_gate_parts: frozenset = frozenset()  # bottoms whose in-place ReLU backward runs here
    zero_copy = None       # ConcatSlots: the producers wrote the parts into one buffer (engine.fuse_concat)
    zero_copy_bwd = False  # ... and the consumers of the output gate its gradient: parts' diffs are views

    def _hip_ok(self, bottoms, ax) -> bool:
        """One-launch HIP path: channel concat of NHWC bf16 device blobs, <= 8 parts."""
        b0 = bottoms[0].data
        return (b0.is_cuda and b0.dtype == torch.bfloat16 and ax == b0.dim() - 1 and len(bottoms) <= 8
                and all(b.data.shape[-1] % 8 == 0 for b in bottoms))

    def forward(self, bottoms, tops):
        if len(bottoms) == 1:
            tops[0].data = bottoms[0].data
            return
        if self.zero_copy is not None:
            buf = self.zero_copy.take()
            if buf is not None and self.zero_copy.holds([b.data for b in bottoms], buf):
                tops[0].data = buf  # every part already sits in its channel slice: no copy
                return
        ax = _phys_axis(bottoms[0], self.axis)
        if self._hip_ok(bottoms, ax):
            from ..ops import hip
            shape = list(bottoms[0].data.shape)
            shape[-1] = sum(b.data.shape[-1] for b in bottoms)
            out = torch.empty(shape, dtype=torch.bfloat16, device=bottoms[0].data.device)
            tops[0].data = hip.concat_channels([b.data for b in bottoms], out)
            return
        if bottoms[0].data.is_cuda:
            lh = _lh()
            shape = list(bottoms[0].data.shape)
            shape[ax] = sum(b.data.shape[ax] for b in bottoms)
            out = torch.empty(shape, dtype=tops[0].dtype, device=bottoms[0].data.device)
            off = 0
            for b in bottoms:
                o, A, i = _oai(b.data, ax)
                lh.axis_copy(b.data, out, o, A, shape[ax], i, 0, off, A)
                off += A
            tops[0].data = out
            return
        tops[0].data = torch.cat([b.data for b in bottoms], dim=ax)

    def backward(self, tops, propagate_down, bottoms):
        ax = _phys_axis(bottoms[0], self.axis)
        if self.zero_copy_bwd and tops[0].diff.is_cuda and tops[0].diff.is_contiguous():
            # the output's consumers already applied the parts' ReLU masks: each part's
            # gradient is a channel-slice view of the output gradient (the producing
            # convolution reads it in place with the slice's pixel stride)
            top_d = tops[0].diff
            for i, (b, (off, c)) in enumerate(zip(bottoms, self.zero_copy.spans)):
                if propagate_down[i]:
                    b.diff = top_d[..., off:off + c]
            return
        gates = [i in self.relu_gate_parts for i in range(len(bottoms))]
        if len(bottoms) > 1 and self._hip_ok(bottoms, ax):
            from ..ops import hip
            diffs = [torch.empty_like(b.data) if propagate_down[i] else None for i, b in enumerate(bottoms)]
            hip.concat_channels_bwd(tops[0].diff, diffs, [b.data if g and d is not None else None
                                                         for b, g, d in zip(bottoms, gates, diffs)],
                                    [b.data.shape[-1] for b in bottoms])
            for b, d in zip(bottoms, diffs):
                if d is not None:
                    b.diff = d
            return
        off = 0
        top_d = tops[0].diff
        for i, b in enumerate(bottoms):
            n = b.shape[self.axis]
            if propagate_down[i]:
                if top_d.is_cuda:
                    o, A, inner = _oai(top_d, ax)
                    d = torch.empty_like(b.data)
                    _lh().axis_copy(top_d, d, o, A, n, inner, off, 0, n)
                    b.diff = ops.relu_backward(d, b.data) if gates[i] else d
                else:
                    d = top_d.narrow(ax, off, n)
                    b.diff = (d * (b.data > 0).to(d.dtype)) if gates[i] else d.contiguous()
            off += n


class ConcatSlots:
    """Zero-copy channel concat (engine.fuse_concat): the producing convolutions write their
    outputs straight into channel slices [off, off + c) of one NHWC buffer — Caffe copies
    every part (concat_layer.cu:9-25).  The buffer is allocated by the first producer of
    an iteration and handed to the Concat layer's output by take()."""

    def __init__(self, chans):
        self.spans, off = [], 0
        for c in chans:
            self.spans.append((off, c))
            off += c
        self.total = off
        self.buf = None

    def slot(self, part: int, nhw, device) -> torch.Tensor:
        nhw = tuple(int(v) for v in nhw)
        if self.buf is None or tuple(self.buf.shape[:3]) != nhw or self.buf.device != device:
            self.buf = torch.empty(nhw + (self.total,), dtype=torch.bfloat16, device=device)
        off, c = self.spans[part]
        return self.buf[..., off:off + c]

    def take(self):
        b, self.buf = self.buf, None
        return b

    def holds(self, parts, buf) -> bool:
        return all(p.dim() == 4 and p.data_ptr() == buf.data_ptr() + 2 * off and p.shape[-1] == c
                   and p.stride(2) == self.total for p, (off, c) in zip(parts, self.spans))


@register("Slice")
class SliceLayer(Layer):
    exact_bottoms = 1
    min_tops = 1

    def layer_setup(self, bottoms, tops):
        p = self.lp.slice_param
        self.axis = bottoms[0].canonical_axis(p.axis if p.HasField("axis") or not p.HasField("slice_dim")
                                              else p.slice_dim)
        self.points = list(p.slice_point)

    def _sizes(self, bottom, n):
        total = bottom.shape[self.axis]
        if self.points:
            if len(self.points) != n - 1:
                raise ValueError("Slice: need num_tops - 1 slice points")
            b = [0] + self.points + [total]
            return [b[i + 1] - b[i] for i in range(n)]
        if total % n:
            raise ValueError("Slice: axis not divisible by the number of tops")
        return [total // n] * n

    def reshape(self, bottoms, tops):
        self.sizes = self._sizes(bottoms[0], len(tops))
        for t, s in zip(tops, self.sizes):
            shape = list(bottoms[0].shape)
            shape[self.axis] = s
            t.reshape(tuple(shape), bottoms[0].dtype)

    def forward(self, bottoms, tops):
        ax = _phys_axis(bottoms[0], self.axis)
        x = bottoms[0].data
        off = 0
        for t, s in zip(tops, self.sizes):
            if x.is_cuda:
                o, A, i = _oai(x, ax)
                y = torch.empty(t.data.shape, dtype=x.dtype, device=x.device)
                _lh().axis_copy(x, y, o, A, s, i, off, 0, s)
                t.data = y
            else:
                t.data = x.narrow(ax, off, s).contiguous()
            off += s

    def backward(self, tops, propagate_down, bottoms):
        if not propagate_down[0]:
            return
        ax = _phys_axis(bottoms[0], self.axis)
        if tops[0].diff.is_cuda:
            g = torch.empty_like(bottoms[0].data)
            o, A, i = _oai(g, ax)
            off = 0
            for t, s in zip(tops, self.sizes):
                _lh().axis_copy(t.diff, g, o, s, A, i, 0, off, s)
                off += s
            bottoms[0].diff = g
            return
        bottoms[0].diff = torch.cat([t.diff for t in tops], dim=ax)


@register("Eltwise")
class EltwiseLayer(Layer):
    min_bottoms = 2
    exact_tops = 1

    def layer_setup(self, bottoms, tops):
        p = self.lp.eltwise_param
        self.op = int(p.operation)  # PROD=0 SUM=1 MAX=2
        self.coeff = list(p.coeff) or [1.0] * len(bottoms)
        if len(self.coeff) != len(bottoms):
            raise ValueError("Eltwise: one coefficient per bottom")
        if self.op != 1 and p.coeff:
            raise ValueError("Eltwise: coefficients only for SUM")
        self.stable = p.stable_prod_grad

    def reshape(self, bottoms, tops):
        for b in bottoms[1:]:
            if b.shape != bottoms[0].shape:
                raise ValueError("Eltwise: bottoms must have the same shape")
        tops[0].reshape(bottoms[0].shape, bottoms[0].dtype)

    def _gpu_inputs(self, bottoms):
        # an in-place top aliases bottom 0: keep the inputs the backward needs
        return [b.data for b in bottoms]

    def forward(self, bottoms, tops):
        if bottoms[0].data.is_cuda:
            lh = _lh()
            xs = [b.data for b in bottoms]
            if len(xs) > 16:
                raise ValueError("Eltwise on the GPU supports at most 16 bottoms")
            if tops[0] is bottoms[0] and self.op == 0:
                xs = [x.clone() for x in xs]
            y, self.mask = lh.eltwise_fwd(self.op, xs, self.coeff)
            self._xs = xs
            tops[0].data = y
            return
        xs = [b.data.float() for b in bottoms]
        if self.op == 0:
            y = xs[0]
            for x in xs[1:]:
                y = y * x
        elif self.op == 1:
            y = xs[0] * self.coeff[0]
            for c, x in zip(self.coeff[1:], xs[1:]):
                y = y + c * x
        else:
            st = torch.stack(xs)
            y, self.argmax = st.max(0)
        self._xs = xs
        tops[0].data = y.to(tops[0].dtype)

    def backward(self, tops, propagate_down, bottoms):
        if tops[0].diff.is_cuda:
            lh = _lh()
            dy, y = tops[0].diff, tops[0].data
            grads = [lh.eltwise_bwd(self.op, self._xs, self.coeff, i, self.stable, y, dy, self.mask)
                     if propagate_down[i] else None for i in range(len(bottoms))]
            for b, g in zip(bottoms, grads):
                if g is not None:
                    b.diff = g
            return
        dy = tops[0].diff.float()
        y = tops[0].data.float()
        for i, b in enumerate(bottoms):
            if not propagate_down[i]:
                continue
            if self.op == 0:
                if self.stable:
                    g = torch.ones_like(dy)
                    for j, x in enumerate(self._xs):
                        if j != i:
                            g = g * x
                else:
                    g = y / self._xs[i]
                g = g * dy
            elif self.op == 1:
                g = dy * self.coeff[i]
            else:
                g = dy * (self.argmax == i).float()
            b.diff = g.to(b.dtype)


@register("Flatten")
class FlattenLayer(Layer):
    exact_bottoms = 1
    exact_tops = 1

    def reshape(self, bottoms, tops):
        p = self.lp.flatten_param
        b = bottoms[0]
        s = b.canonical_axis(p.axis)
        e = b.canonical_axis(p.end_axis)
        shape = b.shape[:s] + (b.count_range(s, e + 1),) + b.shape[e + 1:]
        tops[0].reshape(shape, b.dtype)

    def forward(self, bottoms, tops):
        _logical_copy(bottoms[0], tops[0])

    def backward(self, tops, propagate_down, bottoms):
        if propagate_down[0]:
            _logical_copy_diff(tops[0], bottoms[0])


def _logical_copy(b, t):
    if b.data.is_cuda:
        if not b.is_image and not t.is_image:
            t.data = b.data.view(t.data.shape)  # Caffe ShareData: no copy
        else:
            t.data = _from_logical(_to_logical(b), t)
        return
    logical = b.nchw().contiguous().reshape(t.shape)
    t.data = logical.permute(0, 2, 3, 1).contiguous() if t.is_image else logical


def _logical_copy_diff(t, b):
    if t.diff.is_cuda:
        if not b.is_image and not t.is_image:
            b.diff = t.diff.view(b.data.shape)  # Caffe ShareDiff
        else:
            b.diff = _from_logical(_to_logical(t, diff=True), b)
        return
    logical = t.nchw(diff=True).contiguous().reshape(b.shape)
    b.diff = logical.permute(0, 2, 3, 1).contiguous() if b.is_image else logical


@register("Reshape")
class ReshapeLayer(Layer):
    exact_bottoms = 1
    exact_tops = 1

    def reshape(self, bottoms, tops):
        p = self.lp.reshape_param
        b = bottoms[0]
        axis = b.canonical_axis(p.axis) if p.axis >= 0 else len(b.shape) + 1 + p.axis
        end = len(b.shape) if p.num_axes == -1 else axis + p.num_axes
        dims = list(p.shape.dim)
        out = []
        infer = -1
        for i, d in enumerate(dims):
            if d == 0:
                out.append(b.shape[axis + i])
            elif d == -1:
                infer = len(out)
                out.append(1)
            else:
                out.append(int(d))
        shape = list(b.shape[:axis]) + out + list(b.shape[end:])
        if infer >= 0:
            known = 1
            for i, v in enumerate(shape):
                if i != axis + infer:
                    known *= v
            shape[axis + infer] = b.count // known
        tops[0].reshape(tuple(shape), b.dtype)

    def forward(self, bottoms, tops):
        _logical_copy(bottoms[0], tops[0])

    def backward(self, tops, propagate_down, bottoms):
        if propagate_down[0]:
            _logical_copy_diff(tops[0], bottoms[0])


@register("Silence")
class SilenceLayer(Layer):
    min_bottoms = 1
    exact_tops = 0

    def reshape(self, bottoms, tops):
        pass

    def forward(self, bottoms, tops):
        pass

    def backward(self, tops, propagate_down, bottoms):
        for i, b in enumerate(bottoms):
            if propagate_down[i]:
                b.diff = torch.zeros_like(b.data)


@register("Tile")
class TileLayer(Layer):
    exact_bottoms = 1
    exact_tops = 1

    def reshape(self, bottoms, tops):
        p = self.lp.tile_param
        b = bottoms[0]
        self.axis = b.canonical_axis(p.axis)
        self.tiles = int(p.tiles)
        shape = list(b.shape)
        shape[self.axis] *= self.tiles
        tops[0].reshape(tuple(shape), b.dtype)

    def forward(self, bottoms, tops):
        b, t = bottoms[0], tops[0]
        if b.data.is_cuda:
            ax = _phys_axis(b, self.axis)
            x = b.data
            o, A, i = _oai(x, ax)
            y = torch.empty(t.data.shape, dtype=x.dtype, device=x.device)
            for k in range(self.tiles):
                _lh().axis_copy(x, y, o, A, A * self.tiles, i, 0, k * A, A)
            t.data = y
            return
        x = bottoms[0].nchw()
        reps = [1] * x.dim()
        reps[self.axis] = self.tiles
        y = x.repeat(*reps)
        t = tops[0]
        t.data = y.permute(0, 2, 3, 1).contiguous() if t.is_image else y

    def backward(self, tops, propagate_down, bottoms):
        if propagate_down[0] and tops[0].diff.is_cuda:
            b = bottoms[0]
            ax = _phys_axis(b, self.axis)
            o, A, i = _oai(b.data, ax)
            b.diff = _lh().tile_bwd(tops[0].diff, o, A, i, self.tiles, b.data.shape)
            return
        if propagate_down[0]:
            b = bottoms[0]
            d = tops[0].nchw(diff=True).float()
            shp = list(b.shape)
            d = d.reshape(shp[:self.axis] + [self.tiles, shp[self.axis]] + shp[self.axis + 1:]).sum(self.axis)
            b.diff = (d.permute(0, 2, 3, 1).contiguous() if b.is_image else d).to(b.dtype)


@register("Reduction")
class ReductionLayer(Layer):
    exact_bottoms = 1
    exact_tops = 1

    def reshape(self, bottoms, tops):
        p = self.lp.reduction_param
        b = bottoms[0]
        self.axis = b.canonical_axis(p.axis)
        self.op, self.coeff = int(p.operation), float(p.coeff)
        tops[0].reshape(b.shape[:self.axis], torch.float32)

    def _gpu_segments(self, b, diff=False):
        """(logical-order tensor or physical, segs, L): image blobs reduced over axes >= 2
        are converted to NCHW first (their segments are not contiguous in NHWC)."""
        segs = b.count_range(0, self.axis)
        L = b.count // max(segs, 1)
        t = b.diff if diff else b.data
        if b.is_image and self.axis >= 2:
            return _to_logical(b, diff), segs, L, True
        return t, segs, L, False

    def forward(self, bottoms, tops):
        b = bottoms[0]
        if b.data.is_cuda:
            lh = _lh()
            x, segs, L, _ = self._gpu_segments(b)
            mode = {1: lh.RED_SUM, 2: lh.RED_ABS, 3: lh.RED_SQ, 4: lh.RED_SUM}[self.op]
            scale = self.coeff / L if self.op == 4 else self.coeff
            out = lh.axis_reduce(mode, x, None, 1, 1, segs, L, scale=scale)
            tops[0].data = out.reshape(tops[0].data.shape)
            return
        x = bottoms[0].nchw().float()
        x = x.reshape(x.shape[:self.axis] + (-1,)) if self.axis < x.dim() else x
        if self.op == 1:
            y = x.sum(-1)
        elif self.op == 2:
            y = x.abs().sum(-1)
        elif self.op == 3:
            y = (x * x).sum(-1)
        else:
            y = x.mean(-1)
        tops[0].data = (y * self.coeff).reshape(tops[0].data.shape)

    def backward(self, tops, propagate_down, bottoms):
        if not propagate_down[0]:
            return
        b = bottoms[0]
        if b.data.is_cuda:
            lh = _lh()
            x, segs, L, logical = self._gpu_segments(b)
            g = lh.reduction_bwd(x, tops[0].diff.reshape(-1), segs, L, self.op, self.coeff)
            b.diff = _from_logical(g, b) if logical else g.reshape(b.data.shape)
            return
        x = b.nchw().float().reshape(b.shape[:self.axis] + (-1,))
        dy = tops[0].diff.float().reshape(b.shape[:self.axis] + (1,)) * self.coeff
        if self.op == 1:
            g = dy.expand_as(x)
        elif self.op == 2:
            g = dy * torch.sign(x)
        elif self.op == 3:
            g = dy * 2 * x
        else:
            g = dy.expand_as(x) / x.shape[-1]
        g = g.reshape(b.shape)
        b.diff = (g.permute(0, 2, 3, 1).contiguous() if b.is_image else g).to(b.dtype)


@register("ArgMax")
class ArgMaxLayer(Layer):
    exact_bottoms = 1
    exact_tops = 1

    def layer_setup(self, bottoms, tops):
        p = self.lp.argmax_param
        self.top_k, self.out_max_val = int(p.top_k), p.out_max_val
        self.axis = bottoms[0].canonical_axis(p.axis) if p.HasField("axis") else None

    def reshape(self, bottoms, tops):
        b = bottoms[0]
        if self.axis is None:
            shape = (b.shape[0], 2 if self.out_max_val else 1, self.top_k)
        else:
            shape = list(b.shape)
            shape[self.axis] = self.top_k
            shape = tuple(shape)
        tops[0].reshape(shape, torch.float32)

    def forward(self, bottoms, tops):
        b, t = bottoms[0], tops[0]
        if b.data.is_cuda:
            lh = _lh()
            x = _to_logical(b)  # indices refer to Caffe's logical (C, H, W) order
            if self.axis is None:
                out = lh.topk(x, b.shape[0], b.count // b.shape[0], 1, self.top_k, self.out_max_val, 0,
                              t.data.shape)
            else:
                outer = b.count_range(0, self.axis)
                inner = b.count_range(self.axis + 1)
                lshape = list(b.shape)
                lshape[self.axis] = self.top_k
                out = lh.topk(x, outer, b.shape[self.axis], inner, self.top_k, self.out_max_val, 1, lshape)
                out = _from_logical(out, t)
            t.data = out
            return
        x = bottoms[0].nchw().float()
        if self.axis is None:
            x2 = x.reshape(x.shape[0], -1)
            v, i = x2.topk(self.top_k, dim=1)
            y = torch.stack([i.float(), v], 1) if self.out_max_val else i.float()[:, None, :]
        else:
            v, i = x.topk(self.top_k, dim=self.axis)
            y = v if self.out_max_val else i.float()
        t = tops[0]
        t.data = y.permute(0, 2, 3, 1).contiguous() if t.is_image else y.reshape(t.data.shape)


@register("BatchReindex")
class BatchReindexLayer(Layer):
    exact_bottoms = 2
    exact_tops = 1

    def reshape(self, bottoms, tops):
        tops[0].reshape((bottoms[1].count,) + bottoms[0].shape[1:], bottoms[0].dtype)

    def forward(self, bottoms, tops):
        x = bottoms[0].data
        if x.is_cuda:
            self.idx = bottoms[1].data.reshape(-1).float()
            row = x.numel() // max(x.shape[0], 1)
            tops[0].data = _lh().gather_rows(x, self.idx, self.idx.numel(), row, tops[0].data.shape)
            return
        self.idx = bottoms[1].data.reshape(-1).long()
        tops[0].data = bottoms[0].data.index_select(0, self.idx)

    def backward(self, tops, propagate_down, bottoms):
        if propagate_down[0] and tops[0].diff.is_cuda:
            x = bottoms[0].data
            g = torch.empty_like(x)
            row = x.numel() // max(x.shape[0], 1)
            bottoms[0].diff = _lh().index_add_rows(tops[0].diff, self.idx, x.shape[0], row, g, acc=False)
            return
        if propagate_down[0]:
            g = torch.zeros(bottoms[0].data.shape, dtype=torch.float32, device=self.device)
            g.index_add_(0, self.idx, tops[0].diff.float())
            bottoms[0].diff = g.to(bottoms[0].dtype)


@register("Filter")
class FilterLayer(Layer):
    min_bottoms = 2
    min_tops = 1

    def _host_index(self, bottoms):
        """Selected row indices, read on the host like Caffe's FilterLayer::Reshape
        (filter_layer.cpp:42-62 reads the selector blob's cpu_data)."""
        sel = bottoms[-1].data.reshape(-1).detach().float().cpu()
        return [i for i, v in enumerate(sel.tolist()) if v != 0]

    def reshape(self, bottoms, tops):
        n = len(self._host_index(bottoms)) if bottoms[-1].count else 0
        for b, t in zip(bottoms[:-1], tops):
            t.reshape((n,) + b.shape[1:], b.dtype)

    def forward(self, bottoms, tops):
        host = self._host_index(bottoms)
        if bottoms[0].data.is_cuda:
            self.idx = torch.tensor(host, dtype=torch.int32).to(bottoms[0].data.device, non_blocking=True)
            for b, t in zip(bottoms[:-1], tops):
                t.reshape((len(host),) + b.shape[1:], b.dtype)
                row = b.data.numel() // max(b.data.shape[0], 1)
                t.data = _lh().gather_rows(b.data, self.idx, len(host), row, t.data.shape)
            return
        self.idx = torch.tensor(host, dtype=torch.long)
        for b, t in zip(bottoms[:-1], tops):
            t.reshape((len(self.idx),) + b.shape[1:], b.dtype)
            t.data = b.data.index_select(0, self.idx)

    def backward(self, tops, propagate_down, bottoms):
        for i, (b, t) in enumerate(zip(bottoms[:-1], tops)):
            if propagate_down[i] and t.diff.is_cuda:
                row = b.data.numel() // max(b.data.shape[0], 1)
                b.diff = _lh().index_add_rows(t.diff, self.idx, b.data.shape[0], row, torch.empty_like(b.data),
                                              acc=False)
            elif propagate_down[i]:
                g = torch.zeros_like(b.data)
                g.index_copy_(0, self.idx, t.diff)
                b.diff = g


@register("Embed")
class EmbedLayer(Layer):
    exact_bottoms = 1
    exact_tops = 1

    def layer_setup(self, bottoms, tops):
        p = self.lp.embed_param
        self.N, self.K = int(p.num_output), int(p.input_dim)
        self.weight = self.add_param((self.K, self.N), filler=p.weight_filler if p.HasField("weight_filler") else None)
        self.bias = None
        if p.bias_term:
            self.bias = self.add_param((self.N,), filler=p.bias_filler if p.HasField("bias_filler") else None)

    def reshape(self, bottoms, tops):
        tops[0].reshape(bottoms[0].shape + (self.N,), self.dtype)

    def forward(self, bottoms, tops):
        if bottoms[0].data.is_cuda:
            self.idx = bottoms[0].data.reshape(-1).float()
            tops[0].data = _lh().gather_rows(self.weight.data, self.idx, self.idx.numel(), self.N, tops[0].data.shape,
                                             bias=self.bias.data if self.bias is not None else None,
                                             out_dtype=self.dtype)
            return
        self.idx = bottoms[0].data.reshape(-1).long()
        y = self.weight.data.index_select(0, self.idx)
        if self.bias is not None:
            y = y + self.bias.data
        tops[0].data = y.reshape(tops[0].data.shape).to(self.dtype)

    def backward(self, tops, propagate_down, bottoms):
        if tops[0].diff.is_cuda:
            lh = _lh()
            dy = tops[0].diff
            if self.param_grads_needed(0):
                lh.index_add_rows(dy, self.idx, self.K, self.N, self.weight.diff, acc=True)
            if self.bias is not None and self.param_grads_needed(1):
                lh.axis_reduce(lh.RED_SUM, dy, None, 1, self.idx.numel(), self.N, 1, out=self.bias.diff, acc=True)
            return
        dy = tops[0].diff.float().reshape(-1, self.N)
        if self.param_grads_needed(0):
            self.weight.diff.index_add_(0, self.idx, dy)
        if self.bias is not None and self.param_grads_needed(1):
            self.bias.diff += dy.sum(0)


@register("MVN")
class MVNLayer(Layer):
    exact_bottoms = 1
    exact_tops = 1

    def reshape(self, bottoms, tops):
        tops[0].reshape(bottoms[0].shape, bottoms[0].dtype)

    def _dims(self, x):
        """Reduction dims of one statistic group (mvn_layer.cpp: num = N, or N*C per channel;
        dim = count / num)."""
        p = self.lp.mvn_param
        if x.dim() == 4:
            return (1, 2, 3) if p.across_channels else (1, 2)  # NHWC: spatial dims 1,2 (+channel 3)
        return tuple(range(1, x.dim())) if p.across_channels else tuple(range(2, x.dim()))

    @staticmethod
    def _mean(x, dims):
        return x.mean(dim=dims, keepdim=True) if dims else x  # dim = 1: each element its own group

    def _gpu_geom(self, x):
        """[B][outer][A][inner] of the per-statistic groups: (n, c) over (h, w) in NHWC, or
        n over everything when across_channels (2-D blobs: n over c)."""
        p = self.lp.mvn_param
        N = x.shape[0]
        if x.dim() == 4 and not p.across_channels:
            return N, x.shape[1] * x.shape[2], x.shape[3], 1
        if x.dim() != 4 and not p.across_channels and x.dim() > 1:
            inner = x.numel() // (N * x.shape[1])
            return N, 1, x.shape[1], inner
        return N, 1, 1, x.numel() // N

    def forward(self, bottoms, tops):
        p = self.lp.mvn_param
        if bottoms[0].data.is_cuda:
            lh = _lh()
            x = bottoms[0].data
            B, outer, A, inner = self._gpu_geom(x)
            self.geom = (B, outer, A, inner)
            if p.normalize_variance:
                mean, _, inv = lh.mean_var(x, B, outer, A, inner, p.eps, 1)
            else:
                s1 = lh.axis_reduce(lh.RED_SUM, x, None, B, outer, A, inner)
                mean, _, inv = lh.stats_finalize(s1, None, outer * inner, p.eps, 2)
            self.inv = inv if p.normalize_variance else None
            y = lh.chan_affine(x, mean, self.inv, outer, A, inner)
            self.y = y
            tops[0].data = y
            return
        x = bottoms[0].data.float()
        dims = self._dims(x)
        xm = x - self._mean(x, dims)
        if p.normalize_variance:
            self.std = torch.sqrt(self._mean(xm * xm, dims)) + p.eps
            y = xm / self.std
        else:
            y = xm
        self.y = y
        tops[0].data = y.to(tops[0].dtype)

    def backward(self, tops, propagate_down, bottoms):
        if not propagate_down[0]:
            return
        p = self.lp.mvn_param
        if tops[0].diff.is_cuda:
            lh = _lh()
            B, outer, A, inner = self.geom
            dy = tops[0].diff
            cnt = outer * inner
            m1 = lh.axis_reduce(lh.RED_SUM, dy, None, B, outer, A, inner, scale=1.0 / cnt)
            m2 = (lh.axis_reduce(lh.RED_DOT, dy, self.y, B, outer, A, inner, scale=1.0 / cnt)
                  if p.normalize_variance else None)
            bottoms[0].diff = lh.norm_bwd(dy, self.y if p.normalize_variance else None, m1, m2, self.inv,
                                          outer, A, inner)
            return
        dy = tops[0].diff.float()
        dims = self._dims(dy)
        if p.normalize_variance:
            y = self.y
            g = dy - self._mean(dy, dims) - y * self._mean(dy * y, dims)
            g = g / self.std
        else:
            g = dy - self._mean(dy, dims)
        bottoms[0].diff = g.to(bottoms[0].dtype)


@register("BatchNorm")
class BatchNormLayer(Layer):
    """batch_norm_layer.cpp: normalisation only (no scale/shift), 3 param blobs
    (running mean, running variance, moving-average factor) with lr_mult forced to 0."""
    exact_bottoms = 1
    exact_tops = 1

    def layer_setup(self, bottoms, tops):
        p = self.lp.batch_norm_param
        C = bottoms[0].shape[1]
        self.use_global = p.use_global_stats if p.HasField("use_global_stats") else (self.phase == 1)
        self.frac, self.eps = float(p.moving_average_fraction), float(p.eps)
        self.mean = self.add_param((C,))
        self.var = self.add_param((C,))
        self.factor = self.add_param((1,))
        for ps in range(3):
            if ps >= len(self.lp.param):
                spec = self.lp.param.add()
                spec.lr_mult = 0.0

    def reshape(self, bottoms, tops):
        tops[0].reshape(bottoms[0].shape, bottoms[0].dtype)

    def _red(self, x):
        return tuple(range(x.dim() - 1)) if x.dim() == 4 else tuple(d for d in range(x.dim()) if d != 1)

    def _bc(self, v, x):
        return v.reshape(1, 1, 1, -1) if x.dim() == 4 else v.reshape([1, -1] + [1] * (x.dim() - 2))

    def _gpu_geom(self, x):
        if x.dim() == 4:
            return x.numel() // x.shape[3], x.shape[3], 1
        inner = x.numel() // (x.shape[0] * x.shape[1]) if x.dim() > 1 else 1
        return x.shape[0], x.shape[1] if x.dim() > 1 else 1, inner

    def forward(self, bottoms, tops):
        if bottoms[0].data.is_cuda:
            lh = _lh()
            x = bottoms[0].data
            outer, C_, inner = self._gpu_geom(x)
            self.geom = (outer, C_, inner)
            if self.use_global:
                mean, self.inv_std = lh.bn_global(self.mean.data, self.var.data, self.factor.data, self.eps)
            else:
                mean, var, self.inv_std = lh.mean_var(x, 1, outer, C_, inner, self.eps, 0)
                m = outer * inner
                lh.bn_running(self.mean.data, self.var.data, self.factor.data, mean, var, self.frac,
                              m / max(m - 1, 1))
            y = lh.chan_affine(x, mean, self.inv_std, outer, C_, inner)
            self.xhat = y
            tops[0].data = y
            return
        x = bottoms[0].data.float()
        if self.use_global:
            f = self.factor.data.reshape(())
            s = 0.0 if float(f) == 0 else 1.0 / float(f)
            mean, var = self.mean.data * s, self.var.data * s
        else:
            dims = self._red(x)
            mean = x.mean(dim=dims)
            var = ((x - self._bc(mean, x)) ** 2).mean(dim=dims)
            m = x.numel() // x.shape[-1 if x.dim() == 4 else 1]
            with torch.no_grad():
                self.factor.data.mul_(self.frac).add_(1.0)
                self.mean.data.mul_(self.frac).add_(mean)
                self.var.data.mul_(self.frac).add_(var * (m / max(m - 1, 1)))
        self.inv_std = 1.0 / torch.sqrt(var + self.eps)
        self.xhat = (x - self._bc(mean, x)) * self._bc(self.inv_std, x)
        tops[0].data = self.xhat.to(tops[0].dtype)

    def backward(self, tops, propagate_down, bottoms):
        if not propagate_down[0]:
            return
        if tops[0].diff.is_cuda:
            lh = _lh()
            outer, C_, inner = self.geom
            dy = tops[0].diff
            if self.use_global:
                bottoms[0].diff = lh.norm_bwd(dy, None, None, None, self.inv_std, outer, C_, inner)
                return
            cnt = outer * inner
            m1 = lh.axis_reduce(lh.RED_SUM, dy, None, 1, outer, C_, inner, scale=1.0 / cnt)
            m2 = lh.axis_reduce(lh.RED_DOT, dy, self.xhat, 1, outer, C_, inner, scale=1.0 / cnt)
            bottoms[0].diff = lh.norm_bwd(dy, self.xhat, m1, m2, self.inv_std, outer, C_, inner)
            return
        dy = tops[0].diff.float()
        if self.use_global:
            g = dy * self._bc(self.inv_std, dy)
        else:
            dims = self._red(dy)
            xh = self.xhat
            g = (dy - self._bc(dy.mean(dim=dims), dy) - xh * self._bc((dy * xh).mean(dim=dims), dy))
            g = g * self._bc(self.inv_std, dy)
        bottoms[0].diff = g.to(bottoms[0].dtype)


@register("SPP")
class SPPLayer(Layer):
    """Spatial pyramid pooling (spp_layer.cpp): concat of flattened poolings at levels
    2^l x 2^l bins."""
    exact_bottoms = 1
    exact_tops = 1

    def layer_setup(self, bottoms, tops):
        p = self.lp.spp_param
        self.height = int(p.pyramid_height)
        self.method = int(p.pool)

    def _specs(self, b):
        from ..ops.spec import PoolSpec
        import math
        N, C, H, W = b.shape
        out = []
        for l in range(self.height):
            bins = 2 ** l
            kh, kw = math.ceil(H / bins), math.ceil(W / bins)
            ph, pw = (kh * bins - H + 1) // 2, (kw * bins - W + 1) // 2
            out.append(PoolSpec(N, H, W, C, kh, kw, kh, kw, ph, pw, self.method))
        return out

    def reshape(self, bottoms, tops):
        b = bottoms[0]
        total = sum(s.C * s.P * s.Q for s in self._specs(b))
        tops[0].reshape((b.shape[0], total), b.dtype)

    def forward(self, bottoms, tops):
        from .. import ops
        b = bottoms[0]
        if b.data.is_cuda:
            # each level: HIP pooling (NHWC), then its NCHW-flattened bins copied into the
            # level's column range of the top
            lh = _lh()
            N = b.shape[0]
            total = tops[0].shape[1]
            y = torch.empty((N, total), dtype=tops[0].dtype, device=b.data.device)
            self.aux = []
            off = 0
            for s in self._specs(b):
                p, aux = ops.pool_forward_aux(b.data, s)
                self.aux.append(aux)
                n = s.C * s.P * s.Q
                flat = lh.nhwc_to_nchw(p).reshape(N, n)
                lh.axis_copy(flat, y, N, n, total, 1, 0, off, n)
                off += n
            tops[0].data = y
            return
        outs = []
        for s in self._specs(b):
            y = ops.ref.pool_forward(b.data.float(), s)  # NHWC
            outs.append(y.permute(0, 3, 1, 2).reshape(b.shape[0], -1))
        tops[0].data = torch.cat(outs, 1).to(tops[0].dtype)

    def backward(self, tops, propagate_down, bottoms):
        if not propagate_down[0]:
            return
        from .. import ops
        b = bottoms[0]
        if b.data.is_cuda:
            lh = _lh()
            N = b.shape[0]
            total = tops[0].shape[1]
            grads = []
            off = 0
            for s, aux in zip(self._specs(b), self.aux):
                n = s.C * s.P * s.Q
                d = torch.empty((N, n), dtype=b.data.dtype, device=b.data.device)
                lh.axis_copy(tops[0].diff, d, N, total, n, 1, off, 0, n)
                dy = lh.nchw_to_nhwc(d.reshape(N, s.C, s.P * s.Q), N, s.C, s.P, s.Q)
                grads.append(ops.pool_backward(dy, b.data, s, aux))
                off += n
            b.diff = grads[0] if len(grads) == 1 else _eltwise_sum_gpu(grads)
            return
        g = torch.zeros(b.data.shape, dtype=torch.float32, device=self.device)
        off = 0
        for s in self._specs(b):
            n = s.C * s.P * s.Q
            dy = tops[0].diff[:, off:off + n].float().reshape(b.shape[0], s.C, s.P, s.Q).permute(0, 2, 3, 1)
            g += ops.ref.pool_backward(dy, b.data.float(), s)
            off += n
        b.diff = g.to(b.dtype)


@register("Python")
class PythonLayer(Layer):
    """User-defined layer in Python (caffe/include/caffe/python_layer.hpp:14,
    layer_factory.cpp:202-214): ``python_param { module: "m" layer: "Cls" param_str: "..." }``
    imports ``m.Cls`` and drives it with pycaffe's Layer protocol — ``setup(bottom, top)``,
    ``reshape(bottom, top)``, ``forward(bottom, top)``, ``backward(top, propagate_down,
    bottom)`` — where bottom / top are this engine's blobs (``.data`` / ``.diff`` tensors,
    ``.reshape(shape)``) and ``self.param_str`` holds the string parameter."""

    def layer_setup(self, bottoms, tops):
        import importlib
        pp = self.lp.python_param
        if not pp.module or not pp.layer:
            raise ValueError(f"Python layer {self.name!r} needs python_param.module and .layer")
        cls = getattr(importlib.import_module(pp.module), pp.layer)
        self.impl = cls()
        self.impl.param_str = pp.param_str
        self.impl.phase = self.phase
        if hasattr(self.impl, "setup"):
            self.impl.setup(bottoms, tops)

    def reshape(self, bottoms, tops):
        self.impl.reshape(bottoms, tops)

    def forward(self, bottoms, tops):
        self.impl.forward(bottoms, tops)

    def backward(self, tops, propagate_down, bottoms):
        if hasattr(self.impl, "backward"):
            self.impl.backward(tops, list(propagate_down), bottoms)
