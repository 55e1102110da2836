"""Structural layers: Split, Concat, Slice, Eltwise, Flatten, Reshape, Silence, Tile,
Reduction, ArgMax, BatchReindex, Filter, Embed, MVN, BatchNorm, SPP.

References: caffe/src/caffe/layers/{split,concat,slice,eltwise,flatten,reshape,silence,
tile,reduction,argmax,batch_reindex,filter,embed,mvn,batch_norm,spp}_layer.*.

Channel-axis operations on 4-D blobs (Concat/Slice along axis 1) act on the physical
last axis of the NHWC storage.  Flatten/Reshape keep Caffe's logical (C, H, W) order by
converting through the NCHW view.
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
        acc = d0.float() if d0.dtype != torch.float32 else d0.clone()
        for d in diffs[1:]:
            acc = acc + d.float()
        bottoms[0].diff = acc.to(bottoms[0].dtype)


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

    def _hip_ok(self, bottoms, ax) -> bool:
        """One-launch HIP path: channel concat of NHWC bf16 device blobs, <= 8 parts."""
        b0 = bottoms[0].data
        return (b0.is_cuda and b0.dtype == torch.bfloat16 and ax == b0.dim() - 1 and len(bottoms) <= 8
                and all(b.data.shape[-1] % 8 == 0 for b in bottoms))

    def forward(self, bottoms, tops):
        if len(bottoms) == 1:
            tops[0].data = bottoms[0].data
            return
        ax = _phys_axis(bottoms[0], self.axis)
        if self._hip_ok(bottoms, ax):
            from ..ops import hip
            shape = list(bottoms[0].data.shape)
            shape[-1] = sum(b.data.shape[-1] for b in bottoms)
            out = torch.empty(shape, dtype=torch.bfloat16, device=bottoms[0].data.device)
            tops[0].data = hip.concat_channels([b.data for b in bottoms], out)
            return
        tops[0].data = torch.cat([b.data for b in bottoms], dim=ax)

    def backward(self, tops, propagate_down, bottoms):
        ax = _phys_axis(bottoms[0], self.axis)
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
        for i, b in enumerate(bottoms):
            n = b.shape[self.axis]
            if propagate_down[i]:
                d = tops[0].diff.narrow(ax, off, n)
                b.diff = (d * (b.data > 0).to(d.dtype)) if gates[i] else d.contiguous()
            off += n


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
        off = 0
        for t, s in zip(tops, self.sizes):
            t.data = bottoms[0].data.narrow(ax, off, s).contiguous()
            off += s

    def backward(self, tops, propagate_down, bottoms):
        if propagate_down[0]:
            ax = _phys_axis(bottoms[0], self.axis)
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

    def forward(self, bottoms, tops):
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
    logical = b.nchw().contiguous().reshape(t.shape)
    t.data = logical.permute(0, 2, 3, 1).contiguous() if t.is_image else logical


def _logical_copy_diff(t, b):
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
        b, t = bottoms[0], tops[0]
        logical = b.nchw().contiguous().reshape(t.shape)
        t.data = logical.permute(0, 2, 3, 1).contiguous() if t.is_image else logical

    def backward(self, tops, propagate_down, bottoms):
        if propagate_down[0]:
            b, t = bottoms[0], tops[0]
            logical = t.nchw(diff=True).contiguous().reshape(b.shape)
            b.diff = logical.permute(0, 2, 3, 1).contiguous() if b.is_image else logical


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
        x = bottoms[0].nchw()
        reps = [1] * x.dim()
        reps[self.axis] = self.tiles
        y = x.repeat(*reps)
        t = tops[0]
        t.data = y.permute(0, 2, 3, 1).contiguous() if t.is_image else y

    def backward(self, tops, propagate_down, bottoms):
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

    def forward(self, bottoms, tops):
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
        self.idx = bottoms[1].data.reshape(-1).long()
        tops[0].data = bottoms[0].data.index_select(0, self.idx)

    def backward(self, tops, propagate_down, bottoms):
        if propagate_down[0]:
            g = torch.zeros(bottoms[0].data.shape, dtype=torch.float32, device=self.device)
            g.index_add_(0, self.idx, tops[0].diff.float())
            bottoms[0].diff = g.to(bottoms[0].dtype)


@register("Filter")
class FilterLayer(Layer):
    min_bottoms = 2
    min_tops = 1

    def reshape(self, bottoms, tops):
        sel = bottoms[-1].data.reshape(-1)
        n = int((sel != 0).sum()) if sel.numel() else 0
        for b, t in zip(bottoms[:-1], tops):
            t.reshape((n,) + b.shape[1:], b.dtype)

    def forward(self, bottoms, tops):
        self.idx = torch.nonzero(bottoms[-1].data.reshape(-1) != 0)[:, 0]
        for b, t in zip(bottoms[:-1], tops):
            t.reshape((len(self.idx),) + b.shape[1:], b.dtype)
            t.data = b.data.index_select(0, self.idx)

    def backward(self, tops, propagate_down, bottoms):
        for i, (b, t) in enumerate(zip(bottoms[:-1], tops)):
            if propagate_down[i]:
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
        self.idx = bottoms[0].data.reshape(-1).long()
        y = self.weight.data.index_select(0, self.idx)
        if self.bias is not None:
            y = y + self.bias.data
        tops[0].data = y.reshape(tops[0].data.shape).to(self.dtype)

    def backward(self, tops, propagate_down, bottoms):
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
        p = self.lp.mvn_param
        return (1, 2, 3) if p.across_channels else (1, 2)  # NHWC: spatial dims 1,2 (+channel 3)

    def forward(self, bottoms, tops):
        p = self.lp.mvn_param
        x = bottoms[0].data.float()
        dims = self._dims(x)
        xm = x - x.mean(dim=dims, keepdim=True)
        if p.normalize_variance:
            self.std = torch.sqrt((xm * xm).mean(dim=dims, keepdim=True)) + p.eps
            y = xm / self.std
        else:
            y = xm
        self.y = y
        tops[0].data = y.to(tops[0].dtype)

    def backward(self, tops, propagate_down, bottoms):
        if not propagate_down[0]:
            return
        p = self.lp.mvn_param
        dy = tops[0].diff.float()
        dims = self._dims(dy)
        if p.normalize_variance:
            y = self.y
            g = dy - dy.mean(dim=dims, keepdim=True) - y * (dy * y).mean(dim=dims, keepdim=True)
            g = g / self.std
        else:
            g = dy - dy.mean(dim=dims, keepdim=True)
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

    def forward(self, bottoms, tops):
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
