"""Vision layers: Convolution, Deconvolution, Pooling, LRN, InnerProduct, Im2col.

References: caffe/src/caffe/layers/{base_conv,conv,deconv,pooling,lrn,inner_product,
im2col}_layer.{cpp,cu}.  The reference runs one im2col + SGEMM per image
(conv_layer.cu:14-21); here each pass is ONE implicit-GEMM MFMA launch over the whole
NHWC batch (``ops.hip``), with the bias and (when the net fuses an in-place ReLU) the
activation applied in the GEMM epilogue.
"""
from __future__ import annotations

import torch

from .. import ops, proto
from ..core.layer import Layer, register
from ..ops.spec import POOL_AVE, POOL_MAX, POOL_STOCHASTIC, ConvSpec, PoolSpec


def _conv_hw(cp, name, rep_name, h_name, w_name, default):
    """kernel/stride/pad: repeated field or the _h/_w pair (base_conv_layer.cpp:30-110)."""
    if cp.HasField(h_name) or cp.HasField(w_name):
        return int(getattr(cp, h_name)), int(getattr(cp, w_name))
    rep = list(getattr(cp, rep_name))
    if len(rep) == 0:
        return default, default
    if len(rep) == 1:
        return int(rep[0]), int(rep[0])
    return int(rep[0]), int(rep[1])


def conv_geometry(cp):
    if cp.HasField("kernel_h") or cp.HasField("kernel_w"):
        kh, kw = cp.kernel_h, cp.kernel_w
    else:
        ks = list(cp.kernel_size)
        if not ks:
            raise ValueError("kernel_size is required")
        kh, kw = (ks[0], ks[0]) if len(ks) == 1 else (ks[0], ks[1])
    sh, sw = _conv_hw(cp, "stride", "stride", "stride_h", "stride_w", 1)
    ph, pw = _conv_hw(cp, "pad", "pad", "pad_h", "pad_w", 0)
    return int(kh), int(kw), sh, sw, ph, pw


# --- N-d convolution (base_conv_layer.cpp:16-110: num_spatial_axes != 2, axis != 1 or
# force_nd_im2col) --------------------------------------------------------------------------

def _nd_field(cp, rep: str, h: str, w: str, nsp: int, default):
    """A repeated kernel/stride/pad field given once or per spatial axis, or its _h/_w pair
    (2-D only); Caffe's CHECKs become ValueErrors (base_conv_layer.cpp:26-96)."""
    if cp.HasField(h) or cp.HasField(w):
        if nsp != 2:
            raise ValueError(f"{h} & {w} can only be used for 2D convolution")
        return int(getattr(cp, h)), int(getattr(cp, w))
    vals = [int(v) for v in getattr(cp, rep)]
    if not vals:
        if default is None:
            raise ValueError("kernel_size is required")
        return (default,) * nsp
    if len(vals) not in (1, nsp):
        raise ValueError(f"{rep} must be specified once, or once per spatial dimension "
                         f"({rep} specified {len(vals)} times; {nsp} spatial dims)")
    return tuple(vals * nsp if len(vals) == 1 else vals)


def _canonical_axis(axis: int, nd: int) -> int:
    a = axis + nd if axis < 0 else axis
    if not 0 <= a < nd:
        raise ValueError(f"axis {axis} out of range for a {nd}-axis blob")
    return a


def conv_nd_mode(cp, bottom) -> bool:
    """The N-d path: a blob that is not 4-D, a channel axis other than 1, or force_nd_im2col."""
    nd = len(bottom.shape)
    return nd != 4 or _canonical_axis(int(cp.axis), nd) != 1 or bool(cp.force_nd_im2col)


def _logical(blob, diff=False):
    return blob.nchw(diff=diff)


def _store_logical(blob, t, diff=False):
    """Write a logical-layout tensor into a blob (a 4-D blob's storage is NHWC)."""
    if blob.is_image:
        blob.set_nchw(t.reshape(blob.shape), diff=diff)
    elif diff:
        blob.diff = t.reshape(blob.shape).to(blob.dtype)
    else:
        blob.data = t.reshape(blob.shape).to(blob.dtype)


class _NdGeometry:
    """Channel axis, batch / spatial split and kernel geometry of an N-d Convolution,
    Deconvolution or Im2col (the same parsing as base_conv_layer.cpp:16-110)."""

    def nd_setup(self, cp, bottom):
        nd = len(bottom.shape)
        self.axis = _canonical_axis(int(cp.axis), nd)
        self.nsp = nd - self.axis - 1
        if self.nsp < 1:
            raise ValueError("convolution needs at least one spatial axis")
        self.ks = _nd_field(cp, "kernel_size", "kernel_h", "kernel_w", self.nsp, None)
        self.st = _nd_field(cp, "stride", "stride_h", "stride_w", self.nsp, 1)
        self.pd = _nd_field(cp, "pad", "pad_h", "pad_w", self.nsp, 0)
        if min(self.ks) <= 0 or min(self.st) <= 0:
            raise ValueError("kernel and stride dimensions must be nonzero")
        self.C = int(bottom.shape[self.axis])

    def nd_split(self, shape):
        import math
        return int(math.prod(shape[:self.axis])), int(shape[self.axis]), tuple(int(d) for d in shape[self.axis + 1:])


class ConvolutionNdLayer(_NdGeometry, Layer):
    """Convolution over any number of spatial axes (and any channel axis): N-d im2col +
    the MFMA GEMM on the GPU (ops.hip.conv_nd_*), the fp32 reference on the CPU.  Weights
    keep Caffe's [K][C/g][k_0..k_{n-1}] layout.  Created by ConvolutionLayer.layer_setup when
    conv_nd_mode holds; its type_name keeps the engine's 2-D fusion passes away from it."""
    type_name = "ConvolutionND"

    def layer_setup(self, bottoms, tops):
        cp = self.lp.convolution_param
        if len(bottoms) != len(tops):
            raise ValueError("Convolution needs as many tops as bottoms")
        self.nd_setup(cp, bottoms[0])
        self.K = int(cp.num_output)
        self.groups = int(cp.group)
        if self.K <= 0:
            raise ValueError("num_output must be positive")
        if self.C % self.groups or self.K % self.groups:
            raise ValueError("channels and num_output must be divisible by group")
        self.weight = self.add_param((self.K, self.C // self.groups) + self.ks,
                                     filler=cp.weight_filler if cp.HasField("weight_filler") else None)
        self.bias = None
        if cp.bias_term:
            self.bias = self.add_param((self.K,), filler=cp.bias_filler if cp.HasField("bias_filler") else None)

    def spec(self, b) -> ops.ConvNdSpec:
        num, C, ins = self.nd_split(b.shape)
        if C != self.C:
            raise ValueError(f"{self.name}: input channels changed {self.C} -> {C}")
        return ops.ConvNdSpec(num, C, self.K, ins, self.ks, self.st, self.pd, self.groups)

    def reshape(self, bottoms, tops):
        for b, t in zip(bottoms, tops):
            s = self.spec(b)
            if min(s.outs) <= 0:
                raise ValueError(f"{self.name}: empty convolution output {s.outs}")
            t.reshape(tuple(b.shape[:self.axis]) + (self.K,) + s.outs, self.dtype)

    def forward(self, bottoms, tops):
        w = self.weight.compute
        bias = self.bias.data if self.bias is not None else None
        for b, t in zip(bottoms, tops):
            s = self.spec(b)
            x = _logical(b).reshape((s.num, s.C) + s.ins)
            _store_logical(t, ops.conv_nd_forward(x, w, bias, s))

    def backward(self, tops, propagate_down, bottoms):
        w = self.weight.compute
        dw = self.weight.diff if self.param_grads_needed(0) else None
        db = self.bias.diff if (self.bias is not None and self.param_grads_needed(1)) else None
        for i, (t, b) in enumerate(zip(tops, bottoms)):
            s = self.spec(b)
            x = _logical(b).reshape((s.num, s.C) + s.ins)
            dy = _logical(t, diff=True).reshape((s.num, s.K) + s.outs)
            dx = ops.conv_nd_backward(dy, x, w, s, bool(propagate_down[i]), dw, db)
            if propagate_down[i]:
                _store_logical(b, dx, diff=True)


class DeconvolutionNdLayer(_NdGeometry, Layer):
    """N-d transposed convolution (deconv_layer.cpp): forward = the data gradient of the
    convolution mapping top (num_output channels) -> bottom, backward = that convolution's
    forward (bottom diff) and weight gradient.  Weight Caffe shape [C][K/g][k...]."""
    type_name = "DeconvolutionND"

    def layer_setup(self, bottoms, tops):
        cp = self.lp.convolution_param
        self.nd_setup(cp, bottoms[0])
        self.K = int(cp.num_output)
        self.groups = int(cp.group)
        if self.C % self.groups or self.K % self.groups:
            raise ValueError("channels and num_output must be divisible by group")
        self.weight = self.add_param((self.C, self.K // self.groups) + self.ks,
                                     filler=cp.weight_filler if cp.HasField("weight_filler") else None)
        self.bias = None
        if cp.bias_term:
            self.bias = self.add_param((self.K,), filler=cp.bias_filler if cp.HasField("bias_filler") else None)

    def conv_spec(self, b) -> ops.ConvNdSpec:
        """The convolution top -> bottom whose data gradient this layer's forward is."""
        num, C, ins = self.nd_split(b.shape)
        outs = tuple((i - 1) * st + k - 2 * p for i, k, st, p in zip(ins, self.ks, self.st, self.pd))
        return ops.ConvNdSpec(num, self.K, C, outs, self.ks, self.st, self.pd, self.groups)

    def reshape(self, bottoms, tops):
        for b, t in zip(bottoms, tops):
            sc = self.conv_spec(b)
            if min(sc.ins) <= 0:
                raise ValueError(f"{self.name}: empty deconvolution output {sc.ins}")
            t.reshape(tuple(b.shape[:self.axis]) + (self.K,) + sc.ins, self.dtype)

    def forward(self, bottoms, tops):
        w = self.weight.compute
        for b, t in zip(bottoms, tops):
            sc = self.conv_spec(b)
            x = _logical(b).reshape((sc.num, sc.K) + sc.outs)
            y = ops.conv_nd_backward(x, None, w, sc, True, None, None)
            if self.bias is not None:
                y = (y.float() + self.bias.data.float().view((1, -1) + (1,) * sc.nd)).to(y.dtype)
            _store_logical(t, y)

    def backward(self, tops, propagate_down, bottoms):
        w = self.weight.compute
        dw = self.weight.diff if self.param_grads_needed(0) else None
        for i, (t, b) in enumerate(zip(tops, bottoms)):
            sc = self.conv_spec(b)
            dtop = _logical(t, diff=True).reshape((sc.num, sc.C) + sc.ins)
            if self.bias is not None and self.param_grads_needed(1):
                self.bias.diff += dtop.float().reshape(sc.num, sc.C, -1).sum((0, 2))
            if dw is not None:
                x = _logical(b).reshape((sc.num, sc.K) + sc.outs)
                ops.conv_nd_backward(x, dtop, w, sc, False, dw, None)
            if propagate_down[i]:
                _store_logical(b, ops.conv_nd_forward(dtop, w, None, sc), diff=True)


@register("Convolution")
class ConvolutionLayer(Layer):
    exact_bottoms = -1
    min_bottoms = 1
    min_tops = 1

    fuse_relu = False  # set by the net's fusion pass when an in-place ReLU follows
    relu_gate = False  # ... and when an in-place ReLU PRODUCES the bottom (backward fused into dgrad)
    folded_input = None  # S2D-folded bottom 0 written by a fused augment (engine.fuse_input_fold)
    concat_slot = None  # (ConcatSlots, part): top 0 is written into a zero-copy Concat buffer (engine.fuse_concat)
    flipped_weights = None  # dgrad weights flipped at the start of backward (engine.batch_weight_flips)

    def layer_setup(self, bottoms, tops):
        cp = self.lp.convolution_param
        if conv_nd_mode(cp, bottoms[0]):
            self.__class__ = ConvolutionNdLayer  # N-d path (see conv_nd_mode)
            return self.layer_setup(bottoms, tops)
        if len(bottoms) != len(tops):
            raise ValueError("Convolution needs as many tops as bottoms")
        b = bottoms[0]
        self.R, self.S, self.sh, self.sw, self.ph, self.pw = conv_geometry(cp)
        self.K = int(cp.num_output)
        self.groups = int(cp.group)
        C = b.shape[1]
        if C % self.groups or self.K % self.groups:
            raise ValueError("channels and num_output must be divisible by group")
        Cg = C // self.groups
        R, S = self.R, self.S
        self.C = C
        w = self.add_param((self.K, Cg, R, S), (self.K, R, S, Cg),
                           to_caffe=lambda t: t.permute(0, 3, 1, 2),
                           from_caffe=lambda t: t.permute(0, 2, 3, 1),
                           filler=cp.weight_filler if cp.HasField("weight_filler") else None)
        self.weight = w
        self.bias = None
        if cp.bias_term:
            self.bias = self.add_param((self.K,), filler=cp.bias_filler if cp.HasField("bias_filler") else None)

    def spec(self, b) -> ConvSpec:
        N, C, H, W = b.shape
        if C != self.C:
            raise ValueError(f"{self.name}: input channels changed {self.C} -> {C}")
        return ConvSpec(N, H, W, C, self.K, self.R, self.S, self.sh, self.sw, self.ph, self.pw,
                        1, 1, self.groups)

    def reshape(self, bottoms, tops):
        for b, t in zip(bottoms, tops):
            s = self.spec(b)
            t.reshape((s.N, s.K, s.P, s.Q), self.dtype)

    def forward(self, bottoms, tops):
        w = self.weight.compute
        bias = self.bias.data if self.bias is not None else None
        self._ws = [{} for _ in bottoms]  # forward -> backward scratch (e.g. folded input)
        for i, (b, t) in enumerate(zip(bottoms, tops)):
            s = self.spec(b)
            side = self._fp8_out_side(s) if i == 0 else None
            if side is not None:  # the epilogue also stores the output as the consumer's fp8 input
                from ..ops import gemm as _gemm
                with _gemm.fp8_side_output(side):
                    if self.fp8_slots is not None:
                        t.data = self._forward_fp8(b.data, w, bias, s, out=side.base)
                    else:
                        t.data = ops.conv_forward(b.data, w, bias, s, relu=self.fuse_relu, ws=self._ws[i],
                                                  folded=self.folded_input, out=side.base)
                self.fp8_out[0]._fp8_x_side = side
                continue
            if self.fp8_slots is not None and b.data.is_cuda:
                t.data = self._forward_fp8(b.data, w, bias, s)
                continue
            folded = self.folded_input if i == 0 else None
            if self.concat_slot is not None and i == 0 and b.data.is_cuda:
                slots, part = self.concat_slot
                out = slots.slot(part, (s.N, s.P, s.Q), b.data.device)
                t.data = ops.conv_forward(b.data, w, bias, s, relu=self.fuse_relu, ws=self._ws[i], out=out)
                continue
            t.data = ops.conv_forward(b.data, w, bias, s, relu=self.fuse_relu, ws=self._ws[i], folded=folded)

    fp8_slots = None  # (x slot, w slot) in ctx.fp8 when the forward product runs in e4m3
    fp8_dgrad_slots = None  # (dy slot, flipped-w slot) when the data gradient runs in e4m3
    # the weight gradient runs as an fp8 product too (engine.enable_fp8 wgrad): the forward
    # keeps its e4m3 input (_fp8_xq) for it, and dy's fp8 copy is shared with the data gradient
    fp8_wgrad = False
    _fp8_xq = None
    # engine.fuse_fp8_quant: (consumer conv, its x slot) — this layer's output GEMM also stores
    # the consumer's fp8 input; (producer conv, its dy slot) — this layer's data-gradient GEMM
    # also stores the producer's fp8 output gradient
    fp8_out = None
    fp8_dx_out = None
    fp8_dx_only = False  # store the fp8 input gradient alone (engine.fuse_fp8_quant)
    _fp8_x_side = None
    _fp8_dy_side = None

    def _fp8_ready(self) -> bool:
        sc = getattr(self.ctx, "fp8", None)
        return sc is not None and sc.updates > 0  # delayed-scaling slots initialised

    def _fp8_out_side(self, s):
        if self.fp8_out is None or self.concat_slot is not None or not self._fp8_ready():
            return None
        from ..ops import gemm as _gemm
        cons, ix = self.fp8_out
        sc = self.ctx.fp8
        dev = self.weight.compute.device
        y = torch.empty((s.N, s.P, s.Q, s.K), dtype=torch.bfloat16, device=dev)
        return _gemm.Fp8Side(y, sc.slot(ix), sc.is_e5m2(ix), self._side_part("fwd", dev))

    def _side_part(self, key, dev):
        """Persistent block-|max| partials of this layer's fp8 side output (first allocated
        by an eager step, before any graph capture)."""
        parts = self.__dict__.setdefault("_fp8_parts", {})
        if key not in parts:
            from ..ops import gemm as _gemm
            parts[key] = _gemm.new_side_part(dev)
        return parts[key]

    def fp8_eligible(self, b) -> bool:
        s = self.spec(b)
        return s.C % 16 == 0 and s.Cg % 16 == 0 and s.dh == 1 and s.dw == 1

    def fp8_dgrad_eligible(self, b) -> bool:
        from ..ops import hip
        return hip.fp8_dgrad_ok(self.spec(b))

    def _forward_fp8(self, x, w, bias, s, out=None):
        """e4m3 forward product (delayed per-tensor scales); the weight gradient stays bf16
        on the bf16 activations (fp32 masters are untouched).  The input's e4m3 bytes come
        from the producing conv's epilogue when engine.fuse_fp8_quant paired the two."""
        from ..ops import hip
        sc = self.ctx.fp8
        ix, iw = self.fp8_slots
        from ..ops import gemm as _gemm
        side, self._fp8_x_side = self._fp8_x_side, None
        xq = _gemm.side_bytes(side, x)
        if xq is None:
            xq = hip.quant_fp8(x, sc.slot(ix))
        if self.fp8_wgrad:
            self._fp8_xq = xq
        wq = hip.quant_fp8(w, sc.slot(iw))
        return hip.conv_forward_fp8(xq, wq, bias, s, sc.deq(ix), sc.deq(iw), relu=self.fuse_relu, out=out)

    supports_grad_overwrite = True

    def backward(self, tops, propagate_down, bottoms):
        w = self.weight.compute
        dw = self.weight.diff if self.param_grads_needed(0) else None
        db = self.bias.diff if (self.bias is not None and self.param_grads_needed(1)) else None
        for i, (t, b) in enumerate(zip(tops, bottoms)):
            s = self.spec(b)
            gate = b.data if self.relu_gate else None
            ws = self._ws[i] if i < len(getattr(self, "_ws", ())) else None
            if self.flipped_weights is not None:  # flipped for the whole net (engine.batch_weight_flips)
                ws = {} if ws is None else ws
                ws["wt"] = self.flipped_weights
            if self.fp8_dgrad_slots is not None and t.diff.is_cuda:  # e4m3 data gradient (engine.enable_fp8)
                ws = {} if ws is None else ws
                dy_side, self._fp8_dy_side = self._fp8_dy_side, None
                ws["fp8_dgrad"] = (self.ctx.fp8, *self.fp8_dgrad_slots, dy_side)
                xq, self._fp8_xq = self._fp8_xq, None
                if self.fp8_wgrad and xq is not None and dw is not None and i == 0:
                    ws["fp8_wgrad"] = (self.ctx.fp8, self.fp8_slots[0], xq, self.fp8_dgrad_slots[0])
            if i == 0 and self.fp8_dx_out is not None and propagate_down[i] and self._fp8_ready():
                ws = {} if ws is None else ws
                prod, idy = self.fp8_dx_out
                ws["fp8_dx_side"] = (self.ctx.fp8.slot(idy), self.ctx.fp8.is_e5m2(idy),
                                     self._side_part("bwd", t.diff.device))
            dw_acc = not (dw is not None and self.grad_overwrite(0))
            db_acc = not (db is not None and self.grad_overwrite(1))
            sink = getattr(self, "slab_grad", None)
            if sink is not None and dw is not None and not dw_acc and not (db is not None and db_acc):
                # engine.fuse_splitk_updates: the solver sums this product's split-K slabs
                from ..ops import gemm as _gemm
                with _gemm.defer_reduce(sink):
                    dx = ops.conv_backward(t.diff, b.data, w, s, bool(propagate_down[i]), dw, db, gate, ws,
                                           dw_acc=dw_acc, db_acc=db_acc)
                sink.apply()  # after the data gradient, which reads the old weights
            else:
                if sink is not None:
                    sink.begin()
                    sink.end()  # this pass's gradient went to the flat buffer
                dx = ops.conv_backward(t.diff, b.data, w, s, bool(propagate_down[i]), dw, db, gate, ws,
                                       dw_acc=dw_acc, db_acc=db_acc)
            if ws is not None and "fp8_dx_side_out" in ws:
                self.fp8_dx_out[0]._fp8_dy_side = ws.pop("fp8_dx_side_out")
            if propagate_down[i]:
                b.diff = dx


@register("Deconvolution")
class DeconvolutionLayer(Layer):
    """Transposed convolution (deconv_layer.cpp).  Weight Caffe shape (C_in, K/g, R, S).
    Forward = conv dgrad, backward = conv forward + wgrad with roles swapped; runs
    through the reference path on CPU and the same GEMM engine on GPU."""
    min_bottoms = 1
    min_tops = 1

    def layer_setup(self, bottoms, tops):
        cp = self.lp.convolution_param
        if conv_nd_mode(cp, bottoms[0]):
            self.__class__ = DeconvolutionNdLayer  # N-d path (see conv_nd_mode)
            return self.layer_setup(bottoms, tops)
        self.R, self.S, self.sh, self.sw, self.ph, self.pw = conv_geometry(cp)
        self.K = int(cp.num_output)
        self.groups = int(cp.group)
        C = bottoms[0].shape[1]
        self.C = C
        Kg = self.K // self.groups
        self.weight = self.add_param((C, Kg, self.R, self.S), (C, self.R, self.S, Kg),
                                     to_caffe=lambda t: t.permute(0, 3, 1, 2),
                                     from_caffe=lambda t: t.permute(0, 2, 3, 1),
                                     filler=cp.weight_filler if cp.HasField("weight_filler") else None)
        self.bias = None
        if cp.bias_term:
            self.bias = self.add_param((self.K,), filler=cp.bias_filler if cp.HasField("bias_filler") else None)

    def out_hw(self, H, W):
        return ((H - 1) * self.sh + self.R - 2 * self.ph, (W - 1) * self.sw + self.S - 2 * self.pw)

    def fwd_spec(self, b):
        # the equivalent forward conv maps top (K channels) -> bottom (C channels)
        N, C, H, W = b.shape
        Ho, Wo = self.out_hw(H, W)
        return ConvSpec(N, Ho, Wo, self.K, C, self.R, self.S, self.sh, self.sw, self.ph, self.pw,
                        1, 1, self.groups)

    def reshape(self, bottoms, tops):
        for b, t in zip(bottoms, tops):
            N, C, H, W = b.shape
            Ho, Wo = self.out_hw(H, W)
            t.reshape((N, self.K, Ho, Wo), self.dtype)

    def _w_as_conv(self):
        # deconv weight (C, R, S, K/g) == conv weight of top->bottom conv: (Cout=C, R, S, Cin_g=K/g)
        return self.weight.compute

    def forward(self, bottoms, tops):
        for b, t in zip(bottoms, tops):
            s = self.fwd_spec(b)
            zeros = torch.zeros(t.data.shape, dtype=t.dtype, device=t.device)
            y = ops.conv_backward(b.data, zeros, self._w_as_conv(), s, True, None, None)
            if self.bias is not None:
                y = (y.float() + self.bias.data.float()).to(t.dtype)
            t.data = y

    def backward(self, tops, propagate_down, bottoms):
        dw = self.weight.diff if self.param_grads_needed(0) else None
        for i, (t, b) in enumerate(zip(tops, bottoms)):
            s = self.fwd_spec(b)
            if self.bias is not None and self.param_grads_needed(1):
                self.bias.diff += t.diff.float().reshape(-1, self.K).sum(0)
            if dw is not None:
                # conv(top->bottom) wgrad with x = top diff, dy = bottom data
                ops.conv_backward(b.data, t.diff, self._w_as_conv(), s, False, dw, None)
            if propagate_down[i]:
                b.diff = ops.conv_forward(t.diff, self._w_as_conv(), None, s)


@register("Pooling")
class PoolingLayer(Layer):
    exact_bottoms = 1
    min_tops = 1
    max_tops = 2

    def layer_setup(self, bottoms, tops):
        pp = self.lp.pooling_param
        self.global_pooling = pp.global_pooling
        if pp.HasField("kernel_h") or pp.HasField("kernel_w"):
            self.kh, self.kw = pp.kernel_h, pp.kernel_w
        else:
            self.kh = self.kw = pp.kernel_size
        if pp.HasField("pad_h") or pp.HasField("pad_w"):
            self.ph, self.pw = pp.pad_h, pp.pad_w
        else:
            self.ph = self.pw = pp.pad
        if pp.HasField("stride_h") or pp.HasField("stride_w"):
            self.sh, self.sw = pp.stride_h, pp.stride_w
        else:
            self.sh = self.sw = pp.stride
        self.method = int(pp.pool)
        if self.global_pooling:
            self.ph = self.pw = 0
            self.sh = self.sw = 1
        elif not self.kh or not self.kw:
            raise ValueError("Pooling: kernel size is required")
        self.aux = None

    relu_gate = False  # backward of the slope-0 in-place ReLU producing the bottom is fused here
    fused_lrn = None   # the LRN reading this layer's output, run inside its kernels (engine.fuse_pool_lrn)
    bwd_lrn = None     # the LRN producing this layer's input: backward run here (engine.fuse_lrn_pool_backward)
    # engine.fuse_fp8_quant: (consumer conv, its x slot) / (producer conv, its dy slot) — the
    # pooling kernels also store the consumer's e4m3 input / the producer's fp8 output gradient
    fp8_out = None
    fp8_dx_out = None

    def _fp8_side(self, pair, shape, key, dev):
        sc = getattr(self.ctx, "fp8", None)
        if pair is None or sc is None or sc.updates == 0:
            return None
        from ..ops import gemm as _gemm
        parts = self.__dict__.setdefault("_fp8_parts", {})
        if key not in parts:
            parts[key] = _gemm.new_side_part(dev)
        i = pair[1]
        return _gemm.Fp8Side(torch.empty(shape, dtype=torch.bfloat16, device=dev), sc.slot(i), sc.is_e5m2(i),
                             parts[key])

    def spec(self, b) -> PoolSpec:
        N, C, H, W = b.shape
        kh, kw = (H, W) if self.global_pooling else (self.kh, self.kw)
        return PoolSpec(N, H, W, C, kh, kw, self.sh, self.sw, self.ph, self.pw, self.method)

    def reshape(self, bottoms, tops):
        s = self.spec(bottoms[0])
        tops[0].reshape((s.N, s.C, s.P, s.Q), self.dtype)
        if len(tops) > 1:
            tops[1].reshape((s.N, s.C, s.P, s.Q), self.dtype)

    def forward(self, bottoms, tops):
        s = self.spec(bottoms[0])
        x = bottoms[0].data
        if self.method == POOL_STOCHASTIC and x.is_cuda:
            from ..ops import layers_hip
            if getattr(self, "stream", None) is None:
                self.stream = self.ctx.next_stream_id()
            train = self.phase == proto.TRAIN
            tops[0].data, self.aux = layers_hip.stopool(x, s, self.ctx.rng_state, self.stream, train)
            return
        if self.method == POOL_STOCHASTIC:
            if self.phase == proto.TRAIN:
                # StoPoolForwardTrain (pooling_layer.cu:88-122): draw u ~ U[0,1) per output,
                # take the first window element whose running sum reaches u * window sum
                wins = ops.ref._pool_windows(x.float(), s, 0.0)
                u = torch.rand(wins.shape[:4], generator=self.ctx.gen).to(wins.device)
                csum = wins.cumsum(-1)
                self.aux = (csum >= (u * csum[..., -1])[..., None]).to(torch.uint8).argmax(-1, keepdim=True)
                tops[0].data = ops.ref.nhwc(wins.gather(-1, self.aux).squeeze(-1)).to(x.dtype)
            else:
                # StoPoolForwardTest (pooling_layer.cu:125-155): probability-weighted average
                tops[0].data = _stochastic_test(x.float().clamp_min(0), s).to(x.dtype)
            return
        f = self.fused_lrn
        if f is not None and x.is_cuda:
            from ..ops import hip
            tops[0].data, self.aux, f.top.data = hip.pool_lrn_forward(x, s, self.relu_gate, f.size, f.alpha, f.beta,
                                                                      f.k)
            return
        side = self._fp8_side(self.fp8_out, (s.N, s.P, s.Q, s.C), "fwd", x.device) if x.is_cuda else None
        if side is not None:
            from ..ops import hip
            y, self.aux = hip.pool_forward_mask(x, s, self.relu_gate, side=side)
            self.fp8_out[0]._fp8_x_side = side
        else:
            y, self.aux = ops.pool_forward_aux(x, s, self.relu_gate)
        tops[0].data = y
        if len(tops) > 1:
            tops[1].data = (self.aux.to(tops[1].dtype) if self.aux is not None
                            else torch.zeros_like(y))

    def backward(self, tops, propagate_down, bottoms):
        if not propagate_down[0]:
            return
        s = self.spec(bottoms[0])
        if self.method == POOL_STOCHASTIC and tops[0].diff.is_cuda:
            # the sampled window offsets are a max-pool style mask: gather backward
            import dataclasses
            sm = dataclasses.replace(s, method=0)
            bottoms[0].diff = ops.pool_backward(tops[0].diff, bottoms[0].data, sm, self.aux)
            return
        if self.method == POOL_STOCHASTIC:
            # StoPoolBackward (pooling_layer.cu:270-300): the diff goes to the sampled element
            xl = bottoms[0].data.float().requires_grad_(True)
            with torch.enable_grad():
                y = ops.ref._pool_windows(xl, s, 0.0).gather(-1, self.aux).squeeze(-1)
                g, = torch.autograd.grad(y, xl, ops.ref.nchw(tops[0].diff.float()))
            bottoms[0].diff = g.to(bottoms[0].dtype)
            return
        f = self.fused_lrn
        if f is not None and bottoms[0].data.is_cuda:
            from ..ops import hip
            bottoms[0].diff = hip.lrn_pool_backward(f.top.diff, tops[0].data, self.aux, s, f.size, f.alpha, f.beta,
                                                    f.k)
            return
        f = self.bwd_lrn
        if f is not None and self.aux is not None and self.fp8_dx_out is None and bottoms[0].data.is_cuda:
            from ..ops import hip
            f.bottom.diff = hip.pool_lrn_backward_rev(tops[0].diff, self.aux, f.bottom.data, s, f.size, f.alpha,
                                                      f.beta, f.k, f.relu_gate)
            f.bwd_done = True
            return
        side = (self._fp8_side(self.fp8_dx_out, (s.N, s.H, s.W, s.C), "bwd", bottoms[0].data.device)
                if bottoms[0].data.is_cuda else None)
        if side is not None:
            from ..ops import hip
            bottoms[0].diff = hip.pool_backward(tops[0].diff, bottoms[0].data, s, self.aux, tops[0].data,
                                                self.relu_gate, side=side, side_only=self.fp8_dx_only)
            self.fp8_dx_out[0]._fp8_dy_side = side
            return
        bottoms[0].diff = ops.pool_backward(tops[0].diff, bottoms[0].data, s, self.aux, tops[0].data,
                                            self.relu_gate)


def _stochastic_test(xf, s: PoolSpec):
    sq = ops.ref._pool_windows(xf * xf, s, 0.0).sum(-1)
    lin = ops.ref._pool_windows(xf, s, 0.0).sum(-1)
    out = torch.where(lin > 0, sq / lin.clamp_min(1e-30), torch.zeros_like(lin))
    return ops.ref.nhwc(out)


@register("LRN")
class LRNLayer(Layer):
    exact_bottoms = 1
    exact_tops = 1

    def layer_setup(self, bottoms, tops):
        p = self.lp.lrn_param
        self.size = int(p.local_size)
        if self.size % 2 == 0:
            raise ValueError("LRN only supports odd values for local_size")
        self.alpha, self.beta, self.k = float(p.alpha), float(p.beta), float(p.k)
        self.within = int(p.norm_region) == 1

    def reshape(self, bottoms, tops):
        tops[0].reshape(bottoms[0].shape, self.dtype)

    def forward(self, bottoms, tops):
        if self.pool_fused and bottoms[0].data.is_cuda:
            return  # written by the pooling layer before it (engine.fuse_pool_lrn)
        tops[0].data = ops.lrn_forward(bottoms[0].data, self.size, self.alpha, self.beta, self.k, self.within)

    relu_gate = False  # engine.fuse_relu_backward: the in-place ReLU producing the bottom
    pool_fused = False  # forward and backward run inside the preceding max pooling's kernels
    top = None          # this layer's top Blob (set with pool_fused)
    bottom = None       # this layer's bottom Blob (engine.fuse_lrn_pool_backward)
    bwd_done = False    # this step's backward already run by the max pooling after it

    def backward(self, tops, propagate_down, bottoms):
        if self.bwd_done:
            self.bwd_done = False
            return
        if not propagate_down[0] or (self.pool_fused and bottoms[0].data.is_cuda):
            return
        x = bottoms[0].data
        if self.relu_gate and x.is_cuda:
            from ..ops import hip
            bottoms[0].diff = hip.lrn_backward(tops[0].diff, x, self.size, self.alpha, self.beta, self.k,
                                               self.within, gate=True)
            return
        dx = ops.lrn_backward(tops[0].diff, x, self.size, self.alpha, self.beta, self.k, self.within, tops[0].data)
        bottoms[0].diff = ops.relu_backward(dx, x) if self.relu_gate else dx


@register("InnerProduct")
class InnerProductLayer(Layer):
    exact_bottoms = 1
    exact_tops = 1
    fuse_relu = False
    relu_gate = False
    supports_grad_overwrite = True

    def layer_setup(self, bottoms, tops):
        p = self.lp.inner_product_param
        self.N = int(p.num_output)
        b = bottoms[0]
        self.axis = b.canonical_axis(p.axis)
        self.Kdim = b.count_range(self.axis)
        # 4-D NHWC bottoms flatten in (h, w, c) order; the weight's columns are kept in that
        # order internally and permuted to Caffe's (c, h, w) order at the IO boundary.
        self.perm = None
        if b.is_image and self.axis == 1 and b.shape[2] * b.shape[3] > 1:
            _, C, H, W = b.shape
            self.perm = (C, H, W)
        N, K = self.N, self.Kdim
        if self.perm is not None:
            C, H, W = self.perm
            to_caffe = lambda t: t.reshape(N, H, W, C).permute(0, 3, 1, 2).reshape(N, K)  # noqa: E731
            from_caffe = lambda t: t.reshape(N, C, H, W).permute(0, 2, 3, 1).reshape(N, K)  # noqa: E731
        else:
            to_caffe = from_caffe = None
        self.weight = self.add_param((N, K), (N, K), to_caffe, from_caffe,
                                     filler=p.weight_filler if p.HasField("weight_filler") else None)
        self.bias = None
        if p.bias_term:
            self.bias = self.add_param((N,), filler=p.bias_filler if p.HasField("bias_filler") else None)

    def reshape(self, bottoms, tops):
        b = bottoms[0]
        if b.count_range(self.axis) != self.Kdim:
            raise ValueError(f"{self.name}: input size incompatible with inner product parameters")
        tops[0].reshape(tuple(b.shape[:self.axis]) + (self.N,), self.dtype)

    def forward(self, bottoms, tops):
        b = bottoms[0]
        M = b.count_range(0, self.axis)
        x2 = b.data.reshape(M, self.Kdim)
        bias = self.bias.data if self.bias is not None else None
        d = self.fused_dropout
        drop = (d.ctx.rng_state, d.stream, d.ratio) if d is not None and x2.is_cuda and d.phase == 0 else None
        if self.fp8_slots is not None and x2.is_cuda:
            from ..ops import hip
            sc = self.ctx.fp8
            ix, iw = self.fp8_slots
            xq = hip.quant_fp8(x2, sc.slot(ix))
            wq = hip.quant_fp8(self.weight.compute, sc.slot(iw))
            y = hip.linear_forward_fp8(xq, wq, bias, sc.deq(ix), sc.deq(iw), relu=self.fuse_relu, dropout=drop)
        else:
            if drop is not None:  # TRAIN: the in-place dropout applied in the epilogue
                from ..ops import hip
                y = hip.linear_forward(x2, self.weight.compute, bias, self.fuse_relu, dropout=drop)
            else:
                y = ops.linear_forward(x2, self.weight.compute, bias, self.fuse_relu)
        tops[0].data = y.reshape(tops[0].data.shape)

    fp8_slots = None
    fused_update = None  # solver update applied in the wgrad epilogue (engine.fuse_fc_updates)
    fused_dropout = None  # the in-place Dropout applied in the forward epilogue (engine.fuse_dropout)
    gate_scale = 1.0      # dgrad gate = a fused dropout's output: scale kept values by 1/(1-p)

    def fp8_eligible(self, b) -> bool:
        return self.Kdim % 16 == 0

    def backward(self, tops, propagate_down, bottoms):
        b = bottoms[0]
        M = b.count_range(0, self.axis)
        dy2 = tops[0].diff.reshape(M, self.N)
        x2 = b.data.reshape(M, self.Kdim)
        dw = self.weight.diff if self.param_grads_needed(0) else None
        db = self.bias.diff if (self.bias is not None and self.param_grads_needed(1)) else None
        gate = b.data if self.relu_gate else None
        dw_acc = not (dw is not None and self.grad_overwrite(0))
        db_acc = not (db is not None and self.grad_overwrite(1))
        if self.fused_update is not None and dw is not None and x2.is_cuda:
            # the weight gradient goes straight into the solver update (engine.fuse_fc_updates
            # admits only unshared weights with iter_size 1: this is its one and only write)
            from ..ops import hip
            dx = hip.linear_backward_sgd(dy2, x2, self.weight.compute, bool(propagate_down[0]),
                                         self.fused_update.sgd(), db, gate, db_acc=db_acc, gate_scale=self.gate_scale)
        elif self.gate_scale != 1.0:
            from ..ops import hip
            dx = hip.linear_backward(dy2, x2, self.weight.compute, bool(propagate_down[0]), dw, db, gate,
                                     dw_acc=dw_acc, db_acc=db_acc, gate_scale=self.gate_scale)
        else:
            dx = ops.linear_backward(dy2, x2, self.weight.compute, bool(propagate_down[0]), dw, db, gate,
                                     dw_acc=dw_acc, db_acc=db_acc)
        if propagate_down[0]:
            b.diff = dx.reshape(b.data.shape)


@register("Im2col")
class Im2colLayer(Layer):
    """im2col as a layer (im2col_layer.cpp): top = [N, C*R*S, P, Q] in Caffe order."""
    exact_bottoms = 1
    exact_tops = 1

    def layer_setup(self, bottoms, tops):
        cp = self.lp.convolution_param
        if conv_nd_mode(cp, bottoms[0]):
            self.__class__ = Im2colNdLayer
            return self.layer_setup(bottoms, tops)
        self.R, self.S, self.sh, self.sw, self.ph, self.pw = conv_geometry(cp)

    def reshape(self, bottoms, tops):
        N, C, H, W = bottoms[0].shape
        P = (H + 2 * self.ph - self.R) // self.sh + 1
        Q = (W + 2 * self.pw - self.S) // self.sw + 1
        tops[0].reshape((N, C * self.R * self.S, P, Q), self.dtype)

    def _geom(self, b, t):
        N, C_, H, W = b.shape
        return (N, H, W, C_, t.shape[2], t.shape[3], self.R, self.S, self.sh, self.sw, self.ph, self.pw, 1, 1)

    def forward(self, bottoms, tops):
        if bottoms[0].data.is_cuda:
            from ..ops import layers_hip
            b, t = bottoms[0], tops[0]
            t.data = layers_hip.im2col_caffe(b.data, self._geom(b, t), t.data.shape)
            return
        xn = bottoms[0].nchw().float()
        cols = torch.nn.functional.unfold(xn, (self.R, self.S), padding=(self.ph, self.pw),
                                          stride=(self.sh, self.sw))
        N, CK, L = cols.shape
        t = tops[0]
        t.data = cols.reshape(N, CK, t.shape[2], t.shape[3]).permute(0, 2, 3, 1).contiguous().to(t.dtype)

    def backward(self, tops, propagate_down, bottoms):
        if not propagate_down[0]:
            return
        t, b = tops[0], bottoms[0]
        if t.diff.is_cuda:
            from ..ops import layers_hip
            b.diff = layers_hip.col2im_caffe(t.diff, self._geom(b, t), b.data.shape)
            return
        d = t.nchw(diff=True).float().reshape(t.shape[0], t.shape[1], -1)
        x = torch.nn.functional.fold(d, b.shape[2:], (self.R, self.S), padding=(self.ph, self.pw),
                                     stride=(self.sh, self.sw))
        b.diff = x.permute(0, 2, 3, 1).contiguous().to(b.dtype)


class Im2colNdLayer(_NdGeometry, Layer):
    """N-d im2col layer (im2col_layer.cpp with num_spatial_axes != 2): top =
    shape[:axis] + [C * prod(k)] + outs, each image's columns in (c, taps) order."""
    type_name = "Im2colND"
    exact_bottoms = 1
    exact_tops = 1

    def layer_setup(self, bottoms, tops):
        self.nd_setup(self.lp.convolution_param, bottoms[0])

    def spec(self, b) -> ops.ConvNdSpec:
        num, C, ins = self.nd_split(b.shape)
        return ops.ConvNdSpec(num, C, 1, ins, self.ks, self.st, self.pd, 1)

    def reshape(self, bottoms, tops):
        b = bottoms[0]
        s = self.spec(b)
        tops[0].reshape(tuple(b.shape[:self.axis]) + (s.C * s.T,) + s.outs, self.dtype)

    def forward(self, bottoms, tops):
        b = bottoms[0]
        s = self.spec(b)
        x = _logical(b).reshape((s.num, s.C) + s.ins)
        CT = s.C * s.T
        if x.is_cuda:
            from ..ops import hip, layers_hip
            x = x.contiguous()
            col = torch.empty((s.num * s.P, CT), dtype=x.dtype, device=x.device)
            hip.call("im2col_nd", x, col, s.nd, s.num, s.C, s.C, 0, CT, hip._nd_dims(s), hip._nd_dt(x),
                     hip._nd_dt(col))
            y = layers_hip.transpose(col, s.num, s.P, CT)
        else:
            y = ops.ref.im2col_nd(x.float(), s).reshape(s.num, s.P, CT).transpose(1, 2)
        _store_logical(tops[0], y)

    def backward(self, tops, propagate_down, bottoms):
        if not propagate_down[0]:
            return
        b, t = bottoms[0], tops[0]
        s = self.spec(b)
        CT = s.C * s.T
        dy = _logical(t, diff=True).reshape(s.num, CT, s.P)
        if dy.is_cuda:
            from ..ops import hip, layers_hip
            dcol = layers_hip.transpose(dy.contiguous(), s.num, CT, s.P)
            dx = torch.empty((s.num, s.C) + s.ins, dtype=dy.dtype, device=dy.device)
            hip.call("col2im_nd", dcol, dx, s.nd, s.num, s.C, s.C, 0, CT, hip._nd_dims(s), hip._nd_dt(dcol),
                     hip._nd_dt(dx), 0)
        else:
            x = _logical(b).reshape((s.num, s.C) + s.ins).float().detach().requires_grad_(True)
            col = ops.ref.im2col_nd(x, s).reshape(s.num, s.P, CT).transpose(1, 2)
            dx, = torch.autograd.grad(col, x, dy.float())
        _store_logical(b, dx, diff=True)


__all__ = ["ConvolutionLayer", "DeconvolutionLayer", "PoolingLayer", "LRNLayer", "InnerProductLayer",
           "Im2colLayer", "POOL_MAX", "POOL_AVE"]
