"""Neuron (elementwise) layers: ReLU, Dropout, Sigmoid, TanH, AbsVal, BNLL, Exp, Log,
Power, Threshold, PReLU.

References: caffe/src/caffe/layers/{relu,dropout,sigmoid,tanh,absval,bnll,exp,log,power,
threshold,prelu}_layer.{cpp,cu}.  ReLU and Dropout are on the hot path and run HIP
kernels (ReLU forward is usually fused into the producing conv/IP epilogue by the net);
Dropout regenerates its Philox mask in backward instead of storing it.  The remaining
neurons run one templated HIP elementwise kernel per direction on the GPU
(csrc/kernels/layers.hip ``neuron_fwd_k`` / ``neuron_bwd_k``, fp32 math, 8-wide bf16
vectors) and fp32 tensor math on the CPU reference path.
"""
from __future__ import annotations

import math

import torch

from .. import ops
from ..core.layer import Layer, register


class NeuronLayer(Layer):
    exact_bottoms = 1
    exact_tops = 1

    def reshape(self, bottoms, tops):
        tops[0].reshape(bottoms[0].shape, self.dtype)


@register("ReLU")
class ReLULayer(NeuronLayer):
    fused = False  # forward folded into the producer's GEMM epilogue
    bwd_fused = False  # backward folded into the consumer's backward (gate)

    def layer_setup(self, bottoms, tops):
        self.slope = float(self.lp.relu_param.negative_slope)

    def forward(self, bottoms, tops):
        if self.fused:
            return
        tops[0].data = ops.relu_forward(bottoms[0].data, self.slope)

    def backward(self, tops, propagate_down, bottoms):
        if propagate_down[0] and not self.bwd_fused:
            # in-place: bottom data was overwritten by top data; sign(y) == sign(x) for slope >= 0
            ref = bottoms[0].data
            bottoms[0].diff = ops.relu_backward(tops[0].diff, ref, self.slope)


@register("Dropout")
class DropoutLayer(NeuronLayer):
    relu_gate = False  # backward of the in-place ReLU producing the bottom is fused here
    def layer_setup(self, bottoms, tops):
        self.ratio = float(self.lp.dropout_param.dropout_ratio)
        if not 0.0 <= self.ratio < 1.0:
            raise ValueError("dropout_ratio must be in [0, 1)")
        self.stream = self.ctx.next_stream_id()

    fused_into = None  # the InnerProduct applying this dropout in its epilogue (engine.fuse_dropout)

    def forward(self, bottoms, tops):
        if self.fused_into is not None and self.phase == 0:
            return  # in place, already applied by the producer's GEMM epilogue
        if self.phase == 0 and self.ratio > 0:  # TRAIN
            tops[0].data = ops.dropout_forward(bottoms[0].data, self.ratio, self.ctx.rng_state, self.stream)
        elif tops[0] is not bottoms[0]:
            tops[0].data = bottoms[0].data

    def backward(self, tops, propagate_down, bottoms):
        if not propagate_down[0]:
            return
        if self.fused_into is not None and self.phase == 0:
            return  # mask, scale and ReLU gate applied by the consumer's dgrad epilogue
        if self.phase == 0 and self.ratio > 0:
            gate = bottoms[0].data if self.relu_gate else None
            bottoms[0].diff = ops.dropout_backward(tops[0].diff, self.ratio, self.ctx.rng_state, self.stream, gate)
        elif self.relu_gate:
            bottoms[0].diff = ops.relu_backward(tops[0].diff, bottoms[0].data)
        elif tops[0] is not bottoms[0]:
            bottoms[0].diff = tops[0].diff


class _Elementwise(NeuronLayer):
    """y = f(x), dx = dy * f'(x, y), computed in fp32 and stored in the compute dtype.
    ``kind`` names the HIP kernel (ops.layers_hip.NEURON); ``needs_x`` says whether the
    derivative reads the input (an in-place layer then keeps a copy of it)."""

    kind: str = ""
    needs_x = True

    def hip_params(self):
        return (0.0, 0.0, 0.0)

    def f(self, x):
        raise NotImplementedError

    def df(self, x, y):
        raise NotImplementedError

    def forward(self, bottoms, tops):
        x = bottoms[0].data
        if x.is_cuda:
            from ..ops import layers_hip as lh
            self._x = x.clone() if (tops[0] is bottoms[0] and self.needs_x) else None
            tops[0].data = lh.neuron_fwd(self.kind, x, None, *self.hip_params())
            return
        self._x = x.float() if tops[0] is bottoms[0] else None
        tops[0].data = self.f(x.float()).to(x.dtype)

    def backward(self, tops, propagate_down, bottoms):
        if not propagate_down[0]:
            return
        dy = tops[0].diff
        if dy.is_cuda:
            from ..ops import layers_hip as lh
            x = (self._x if self._x is not None else bottoms[0].data) if self.needs_x else None
            bottoms[0].diff = lh.neuron_bwd(self.kind, x, tops[0].data, dy, *self.hip_params())
            return
        x = self._x if self._x is not None else bottoms[0].data.float()
        y = tops[0].data.float()
        bottoms[0].diff = (tops[0].diff.float() * self.df(x, y)).to(tops[0].diff.dtype)


@register("Sigmoid")
class SigmoidLayer(_Elementwise):
    kind, needs_x = "Sigmoid", False

    def f(self, x):
        return torch.sigmoid(x)

    def df(self, x, y):
        return y * (1 - y)


@register("TanH")
class TanHLayer(_Elementwise):
    kind, needs_x = "TanH", False

    def f(self, x):
        return torch.tanh(x)

    def df(self, x, y):
        return 1 - y * y


@register("AbsVal")
class AbsValLayer(_Elementwise):
    kind = "AbsVal"

    def f(self, x):
        return x.abs()

    def df(self, x, y):
        return torch.sign(x)


@register("BNLL")
class BNLLLayer(_Elementwise):
    kind = "BNLL"

    def f(self, x):
        return torch.where(x > 0, x + torch.log1p(torch.exp(-x)), torch.log1p(torch.exp(x)))

    def df(self, x, y):
        e = torch.exp(torch.clamp(x, max=50.0))
        return e / (e + 1)


@register("Exp")
class ExpLayer(_Elementwise):
    kind, needs_x = "Exp", False

    def hip_params(self):
        return (self.log_base * self.scale, self.log_base * self.shift, 0.0)

    def layer_setup(self, bottoms, tops):
        p = self.lp.exp_param
        base, self.scale, self.shift = float(p.base), float(p.scale), float(p.shift)
        self.log_base = 1.0 if base == -1 else math.log(base)
        if base != -1 and base <= 0:
            raise ValueError("base must be strictly positive")

    def f(self, x):
        return torch.exp((self.shift + self.scale * x) * self.log_base)

    def df(self, x, y):
        return y * self.log_base * self.scale


@register("Log")
class LogLayer(_Elementwise):
    kind = "Log"

    def hip_params(self):
        return (self.scale, self.shift, self.inv_log_base)

    def layer_setup(self, bottoms, tops):
        p = self.lp.log_param
        base, self.scale, self.shift = float(p.base), float(p.scale), float(p.shift)
        self.inv_log_base = 1.0 if base == -1 else 1.0 / math.log(base)

    def f(self, x):
        return torch.log(self.shift + self.scale * x) * self.inv_log_base

    def df(self, x, y):
        return self.scale * self.inv_log_base / (self.shift + self.scale * x)


@register("Power")
class PowerLayer(_Elementwise):
    kind = "Power"

    def hip_params(self):
        return (self.power, self.scale, self.shift)

    def layer_setup(self, bottoms, tops):
        p = self.lp.power_param
        self.power, self.scale, self.shift = float(p.power), float(p.scale), float(p.shift)

    def f(self, x):
        return torch.pow(self.shift + self.scale * x, self.power)

    def df(self, x, y):
        if self.power == 0 or self.scale == 0:
            return torch.zeros_like(x)
        return self.power * self.scale * torch.pow(self.shift + self.scale * x, self.power - 1)


@register("Threshold")
class ThresholdLayer(NeuronLayer):
    def layer_setup(self, bottoms, tops):
        self.t = float(self.lp.threshold_param.threshold)

    def forward(self, bottoms, tops):
        x = bottoms[0].data
        if x.is_cuda:
            from ..ops import layers_hip as lh
            tops[0].data = lh.neuron_fwd("Threshold", x, self.dtype, self.t)
            return
        tops[0].data = (x.float() > self.t).to(self.dtype)

    def backward(self, tops, propagate_down, bottoms):
        if propagate_down[0]:
            raise NotImplementedError("Threshold layer has no backward")


@register("PReLU")
class PReLULayer(NeuronLayer):
    def layer_setup(self, bottoms, tops):
        p = self.lp.prelu_param
        C = bottoms[0].shape[1] if len(bottoms[0].shape) > 1 else 1
        self.shared = p.channel_shared
        filler = p.filler if p.HasField("filler") else None
        if filler is None:
            from .. import proto
            filler = proto.FillerParameter(type="constant", value=0.25)
        self.slope = self.add_param((1,) if self.shared else (C,), filler=filler)

    def _a(self, x):
        a = self.slope.data.float()
        return a.reshape(-1) if (self.shared or x.dim() != 4) else a  # NHWC: channel is last

    def _bcast(self, a, x):
        if self.shared:
            return a.reshape([1] * x.dim())
        if x.dim() == 4:
            return a.reshape(1, 1, 1, -1)
        return a.reshape([1, -1] + [1] * (x.dim() - 2))

    def _geom(self, x):
        """(C, inner, outer) of the channel axis in the physical layout (NHWC: inner 1)."""
        if self.shared:
            return 1, 1, x.numel()
        if x.dim() == 4:
            return x.shape[-1], 1, x.numel() // x.shape[-1]
        inner = 1
        for d in x.shape[2:]:
            inner *= d
        return x.shape[1], inner, x.shape[0]

    def forward(self, bottoms, tops):
        if bottoms[0].data.is_cuda:
            from ..ops import layers_hip as lh
            x = bottoms[0].data
            self._x = x.clone() if tops[0] is bottoms[0] else x
            C_, inner, _ = self._geom(x)
            tops[0].data = lh.prelu_fwd(x, self.slope.data, C_, inner, out_dtype=tops[0].dtype)
            return
        x = bottoms[0].data.float()
        self._x = x
        a = self._bcast(self.slope.data.float(), x)
        tops[0].data = torch.where(x > 0, x, x * a).to(self.dtype)

    def backward(self, tops, propagate_down, bottoms):
        if tops[0].diff.is_cuda:
            from ..ops import layers_hip as lh
            x, dy = self._x, tops[0].diff
            C_, inner, outer = self._geom(x)
            if self.param_grads_needed(0):
                # slope gradient: sum over everything but the channel of dy * x * [x <= 0]
                lh.axis_reduce(lh.RED_PRELU, dy, x, 1, outer, C_, inner, out=self.slope.diff.view(-1), acc=True)
            if propagate_down[0]:
                bottoms[0].diff = lh.prelu_bwd(x, dy, self.slope.data, C_, inner)
            return
        x = self._x
        dy = tops[0].diff.float()
        a = self._bcast(self.slope.data.float(), x)
        if self.param_grads_needed(0):
            g = dy * x * (x <= 0)
            if self.shared:
                self.slope.diff += g.sum().reshape(1)
            elif x.dim() == 4:
                self.slope.diff += g.sum(dim=(0, 1, 2))
            else:
                dims = [d for d in range(x.dim()) if d != 1]
                self.slope.diff += g.sum(dim=dims)
        if propagate_down[0]:
            bottoms[0].diff = (dy * torch.where(x > 0, torch.ones_like(x), a)).to(self.dtype)
