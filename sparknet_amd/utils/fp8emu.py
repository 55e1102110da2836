"""e4m3 storage emulation on the CPU engine: the floor of the fp8 fidelity gates.

The GPU fp8 mode (:func:`sparknet_amd.engine.enable_fp8`) quantises per tensor, at three kinds
of product, to OCP e4m3 with a scale ``s = 448 / amax`` and dequantises in the fp32 epilogue:

* forward (``layer.fp8_slots``): the layer input x and the bf16 weights;
* data gradient (``layer.fp8_dgrad_slots``, stride-1 convs): the output gradient dy and the
  (flip-transposed) weights;
* weight gradient (``layer.fp8_wgrad``): dy's fp8 copy (shared with the data gradient) and the
  forward's fp8 x; the bias gradient is the column sum of the quantised dy (the e4m3 ones column,
  ``features fp8_wgrad_bias``).

:func:`emulate` applies the same quantisation points to a CPU (fp32-compute) net's operands —
``q(t) = e4m3(t * s) / s`` with the tensor's own amax, which is the GPU's scaling on an
iteration whose slots are uninitialised (the first; later iterations take the amax history,
``csrc/kernels/fp8.hip``).  Run on a bf16-storage CPU net it isolates what e4m3 (plus bf16)
storage alone does to an update, independent of any GPU kernel: the yardstick the one-step
fp8 gate (tests/test_fp8_update_gate_gpu.py) bounds the GPU's deviation by.

Reference: Caffe has no reduced-precision mode (libccaffe/ccaffe.h:3 ``#define DTYPE float``);
the gate's pattern is caffe/src/caffe/test/test_gradient_based_solver.cpp:225-320.
"""
from __future__ import annotations

import contextlib
import threading

import torch

from ..ops import ref

E4M3_MAX = 448.0
_cur = threading.local()


def quant(t: torch.Tensor, block: int = 0, dim: int = -1) -> torch.Tensor:
    """fp32 values of ``t`` stored as e4m3 with per-tensor current scaling (RNE, saturating
    at 448 by construction of the scale); an all-zero tensor stays zero.

    ``block`` > 0: CDNA4 block scaling instead (what ``v_mfma_scale_f32_16x16x128_f8f6f4``'s
    E8M0 operands would carry): every run of ``block`` consecutive elements along ``dim`` (the
    product's reduction dimension) gets its own power-of-two scale, the smallest that keeps the
    run's |max| within 448."""
    tf = t.detach().float()
    if block:
        v = tf.movedim(dim, -1)
        shp = v.shape
        n = shp[-1]
        pad = -n % block
        v = torch.nn.functional.pad(v.reshape(-1, n), (0, pad)).reshape(-1, block)
        amax = v.abs().amax(1, keepdim=True)
        e = torch.ceil(torch.log2(amax.clamp_min(1e-30) / E4M3_MAX))
        sc = torch.where(amax > 0, torch.exp2(e), torch.ones_like(amax))
        q = (v / sc).clamp_(-E4M3_MAX, E4M3_MAX).to(torch.float8_e4m3fn).float() * sc
        q = q.reshape(-1, n + pad)[:, :n].reshape(shp)
        return q.movedim(-1, dim).contiguous()
    a = float(tf.abs().max()) if tf.numel() else 0.0
    if not a > 0.0 or a == float("inf"):
        return tf
    s = torch.tensor(E4M3_MAX, dtype=torch.float32) / a
    return (tf * s).clamp_(-E4M3_MAX, E4M3_MAX).to(torch.float8_e4m3fn).float() / s


def _q(t, dim=-1):
    """quant() with the active emulation's block size (0: per tensor)."""
    return quant(t, getattr(_cur, "block", 0), dim)


def _rows(t):
    """NHWC activation / gradient as [pixels][channels] (the weight gradient reduces over pixels)."""
    return t.reshape(-1, t.shape[-1])


def fp8_modes(net) -> dict:
    """{layer name: (fwd, dgrad, wgrad)} of the fp8 products an fp8-enabled (GPU) net runs."""
    out = {}
    for layer in net.layers:
        m = (getattr(layer, "fp8_slots", None) is not None, getattr(layer, "fp8_dgrad_slots", None) is not None,
             bool(getattr(layer, "fp8_wgrad", False)))
        if any(m):
            out[layer.name] = m
    return out


def _mode():
    return getattr(_cur, "mode", None)


def _conv_forward(orig):
    def fn(x, w, b, s, relu=False, ws=None, folded=None):
        m = _mode()
        if not (m and m[0]):
            return orig(x, w, b, s, relu=relu, ws=ws, folded=folded)
        return orig(_q(x), _q(w), b, s, relu=relu).to(x.dtype)
    return fn


def _conv_backward(orig):
    def fn(dy, x, w, s, need_dx, dw=None, db=None, gate=None, ws=None, dw_acc=True, db_acc=True, **kw):
        m = _mode()
        if not (m and (m[1] or m[2])):
            return orig(dy, x, w, s, need_dx, dw=dw, db=db, gate=gate, ws=ws, dw_acc=dw_acc, db_acc=db_acc, **kw)
        if dw is not None or db is not None:
            if m[2]:  # reduction over pixels
                qdy = _q(_rows(dy), 0).reshape(dy.shape)
                orig(qdy, _q(_rows(x), 0).reshape(x.shape), w, s, False, dw=dw, db=db, dw_acc=dw_acc, db_acc=db_acc)
            else:
                orig(dy, x, w, s, False, dw=dw, db=db, dw_acc=dw_acc, db_acc=db_acc)
        if not need_dx:
            return None
        if not m[1]:
            return orig(dy, x, w, s, True, gate=gate)
        # reduction over output channels: dy's channels, the weights' rows
        return orig(_q(dy), x, _q(w.reshape(s.K, -1), 0).reshape(w.shape), s, True, gate=gate).to(x.dtype)
    return fn


def _linear_forward(orig):
    def fn(x2, w, b, relu=False, **kw):
        m = _mode()
        if not (m and m[0]):
            return orig(x2, w, b, relu=relu, **kw)
        return orig(_q(x2), _q(w), b, relu=relu).to(x2.dtype)
    return fn


def _scoped(fn, mode):
    def call(*a, **k):
        prev = _mode()
        _cur.mode = mode
        try:
            return fn(*a, **k)
        finally:
            _cur.mode = prev
    return call


@contextlib.contextmanager
def emulate(net, modes: dict, block: int = 0):
    """Within the block, the CPU ``net``'s layers named in ``modes`` ({name: (fwd, dgrad,
    wgrad)}, e.g. :func:`fp8_modes` of the GPU net) quantise their product operands to e4m3
    (``block``: per-``block`` power-of-two scales along each product's reduction dimension
    instead of one scale per tensor)."""
    assert net.device.type == "cpu"
    prev_block = getattr(_cur, "block", 0)
    _cur.block = block
    patched = {"conv_forward": _conv_forward, "conv_backward": _conv_backward, "linear_forward": _linear_forward}
    saved = {k: getattr(ref, k) for k in patched}
    wrapped = []
    try:
        for k, mk in patched.items():
            setattr(ref, k, mk(saved[k]))
        for layer in net.layers:
            if layer.name in modes:
                wrapped.append(layer)
                layer.forward = _scoped(type(layer).forward.__get__(layer), modes[layer.name])
                layer.backward = _scoped(type(layer).backward.__get__(layer), modes[layer.name])
        yield
    finally:
        _cur.block = prev_block
        for k, v in saved.items():
            setattr(ref, k, v)
        for layer in wrapped:
            del layer.forward, layer.backward
