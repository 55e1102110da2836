"""Device-dispatching op layer.

Every op has two implementations with identical semantics:

* :mod:`.hip` — hand-written HIP/CDNA4 kernels from ``libsn_kernels.so`` (used for every
  tensor on a ROCm device; there is NO silent PyTorch fallback on the GPU — if the
  native library is missing the call raises);
* :mod:`.ref` — PyTorch fp32 reference (CPU tensors; also the test oracle).
"""
from __future__ import annotations

import contextlib
import threading

import torch

from . import ref
from .spec import POOL_AVE, POOL_MAX, POOL_STOCHASTIC, ConvNdSpec, ConvSpec, PoolSpec  # noqa: F401

_hip = None
_state = threading.local()


def _hipmod():
    global _hip
    if _hip is None:
        from . import hip as _h
        _hip = _h
    return _hip


def f32_active() -> bool:
    """Inside ``precision(torch.float32)``: GPU tensors take the fp32 device path."""
    return getattr(_state, "f32", False)


@contextlib.contextmanager
def precision(dtype):
    """Net forward / backward of a ``dtype`` net: fp32 nets on the GPU route every op to
    :mod:`.f32dev` (fp32 MFMA products + the reference formulas), bf16 nets to :mod:`.hip`."""
    prev = f32_active()
    _state.f32 = dtype == torch.float32
    try:
        yield
    finally:
        _state.f32 = prev


def _gpu(t: torch.Tensor) -> bool:
    """The bf16 HIP engine serves this tensor (a GPU tensor outside the fp32 device mode)."""
    return t.is_cuda and not f32_active()


def _impl(t: torch.Tensor):
    if not t.is_cuda:
        return ref
    if f32_active():
        from . import f32dev
        return f32dev
    return _hipmod()


def _dispatch(name):
    def fn(first, *args, **kwargs):
        return getattr(_impl(first), name)(first, *args, **kwargs)
    fn.__name__ = name
    return fn


conv_forward = _dispatch("conv_forward")
conv_backward = _dispatch("conv_backward")
conv_nd_forward = _dispatch("conv_nd_forward")
conv_nd_backward = _dispatch("conv_nd_backward")
linear_forward = _dispatch("linear_forward")
linear_backward = _dispatch("linear_backward")
pool_forward = _dispatch("pool_forward")
lrn_forward = _dispatch("lrn_forward")
lrn_backward = _dispatch("lrn_backward")
relu_forward = _dispatch("relu_forward")
relu_backward = _dispatch("relu_backward")
softmax_forward = _dispatch("softmax_forward")
softmax_backward = _dispatch("softmax_backward")
accuracy = _dispatch("accuracy")


def pool_backward(dy, x, s, aux=None, y=None, gate=False):
    """gate=True: x is a slope-0 in-place ReLU output whose backward is fused here (MAX
    pooling on the GPU encodes it in the forward's argmax mask)."""
    if _gpu(dy):
        return _hipmod().pool_backward(dy, x, s, aux, y, gate)
    if dy.is_cuda:  # fp32 device mode
        from . import f32dev
        return f32dev.pool_backward(dy, x, s, aux, y, gate)
    return ref.pool_backward(dy, x, s, gate)


def pool_forward_aux(x, s, gate=False):
    """Forward returning (y, aux) where aux is the GPU argmax mask (None on CPU)."""
    if _gpu(x):
        return _hipmod().pool_forward_mask(x, s, gate)
    if x.is_cuda:  # fp32 device mode
        from . import f32dev
        return f32dev.pool_forward_aux(x, s, gate)
    return ref.pool_forward(x, s), None


def dropout_forward(x, ratio, rng_state, stream):
    if _gpu(x):
        return _hipmod().dropout_forward(x, ratio, rng_state, stream)
    if x.is_cuda:
        from . import f32dev
        return f32dev.dropout_forward(x, ratio, rng_state, stream)
    seed, counter = (int(v) for v in rng_state.tolist())
    return ref.dropout_forward(x, ratio, seed, counter, stream)


def dropout_backward(dy, ratio, rng_state, stream, gate=None):
    if _gpu(dy):
        return _hipmod().dropout_backward(dy, ratio, rng_state, stream, gate)
    if dy.is_cuda:
        from . import f32dev
        return f32dev.dropout_backward(dy, ratio, rng_state, stream, gate)
    seed, counter = (int(v) for v in rng_state.tolist())
    return ref.dropout_backward(dy, ratio, seed, counter, stream, gate)


def softmax_loss_forward(x2, labels, ignore_label=None, normalize=True, outer_num=None):
    return _impl(x2).softmax_loss_forward(x2, labels, ignore_label, normalize, outer_num)


def softmax_loss_backward(prob, labels, loss_weight, norm, ignore_label=None, dtype=torch.float32):
    return _impl(prob).softmax_loss_backward(prob, labels, loss_weight, norm, ignore_label, dtype)


def sum_bf16(tensors):
    """Elementwise sum of same-shape bf16 device tensors (fp32 accumulation)."""
    return _hipmod().sum_bf16([t.contiguous() for t in tensors])


def cast_f32_to_bf16(src: torch.Tensor, dst: torch.Tensor) -> None:
    if src.is_cuda:
        _hipmod().cast_f32_to_bf16(src, dst)
    else:
        dst.copy_(src)


def advance_rng(rng_state: torch.Tensor) -> None:
    """Bump the Philox counter once per iteration (device-side, graph-capturable)."""
    if rng_state.is_cuda:
        _hipmod().advance_rng(rng_state)
    else:
        rng_state[1] += 1


def solver_tables(segments, total: int, device, slab_chunks=None) -> dict:
    """Per-element multipliers (CPU reference) or the chunk table of the fused HIP update
    (``slab_chunks``: gradients read from split-K slabs, GPU only)."""
    device = torch.device(device)
    if device.type == "cuda":
        return _hipmod().solver_tables(segments, total, device, slab_chunks)
    assert not slab_chunks
    lr = torch.zeros(max(total, 1))
    dc = torch.zeros(max(total, 1))
    for off, cnt, lm, dm in segments:
        lr[off:off + cnt] = lm
        dc[off:off + cnt] = dm
    return {"lr": lr, "decay": dc}


def solver_update(kind, data, diff, history, compute, tables, hyper, l1: bool, clip: bool,
                  grid_limit: int = 0) -> None:
    if data.is_cuda:
        _hipmod().solver_update(kind, data, diff, history, compute, tables, hyper, l1, clip, grid_limit)
        return
    h = hyper.tolist()
    ref.solver_update_ref(kind, data, diff, history, tables["lr"], tables["decay"], h, l1, clip)
    if compute is not None and compute is not data:
        compute.copy_(data)
