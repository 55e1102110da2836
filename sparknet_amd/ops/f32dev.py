"""fp32 device mode: the reference's numerics on the MI355X.

Caffe computes every layer in fp32 (``/root/reference/libccaffe/ccaffe.h:3`` ``#define DTYPE
float``; its convolutions are im2col + SGEMM, ``caffe/src/caffe/layers/base_conv_layer.cpp:
312-376``, ``caffe/src/caffe/util/math_functions.cu:14-28``).  A net built with
``dtype=torch.float32`` on a ROCm device runs its products on ``csrc/kernels/fp32.hip``:
exact-f32 matrix cores (``v_mfma_f32_16x16x4_f32``, a k-ordered fmaf chain per output) fed
by an explicit NHWC im2col — the reference's own algorithm, on MFMA instead of SGEMM.  The
remaining (bandwidth-bound) layers run the fp32 formulas of :mod:`.ref` on device tensors.
The production bf16 engine is untouched: ``ops.precision(torch.float32)`` (entered by
``Net`` for fp32 nets on the GPU) routes the dispatch here.

Layouts: activations NHWC fp32, weights [K][R][S][Cg] (the engine's internal layout).
"""
from __future__ import annotations

import torch

from . import _lib, ref
from .spec import ConvSpec

F32 = torch.float32


_BK = 32  # the kernel's k per stage: split-K chunks are multiples of it


def gemm(a: torch.Tensor, b: torch.Tensor, out: torch.Tensor, M: int, N: int, K: int, a_t: bool = False,
         b_t: bool = False, bias=None, relu=False, accumulate=False):
    """out[M][N] (+)= A[M][K] @ B[N][K]^T (+ bias, ReLU), fp32.  ``a_t`` / ``b_t``: the operand
    is stored k-major ([K][M] / [K][N], unit stride along its rows) and is read in place —
    the weight gradients' activations and output gradients, the data gradients' weights — with
    its row stride taken from the tensor.  Products with few 128x128 output tiles and a long
    reduction (the weight gradients: K = pixels) split K over up to ~512 blocks into fp32 slabs
    summed in split order."""
    assert a.dtype == b.dtype == out.dtype == F32 and a.stride(-1) == 1 and b.stride(-1) == 1 and out.stride(1) == 1
    assert out.shape[0] == M and out.shape[1] == N
    assert (a.shape[0], a.shape[1]) == ((K, M) if a_t else (M, K)) and (b.shape[0], b.shape[1]) == ((K, N) if b_t else (N, K))
    trans = int(a_t) | (int(b_t) << 1)
    tiles = -(-M // 128) * -(-N // 128)
    splits = max(1, min(512 // tiles, K // 2048)) if tiles < 256 else 1
    if splits > 1:
        kchunk = -(-(-(-K // splits)) // _BK) * _BK
        splits = -(-K // kchunk)
    if splits == 1:
        _lib.call("gemm_f32", a, a.stride(0), b, b.stride(0), out, out.stride(0), M, N, K,
                  bias if bias is not None else None, int(accumulate), int(relu), 1, K, trans)
        return out
    ws = torch.empty((splits, M, N), dtype=F32, device=out.device)
    _lib.call("gemm_f32", a, a.stride(0), b, b.stride(0), ws, N, M, N, K, None, 0, 0, splits, kchunk, trans)
    r = ws.sum(0)
    if bias is not None:
        r += bias
    if relu:
        r.clamp_(min=0)
    if accumulate:
        out += r
    else:
        out.copy_(r)
    return out


def gemm_nt(a: torch.Tensor, b: torch.Tensor, out: torch.Tensor, bias=None, relu=False, accumulate=False):
    """out[M][N] (+)= a[M][K] @ b[N][K]^T, both operands K-contiguous."""
    return gemm(a, b, out, a.shape[0], b.shape[0], a.shape[1], bias=bias, relu=relu, accumulate=accumulate)


def _c(t):
    return t if t.is_contiguous() else t.contiguous()


def _im2col(x, s: ConvSpec, g: int) -> torch.Tensor:
    col = torch.empty((s.N * s.P * s.Q, s.R * s.S * s.Cg), dtype=F32, device=x.device)
    _lib.call("im2col_f32", x, col, s.N, s.H, s.W, s.C, s.P, s.Q, s.R, s.S, s.sh, s.sw, s.ph, s.pw, s.dh, s.dw,
              s.Cg, g * s.Cg)
    return col


def conv_forward(x, w, b, s: ConvSpec, relu=False, ws=None, folded=None):
    x = _c(x.to(F32))
    y = torch.empty((s.N, s.P, s.Q, s.K), dtype=F32, device=x.device)
    y2 = y.view(-1, s.K)
    w2 = _c(w.to(F32)).view(s.K, -1)
    for g in range(s.groups):
        col = _im2col(x, s, g)
        gemm_nt(col, w2[g * s.Kg:(g + 1) * s.Kg], y2[:, g * s.Kg:(g + 1) * s.Kg],
                bias=b[g * s.Kg:(g + 1) * s.Kg].float().contiguous() if b is not None else None, relu=relu)
    return y


def conv_backward(dy, x, w, s: ConvSpec, need_dx: bool, dw=None, db=None, gate=None, ws=None,
                  dw_acc=True, db_acc=True, dx_out=None):
    """Caffe's order (base_conv_layer.cpp:338-376): per group, dW += dY^T col (col = im2col(x)),
    dcol = dY W, dx = col2im(dcol); db = the column sum of dY."""
    dy = _c(dy.to(F32))
    x = _c(x.to(F32))
    dy2 = dy.view(-1, s.K)
    w2 = _c(w.to(F32)).view(s.K, -1)
    if db is not None:
        ref._acc(db, dy2.sum(0), db_acc)
    dx = torch.empty((s.N, s.H, s.W, s.C), dtype=F32, device=x.device) if need_dx else None
    for g in range(s.groups):
        dyg = dy2[:, g * s.Kg:(g + 1) * s.Kg]
        if dw is not None:
            col = _im2col(x, s, g)
            dwg = dw.view(s.K, -1)[g * s.Kg:(g + 1) * s.Kg]
            # reduction over pixels: both operands read k-major in place (dy's channel slice, col)
            gemm(dyg, col, dwg, s.Kg, col.shape[1], col.shape[0], a_t=True, b_t=True, accumulate=dw_acc)
        if need_dx:
            dcol = torch.empty((s.N * s.P * s.Q, s.R * s.S * s.Cg), dtype=F32, device=x.device)
            wg = w2[g * s.Kg:(g + 1) * s.Kg]  # [Kg][kred]: k-major B of dcol = dy_g @ w_g
            gemm(dyg, wg, dcol, dcol.shape[0], wg.shape[1], s.Kg, b_t=True)
            _lib.call("col2im_f32", dcol, dx, s.N, s.H, s.W, s.C, s.P, s.Q, s.R, s.S, s.sh, s.sw, s.ph, s.pw,
                      s.dh, s.dw, s.Cg, g * s.Cg, 0)
    if dx is not None:
        dx = ref._gated(dx, gate.to(F32) if gate is not None else None)
        if dx_out is not None:
            dx_out.copy_(dx)
            return dx_out
    return dx


def linear_forward(x2, w, b, relu=False):
    x2 = _c(x2.to(F32))
    y = torch.empty((x2.shape[0], w.shape[0]), dtype=F32, device=x2.device)
    return gemm_nt(x2, _c(w.to(F32)), y, bias=b.float().contiguous() if b is not None else None, relu=relu)


def linear_backward(dy2, x2, w, need_dx, dw=None, db=None, gate=None, dw_acc=True, db_acc=True):
    """inner_product_layer.cu:22-54: dW (+)= dY^T X, db (+)= colsum(dY), dX = dY W."""
    dy2 = _c(dy2.to(F32))
    x2 = _c(x2.to(F32))
    if dw is not None:
        gemm(dy2, x2, dw, dy2.shape[1], x2.shape[1], dy2.shape[0], a_t=True, b_t=True, accumulate=dw_acc)
    if db is not None:
        ref._acc(db, dy2.sum(0), db_acc)
    if not need_dx:
        return None
    dx = torch.empty_like(x2)
    wf = _c(w.to(F32))  # [N][K]: k-major B of dx = dy @ w
    gemm(dy2, wf, dx, dy2.shape[0], wf.shape[1], wf.shape[0], b_t=True)
    return ref._gated(dx, gate.reshape(x2.shape).to(F32) if gate is not None else None)


def dropout_forward(x, ratio, rng_state, stream):
    """dropout_layer.cu: the device Philox keep mask of the bf16 engine (same bits)."""
    x = _c(x.to(F32))
    y = torch.empty_like(x)
    _lib.call("dropout_f32", x, y, x.numel(), rng_state, int(stream), float(ratio), None)
    return y


def dropout_backward(dy, ratio, rng_state, stream, gate=None):
    dy = _c(dy.to(F32))
    dx = torch.empty_like(dy)
    _lib.call("dropout_f32", dy, dx, dy.numel(), rng_state, int(stream), float(ratio),
              _c(gate.to(F32)) if gate is not None else None)
    return dx


def _pool_args(s):
    return (s.N, s.H, s.W, s.C, s.P, s.Q, s.kh, s.kw, s.sh, s.sw, s.ph, s.pw)


def pool_forward_aux(x, s, gate=False):
    """pooling_layer.cu MaxPoolForward / AvePoolForward on NHWC fp32: (y, argmax flat index
    h * W + w per output for MAX, else None)."""
    from .spec import POOL_AVE, POOL_MAX
    if s.method not in (POOL_MAX, POOL_AVE):  # stochastic pooling: the reference formulas
        return ref.pool_forward(x, s), None
    x = _c(x.to(F32))
    mx = s.method == POOL_MAX
    y = torch.empty((s.N, s.P, s.Q, s.C), dtype=F32, device=x.device)
    mask = torch.empty((s.N, s.P, s.Q, s.C), dtype=torch.int32, device=x.device) if mx else None
    _lib.call("pool_f32", x, y, mask, *_pool_args(s), int(mx))
    return y, mask


def pool_forward(x, s):
    return pool_forward_aux(x, s)[0]


def pool_backward(dy, x, s, aux=None, y=None, gate=False):
    """MaxPoolBackward / AvePoolBackward: the gather over the windows covering each input."""
    from .spec import POOL_AVE, POOL_MAX
    mx = s.method == POOL_MAX
    if s.method not in (POOL_MAX, POOL_AVE) or (mx and aux is None):
        return ref.pool_backward(dy, x, s, gate)
    dy = _c(dy.to(F32))
    dx = torch.empty((s.N, s.H, s.W, s.C), dtype=F32, device=dy.device)
    _lib.call("pool_f32_bwd", dy, aux if mx else None, dx, *_pool_args(s), int(mx))
    return ref._gated(dx, x if gate else None)


def relu_forward(x, slope=0.0):
    """relu_layer.cu forward, one pass (same operations as the reference formula)."""
    x = _c(x.to(F32))
    y = torch.empty_like(x)
    _lib.call("relu_f32", x, y, x.numel(), float(slope))
    return y


def relu_backward(dy, x, slope=0.0):
    dy, x = _c(dy.to(F32)), _c(x.to(F32))
    dx = torch.empty_like(dy)
    _lib.call("relu_f32_bwd", dy, x, dx, dy.numel(), float(slope))
    return dx


def __getattr__(name):
    # every other op: the fp32 formulas of the reference module, on device tensors.  (LRN stays
    # there on purpose: an LRN kernel with the same formula but its own rounding moved CaffeNet's
    # conv1 one-step update by 1.4e-3 relative to the CPU engine — that update is a sum of nearly
    # cancelling terms — against 0.9e-3 with the reference's own operations; scripts/fp32_gate_probe.py)
    return getattr(ref, name)
