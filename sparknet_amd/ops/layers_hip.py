"""ctypes wrappers of ``csrc/kernels/layers.hip``: the non-hot Caffe layer families on the
GPU (neurons, PReLU, Eltwise, BatchNorm / MVN, axis copies, layout changes, row gathers /
scatter-adds, Reduction, ArgMax, Caffe-ordered Im2col, the loss family).

Every function launches HIP kernels on torch's current stream (graph-capturable); torch is
used only to allocate outputs.  Tensors must be contiguous bf16 or fp32 device tensors.
Shapes are described as ``[B][outer][A][inner]`` decompositions of the PHYSICAL layout.
"""
from __future__ import annotations

import ctypes as C

import torch

from . import _lib

call = _lib.call

NEURON = {"Sigmoid": 0, "TanH": 1, "AbsVal": 2, "BNLL": 3, "Exp": 4, "Log": 5, "Power": 6, "Threshold": 7}
RED_SUM, RED_DOT, RED_SQ, RED_PRELU, RED_ABS, RED_CSQ = 0, 1, 2, 3, 4, 5
LOSS = {"Euclidean": 0, "HingeL1": 1, "HingeL2": 2, "Multinomial": 3, "Infogain": 4, "SigmoidXent": 5,
        "Contrastive": 6}


def dt(t: torch.Tensor) -> int:
    if t.dtype == torch.float32:
        return 1
    if t.dtype == torch.bfloat16:
        return 0
    raise TypeError(f"layers_hip: unsupported dtype {t.dtype}")


def _c(t):
    if t is None:
        return None
    return t if t.is_contiguous() else t.contiguous()


# -- neurons -------------------------------------------------------------------------------
def neuron_fwd(kind: str, x, out_dtype=None, a=0.0, b=0.0, c=0.0):
    x = _c(x)
    y = torch.empty(x.shape, dtype=out_dtype or x.dtype, device=x.device)
    call("neuron_fwd", NEURON[kind], x, y, x.numel(), dt(x), dt(y), float(a), float(b), float(c))
    return y


def neuron_bwd(kind: str, x, y, dy, a=0.0, b=0.0, c=0.0):
    dy = _c(dy)
    dx = torch.empty_like(dy)
    call("neuron_bwd", NEURON[kind], _c(x), _c(y), dy, dx, dy.numel(), dt(x) if x is not None else 0,
         dt(y) if y is not None else 0, dt(dy), float(a), float(b), float(c))
    return dx


def prelu_fwd(x, slope, C_, inner, out_dtype=None):
    x = _c(x)
    y = torch.empty(x.shape, dtype=out_dtype or x.dtype, device=x.device)
    call("prelu_fwd", x, _c(slope), y, x.numel(), C_, inner, dt(x), dt(y))
    return y


def prelu_bwd(x, dy, slope, C_, inner):
    """dx in dy's dtype; x may be in another dtype (an fp32 2-D Input blob)."""
    dy = _c(dy)
    dx = torch.empty_like(dy)
    call("prelu_bwd", _c(x), dy, _c(slope), dx, dy.numel(), C_, inner, dt(x), dt(dy))
    return dx


# -- deterministic reductions --------------------------------------------------------------
def axis_reduce(mode, p, q, B, outer, A, inner, out=None, scale=1.0, acc=False):
    """out[b*A + a] (+)= scale * sum over (outer, inner) of f(p, q) (fp32, deterministic)."""
    p = _c(p)
    q = _c(q)
    k = _lib.kernels()
    k.sn_axis_reduce_splits.restype = C.c_longlong
    splits = int(k.sn_axis_reduce_splits(C.c_longlong(B), C.c_longlong(outer), C.c_longlong(A),
                                         C.c_longlong(inner)))
    part = torch.empty(splits * B * A, dtype=torch.float32, device=p.device)
    if out is None:
        out = torch.empty(B * A, dtype=torch.float32, device=p.device)
        acc = False
    call("axis_reduce", mode, p, q, dt(p), dt(q) if q is not None else 0, B, outer, A, inner, part, out,
         float(scale), int(acc))
    return out


def stats_finalize(s1, s2, count, eps, mode):
    n = s1.numel()
    mean = torch.empty(n, dtype=torch.float32, device=s1.device)
    var = torch.empty_like(mean)
    inv = torch.empty_like(mean)
    call("stats_finalize", s1, s2, n, 1.0 / max(count, 1), float(eps), mode, mean, var, inv)
    return mean, var, inv


def mean_var(x, B, outer, A, inner, eps, mode):
    """Per-(b, a) mean, variance and inverse scale of x over (outer, inner) in two
    deterministic passes: the mean, then the CENTRED second moment E[(x - mean)^2]
    (Caffe's batch_norm_layer.cu:50-59 / mvn_layer.cu:31-36 order, no E[x^2] - EX^2
    cancellation).  mode as stats_finalize: 0 BatchNorm, 1 MVN."""
    count = outer * inner
    s1 = axis_reduce(RED_SUM, x, None, B, outer, A, inner)
    mean, _, _ = stats_finalize(s1, None, count, eps, 2)
    s2 = axis_reduce(RED_CSQ, x, mean, B, outer, A, inner)
    return stats_finalize(s1, s2, count, eps, mode | 4)


def chan_affine(x, mean, inv, outer, A, inner, out_dtype=None):
    x = _c(x)
    y = torch.empty(x.shape, dtype=out_dtype or x.dtype, device=x.device)
    call("chan_affine", x, y, x.numel(), outer, A, inner, mean, inv, dt(x), dt(y))
    return y


def norm_bwd(dy, xhat, m1, m2, inv, outer, A, inner):
    dy = _c(dy)
    dx = torch.empty_like(dy)
    call("norm_bwd", dy, _c(xhat), dx, dy.numel(), outer, A, inner, m1, m2, inv, dt(dy),
         dt(xhat) if xhat is not None else 0)
    return dx


def bn_running(mean, var, factor, bmean, bvar, frac, unbias):
    call("bn_running", mean, var, factor, bmean, bvar, mean.numel(), float(frac), float(unbias))


def bn_global(rm, rv, factor, eps):
    Cn = rm.numel()
    mean = torch.empty(Cn, dtype=torch.float32, device=rm.device)
    inv = torch.empty_like(mean)
    call("bn_global", rm, rv, factor, Cn, float(eps), mean, inv)
    return mean, inv


# -- eltwise -------------------------------------------------------------------------------
def _ptrs(xs):
    arr = (C.c_void_p * len(xs))(*[t.data_ptr() for t in xs])
    return arr


def eltwise_fwd(op, xs, coeffs):
    xs = [_c(x) for x in xs]
    y = torch.empty_like(xs[0])
    mask = torch.empty(xs[0].shape, dtype=torch.int32, device=y.device) if op == 2 else None
    co = (C.c_float * len(xs))(*[float(c) for c in coeffs])
    call("eltwise_fwd", _ptrs(xs), co, len(xs), op, y, mask, y.numel(), dt(y))
    return y, mask


def eltwise_bwd(op, xs, coeffs, which, stable, y, dy, mask):
    xs = [_c(x) for x in xs]
    dy = _c(dy)
    dx = torch.empty_like(dy)
    co = (C.c_float * len(xs))(*[float(c) for c in coeffs])
    call("eltwise_bwd", _ptrs(xs), co, len(xs), op, which, int(stable), _c(y), dy, mask, dx, dy.numel(), dt(dy))
    return dx


# -- copies / layout -----------------------------------------------------------------------
def axis_copy(src, dst, outer, srcA, dstA, inner, src_off, dst_off, cnt, acc=False):
    call("axis_copy", _c(src), dst, outer, srcA, dstA, inner, src_off, dst_off, cnt, dt(src), dt(dst), int(acc))


def tile_bwd(src, outer, A, inner, tiles, out_shape):
    dst = torch.empty(out_shape, dtype=src.dtype, device=src.device)
    call("tile_bwd", _c(src), dst, outer, A, inner, tiles, dt(src))
    return dst


def transpose(src, N, R, Ccols, out_shape=None, out_dtype=None):
    """[N][R][Ccols] -> [N][Ccols][R] (NHWC <-> NCHW with R = HW / C)."""
    dst = torch.empty(out_shape if out_shape is not None else (N, Ccols, R), dtype=out_dtype or src.dtype,
                      device=src.device)
    call("transpose", _c(src), dst, N, R, Ccols, dt(src), dt(dst))
    return dst


def nhwc_to_nchw(t, out_dtype=None):
    N, H, W, Cn = t.shape
    return transpose(t, N, H * W, Cn, (N, Cn, H, W), out_dtype)


def nchw_to_nhwc(t, N, Cn, H, W, out_dtype=None):
    return transpose(t, N, Cn, H * W, (N, H, W, Cn), out_dtype)


# -- gathers / scatter-adds ----------------------------------------------------------------
def gather_rows(src, idx, rows, row_len, out_shape, bias=None, out_dtype=None):
    idx = _c(idx)
    dst = torch.empty(out_shape, dtype=out_dtype or src.dtype, device=src.device)
    call("gather_rows", _c(src), idx, int(idx.dtype == torch.int32), dst, rows, row_len, bias, dt(src), dt(dst))
    return dst


def index_add_rows(src, idx, n_dst, row_len, dst, acc):
    idx = _c(idx)
    call("index_add_rows", _c(src), idx, int(idx.dtype == torch.int32), idx.numel(), dst, n_dst, row_len,
         dt(src), dt(dst), int(acc))
    return dst


# -- Reduction / ArgMax / Im2col ------------------------------------------------------------
def reduction_bwd(x, dy, segs, L, op, coeff):
    x = _c(x)
    dx = torch.empty_like(x)
    call("reduction_bwd", x, _c(dy), dx, segs, L, op, float(coeff), dt(x))
    return dx


def topk(x, outer, A, inner, k, out_max_val, axis_mode, out_shape):
    out = torch.empty(out_shape, dtype=torch.float32, device=x.device)
    call("topk", _c(x), outer, A, inner, k, int(out_max_val), int(axis_mode), out, dt(x))
    return out


def im2col_caffe(x, g, out_shape):
    col = torch.empty(out_shape, dtype=x.dtype, device=x.device)
    call("im2col_caffe", _c(x), col, *g, dt(x))
    return col


def col2im_caffe(dcol, g, out_shape):
    dx = torch.empty(out_shape, dtype=dcol.dtype, device=dcol.device)
    call("col2im_caffe", _c(dcol), dx, *g, dt(dcol))
    return dx


# -- losses --------------------------------------------------------------------------------
def loss_rows_fwd(kind, x, t, label, H, M, C_, margin=0.0, legacy=False):
    """Per-row loss terms [M] (and d2 [M] for Contrastive) -> (row_loss, workspace)."""
    x = _c(x)
    ws = torch.empty(3 * M, dtype=torch.float32, device=x.device)
    call("loss_rows_fwd", LOSS[kind], x, _c(t), _c(label), _c(H), M, C_, dt(x), dt(t) if t is not None else 0,
         float(margin), int(legacy), ws)
    return ws


def loss_sum(ws, M, scale):
    """0-d fp32 loss = scale * sum(ws[:M]) (device, no host sync)."""
    out = torch.empty((), dtype=torch.float32, device=ws.device)
    call("vsum", ws, M, out, float(scale), 0)
    return out


def loss_rows_bwd(kind, x, t, label, H, M, C_, loss_weight, scale, sign=1.0, ws=None, margin=0.0, legacy=False):
    x = _c(x)
    dx = torch.empty_like(x)
    d2 = ws[M:2 * M] if ws is not None else None
    call("loss_rows_bwd", LOSS[kind], x, _c(t), _c(label), _c(H), M, C_, dt(x), dt(t) if t is not None else 0,
         float(margin), int(legacy), _c(loss_weight.reshape(-1).float()), float(scale), float(sign), d2, dx)
    return dx


# -- stochastic pooling ----------------------------------------------------------------------
def stopool(x, s, rng_state, stream, train):
    """(y, mask): mask holds the sampled window offset (train) for the max-pool backward."""
    x = _c(x)
    y = torch.empty((s.N, s.P, s.Q, s.C), dtype=x.dtype, device=x.device)
    mask = torch.empty((s.N, s.P, s.Q, s.C), dtype=torch.uint8, device=x.device) if train else None
    call("stopool", x, y, mask, s.N, s.H, s.W, s.C, s.P, s.Q, s.kh, s.kw, s.sh, s.sw, rng_state, int(stream),
         int(train))
    return y, mask
