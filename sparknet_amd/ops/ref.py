"""PyTorch fp32 reference implementations of every op (CPU path and test oracle).

Each function mirrors the Caffe CPU/GPU semantics of the corresponding layer (file:line
cited per function) on NHWC tensors.  Complex backward passes are obtained with
autograd on the forward formula, which gives the exact analytic gradient that the
reference's hand-written backward kernels implement.  These run on the CPU reference
path (``device='cpu'``) and serve as the oracle for the HIP kernel tests.
"""
from __future__ import annotations

import math

import torch
import torch.nn.functional as F

from .spec import POOL_AVE, POOL_MAX, ConvNdSpec, ConvSpec, PoolSpec


def nchw(x):
    return x.permute(0, 3, 1, 2)


def nhwc(x):
    return x.permute(0, 2, 3, 1).contiguous()


def _w_oihw(w, s: ConvSpec):
    return w.reshape(s.K, s.R, s.S, s.Cg).permute(0, 3, 1, 2)


# --- convolution (base_conv_layer.cpp:312-376, conv_layer.cpp) -----------------------

def conv_forward(x, w, b, s: ConvSpec, relu=False, ws=None, folded=None):
    y = F.conv2d(nchw(x.float()), _w_oihw(w.float(), s), b.float() if b is not None else None,
                 stride=(s.sh, s.sw), padding=(s.ph, s.pw), dilation=(s.dh, s.dw), groups=s.groups)
    if relu:
        y = F.relu(y)
    return nhwc(y).to(x.dtype)


# --- N-d convolution (base_conv_layer.cpp:16-40, im2col.cpp im2col_nd_cpu) ------------

def im2col_nd(x, s: ConvNdSpec, g: int = 0):
    """[num][C][ins] -> col [num * P][Cg * T] of channel group g (Caffe's (c, taps) order)."""
    xp = F.pad(x[:, g * s.Cg:(g + 1) * s.Cg], [p for d in reversed(s.pd) for p in (d, d)])
    taps = []
    import itertools
    for kk in itertools.product(*[range(k) for k in s.ks]):
        idx = [slice(None), slice(None)] + [slice(k0, k0 + st * (o - 1) + 1, st)
                                            for k0, st, o in zip(kk, s.st, s.outs)]
        taps.append(xp[tuple(idx)])
    col = torch.stack(taps, 2)  # [num][Cg][T][outs]
    return col.reshape(s.num, s.Cg * s.T, s.P).transpose(1, 2).reshape(s.num * s.P, s.Cg * s.T)


def conv_nd_forward(x, w, b, s: ConvNdSpec):
    """x [num][C][ins], w [K][Cg][ks] (Caffe layout) -> y [num][K][outs]."""
    x, w = x.float(), w.float()
    ys = []
    for g in range(s.groups):
        col = im2col_nd(x, s, g)
        wg = w[g * s.Kg:(g + 1) * s.Kg].reshape(s.Kg, -1)
        ys.append((col @ wg.t()).reshape(s.num, s.P, s.Kg).transpose(1, 2))
    y = torch.cat(ys, 1)
    if b is not None:
        y = y + b.float().view(1, -1, 1)
    return y.reshape((s.num, s.K) + s.outs)


def conv_nd_backward(dy, x, w, s: ConvNdSpec, need_dx: bool, dw=None, db=None):
    """Gradients of conv_nd_forward by autograd on the same formula; dw / db accumulate
    (Caffe's Backward adds into the param diffs).  x may be None when dw is None (the data
    gradient alone: a Deconvolution forward)."""
    if x is None:
        assert dw is None
        x = torch.zeros((s.num, s.C) + tuple(s.ins), dtype=dy.dtype)
    xr = x.float().detach().requires_grad_(need_dx)
    wr = w.float().detach().requires_grad_(dw is not None)
    y = conv_nd_forward(xr, wr, None, s)
    ins = [t for t in (xr, wr) if t.requires_grad]
    grads = torch.autograd.grad(y, ins, dy.float()) if ins else ()
    gi = iter(grads)
    dx = next(gi) if need_dx else None
    if dw is not None:
        dw += next(gi).reshape(dw.shape)
    if db is not None:
        db += dy.float().reshape(s.num, s.K, -1).sum((0, 2))
    return dx.to(x.dtype) if dx is not None else None


def _gated(dx, gate):
    """Backward of a slope-0 ReLU whose output is ``gate`` (fused into the producer)."""
    return dx if gate is None else dx * (gate > 0).to(dx.dtype)


def _acc(dst, val, accumulate):
    if accumulate:
        dst += val
    else:
        dst.copy_(val)


def conv_backward(dy, x, w, s: ConvSpec, need_dx: bool, dw=None, db=None, gate=None, ws=None,
                  dw_acc=True, db_acc=True):
    dyn = nchw(dy.float())
    xn = nchw(x.float())
    wo = _w_oihw(w.float(), s)
    dx = None
    if need_dx:
        dx = torch.nn.grad.conv2d_input(xn.shape, wo, dyn, stride=(s.sh, s.sw), padding=(s.ph, s.pw),
                                        dilation=(s.dh, s.dw), groups=s.groups)
        dx = _gated(nhwc(dx).to(x.dtype), gate)
    if dw is not None:
        gw = torch.nn.grad.conv2d_weight(xn, wo.shape, dyn, stride=(s.sh, s.sw), padding=(s.ph, s.pw),
                                         dilation=(s.dh, s.dw), groups=s.groups)
        _acc(dw, gw.permute(0, 2, 3, 1).reshape(dw.shape), dw_acc)
    if db is not None:
        _acc(db, dyn.sum(dim=(0, 2, 3)), db_acc)
    return dx


# --- deconvolution (deconv_layer.cpp): conv with roles of fwd/dgrad swapped ------------

def deconv_forward(x, w, b, s: ConvSpec):
    """x: [N,H,W,C=num_input]; w internal (C, R, S, K/g) i.e. Caffe (C, K/g, R, S) permuted."""
    wo = w.float().reshape(s.C, s.R, s.S, s.Kg).permute(0, 3, 1, 2)
    y = F.conv_transpose2d(nchw(x.float()), wo, b.float() if b is not None else None,
                           stride=(s.sh, s.sw), padding=(s.ph, s.pw), dilation=(s.dh, s.dw),
                           groups=s.groups)
    return nhwc(y).to(x.dtype)


# --- inner product (inner_product_layer.cpp) ------------------------------------------

def linear_forward(x2, w, b, relu=False):
    y = x2.float() @ w.float().t()
    if b is not None:
        y = y + b.float()
    if relu:
        y = F.relu(y)
    return y.to(x2.dtype)


def linear_backward(dy2, x2, w, need_dx, dw=None, db=None, gate=None, dw_acc=True, db_acc=True):
    dyf = dy2.float()
    if dw is not None:
        _acc(dw, dyf.t() @ x2.float(), dw_acc)
    if db is not None:
        _acc(db, dyf.sum(0), db_acc)
    if not need_dx:
        return None
    return _gated((dyf @ w.float()).to(x2.dtype), gate.reshape(x2.shape) if gate is not None else None)


# --- pooling (pooling_layer.cpp / .cu) -------------------------------------------------

def _pool_windows(x, s: PoolSpec, fill):
    """Padded NCHW input and its [N, C, P, Q, kh*kw] window view."""
    P, Q = s.P, s.Q
    Hp = (P - 1) * s.sh + s.kh
    Wp = (Q - 1) * s.sw + s.kw
    xn = nchw(x)
    pad_b = Hp - s.H - s.ph
    pad_r = Wp - s.W - s.pw
    xp = F.pad(xn, (s.pw, max(pad_r, 0), s.ph, max(pad_b, 0)), value=fill)
    xp = xp[:, :, :Hp, :Wp]
    win = xp.unfold(2, s.kh, s.sh).unfold(3, s.kw, s.sw)  # N,C,P,Q,kh,kw
    return win.reshape(*win.shape[:4], s.kh * s.kw)


def _ave_divisor(s: PoolSpec, device):
    P, Q = s.P, s.Q
    hs = torch.arange(P, device=device) * s.sh - s.ph
    ws = torch.arange(Q, device=device) * s.sw - s.pw
    he = torch.clamp(hs + s.kh, max=s.H + s.ph)
    we = torch.clamp(ws + s.kw, max=s.W + s.pw)
    return ((he - hs)[:, None] * (we - ws)[None, :]).float()


def _pool_fwd_f32(x, s: PoolSpec):
    if s.method == POOL_MAX:
        return _pool_windows(x, s, float("-inf")).max(dim=-1).values
    win = _pool_windows(x, s, 0.0)
    return win.sum(dim=-1) / _ave_divisor(s, x.device)


def pool_forward(x, s: PoolSpec):
    y = _pool_fwd_f32(x.float(), s)
    return nhwc(y).to(x.dtype)


def pool_backward(dy, x, s: PoolSpec, gate=False):
    xf = x.float().detach().requires_grad_(True)
    y = _pool_fwd_f32(xf, s)
    (g,) = torch.autograd.grad(y, xf, nchw(dy.float()))
    return _gated(g.to(x.dtype), x if gate else None)


# --- LRN (lrn_layer.cpp / .cu) -------------------------------------------------------

def _lrn_across_f32(x, size, alpha, beta, k):
    pre = (size - 1) // 2
    post = size - pre - 1
    sq = x * x
    sq = F.pad(sq, (pre, post))  # pad the channel (last) axis
    win = sq.unfold(-1, size, 1).sum(-1)
    scale = k + alpha / size * win
    return x * scale.pow(-beta)


def _lrn_within_f32(x, size, alpha, beta):
    pre = (size - 1) // 2
    s = PoolSpec(x.shape[0], x.shape[1], x.shape[2], x.shape[3], size, size, 1, 1, pre, pre, POOL_AVE)
    pooled = nhwc(_pool_fwd_f32(x * x, s))
    return x * (1 + alpha * pooled).pow(-beta)


def lrn_forward(x, size, alpha, beta, k, within=False):
    xf = x.float()
    y = _lrn_within_f32(xf, size, alpha, beta) if within else _lrn_across_f32(xf, size, alpha, beta, k)
    return y.to(x.dtype)


def lrn_backward(dy, x, size, alpha, beta, k, within=False, y=None):
    xf = x.float().detach().requires_grad_(True)
    y = _lrn_within_f32(xf, size, alpha, beta) if within else _lrn_across_f32(xf, size, alpha, beta, k)
    (g,) = torch.autograd.grad(y, xf, dy.float())
    return g.to(x.dtype)


# --- neurons (relu/sigmoid/tanh/... layers) --------------------------------------------

def relu_forward(x, slope=0.0):
    xf = x.float()
    return torch.where(xf > 0, xf, xf * slope).to(x.dtype)


def relu_backward(dy, x, slope=0.0):
    xf = x.float()
    return (dy.float() * torch.where(xf > 0, torch.ones_like(xf), torch.full_like(xf, slope))).to(dy.dtype)


# --- dropout (dropout_layer.cpp:14-18, .cu): keep iff u32 > UINT_MAX*p -----------------

_M0, _M1 = 0xD2511F53, 0xCD9E8D57
_W0, _W1 = 0x9E3779B9, 0xBB67AE85
_MASK32 = 0xFFFFFFFF


def philox_u32(n: int, seed: int, counter: int, stream: int) -> torch.Tensor:
    """Dropout words for element indices 0..n-1: element e takes word e % 4 of
    Philox4x32-10 at counter e // 4 — bit-identical to the HIP kernels
    (csrc/kernels/common.h dropout_bits4) so CPU and GPU dropout masks agree."""
    n4 = -(-n // 4)
    return _philox4(n4, seed, counter, stream).reshape(-1)[:n]


def _philox4(n4: int, seed: int, counter: int, stream: int) -> torch.Tensor:
    """[n4, 4] Philox4x32-10 output words for counters 0..n4-1."""
    idx = torch.arange(n4, dtype=torch.int64)
    c0 = idx & _MASK32
    c1 = (idx >> 32) & _MASK32
    c1 = c1 | ((stream & 0xFFFF) << 16)
    c2 = torch.full_like(idx, counter & _MASK32)
    c3 = torch.full_like(idx, (counter >> 32) & _MASK32)
    k0 = seed & _MASK32
    k1 = (seed >> 32) & _MASK32
    for _ in range(10):
        p0 = c0 * _M0
        p1 = c2 * _M1
        hi0, lo0 = (p0 >> 32) & _MASK32, p0 & _MASK32
        hi1, lo1 = (p1 >> 32) & _MASK32, p1 & _MASK32
        c0, c1, c2, c3 = hi1 ^ c1 ^ k0, lo1, hi0 ^ c3 ^ k1, lo0
        k0 = (k0 + _W0) & _MASK32
        k1 = (k1 + _W1) & _MASK32
    return torch.stack([c0, c1, c2, c3], dim=1)


def philox4_counters(seed: int, c0, c1: int, c2: int, c3: int) -> torch.Tensor:
    """Philox4x32-10 of arbitrary counters (c0 a tensor, c1..c3 scalars): [len(c0), 4]."""
    c0 = torch.as_tensor(c0, dtype=torch.int64) & _MASK32
    c1 = torch.full_like(c0, c1 & _MASK32)
    c2 = torch.full_like(c0, c2 & _MASK32)
    c3 = torch.full_like(c0, c3 & _MASK32)
    k0, k1 = seed & _MASK32, (seed >> 32) & _MASK32
    for _ in range(10):
        p0 = c0 * _M0
        p1 = c2 * _M1
        hi0, lo0 = (p0 >> 32) & _MASK32, p0 & _MASK32
        hi1, lo1 = (p1 >> 32) & _MASK32, p1 & _MASK32
        c0, c1, c2, c3 = hi1 ^ c1 ^ k0, lo1, hi0 ^ c3 ^ k1, lo0
        k0 = (k0 + _W0) & _MASK32
        k1 = (k1 + _W1) & _MASK32
    return torch.stack([c0, c1, c2, c3], dim=1)


def augment_params(N: int, seed: int, counter: int, Hs: int, Ws: int, crop_h: int, crop_w: int, mirror: bool):
    """Per-image (row offset, column offset, mirror) of a training crop — the draw of the
    augment / augment_s2d kernels (csrc/kernels/augment.hip: Philox(seed) at counter
    (n, 0xA5A50000, counter)), so a CPU feeder reproduces the device crops exactly."""
    u = philox4_counters(seed, torch.arange(N), 0xA5A50000, counter & _MASK32, (counter >> 32) & _MASK32)
    ho = (u[:, 0] % (Hs - crop_h + 1)).tolist()
    wo = (u[:, 1] % (Ws - crop_w + 1)).tolist()
    mir = (u[:, 2] & 1).tolist() if mirror else [0] * N
    return list(zip(ho, wo, [bool(m) for m in mir]))


def dropout_mask(shape, ratio, seed, counter, stream, device):
    n = math.prod(shape)
    u = philox_u32(n, seed, counter, stream)
    thr = int(_MASK32 * ratio)
    return (u > thr).reshape(shape).to(device)


def dropout_forward(x, ratio, seed, counter, stream):
    scale = 1.0 / (1.0 - ratio)
    m = dropout_mask(x.shape, ratio, seed, counter, stream, x.device)
    return (x.float() * m * scale).to(x.dtype)


def dropout_backward(dy, ratio, seed, counter, stream, gate=None):
    return _gated(dropout_forward(dy, ratio, seed, counter, stream), gate)


# --- softmax / softmax-with-loss (softmax_loss_layer.cpp / .cu) ------------------------

def softmax_forward(x2):
    return torch.softmax(x2.float(), dim=-1).to(x2.dtype)


def softmax_backward(dy2, y2):
    y = y2.float()
    d = dy2.float()
    return (y * (d - (d * y).sum(-1, keepdim=True))).to(dy2.dtype)


def softmax_loss_forward(x2, labels, ignore_label=None, normalize=True, outer_num=None):
    """SoftmaxWithLoss forward (softmax_loss_layer.cpp:Forward_cpu).
    Returns (loss, prob, normalizer): loss = -sum log(max(p_label, FLT_MIN)) / normalizer,
    normalizer = #valid labels if ``normalize`` else outer_num."""
    prob = torch.softmax(x2.float(), dim=-1)
    lab = labels.reshape(-1).long()
    valid = torch.ones_like(lab, dtype=torch.bool)
    if ignore_label is not None:
        valid = lab != ignore_label
    safe = torch.where(valid, lab, torch.zeros_like(lab))
    p = prob.gather(1, safe[:, None])[:, 0].clamp_min(torch.finfo(torch.float32).tiny)
    nll = torch.where(valid, -torch.log(p), torch.zeros_like(p))
    if normalize:
        norm = valid.sum().float()
    else:
        norm = torch.tensor(float(outer_num if outer_num is not None else x2.shape[0]))
    norm = torch.clamp(norm, min=1.0)
    return nll.sum() / norm, prob, norm


def softmax_loss_backward(prob, labels, loss_weight, norm, ignore_label=None, dtype=torch.float32):
    lab = labels.reshape(-1).long()
    g = prob.clone()
    valid = torch.ones_like(lab, dtype=torch.bool)
    if ignore_label is not None:
        valid = lab != ignore_label
    safe = torch.where(valid, lab, torch.zeros_like(lab))
    g.scatter_add_(1, safe[:, None], torch.where(valid, -1.0, 0.0)[:, None])
    g = g * valid[:, None].float()
    lw = loss_weight.reshape(-1)[0].float() if torch.is_tensor(loss_weight) else loss_weight
    g = g * (lw / norm)
    return g.to(dtype)


def accuracy(x2, labels, top_k=1, ignore_label=None):
    lab = labels.reshape(-1).long()
    xf = x2.float()
    # Caffe counts a hit when fewer than top_k classes score strictly higher.
    lab_score = xf.gather(1, lab.clamp(0, xf.shape[1] - 1)[:, None])
    higher = (xf > lab_score).sum(1)
    hit = (higher < top_k).float()
    valid = torch.ones_like(hit, dtype=torch.bool)
    if ignore_label is not None:
        valid = lab != ignore_label
    n = valid.sum().float()
    return (hit * valid).sum() / torch.clamp(n, min=1.0)


# --- solver (sgd_solver.cpp:102-239) ----------------------------------------------------

def sgd_update(data, diff, hist, lr_vec, decay_vec, momentum, l1: bool, clip_scale: float):
    """In-place fused SGD on flat fp32 buffers; lr_vec/decay_vec are per-element
    (lr*lr_mult, wd*decay_mult)."""
    g = diff * clip_scale if clip_scale != 1.0 else diff.clone()
    if l1:
        g += decay_vec * torch.sign(data)
    else:
        g += decay_vec * data
    hist.mul_(momentum).add_(lr_vec * g)
    diff.copy_(hist)
    data.sub_(hist)


def solver_update_ref(kind, data, diff, hist, lr_mult, decay_mult, h, l1, clip):
    """Reference for every solver kind on flat fp32 buffers (CPU).  ``h`` = hyper list.
    Order: clip (global L2 of raw diffs) -> 1/iter_size -> L1/L2 decay -> update rule."""
    lr, mom, wd, clipv, norm, delta, mom2, rms, corr = h[0], h[1], h[2], h[3], h[4], h[5], h[6], h[7], h[8]
    scale = norm
    if clip and clipv > 0:
        l2 = float(torch.sqrt((diff.double() ** 2).sum()))
        if l2 > clipv:
            scale *= clipv / l2
    g = diff * scale
    w = data
    if l1:
        g = g + (wd * decay_mult) * torch.sign(w)
    else:
        g = g + (wd * decay_mult) * w
    rate = lr * lr_mult
    if kind == 0:      # SGD
        hist[0].mul_(mom).add_(rate * g)
        upd = hist[0]
    elif kind == 1:    # Nesterov
        prev = hist[0].clone()
        hist[0].mul_(mom).add_(rate * g)
        upd = (1 + mom) * hist[0] - mom * prev
    elif kind == 2:    # AdaGrad
        hist[0].add_(g * g)
        upd = rate * g / (torch.sqrt(hist[0]) + delta)
    elif kind == 3:    # RMSProp
        hist[0].mul_(rms).add_((1 - rms) * g * g)
        upd = rate * g / (torch.sqrt(hist[0]) + delta)
    elif kind == 4:    # AdaDelta
        hist[0].mul_(mom).add_((1 - mom) * g * g)
        u = g * torch.sqrt((hist[1] + delta) / (hist[0] + delta))
        hist[1].mul_(mom).add_((1 - mom) * u * u)
        upd = rate * u
    elif kind == 5:    # Adam
        hist[0].mul_(mom).add_((1 - mom) * g)
        hist[1].mul_(mom2).add_((1 - mom2) * g * g)
        upd = rate * corr * hist[0] / (torch.sqrt(hist[1]) + delta)
    else:
        raise ValueError(kind)
    diff.copy_(upd)
    data.sub_(upd)
