"""HIP implementations of the op API (MI355X / gfx950).

Every function here launches hand-written kernels from ``libsn_kernels.so`` on torch's
current stream (so a whole iteration can be captured into a hipGraph).  PyTorch is only
used for allocation and for trivial glue on uncommon shapes (zero-padding operands whose
channel counts are not multiples of 8).
"""
from __future__ import annotations

import contextlib
import ctypes as C
import dataclasses
import os

import torch

from . import _lib
from ..utils import features
from .gemm import (EPI_BF16, EPI_F32, EPI_F32_ACC, ConvGeom, Dense, FlipW, Im2col, colsum, gemm,
                   linear_dgrad, linear_fwd, linear_wgrad)
from .spec import POOL_MAX, ConvNdSpec, ConvSpec, PoolSpec

call = _lib.call
BF16 = torch.bfloat16
DGRAD_INPLACE_WEIGHTS = False  # conv dgrad: read W via the FLIPW operand instead of a flip pass


def _c(t: torch.Tensor) -> torch.Tensor:
    return t if t.is_contiguous() else t.contiguous()


def chan_stride(t: torch.Tensor) -> int:
    """Pixel stride (elements) of an NHWC tensor that is either contiguous or a channel
    slice [..., c0:c0+C] of a contiguous [N, H, W, Ctot] tensor (the zero-copy concat
    layout: a tower writes / reads its channels in place); 0 for any other layout."""
    if t.is_contiguous():
        return t.shape[-1]
    if t.dim() != 4 or t.stride(-1) != 1:
        return 0
    N, H, W, Cc = t.shape
    ld = t.stride(2)
    if ld < Cc or t.stride(1) != W * ld or (N > 1 and t.stride(0) != H * W * ld):
        return 0
    return ld


def as_bf16(t: torch.Tensor | None) -> torch.Tensor | None:
    """Contiguous bf16 view of a GPU activation.  Non-image blobs fed by Input / data
    layers stay fp32 (labels, 2-D features); the bf16-only kernels below get a bf16 copy
    made by the native cast kernel instead of reading fp32 bytes as bf16."""
    if t is None:
        return None
    t = _c(t)
    if t.dtype == BF16:
        return t
    if t.dtype != torch.float32:
        raise TypeError(f"GPU activations are bf16 or fp32, got {t.dtype}")
    out = torch.empty(t.shape, dtype=BF16, device=t.device)
    call("cast_f32_bf16", t, out, t.numel())
    return out


def _round8(n: int) -> int:
    return -(-n // 8) * 8


# --------------------------------------------------------------------------------------
# Convolution
# --------------------------------------------------------------------------------------

def _implicit_ok(s: ConvSpec) -> bool:
    return s.Cg % 8 == 0 and s.C % 8 == 0


def _weight_kpad(w: torch.Tensor, s: ConvSpec) -> tuple[torch.Tensor, int]:
    """Weights as [K, Kpad] bf16 with K-dim (r, s, c) zero-padded to a multiple of 8."""
    kred = s.R * s.S * s.Cg
    kpad = _round8(kred)
    w2 = w.reshape(s.K, kred)
    if kpad == kred:
        return _c(w2), kpad
    out = torch.zeros((s.K, kpad), dtype=BF16, device=w.device)
    out[:, :kred].copy_(w2)
    return out, kpad


def _im2col(x: torch.Tensor, s: ConvSpec, g: int, kpad: int) -> torch.Tensor:
    M = s.N * s.P * s.Q
    col = torch.empty((M, kpad), dtype=BF16, device=x.device)
    call("im2col", x, col, s.N, s.H, s.W, s.C, s.P, s.Q, s.R, s.S, s.sh, s.sw, s.ph, s.pw, s.dh, s.dw,
         s.Cg, kpad, g * s.Cg)
    return col


def _geom(s: ConvSpec) -> ConvGeom:
    return ConvGeom(s.N, s.H, s.W, s.C, s.P, s.Q, s.R, s.S, s.sh, s.sw, s.ph, s.pw, s.dh, s.dw, s.Cg)


def _s2d_plan(s: ConvSpec):
    """Space-to-depth fold for low-channel, ungrouped convs (input layers): returns
    (f, Cp, Rf, Sf, folded ConvSpec) or None.  Stride f >= 2 folds f x f pixels into the
    channels (AlexNet conv1: 3 -> 48 channels, 11x11/4 -> 3x3/1); stride 1 is the f = 1
    case — channels zero-padded to 8 and the spatial padding materialised (VGG conv1_1,
    LeNet / CIFAR conv1) — so every input conv runs on the implicit-GEMM path instead of
    an explicit im2col buffer."""
    if _implicit_ok(s) or s.groups != 1 or s.sh != s.sw or s.dh != 1 or s.dw != 1:
        return None
    f = s.sh
    cp = s.C
    while (f * f * cp) % 8:
        cp += 1
    rf, sf = -(-s.R // f), -(-s.S // f)
    hs, ws = s.P + rf - 1, s.Q + sf - 1
    s2 = ConvSpec(s.N, hs, ws, f * f * cp, s.K, rf, sf, 1, 1, 0, 0, 1, 1, 1)
    assert s2.P == s.P and s2.Q == s.Q
    return f, cp, rf, sf, s2


def _s2d_input(x, s: ConvSpec, plan):
    f, cp, rf, sf, s2 = plan
    x2 = torch.empty((s.N, s2.H, s2.W, s2.C), dtype=BF16, device=x.device)
    call("s2d_input", x, x2, s.N, s.H, s.W, s.C, s2.H, s2.W, f, cp, s.ph, s.pw)
    return x2


def _slice_ok(s: ConvSpec) -> bool:
    """Convs whose input may be / output may go to a channel slice of a wider NHWC
    tensor: ungrouped implicit-GEMM products (channel offsets stay 16-B aligned)."""
    return s.groups == 1 and _implicit_ok(s) and s.Kg % 8 == 0


# The implicit-GEMM index decode (fp32 reciprocal division) is exact below 2^24 pixels per
# launch; larger batches (e.g. VGG-16 at batch 512, sized for 288 GB of HBM) run as
# consecutive launches over image chunks — forward / dgrad write disjoint output slices,
# weight gradients accumulate.
_MAX_PIX = 1 << 24


def _image_chunk(s: ConvSpec) -> int:
    """Images per launch (s.N when one launch holds the whole batch)."""
    per = max(s.H * s.W, s.P * s.Q, 1)
    plan = _s2d_plan(s)
    if plan is not None:  # the folded input materialises the spatial padding
        per = max(per, plan[4].H * plan[4].W)
    return s.N if s.N * per < _MAX_PIX else max(1, (_MAX_PIX - 1) // per)


def conv_forward(x, w, b, s: ConvSpec, relu=False, ws=None, folded=None, out=None):
    nb = _image_chunk(s)
    if nb < s.N:
        y = out if out is not None else torch.empty((s.N, s.P, s.Q, s.K), dtype=BF16, device=x.device)
        for n0 in range(0, s.N, nb):
            n1 = min(s.N, n0 + nb)
            conv_forward(x[n0:n1], w, b, s.with_batch(n1 - n0), relu, None,
                         folded[n0:n1] if folded is not None else None, out=y[n0:n1])
        if ws is not None and folded is not None:
            # the chunked weight gradient must read the fused augment's folded input: the
            # NHWC data blob is not written when the fold is fused (engine.fuse_input_fold)
            ws["s2d_full"] = (x.data_ptr(), x._version, folded)
        return y
    return _conv_forward(x, w, b, s, relu, ws, folded, out)


def _conv_forward(x, w, b, s: ConvSpec, relu=False, ws=None, folded=None, out=None):
    """ws: optional per-layer dict kept from forward to backward (the space-to-depth
    folded input is stored there so the weight-gradient pass does not rebuild it).
    folded: the S2D-folded input already produced upstream (fused augment + fold); x is
    then not read.  out: a [N, P, Q, K] channel-slice view of a wider NHWC tensor to
    write the output into (GEMM ldc = its pixel stride: a zero-copy Concat part); x may
    itself be such a slice."""
    ldx = chan_stride(x)
    if not (ldx and _slice_ok(s)):
        x, ldx = _c(x), s.C
    assert x.dtype == BF16 and w.dtype == BF16, (x.dtype, w.dtype)
    if out is not None:
        ldo = chan_stride(out)
        assert (out.is_contiguous() or _slice_ok(s)) and ldo and tuple(out.shape) == (s.N, s.P, s.Q, s.K) \
            and out.dtype == BF16, "conv output slice needs an ungrouped implicit conv and an NHWC channel-slice view"
    plan = _s2d_plan(s)
    if plan is not None:
        f, cp, rf, sf, s2 = plan
        w2 = torch.empty((s.K, rf, sf, s2.C), dtype=BF16, device=x.device)
        call("s2d_weight", _c(w), w2, s.K, s.R, s.S, s.C, f, cp, rf, sf)
        x2 = folded if folded is not None else _s2d_input(x, s, plan)
        if ws is not None:
            ws["s2d"] = (x.data_ptr(), x._version, x2)
        return conv_forward(x2, w2, b, s2, relu, out=out)
    M = s.N * s.P * s.Q
    if out is not None:
        y, ldy = out, chan_stride(out)
    else:
        y, ldy = torch.empty((s.N, s.P, s.Q, s.K), dtype=BF16, device=x.device), s.K
    if ldx == s.C and ldy == s.K and x.is_contiguous() and packed3x3k64_ok(s):
        # the packed kernel also stores a fused fp8 side output (engine.fuse_fp8_quant: conv1_2's
        # e4m3 input under --dtype fp8), in the e4m3 format only
        from . import gemm as G
        side = G._SIDE if _side_covers(y) else None
        if side is None or not side.e5m2:
            q = (None, None, None)
            if side is not None:
                q = (side.q.data_ptr() + (y.data_ptr() - side.base.data_ptr()) // 2, side.slot, side.part)
                side.launches += 1
            call("conv_packed3x3k64", x, _c(w), b, y, s.N, s.H, s.W, s.C, s.K, int(relu), *q)
            return y
    direct_io = ldx == s.C and ldy == s.K and x.is_contiguous() and not _side_covers(y)
    if direct_io and packed_conv_ok(s):
        call("conv_packed3x3", x, _c(w), b, y, s.N, s.H, s.W, s.C, s.K, int(relu))
        return y
    if direct_io and packed11_conv_ok(s):
        call("conv_packed1x1", x, _c(w), b, y, s.N, s.H, s.W, s.C, s.K, int(relu))
        return y
    if direct_io and packed44_conv_ok(s):
        call("conv_packed4x4", x, _c(w), b, y, s.N, s.H, s.W, s.C, s.K, int(relu))
        return y
    if direct_io and direct_conv_ok(s):
        call("conv3x3_direct", x, _c(w), b, None, y, s.N, s.H, s.W, s.C, s.K, s.ph, int(relu), 0)
        return y
    if direct_io and direct96_split_ok(s):
        # K / 96 launches of the 96-output direct kernel, each into its channel slice of y
        wc = _c(w)
        for j in range(0, s.K, 96):
            call("conv3x3_direct", x, wc[j:j + 96], b[j:j + 96] if b is not None else None, None, y[..., j:],
                 s.N, s.H, s.W, s.C, 96, s.ph, int(relu), s.K)
        return y
    if _implicit_ok(s):
        kred = s.R * s.S * s.Cg
        g = _geom(s)
        g.C = ldx  # pixel stride of the (possibly channel-sliced) input
        A = Im2col(x, g, kcontig=True, gstride=s.Cg)
        B = Dense(_c(w.reshape(s.K, kred)), kred, True, gstride=s.Kg * kred)
        gemm(M, s.Kg, kred, A, B, y, ldy, epi=EPI_BF16, groups=s.groups, c_gstride=s.Kg, bias=b, relu=relu)
        return y
    assert ldy == s.K, "explicit im2col path writes contiguous outputs"
    wp, kpad = _weight_kpad(w, s)
    y2 = y.view(M, s.K)
    for g in range(s.groups):
        col = _im2col(x, s, g, kpad)
        wg = wp[g * s.Kg:(g + 1) * s.Kg]
        bg = b[g * s.Kg:(g + 1) * s.Kg] if b is not None else None
        gemm(M, s.Kg, kpad, Dense(col, kpad, True), Dense(_c(wg), kpad, True), y2[:, g * s.Kg:], s.K,
             epi=EPI_BF16, bias=bg, relu=relu)
    return y


# Direct 3x3 / stride-1 conv (csrc/kernels/conv3x3.hip: resident weights, input patch in LDS)
# instead of the implicit GEMM for two thin shapes: 64 -> 64 channels with pad 1 (VGG-16's
# conv1_2 forward and data gradient) and 48 -> 96 with pad 0 (CaffeNet / AlexNet conv1 after
# the space-to-depth fold)
_DIRECT_C64 = features.enabled("conv_direct_c64")
_DIRECT_K96 = features.enabled("conv_direct_k96")


def direct_c64_ok(s: ConvSpec) -> bool:
    return (_DIRECT_C64 and s.C == 64 and s.K == 64 and s.groups == 1 and s.R == 3 and s.S == 3 and s.sh == 1
            and s.sw == 1 and s.ph == 1 and s.pw == 1 and s.dh == 1 and s.dw == 1)


def direct_conv_ok(s: ConvSpec) -> bool:
    """Forward products the direct kernel takes (the data gradient: direct_c64_ok only)."""
    if direct_c64_ok(s):
        return True
    return (_DIRECT_K96 and s.C == 48 and s.K == 96 and s.groups == 1 and s.R == 3 and s.S == 3 and s.sh == 1
            and s.sw == 1 and s.ph == 0 and s.pw == 0 and s.dh == 1 and s.dw == 1)


# 3x3 / stride-1 / pad-1 convolutions with <= 64 input channels and a multiple of 96 (> 96)
# outputs — GoogLeNet's conv2/3x3, 64 -> 192 — as 96-output direct launches writing channel
# slices of the output: 2 x 64.6 us vs 155 us for the implicit GEMM at b128 (the GEMM re-reads
# its 9x im2col A operand and the whole weight panel per 128-row tile; scripts/direct96_probe.py).
# (SN_FEATURES=conv_direct96=0 keeps the GEMM.)
_DIRECT96 = features.enabled("conv_direct96")


# 1x1 convolutions with <= 64 inputs and 64 outputs (GoogLeNet's conv2/3x3_reduce) on the
# tap-packed direct kernel's <1, 64> instance (SN_FEATURES=conv_packed11=1; measured in
# profiles/r5_packed11.txt)
_PACKED11 = features.enabled("conv_packed11")


def packed11_conv_ok(s: ConvSpec) -> bool:
    return (_PACKED11 and 0 < s.C <= 64 and s.C % 8 == 0 and s.K == 64 and s.groups == 1 and s.R == 1
            and s.S == 1 and s.sh == 1 and s.sw == 1 and s.ph == 0 and s.pw == 0 and s.dh == 1 and s.dw == 1
            and s.W * s.C * 2 * min(s.H, (191 + s.W - 1) // s.W + 1) <= 36864)


def direct96_split_ok(s: ConvSpec) -> bool:
    return (_DIRECT96 and 0 < s.C <= 64 and s.C % 8 == 0 and s.K > 96 and s.K % 96 == 0 and s.groups == 1
            and s.R == 3 and s.S == 3 and s.sh == 1 and s.sw == 1 and s.ph == 1 and s.pw == 1 and s.dh == 1
            and s.dw == 1)


# CaffeNet / AlexNet conv1 after the fold (48 -> 96, 3x3, pad 0) on the tap-packed direct kernel
# (csrc/kernels/conv_packed.hip: 14 instead of 18 K steps, 192-pixel row-major tiles instead of
# 16 x 16 ones); SN_FEATURES=conv_packed=0 returns it to the 64-channel direct kernel
_PACKED = features.enabled("conv_packed")


def packed_conv_ok(s: ConvSpec) -> bool:
    if not (_PACKED and s.K == 96 and 0 < s.C <= 48 and s.C % 8 == 0 and s.groups == 1 and s.R == 3 and s.S == 3
            and s.sh == 1 and s.sw == 1 and s.ph == 0 and s.pw == 0 and s.dh == 1 and s.dw == 1 and s.Q > 0):
        return False
    rows = min(s.H, (191 + s.Q - 1) // s.Q + 3)  # input rows one 192-pixel tile touches
    return rows * s.W * s.C * 2 <= 38400 and s.P * s.Q * 96 < 2 ** 31


# GoogLeNet conv1 after the 2x2 fold (115 x 115 x 16 -> 112 x 112 x 64, 4x4 taps, pad 0) on the
# same tap-packed direct kernel's <4, 64> instance: the input rows of a 192-pixel tile staged
# once in LDS instead of the implicit GEMM's per-tap re-reads of its 256x64 tiles;
# SN_FEATURES=conv_packed44=0 returns it to the GEMM
_PACKED44 = features.enabled("conv_packed44")


def packed44_conv_ok(s: ConvSpec) -> bool:
    if not (_PACKED44 and s.K == 64 and s.C in (8, 16) and s.groups == 1 and s.R == 4 and s.S == 4
            and s.sh == 1 and s.sw == 1 and s.ph == 0 and s.pw == 0 and s.dh == 1 and s.dw == 1 and s.Q > 0):
        return False
    rows = min(s.H, (191 + s.Q - 1) // s.Q + 4)  # input rows one 192-pixel tile touches
    return rows * s.W * s.C * 2 <= 22528 and s.P * s.Q * 64 < 2 ** 31


# VGG-16 conv1_1 after its fold (226 x 226 x 8 -> 224 x 224 x 64, 3x3, pad 0) on the tap-packed
# kernel's <3, 64> instance: 3 K steps of 32 instead of the implicit GEMM's two 64-deep steps per
# 128-row tile; SN_FEATURES=conv_packed_k64=0 returns it to the GEMM
_PACKED_K64 = features.enabled("conv_packed_k64")


def packed3x3k64_ok(s: ConvSpec) -> bool:
    if not (_PACKED_K64 and s.K == 64 and s.C == 8 and s.groups == 1 and s.R == 3 and s.S == 3
            and s.sh == 1 and s.sw == 1 and s.ph == 0 and s.pw == 0 and s.dh == 1 and s.dw == 1 and s.Q > 0):
        return False
    rows = min(s.H, (191 + s.Q - 1) // s.Q + 3)  # input rows one 192-pixel tile touches
    return rows * s.W * s.C * 2 <= 16384 and s.P * s.Q * 64 < 2 ** 31


# the e4m3 direct kernel (csrc/kernels/conv3x3_fp8.hip) for the same 64 -> 64 products under
# engine.enable_fp8 (forward, and the data gradient with an e4m3 output gradient; the layer's
# weight gradient then runs fp8 too): forward 1.37x the bf16 direct kernel at VGG conv1_2's
# shape (profiles/r4_direct8_probe.txt), VGG-16 b2048 fp8 step 186 -> 181 ms with the thin tiles
# and 192 -> 182 ms without (profiles/r4_vgg16_fp8_variants.jsonl).  SN_FEATURES=conv_direct_fp8=0 keeps
# these layers bf16.
_DIRECT_FP8 = features.enabled("conv_direct_fp8")


def direct_fp8_ok(s: ConvSpec) -> bool:
    return _DIRECT_FP8 and direct_c64_ok(s)


def _side_covers(t: torch.Tensor) -> bool:
    from . import gemm as G
    return G._SIDE is not None and G._SIDE.covers(t)  # a fused fp8 side output needs the GEMM epilogue


def dgrad_uses_flip(s: ConvSpec) -> bool:
    """Does conv_backward compute this conv's data gradient as a forward conv over
    flip-transposed weights (the path FlipBatch pre-computes the weights for)?"""
    return (s.sh == 1 and s.sw == 1 and s.dh == 1 and s.dw == 1 and _implicit_ok(s) and s.Kg % 8 == 0
            and not DGRAD_INPLACE_WEIGHTS)


class FlipBatch:
    """Flip-transpose the weights of several convolutions in ONE launch
    (flip_weights_multi): items are (w, wt, G, Kg, R, S, Cg) with w the bf16 compute
    weights [K][R][S][Cg] and wt the persistent [G][Cg][R][S][Kg] output.  The device
    descriptor table holds raw pointers, so run() re-checks them on the host and rebuilds
    the table if a tensor was re-allocated."""

    def __init__(self, items, device):
        self.items = list(items)
        self.device = torch.device(device)
        self._build()

    def _ptrs(self):
        return [(w.data_ptr(), wt.data_ptr()) for w, wt, *_ in self.items]

    def _build(self):
        lib = _lib.kernels()
        lib.sn_flip_desc_size.restype = C.c_int
        size = lib.sn_flip_desc_size()
        buf = (C.c_char * (size * len(self.items)))()
        for i, (w, wt, G, Kg, R, S, Cg) in enumerate(self.items):
            assert w.is_contiguous() and wt.is_contiguous() and w.dtype == BF16 and wt.dtype == BF16
            assert w.numel() == wt.numel() == G * Kg * R * S * Cg < (1 << 31)
            lib.sn_flip_desc(C.byref(buf, i * size), C.c_void_p(w.data_ptr()), C.c_void_p(wt.data_ptr()),
                             *(C.c_longlong(v) for v in (G, Kg, R, S, Cg)))
        self.descs = torch.frombuffer(bytearray(buf), dtype=torch.uint8).to(self.device)
        # 64 x 64 transpose tiles of the largest descriptor = the launch's grid width
        self.max_tiles = max(G * R * S * -(-Kg // 64) * -(-Cg // 64) for _, _, G, Kg, R, S, Cg in self.items)
        self.ptrs = self._ptrs()

    def run(self) -> None:
        if self._ptrs() != self.ptrs:
            self._build()
        call("flip_weights_multi", self.descs, len(self.items), self.max_tiles)


def _pad_cols(t2: torch.Tensor, n: int) -> torch.Tensor:
    out = torch.zeros((t2.shape[0], n), dtype=t2.dtype, device=t2.device)
    out[:, :t2.shape[1]].copy_(t2)
    return out


def conv_backward(dy, x, w, s: ConvSpec, need_dx: bool, dw=None, db=None, gate=None, ws=None,
                  dw_acc=True, db_acc=True, dx_out=None):
    """``dx_out``: write the data gradient there — contiguous, or a channel slice of a wider
    NHWC buffer, which the stride-1 implicit dgrad writes in place (ldc = the slice's pixel
    stride)."""
    if dx_out is not None and need_dx:
        if chan_stride(dx_out) == s.C or (_implicit_ok(s) and s.sh == s.sw == 1 and s.dh == s.dw == 1
                                          and s.Kg % 8 == 0 and chan_stride(dx_out) and _image_chunk(s) >= s.N
                                          and not (ws and ("fp8_dgrad" in ws or "fp8_dx_side" in ws))):
            return _conv_backward_chunked(dy, x, w, s, need_dx, dw, db, gate, ws, dw_acc, db_acc, dx_out)
        dx = conv_backward(dy, x, w, s, need_dx, dw, db, gate, ws, dw_acc, db_acc)
        dx_out.copy_(dx)
        return dx_out
    side_req = ws.pop("fp8_dx_side", None) if ws else None
    if side_req is not None and need_dx:
        # the data-gradient GEMM epilogue also stores dx as fp8 for the layer below's fp8 data
        # gradient (engine.fuse_fp8_quant); ws["fp8_dx_side_out"] is that fp8 copy's Fp8Side
        from .gemm import Fp8Side, fp8_side_output
        dx = torch.empty((s.N, s.H, s.W, s.C), dtype=BF16, device=x.device)
        side = Fp8Side(dx, *side_req)
        with fp8_side_output(side):
            out = _conv_backward_chunked(dy, x, w, s, need_dx, dw, db, gate, ws, dw_acc, db_acc, dx)
        ws["fp8_dx_side_out"] = side if out is dx else None
        return out
    return _conv_backward_chunked(dy, x, w, s, need_dx, dw, db, gate, ws, dw_acc, db_acc)


def _conv_backward_chunked(dy, x, w, s: ConvSpec, need_dx: bool, dw=None, db=None, gate=None, ws=None,
                           dw_acc=True, db_acc=True, dx=None):
    nb = _image_chunk(s)
    if nb < s.N:
        if dx is None:
            dx = torch.empty((s.N, s.H, s.W, s.C), dtype=BF16, device=x.device) if need_dx else None
        full = ws.get("s2d_full") if ws else None
        if full is not None and not (full[0] == x.data_ptr() and full[1] == x._version):
            full = None
        dyq_full = _fp8_dyq(dy, ws, s) if ws else None  # one fp8 copy of dy shared by the chunks
        for n0 in range(0, s.N, nb):
            n1 = min(s.N, n0 + nb)
            cws = {k: ws[k] for k in ("wt", "fp8_dgrad") if k in ws} if ws else None
            if dyq_full is not None:
                cws["fp8_dyq"] = dyq_full[n0:n1]
            if ws and "fp8_wgrad" in ws:
                sc, ix, xq, idy = ws["fp8_wgrad"]
                cws["fp8_wgrad"] = (sc, ix, xq[n0:n1], idy)
            if full is not None:
                xc = x[n0:n1]
                cws["s2d"] = (xc.data_ptr(), xc._version, full[2][n0:n1])
            _conv_backward(dy[n0:n1], x[n0:n1], w, s.with_batch(n1 - n0), need_dx, dw,
                           db, gate[n0:n1] if gate is not None else None, cws, dw_acc, db_acc,
                           dx_out=dx[n0:n1] if need_dx else None)
            dw_acc = db_acc = True  # later chunks accumulate into the weight gradients
        return dx
    return _conv_backward(dy, x, w, s, need_dx, dw, db, gate, ws, dw_acc, db_acc, dx_out=dx)


def _conv_backward(dy, x, w, s: ConvSpec, need_dx: bool, dw=None, db=None, gate=None, ws=None,
                   dw_acc=True, db_acc=True, dx_out=None):
    """gate: optional bf16 NHWC tensor shaped like x; dx is zeroed where gate <= 0
    (the backward of a slope-0 in-place ReLU that produced x, fused into the dgrad).
    dw_acc / db_acc False: overwrite the gradient instead of accumulating (its buffer
    was not cleared, see Net.clear_param_diffs(lazy=True))."""
    kred = s.R * s.S * s.Cg
    plan = _s2d_plan(s) if s.Kg % 8 == 0 else None
    ldd, ldx = chan_stride(dy), chan_stride(x)
    if plan is not None or not _slice_ok(s) or not (ldd and ldx):
        dy, ldd, x, ldx = _c(dy), s.K, _c(x), s.C
    M = s.N * s.P * s.Q
    # dy2: the [M, K] gradient matrix (row stride ldd: a channel slice of a zero-copy concat
    # diff when ldd > K; only the ungrouped implicit paths below see such a view)
    dy2 = dy.view(M, s.K) if ldd == s.K else dy
    # the bias gradient rides on the weight-gradient GEMM (ones column) on its implicit
    # paths; otherwise (no dw, explicit im2col) it is a separate column sum
    fused_db = db is not None and dw is not None and (
        plan is not None or (_implicit_ok(s) and s.Kg % 8 == 0))
    f8w = ws.get("fp8_wgrad") if ws is not None else None
    if (f8w is not None and dw is not None and plan is None and ldd == s.K and ldx == s.C
            and fp8_wgrad_ok(s) and f8w[2].shape[0] == s.N):
        dyq = ws.get("fp8_dyq")
        if dyq is None:
            dyq = ws["fp8_dyq"] = _fp8_dyq(dy, ws, s)
        _conv_wgrad_fp8(dy2, dyq, s, M, kred, f8w, dw, db, dw_acc, db_acc, _dy_fp8_only(ws))
        dw = None
        if db is not None:
            db, fused_db = None, False
    if (dw is not None or db is not None) and _dy_fp8_only(ws):
        _no_bf16_dy("a bf16 weight / bias gradient")
    _conv_wgrad(dy2, x, s, M, kred, plan, fused_db, dw, db, ws, dw_acc, db_acc, ldd, ldx)
    if not need_dx:
        return None
    return _conv_dgrad(dy, x, w, s, M, gate, ws, ldd, ldx, dx_out)


def _conv_wgrad(dy2, x, s, M, kred, plan, fused_db, dw, db, ws, dw_acc, db_acc, ldd=0, ldx=0):
    ldd, ldx = ldd or s.K, ldx or s.C
    if db is not None and not fused_db:
        assert ldd == s.K
        colsum(dy2, db, accumulate=db_acc)
    if dw is not None and plan is not None:
        f, cp, rf, sf, s2 = plan
        cached = ws.get("s2d") if ws is not None else None
        if cached is not None and cached[0] == x.data_ptr() and cached[1] == x._version:
            x2 = cached[2]
        else:
            x2 = _s2d_input(x, s, plan)
        k2 = rf * sf * s2.C
        dw2 = torch.empty((s.K, k2), dtype=torch.float32, device=x.device)
        gemm(s.K, k2, M, Dense(dy2, s.K, kcontig=False), Im2col(x2, _geom(s2), kcontig=False), dw2, k2,
             epi=EPI_F32, bias_grad=db if fused_db else None, bias_acc=db_acc)
        call("s2d_weight_grad", dw2, dw, s.K, s.R, s.S, s.C, f, cp, rf, sf, int(dw_acc))
        dw = None
    if dw is not None:
        if _implicit_ok(s) and s.Kg % 8 == 0:
            A = Dense(dy2, ldd, kcontig=False, gstride=s.Kg)
            g = _geom(s)
            g.C = ldx
            B = Im2col(x, g, kcontig=False, gstride=s.Cg)
            gemm(s.Kg, kred, M, A, B, dw, kred, epi=EPI_F32_ACC if dw_acc else EPI_F32, groups=s.groups,
                 c_gstride=s.Kg * kred, bias_grad=db if fused_db else None, bias_acc=db_acc)
        else:
            kpad = _round8(kred)
            kgp = _round8(s.Kg)
            dw2 = dw.view(s.K, kred)
            for g in range(s.groups):
                col = _im2col(x, s, g, kpad)
                dyg = dy2[:, g * s.Kg:(g + 1) * s.Kg]
                dyg = _c(dyg) if kgp == s.Kg else _pad_cols(dyg, kgp)
                tmp = torch.zeros((kgp, kpad), dtype=torch.float32, device=x.device)
                gemm(kgp, kpad, M, Dense(dyg, dyg.stride(0), False), Dense(col, kpad, False), tmp, kpad,
                     epi=EPI_F32)
                if dw_acc:
                    dw2[g * s.Kg:(g + 1) * s.Kg].add_(tmp[:s.Kg, :kred])
                else:
                    dw2[g * s.Kg:(g + 1) * s.Kg].copy_(tmp[:s.Kg, :kred])


# Bias gradient of the fp8 weight-gradient products.  1 (default): a virtual e4m3 ones column
# of the product, i.e. the column sum of the QUANTISED output gradient (e4m3 / e5m2 with the
# tensor's delayed scale: small entries are rounded or flushed); 0: an exact column sum of the
# bf16 output gradient in a separate pass.  Measured on VGG-16 b2048 fp8, one box
# (profiles/r5_fp8_bias_ab.txt): the separate pass reads every dy once more (6.3 ms / step,
# 11.27-11.31k vs 11.51-11.55k img/s) and tests/test_fp8_fidelity_gpu.py passes both ways
# (max deviation 0.071 exact vs 0.093 quantised, bound 0.234).
FP8_WGRAD_BIAS = features.enabled("fp8_wgrad_bias")


def fp8_wgrad_ok(s: ConvSpec) -> bool:
    """Can this conv's weight gradient run as an e4m3 / e5m2 product (fp8 MC operands read
    with ds_read_b64_tr_b8: whole 16-channel chunks on both sides, implicit im2col of x)?"""
    return _implicit_ok(s) and s.Kg % 16 == 0 and s.Cg % 16 == 0 and s.C % 16 == 0 and s.K % 16 == 0


def conv_dy_fp8_only_ok(layer, s: ConvSpec) -> bool:
    """Would this conv's backward read its output gradient only as fp8 bytes — e4m3 data
    gradient (the flip path), e4m3 weight gradient with the bias on its ones column, no
    space-to-depth plan?  Then the max pooling above may store that gradient as fp8 alone
    (engine.fuse_fp8_quant fp8_dx_only); conv_backward raises if a bf16 read happens anyway."""
    if layer.fp8_dgrad_slots is None or not fp8_dgrad_ok(s) or _s2d_plan(s) is not None:
        return False
    if not (s.sh == 1 and s.sw == 1 and s.dh == 1 and s.dw == 1 and _implicit_ok(s) and s.Kg % 8 == 0):
        return False
    need_w = layer.param_grads_needed(0)
    need_b = layer.bias is not None and layer.param_grads_needed(1)
    if need_w and not (layer.fp8_wgrad and fp8_wgrad_ok(s)):
        return False
    return not need_b or (need_w and (s.R * s.S * s.Cg) % 16 == 0 and FP8_WGRAD_BIAS)


def _dy_fp8_only(ws) -> bool:
    """The output gradient exists only as the fp8 side output of the layer above (a max
    pooling's backward with side_only): its bf16 tensor was never written."""
    f8 = ws.get("fp8_dgrad") if ws else None
    return bool(f8 is not None and len(f8) > 3 and f8[3] is not None and getattr(f8[3], "only", False))


def _no_bf16_dy(what: str):
    raise RuntimeError(f"conv backward: {what} would read the bf16 output gradient, which the max pooling "
                       "above stored only as fp8 (engine.fuse_fp8_quant fp8_dx_only; SN_FEATURES=fp8_dx_only=0)")


def _fp8_dyq(dy, ws, s):
    """fp8 bytes of the output gradient for this layer's fp8 data / weight gradients: the
    side output of the layer above's dgrad epilogue when it covers dy, else one pass."""
    f8 = ws.get("fp8_dgrad") if ws else None
    f8w = ws.get("fp8_wgrad") if ws else None
    if f8 is None and f8w is None:
        return None
    if f8 is not None:
        sc, idy = f8[0], f8[1]
        side = f8[3] if len(f8) > 3 else None
    else:
        sc, idy, side = f8w[0], f8w[3], None
    e5 = sc.is_e5m2(idy)
    from .gemm import side_bytes
    dyq = side_bytes(side, dy, e5)
    if dyq is None and _dy_fp8_only(ws):
        _no_bf16_dy("quantising dy")
    return dyq if dyq is not None else quant_fp8(_c(dy), sc.slot(idy), e5m2=e5)


def _conv_wgrad_fp8(dy2, dyq, s, M, kred, f8w, dw, db, dw_acc, db_acc, dy_fp8_only=False):
    """Weight gradient as an fp8 product with the reduction over pixels: A = the output
    gradient (e4m3 / e5m2, MC: [pixels][K]), B = the implicit im2col of the layer input's
    e4m3 copy kept from the forward (MC), both read transposed from LDS by
    ds_read_b64_tr_b8; fp32 accumulation, split-K slabs, dequantised epilogue.  The bias
    gradient, by default, rides on the product as an e4m3 ones column, i.e. it is the column
    sum of the QUANTISED dy, whose small entries are rounded or flushed; SN_FEATURES=fp8_wgrad_bias=0
    computes the exact column sum of the bf16 dy in a separate pass instead (FP8_WGRAD_BIAS;
    reference: base_conv_layer.cpp:338-376, conv_layer.cu:35-53)."""
    sc, ix, xq, idy = f8w
    # the ones column of B is an e4m3 1.0 dequantised by dy's factor only
    fused_db = db is not None and kred % 16 == 0 and FP8_WGRAD_BIAS
    if db is not None and not fused_db:
        if dy_fp8_only:
            _no_bf16_dy("the exact bias gradient")
        colsum(dy2, db, accumulate=db_acc)
    A = Dense(dyq.view(M, s.K), s.K, kcontig=False, gstride=s.Kg)
    B = Im2col(xq, _geom(s), kcontig=False, gstride=s.Cg)
    gemm(s.Kg, kred, M, A, B, dw, kred, epi=EPI_F32_ACC if dw_acc else EPI_F32, groups=s.groups,
         c_gstride=s.Kg * kred, deq=(sc.deq(idy), sc.deq(ix), 2 if sc.is_e5m2(idy) else 1),
         bias_grad=db if fused_db else None, bias_acc=db_acc)


def _conv_dgrad(dy, x, w, s, M, gate, ws, ldd=0, ldx=0, dx_out=None):
    ldd, ldx = ldd or s.K, ldx or s.C
    dx = dx_out if dx_out is not None else torch.empty((s.N, s.H, s.W, s.C), dtype=BF16, device=x.device)
    ldo = chan_stride(dx)  # C, or the pitch of a channel-slice destination (conv_backward dx_out)
    if gate is not None and chan_stride(gate) != ldo:  # the gate (= x) must share dx's layout
        gate = _c(gate)
    if _dy_fp8_only(ws) and not (s.sh == 1 and s.sw == 1 and s.dh == 1 and s.dw == 1 and _implicit_ok(s)
                                 and s.Kg % 8 == 0):
        _no_bf16_dy("a bf16 data gradient")
    if s.sh == 1 and s.sw == 1 and s.dh == 1 and s.dw == 1 and _implicit_ok(s) and s.Kg % 8 == 0:
        # dgrad == forward conv of dy with flipped / transposed weights, pad' = R-1-pad.
        # A flip pass + KC (ds_read_b128) B operand measures faster than reading the
        # weights in place through the FLIPW operand (MC, tr_b16 reads): 81k vs 86k img/s
        # on CaffeNet; FLIPW stays available via DGRAD_INPLACE_WEIGHTS.
        g2 = ConvGeom(s.N, s.P, s.Q, ldd, s.H, s.W, s.R, s.S, 1, 1, s.R - 1 - s.ph, s.S - 1 - s.pw, 1, 1, s.Kg)
        kr2 = s.R * s.S * s.Kg
        pre = ws.get("wt") if ws is not None else None  # flipped once for the net (FlipBatch)
        f8 = ws.get("fp8_dgrad") if ws is not None else None
        if f8 is not None and fp8_dgrad_ok(s) and ldd == s.K:
            return _conv_dgrad_fp8(dy, w, s, g2, kr2, pre, gate, dx, f8, ws.get("fp8_dyq"))
        if _dy_fp8_only(ws):
            _no_bf16_dy("a bf16 data gradient")
        if (direct_c64_ok(s) and ldd == s.K and ldx == s.C and dy.is_contiguous() and dx.is_contiguous()
                and not DGRAD_INPLACE_WEIGHTS and not _side_covers(dx)):
            if pre is None:
                pre = torch.empty((s.groups, s.Cg, s.R, s.S, s.Kg), dtype=BF16, device=x.device)
                call("flip_weights", _c(w), pre, s.groups, s.Kg, s.R, s.S, s.Cg)
            call("conv3x3_direct", dy, pre, None, _c(gate) if gate is not None else None, dx, s.N, s.H, s.W, 64, 64, 1,
                 0, 0)
            return dx
        A = Im2col(dy, g2, kcontig=True, gstride=s.Kg)
        if DGRAD_INPLACE_WEIGHTS:
            B = FlipW(_c(w), s.Kg, s.R, s.S, s.Cg)
        else:
            if pre is not None:
                wt = pre
            else:
                wt = torch.empty((s.groups, s.Cg, s.R, s.S, s.Kg), dtype=BF16, device=x.device)
                call("flip_weights", _c(w), wt, s.groups, s.Kg, s.R, s.S, s.Cg)
            B = Dense(wt.view(s.C, kr2), kr2, True, gstride=s.Cg * kr2)
        gemm(s.N * s.H * s.W, s.Cg, kr2, A, B, dx, ldo, epi=EPI_BF16, groups=s.groups, c_gstride=s.Cg,
             gate=gate)
        return dx
    # generic: dcol = dy_g @ W_g, then col2im (gather, no atomics)
    assert ldd == s.K
    dy2 = dy.view(M, s.K)
    wp, kpad = _weight_kpad(w, s)
    kgp = _round8(s.Kg)
    for g in range(s.groups):
        dyg = dy2[:, g * s.Kg:(g + 1) * s.Kg]
        dyg = _c(dyg) if kgp == s.Kg else _pad_cols(dyg, kgp)
        wg = wp[g * s.Kg:(g + 1) * s.Kg]
        if kgp != s.Kg:
            wg = torch.cat([wg, torch.zeros((kgp - s.Kg, kpad), dtype=BF16, device=x.device)])
        dcol = torch.empty((M, kpad), dtype=BF16, device=x.device)
        gemm(M, kpad, kgp, Dense(dyg, dyg.stride(0), True), Dense(_c(wg), kpad, False), dcol, kpad, epi=EPI_BF16)
        call("col2im", dcol, dx, s.N, s.H, s.W, s.C, s.P, s.Q, s.R, s.S, s.sh, s.sw, s.ph, s.pw, s.dh, s.dw,
             s.Cg, kpad, g * s.Cg)
    if gate is not None:
        dx = relu_backward(dx, gate)
        if dx_out is not None:
            dx_out.copy_(dx)
            dx = dx_out
    return dx


def fp8_dgrad_ok(s: ConvSpec) -> bool:
    """Can this conv's data gradient run as an e4m3 product (the flip path with output-
    gradient channels in whole 16-byte fp8 chunks)?"""
    return dgrad_uses_flip(s) and s.Kg % 16 == 0 and s.C % 8 == 0


def _conv_dgrad_fp8(dy, w, s, g2, kr2, wt, gate, dx, f8, ws_dyq=None):
    """Data gradient as an e4m3 forward conv of the output gradient with the flip-
    transposed weights (v_mfma_scale_f32_16x16x128_f8f6f4, fp32 accumulation): the output
    gradient (e4m3, or e5m2 when its slot says so) and the flipped weights are quantised
    per tensor with their own delayed-
    scaling slots (a slot not yet initialised scales from the current tensor), the
    epilogue dequantises and applies the ReLU-backward gate, dx stays bf16.  The weight
    gradient keeps reading the bf16 output gradient."""
    sc, idy, iwt = f8[:3]
    if wt is None:
        wt = torch.empty((s.groups, s.Cg, s.R, s.S, s.Kg), dtype=BF16, device=dy.device)
        call("flip_weights", _c(w), wt, s.groups, s.Kg, s.R, s.S, s.Cg)
    e5 = sc.is_e5m2(idy)
    dyq = ws_dyq
    if dyq is None:
        side = f8[3] if len(f8) > 3 else None  # dy's fp8 bytes stored by the layer above's dgrad epilogue
        from .gemm import side_bytes
        dyq = side_bytes(side, dy, e5)
    if dyq is None:
        if len(f8) > 3 and getattr(f8[3], "only", False):
            _no_bf16_dy("quantising dy for the data gradient")
        dyq = quant_fp8(dy, sc.slot(idy), e5m2=e5)
    wtq = quant_fp8(wt, sc.slot(iwt))
    if direct_fp8_ok(s) and not e5 and dx.is_contiguous() and not _side_covers(dx):
        call("conv3x3_fp8", _c(dyq), wtq, sc.deq(idy), sc.deq(iwt), None, _c(gate) if gate is not None else None, dx,
             s.N, s.H, s.W, 0)
        return dx
    A = Im2col(dyq, g2, kcontig=True, gstride=s.Kg)
    B = Dense(wtq.view(s.C, kr2), kr2, True, gstride=s.Cg * kr2)
    gemm(s.N * s.H * s.W, s.Cg, kr2, A, B, dx, s.C, epi=EPI_BF16, groups=s.groups, c_gstride=s.Cg,
         gate=_c(gate) if gate is not None else None, deq=(sc.deq(idy), sc.deq(iwt), 2 if e5 else 1))
    return dx


# --------------------------------------------------------------------------------------
# InnerProduct
# --------------------------------------------------------------------------------------

def linear_forward(x2, w, b, relu=False, dropout=None):
    """dropout: (rng_state, stream id, ratio) — a following in-place Dropout applied in
    the epilogue (engine.fuse_dropout)."""
    return linear_fwd(_c(x2), _c(w), b, relu, dropout=dropout)


def linear_backward(dy2, x2, w, need_dx, dw=None, db=None, gate=None, dw_acc=True, db_acc=True, gate_scale=1.0):
    dy2 = _c(dy2)
    if dw is not None:
        # the bias gradient comes out of the weight-gradient GEMM when it can (ones column)
        if not linear_wgrad(dy2, _c(x2), dw, accumulate=dw_acc, db=db, db_acc=db_acc) and db is not None:
            colsum(dy2, db, accumulate=db_acc)
    elif db is not None:
        colsum(dy2, db, accumulate=db_acc)
    if not need_dx:
        return None
    return linear_dgrad(dy2, _c(w), gate=gate.reshape(x2.shape) if gate is not None else None,
                        gate_scale=gate_scale)


def linear_backward_sgd(dy2, x2, w, need_dx, sgd, db=None, gate=None, db_acc=True, gate_scale=1.0):
    """InnerProduct backward whose weight gradient is consumed by the solver update in the
    GEMM epilogue (gemm.linear_wgrad_sgd).  The data gradient runs FIRST: it reads the
    bf16 compute weights ``w`` that the fused update then overwrites."""
    dy2, x2 = _c(dy2), _c(x2)
    dx = None
    if need_dx:
        dx = linear_dgrad(dy2, _c(w), gate=gate.reshape(x2.shape) if gate is not None else None,
                          gate_scale=gate_scale)
    from .gemm import linear_wgrad_sgd
    if not linear_wgrad_sgd(dy2, x2, sgd, db, db_acc) and db is not None:
        colsum(dy2, db, accumulate=db_acc)
    return dx


# --------------------------------------------------------------------------------------
# N-d convolution (csrc/kernels/conv_nd.hip: N-d im2col / col2im) on the MFMA GEMM engine
# --------------------------------------------------------------------------------------

def _nd_dims(s: ConvNdSpec):
    v = list(s.ins) + list(s.outs) + list(s.ks) + list(s.st) + list(s.pd)
    return (C.c_int * len(v))(*v)


def _nd_dt(t: torch.Tensor) -> int:
    assert t.dtype in (BF16, torch.float32), t.dtype
    return int(t.dtype == torch.float32)


def _nd_col(x, s: ConvNdSpec, g: int) -> torch.Tensor:
    """im2col of channel group g: [num * P][ld] bf16 (ld = Cg*T rounded up to 8, pad = 0)."""
    ld = _round8(s.Cg * s.T)
    col = torch.empty((s.num * s.P, ld), dtype=BF16, device=x.device)
    call("im2col_nd", x, col, s.nd, s.num, s.C, s.Cg, g * s.Cg, ld, _nd_dims(s), _nd_dt(x), 0)
    return col


def _nd_chan_cl(t, s: ConvNdSpec, chans: int, g: int, per: int) -> torch.Tensor:
    """[num][chans][P] channel group g (per channels) -> channels-last [num * P][per]."""
    from . import layers_hip as lh
    if s.groups == 1:
        return lh.transpose(t, s.num, chans, s.P).view(s.num * s.P, chans)
    tmp = torch.empty((s.num, per, s.P), dtype=t.dtype, device=t.device)
    lh.axis_copy(t, tmp, s.num, chans, per, s.P, g * per, 0, per)
    return lh.transpose(tmp, s.num, per, s.P).view(s.num * s.P, per)


def conv_nd_forward(x, w, b, s: ConvNdSpec):
    """x [num][C][ins] bf16, w [K][Cg][ks] bf16 (Caffe layout) -> y [num][K][outs] bf16: per
    group an N-d im2col, one NT MFMA product with the bias epilogue, and a transpose of the
    channels-last result into the group's channel slice."""
    from . import layers_hip as lh
    x = _c(x)
    CT = s.Cg * s.T
    y = torch.empty((s.num, s.K, s.P), dtype=BF16, device=x.device)
    for g in range(s.groups):
        col = _nd_col(x, s, g)
        wg = torch.zeros((s.Kg, col.shape[1]), dtype=BF16, device=x.device)
        wg[:, :CT] = w[g * s.Kg:(g + 1) * s.Kg].reshape(s.Kg, CT)
        bg = b[g * s.Kg:(g + 1) * s.Kg].float().contiguous() if b is not None else None
        yc = linear_fwd(col, wg, bg)  # [num * P][Kg]
        if s.groups == 1:
            y = lh.transpose(yc, s.num, s.P, s.Kg, out_shape=(s.num, s.K, s.P))
        else:
            lh.axis_copy(lh.transpose(yc, s.num, s.P, s.Kg), y, s.num, s.Kg, s.K, s.P, 0, g * s.Kg, s.Kg)
    return y.view((s.num, s.K) + s.outs)


def conv_nd_backward(dy, x, w, s: ConvNdSpec, need_dx: bool, dw=None, db=None):
    """Weight / bias gradients (accumulated into dw [K][Cg][ks], db [K], fp32) from one TN
    product per group over the channels-last dy and the im2col of x (bias through the
    ones column); the data gradient from one NN product per group and the N-d col2im."""
    dy = _c(dy).to(BF16)
    if x is not None:
        x = _c(x)
    assert x is not None or dw is None, "the weight gradient needs the input"
    CT = s.Cg * s.T
    dx = torch.empty((s.num, s.C) + s.ins, dtype=dy.dtype, device=dy.device) if need_dx else None
    for g in range(s.groups):
        dyc = _nd_chan_cl(dy, s, s.K, g, s.Kg)  # [num * P][Kg]
        if dw is not None:
            col = _nd_col(x, s, g)
            dwg = dw.view(s.K, CT)[g * s.Kg:(g + 1) * s.Kg]
            dbg = db[g * s.Kg:(g + 1) * s.Kg] if db is not None else None
            if not linear_wgrad(dyc, col[:, :CT], dwg, accumulate=True, db=dbg, db_acc=True) and dbg is not None:
                colsum(dyc, dbg, accumulate=True)
        elif db is not None:
            colsum(dyc, db[g * s.Kg:(g + 1) * s.Kg], accumulate=True)
        if need_dx:
            wg = w[g * s.Kg:(g + 1) * s.Kg].reshape(s.Kg, CT).contiguous()
            dcol = linear_dgrad(dyc, wg)  # [num * P][CT] (possibly a view of a padded buffer)
            call("col2im_nd", dcol, dx, s.nd, s.num, s.C, s.Cg, g * s.Cg, dcol.stride(0), _nd_dims(s), 0,
                 _nd_dt(dx), 0)
    return dx


# --------------------------------------------------------------------------------------
# Pooling / LRN
# --------------------------------------------------------------------------------------

def _pool_args(s: PoolSpec):
    return (s.N, s.H, s.W, s.C, s.P, s.Q, s.kh, s.kw, s.sh, s.sw, s.ph, s.pw, s.method)


# the pooling / LRN kernels decode NHWC element indices in 32 bits: larger batches run as
# several launches over image ranges (contiguous NHWC slices)
_MAX_ELEMS = 1 << 31


def _pool_images(s: PoolSpec) -> int:
    per = s.H * s.W * s.C
    return s.N if s.N * per < _MAX_ELEMS else max(1, (_MAX_ELEMS - 1) // per)


def pool_side_ok(s: PoolSpec, backward: bool) -> bool:
    """Can the pooling kernels store an fp8 side output (ops.gemm.Fp8Side) of this pool's
    output (forward: vectorised 2x2 / 3x3 max pooling) or input gradient (backward: the
    pool_bwd_k gathers, not the 3x3 / stride-2 blocked kernel)?"""
    if s.C % 8:
        return False
    if not backward:
        return s.method == POOL_MAX and s.kh == s.kw and s.kh in (2, 3)
    nh, nw = -(-s.kh // s.sh), -(-s.kw // s.sw)
    return not (s.kh == 3 and s.kw == 3 and s.sh == 2 and s.sw == 2) and nh == nw and 1 <= nh <= 3


def _side_args(side, t, n0, n1):
    if side is None:
        return (None, None, None, 0)
    return (side.q[n0:n1], side.slot, side.part, int(side.e5m2))


def pool_forward_mask(x, s: PoolSpec, gate: bool = False, side=None):
    """gate=True (MAX only): x is the output of a slope-0 in-place ReLU whose backward is
    folded into the argmax mask (windows with max <= 0 pass no gradient).  side: an
    ops.gemm.Fp8Side over the output (pool_side_ok): the kernel also stores its fp8 bytes."""
    x = _c(x)
    if side is not None:
        assert pool_side_ok(s, False) and tuple(side.base.shape) == (s.N, s.P, s.Q, s.C)
        y = side.base
    else:
        y = torch.empty((s.N, s.P, s.Q, s.C), dtype=BF16, device=x.device)
    mask = torch.empty((s.N, s.P, s.Q, s.C), dtype=torch.uint8, device=x.device) if s.method == POOL_MAX else None
    nb = _pool_images(s)
    for n0 in range(0, s.N, nb):
        n1 = min(s.N, n0 + nb)
        call("pool_fwd", x[n0:n1], y[n0:n1], mask[n0:n1] if mask is not None else None,
             *_pool_args(dataclasses.replace(s, N=n1 - n0)), int(gate and s.method == POOL_MAX),
             *_side_args(side, y, n0, n1))
    if side is not None:
        side.launches += 1
        side.finish()
    return y, mask


def pool_forward(x, s: PoolSpec):
    return pool_forward_mask(x, s)[0]


def pool_backward(dy, x, s: PoolSpec, mask=None, y=None, gate=False, side=None, side_only=False):
    """side: an ops.gemm.Fp8Side over dx (pool_side_ok backward; not with a non-MAX gate).
    side_only: store the fp8 bytes alone — the returned bf16 dx is NOT written (its only
    reader takes the fp8 copy, engine.fuse_fp8_quant's fp8_dx_only; side.only marks it so
    conv_backward refuses any path that would read the bf16 values)."""
    if side_only:
        assert side is not None and s.method == POOL_MAX
        side.only = True
    if side is not None:
        assert pool_side_ok(s, True) and not (gate and s.method != POOL_MAX)
        assert tuple(side.base.shape) == (s.N, s.H, s.W, s.C)
        dx = side.base
    else:
        dx = torch.empty((s.N, s.H, s.W, s.C), dtype=BF16, device=dy.device)
    if s.method == POOL_MAX and mask is None:
        _, mask = pool_forward_mask(x, s, gate)
    dy = _c(dy)
    nb = _pool_images(s)
    for n0 in range(0, s.N, nb):
        n1 = min(s.N, n0 + nb)
        call("pool_bwd", dy[n0:n1], mask[n0:n1] if mask is not None else None, None if side_only else dx[n0:n1],
             *_pool_args(dataclasses.replace(s, N=n1 - n0)), *_side_args(side, dx, n0, n1))
    if side is not None:
        side.launches += 1
        side.finish()
    if gate and s.method != POOL_MAX:
        dx = relu_backward(dx, x)
    return dx


def pool_lrn_eligible(s: PoolSpec, size: int, within: bool) -> bool:
    """Max pooling 3x3 / stride 2 followed by a cross-channel LRN that the fused
    sn_pool_lrn_fwd / sn_lrn_pool_bwd pair covers (csrc/kernels/pool_lrn.hip)."""
    if s.method != POOL_MAX or within or (s.kh, s.kw, s.sh, s.sw) != (3, 3, 2, 2) or s.C % 8 or size not in (3, 5, 7, 9):
        return False
    if s.ph >= 3 or s.pw >= 3 or s.N * s.H * s.W * s.C >= 1 << 32:
        return False
    # the kernels' own host tests (plrn_ok, the backward tile search of plrn_bwd_tile with the
    # LDS-staged mask's 24-B items and >= 4-chunk groups, row coverage): one source of truth
    fn = _lib.kernels().sn_pool_lrn_supported
    fn.restype = C.c_int
    return bool(fn(*(C.c_longlong(v) for v in (s.N, s.H, s.W, s.C, s.P, s.Q, s.ph, s.pw, size))))


def pool_lrn_forward(x, s: PoolSpec, gate: bool, size: int, alpha: float, beta: float, k: float):
    """-> (pooled, argmax mask, LRN output): max pooling and the cross-channel LRN of its
    output in one launch (the pooled tensor is kept: the LRN backward reads it)."""
    x = _c(x)
    pooled = torch.empty((s.N, s.P, s.Q, s.C), dtype=BF16, device=x.device)
    mask = torch.empty((s.N, s.P, s.Q, s.C), dtype=torch.uint8, device=x.device)
    y = torch.empty_like(pooled)
    call("pool_lrn_fwd", x, pooled, mask, y, s.N, s.H, s.W, s.C, s.P, s.Q, s.ph, s.pw, int(gate), int(size),
         float(alpha), float(beta), float(k))
    return pooled, mask, y


def lrn_pool_backward(dy, pooled, mask, s: PoolSpec, size: int, alpha: float, beta: float, k: float):
    """Gradient at the pooling input from the gradient at the LRN output (the pooled
    gradient lives only in LDS)."""
    dx = torch.empty((s.N, s.H, s.W, s.C), dtype=BF16, device=dy.device)
    call("lrn_pool_bwd", _c(pooled), _c(dy), mask, dx, s.N, s.H, s.W, s.C, s.P, s.Q, s.ph, s.pw, int(size),
         float(alpha), float(beta), float(k))
    return dx


def pool_lrn_rev_eligible(s: PoolSpec, size: int, within: bool) -> bool:
    """A cross-channel LRN feeding a 3x3 / stride-2 max pooling whose backwards
    sn_pool_lrn_bwd_rev runs as one launch (csrc/kernels/pool_lrn.hip: plrn_ok and the
    2x2-block row coverage, mirrored here)."""
    if s.method != POOL_MAX or within or (s.kh, s.kw, s.sh, s.sw) != (3, 3, 2, 2) or s.C % 8 or size not in (3, 5, 7, 9):
        return False
    if s.ph >= 3 or s.pw >= 3 or s.N * s.H * s.W * s.C >= 1 << 32 or s.C > 8192:
        return False
    if 2 * (s.P - 1) - s.ph >= s.H or 2 * (s.Q - 1) - s.pw >= s.W:
        return False
    return (s.H + s.ph + 1) // 2 <= s.P + 1 and (s.W + s.pw + 1) // 2 <= s.Q + 1


def pool_lrn_backward_rev(dy, mask, x, s: PoolSpec, size: int, alpha: float, beta: float, k: float,
                          gate: bool = False):
    """Gradient at an LRN's input from the gradient at the output of the max pooling that
    reads the LRN's output (pool_bwd_k3s2 then lrn_across_bwd in one launch; the LRN-output
    gradient lives only in registers).  x: the LRN input; gate: the in-place ReLU that
    produced x."""
    x = _c(x)
    assert tuple(x.shape) == (s.N, s.H, s.W, s.C) and tuple(mask.shape) == (s.N, s.P, s.Q, s.C)
    dx = torch.empty_like(x)
    call("pool_lrn_bwd_rev", _c(dy), _c(mask), x, dx, s.N, s.H, s.W, s.C, s.P, s.Q, s.ph, s.pw, int(size),
         float(alpha), float(beta), float(k), int(gate))
    return dx


def lrn_forward(x, size, alpha, beta, k, within=False):
    x = _c(x)
    N, H, W, Cc = x.shape
    y = torch.empty_like(x)
    if within:
        call("lrn_within_fwd", x, y, None, N, H, W, Cc, size, float(alpha), float(beta))
    else:
        call("lrn_across_fwd", x, y, N, H, W, Cc, size, float(alpha), float(beta), float(k))
    return y


def lrn_backward(dy, x, size, alpha, beta, k, within=False, y=None, gate=False):
    """gate: also apply the backward of the slope-0 in-place ReLU that produced x (dx = 0
    where x <= 0) — inside the across-channel kernel, as a pass after the within one."""
    x, dy = _c(x), _c(dy)
    N, H, W, Cc = x.shape
    dx = torch.empty_like(x)
    if within:
        sbuf = torch.empty(x.shape, dtype=torch.float32, device=x.device)
        u = torch.empty(x.shape, dtype=torch.float32, device=x.device)
        call("lrn_within_bwd", x, dy, sbuf, u, dx, N, H, W, Cc, size, float(alpha), float(beta))
        if gate:
            dx = relu_backward(dx, x)
    else:
        call("lrn_across_bwd", x, dy, dx, N, H, W, Cc, size, float(alpha), float(beta), float(k), int(gate))
    return dx


# --------------------------------------------------------------------------------------
# Elementwise
# --------------------------------------------------------------------------------------

def relu_forward(x, slope=0.0):
    x = as_bf16(x)
    y = torch.empty_like(x)
    call("relu_fwd", x, y, x.numel(), float(slope))
    return y


def relu_backward(dy, x, slope=0.0):
    dy, x = as_bf16(dy), as_bf16(x)
    dx = torch.empty_like(dy)
    call("relu_bwd", dy, x, dx, x.numel(), float(slope))
    return dx


def _dropout(x, ratio, rng_state, stream, gate=None):
    x = as_bf16(x)
    y = torch.empty_like(x)
    call("dropout", x, y, x.numel(), rng_state, int(stream), float(ratio), as_bf16(gate))
    return y


def dropout_forward(x, ratio, rng_state, stream):
    return _dropout(x, ratio, rng_state, stream)


def dropout_backward(dy, ratio, rng_state, stream, gate=None):
    return _dropout(dy, ratio, rng_state, stream, gate)


def cast_f32_to_bf16(src, dst):
    call("cast_f32_bf16", src, dst, src.numel())


def advance_rng(rng_state):
    call("advance_rng", rng_state)


def concat_channels(parts, out):
    """NHWC channel concat of bf16 ``parts`` into ``out`` (one launch, <= 8 parts)."""
    pix = out.numel() // out.shape[-1]
    parts = [_c(t) for t in parts]
    assert sum(t.shape[-1] for t in parts) == out.shape[-1] and all(t.numel() // t.shape[-1] == pix for t in parts)
    _concat(parts, None, [t.shape[-1] for t in parts], out, pix, 0)
    return out


def concat_channels_bwd(dy, diffs, gates, chans):
    """Backward of concat_channels: ``diffs[i]`` (pre-allocated, or None to skip the part)
    get channels [sum(chans[:i]), +chans[i]) of ``dy``, masked by ``gates[i] > 0`` when a
    gate is given."""
    dy = _c(dy)
    pix = dy.numel() // dy.shape[-1]
    assert sum(chans) == dy.shape[-1]
    for d, g, c in zip(diffs, gates, chans):
        assert d is None or (d.is_contiguous() and d.shape[-1] == c and d.numel() // c == pix)
        assert g is None or (g.is_contiguous() and d is not None and g.shape == d.shape)
    _concat(diffs, gates, chans, dy, pix, 1)


def _concat(parts, gates, chans, top, pix, bwd):
    n = len(parts)
    P = (C.c_void_p * 8)(*[(t.data_ptr() if t is not None else 0) for t in parts] + [0] * (8 - n))
    G = (C.c_void_p * 8)(*[(g.data_ptr() if g is not None else 0) for g in (gates or [None] * n)] + [0] * (8 - n))
    Ch = (C.c_longlong * 8)(*list(chans) + [0] * (8 - n))
    _lib.check(_lib.kernels().sn_concat_nhwc(P, G, Ch, C.c_longlong(n), C.c_void_p(top.data_ptr()),
                                             C.c_longlong(pix), C.c_longlong(bwd), C.c_void_p(_lib.stream_ptr())),
               "concat_nhwc")
    if _lib.DEBUG_SYNC:
        _lib.debug_sync("concat_nhwc")


def sum_bf16(tensors, out=None):
    out = torch.empty_like(tensors[0]) if out is None else out
    n = out.numel()
    for i in range(0, len(tensors), 8):
        chunk = [_c(t) for t in tensors[i:i + 8]]
        if i:
            chunk = [out] + chunk[:7]
        arr = (C.c_void_p * 8)(*[t.data_ptr() for t in chunk] + [0] * (8 - len(chunk)))
        _lib.check(_lib.kernels().sn_sum_bf16(arr, C.c_longlong(len(chunk)), C.c_void_p(out.data_ptr()),
                                              C.c_longlong(n), C.c_void_p(_lib.stream_ptr())), "sum_bf16")
    return out


# --------------------------------------------------------------------------------------
# Softmax / loss / accuracy
# --------------------------------------------------------------------------------------

def softmax_loss_forward(x2, labels, ignore_label=None, normalize=True, outer_num=None):
    x2 = _c(x2)
    M, Cn = x2.shape
    dev = x2.device
    prob = torch.empty((M, Cn), dtype=torch.float32, device=dev)
    rows = torch.empty((2, M), dtype=torch.float32, device=dev)
    out = torch.empty(2, dtype=torch.float32, device=dev)
    lab = _c(labels.reshape(-1).float())
    call("softmax_xent_fwd", x2, lab, prob, rows[0], rows[1], out[0:1], out[1:2], M, Cn,
         int(ignore_label is not None), int(ignore_label or 0), int(normalize),
         int(outer_num if outer_num is not None else M))
    return out[0], prob, out[1:2]


def softmax_loss_backward(prob, labels, loss_weight, norm, ignore_label=None, dtype=BF16):
    M, Cn = prob.shape
    dx = torch.empty((M, Cn), dtype=BF16, device=prob.device)
    lw = loss_weight.reshape(-1).float()
    call("softmax_xent_bwd", prob, _c(labels.reshape(-1).float()), lw, norm, dx, M, Cn,
         int(ignore_label is not None), int(ignore_label or 0))
    return dx if dtype == BF16 else dx.to(dtype)


def softmax_forward(x2):
    x2 = as_bf16(x2)
    y = torch.empty_like(x2)
    call("softmax_fwd", x2, y, x2.shape[0], x2.shape[1])
    return y


def softmax_backward(dy2, y2):
    dy2, y2 = as_bf16(dy2), as_bf16(y2)
    dx = torch.empty_like(y2)
    call("softmax_bwd", dy2, y2, dx, y2.shape[0], y2.shape[1])
    return dx


def accuracy(x2, labels, top_k=1, ignore_label=None):
    x2 = _c(x2)
    M, Cn = x2.shape
    rows = torch.empty((2, M), dtype=torch.float32, device=x2.device)
    out = torch.empty(2, dtype=torch.float32, device=x2.device)
    call("accuracy", x2, _c(labels.reshape(-1).float()), rows[0], rows[1], out[0:1], out[1:2], M, Cn,
         int(top_k), int(ignore_label is not None), int(ignore_label or 0))
    return out[0]


# --------------------------------------------------------------------------------------
# Solver
# --------------------------------------------------------------------------------------

CHUNK = 8192


def solver_tables(segments, total: int, device, slab_chunks=None) -> dict:
    """Chunk table of the fused update kernel.  ``slab_chunks``: {segment offset: [(start,
    count, slab byte address, slab stride, splits, element stride), ...]} replaces the
    flat-gradient chunks of those segments by chunks whose gradient the kernel sums from
    split-K slabs (engine.fuse_splitk_updates)."""
    pos, mult, src = [], [], []
    slab_chunks = slab_chunks or {}
    for off, cnt, lm, dm in segments:
        if off in slab_chunks:
            for start, n, ptr, ss, splits, es in slab_chunks[off]:
                for s in range(0, n, CHUNK):
                    pos.append((start + s, min(CHUNK, n - s)))
                    mult.append((lm, dm))
                    src.append((ptr + 4 * s * es, ss, splits, es))
            continue
        padded = -(-cnt // 64) * 64
        for s in range(0, padded, CHUNK):
            pos.append((off + s, min(CHUNK, padded - s)))
            mult.append((lm, dm))
            src.append((0, 0, 0, 0))
    nparts = max(1, min(1024, -(-total // (256 * 16))))
    return {
        "pos": torch.tensor(pos or [(0, 0)], dtype=torch.int64, device=device),
        "mult": torch.tensor(mult or [(0.0, 0.0)], dtype=torch.float32, device=device),
        "src": (torch.tensor(src, dtype=torch.int64, device=device) if slab_chunks and src else None),
        "n": len(pos),
        "part": torch.empty(nparts, dtype=torch.float32, device=device),
        "total": total,
    }


def solver_update(kind, data, diff, history, compute, tables, hyper, l1, clip, grid_limit=0):
    h0 = history[0]
    h1 = history[1] if len(history) > 1 else history[0]
    call("solver_update", int(kind), data, diff, h0, h1, compute, tables["pos"], tables["mult"], tables["n"],
         hyper, int(l1), int(clip), tables["part"], tables["part"].numel(), tables["total"], int(grid_limit),
         tables.get("src"))


def scale_shadow(flat, shadow, scale: float):
    call("scale_shadow", flat, shadow, flat.numel(), float(scale))


# --------------------------------------------------------------------------------------
# Data augmentation
# --------------------------------------------------------------------------------------

def s2d_plan(s: ConvSpec):
    return _s2d_plan(s)


def _labels(labels, label_out):
    if labels is None:
        return None, None
    assert labels.dtype == torch.int32 and label_out.dtype == torch.float32 and label_out.numel() == labels.numel()
    return _c(labels), label_out


def augment_s2d(src_u8, x2, crop, plan, s: ConvSpec, mean=None, mean_mode=0, scale=1.0, rng_state=None,
                train=True, mirror=False, labels=None, label_out=None):
    """Fused augment + space-to-depth fold into x2 (see conv_forward(folded=...)); with
    ``labels`` (int32 [N]) the same launch also writes them as floats into ``label_out``."""
    N, Cc, Hs, Ws = src_u8.shape
    f, cp, rf, sf, s2 = plan
    assert tuple(x2.shape) == (N, s2.H, s2.W, s2.C) and x2.dtype == BF16 and x2.is_contiguous()
    assert s.C == Cc and s.H == crop and s.W == crop
    assert labels is None or labels.numel() == N
    call("augment_s2d", _c(src_u8), x2, N, Cc, Hs, Ws, crop, crop, mean, int(mean_mode), float(scale), rng_state,
         int(train), int(mirror), s2.H, s2.W, f, cp, s.ph, s.pw, *_labels(labels, label_out))
    return x2


def augment(src_u8, dst, crop, mean=None, mean_mode=0, scale=1.0, rng_state=None, train=True, mirror=False,
            offs_out=None, labels=None, label_out=None):
    N, Cc, Hs, Ws = src_u8.shape
    assert labels is None or labels.numel() == N
    # an fp32 data blob (the fp32 device mode) gets the fp32 twin of the kernel
    call("augment_f32" if dst.dtype == torch.float32 else "augment", _c(src_u8), dst, N, Cc, Hs, Ws, crop, crop,
         mean, int(mean_mode), float(scale), rng_state, int(train), int(mirror), offs_out,
         *_labels(labels, label_out))
    return dst


# --------------------------------------------------------------------------------------
# FP8 (e4m3) forward products with per-tensor delayed scaling
# --------------------------------------------------------------------------------------

FP8_MARGIN = float(os.environ.get("SN_FP8_MARGIN", "1.0"))  # quantisation scale = 448 / (amax * margin)
# delayed scaling over the max of the last FP8_HISTORY iterations' amaxes (0: last iteration only)
FP8_HISTORY = int(os.environ.get("SN_FP8_HISTORY", "16"))


E4M3_MAX, E5M2_MAX = 448.0, 57344.0


class Fp8Scales:
    """Device-resident scale slots (csrc/kernels/fp8.hip): [n][scale, amax, 1/scale,
    initialised, format max, -, -, -].  Slots are e4m3 unless :meth:`set_e5m2` is called."""

    def __init__(self, n: int, device):
        self.updates = 0  # fp8_update_scales launches issued (slots are initialised after the first)
        self.slots = torch.zeros((max(n, 1), 8), dtype=torch.float32, device=device)
        self.slots[:, 0] = 1.0
        self.slots[:, 2] = 1.0
        self.slots[:, 4] = E4M3_MAX
        self.n = n
        self._e5m2 = set()
        self.history = FP8_HISTORY
        self.hist = torch.zeros((max(n, 1), max(1, self.history)), dtype=torch.float32, device=device)

    def set_e5m2(self, i: int) -> None:
        self.slots[i, 4] = E5M2_MAX
        self._e5m2.add(i)

    def is_e5m2(self, i: int) -> bool:
        return i in self._e5m2

    def slot(self, i: int) -> torch.Tensor:
        return self.slots[i]

    def deq(self, i: int) -> torch.Tensor:
        return self.slots[i, 2:3]

    def update(self) -> None:
        call("fp8_update_scales", self.slots, self.hist, int(self.history), self.n, float(FP8_MARGIN))
        self.updates += 1


def quant_fp8(x: torch.Tensor, slot: torch.Tensor, out: torch.Tensor | None = None,
              e5m2: bool = False) -> torch.Tensor:
    """e4m3 (or e5m2) bytes of bf16 ``x`` scaled by slot[0]; folds |x|max into slot[1]
    (an uninitialised slot is scaled from the current tensor, see csrc/kernels/fp8.hip)."""
    x = _c(x)
    q = torch.empty(x.shape, dtype=torch.uint8, device=x.device) if out is None else out
    call("quant_fp8", x, q, x.numel(), slot, bool(e5m2))
    return q


def conv_forward_fp8(xq, wq, b, s: ConvSpec, deq_x, deq_w, relu=False, out=None):
    """Implicit-GEMM convolution on e4m3 operands (v_mfma_scale_f32_16x16x128_f8f6f4),
    fp32 accumulation, dequantised + bias + ReLU epilogue, bf16 NHWC output (written into
    ``out`` when given: image chunks of a large batch write their slice in place)."""
    assert s.Cg % 16 == 0 and s.C % 16 == 0 and xq.dtype == torch.uint8 and wq.dtype == torch.uint8
    nb = _image_chunk(s)
    if nb < s.N:
        y = out if out is not None else torch.empty((s.N, s.P, s.Q, s.K), dtype=BF16, device=xq.device)
        for n0 in range(0, s.N, nb):
            n1 = min(s.N, n0 + nb)
            conv_forward_fp8(xq[n0:n1], wq, b, s.with_batch(n1 - n0), deq_x, deq_w, relu, out=y[n0:n1])
        return y
    M = s.N * s.P * s.Q
    kred = s.R * s.S * s.Cg
    y = out if out is not None else torch.empty((s.N, s.P, s.Q, s.K), dtype=BF16, device=xq.device)
    assert y.is_contiguous()
    if direct_fp8_ok(s) and not _side_covers(y):
        call("conv3x3_fp8", _c(xq), _c(wq), deq_x, deq_w, b, None, y, s.N, s.H, s.W, int(relu))
        return y
    A = Im2col(xq, _geom(s), kcontig=True, gstride=s.Cg)
    B = Dense(wq.view(s.K, kred), kred, True, gstride=s.Kg * kred)
    gemm(M, s.Kg, kred, A, B, y, s.K, epi=EPI_BF16, groups=s.groups, c_gstride=s.Kg, bias=b, relu=relu,
         deq=(deq_x, deq_w))
    return y


def linear_forward_fp8(xq, wq, b, deq_x, deq_w, relu=False, dropout=None):
    M, K = xq.shape
    N = wq.shape[0]
    assert K % 16 == 0
    y = torch.empty((M, N), dtype=BF16, device=xq.device)
    gemm(M, N, K, Dense(xq, K, True), Dense(wq, K, True), y, N, epi=EPI_BF16, bias=b, relu=relu,
         deq=(deq_x, deq_w), dropout=dropout)
    return y
