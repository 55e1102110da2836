"""Python front-end of the MFMA GEMM (``csrc/kernels/gemm.hip``).

All products are expressed as ``C_g[m, n] (op)= sum_k A_g(m, k) * B_g(n, k)`` over
"virtual row-major matrices" (see the kernel header):

* ``Dense(t, ld, kcontig)`` — a 2-D bf16 view;  ``kcontig=True`` means rows are the
  M/N axis and the reduction axis is contiguous (KC), otherwise rows are the reduction
  axis (MC, read through ds_read_b64_tr_b16).
* ``Im2col(x, geom)`` — the implicit [N*P*Q] x [R*S*Cg] patch matrix of an NHWC tensor.

Split-K is chosen so a launch has enough workgroups for 256 CUs; partial products go to
an fp32 workspace and are combined by a deterministic reduce kernel.
"""
from __future__ import annotations

import ctypes as C
from dataclasses import dataclass

import torch

from . import _lib

OP_DENSE, OP_IM2COL = 0, 1
EPI_BF16, EPI_F32, EPI_F32_ACC = 0, 1, 2
BM = BN = 128
BK = 64
TARGET_BLOCKS = 512  # 2 blocks per CU on 256 CUs


@dataclass
class Dense:
    t: torch.Tensor
    ld: int
    kcontig: bool
    gstride: int = 0  # elements between groups


@dataclass
class ConvGeom:
    N: int
    H: int
    W: int
    C: int
    P: int
    Q: int
    R: int
    S: int
    sh: int = 1
    sw: int = 1
    ph: int = 0
    pw: int = 0
    dh: int = 1
    dw: int = 1
    Cg: int = 0

    def c_struct(self) -> _lib.SnConvGeom:
        return _lib.SnConvGeom(self.N, self.H, self.W, self.C, self.P, self.Q, self.R, self.S,
                               self.sh, self.sw, self.ph, self.pw, self.dh, self.dw, self.Cg)


@dataclass
class Im2col:
    x: torch.Tensor  # NHWC bf16
    geom: ConvGeom
    kcontig: bool
    gstride: int = 0  # channels between groups


def _operand(op) -> tuple[_lib.SnOperand, int, int]:
    if isinstance(op, Dense):
        assert op.t.dtype == torch.bfloat16, op.t.dtype
        assert op.t.data_ptr() % 16 == 0 and op.ld % 8 == 0, "dense operand must be 16-B aligned"
        s = _lib.SnOperand(op.t.data_ptr(), op.ld, op.gstride, _lib.SnConvGeom())
        return s, 0 if op.kcontig else 1, OP_DENSE
    assert op.x.dtype == torch.bfloat16 and op.x.is_contiguous()
    g = op.geom
    assert g.Cg % 8 == 0 and g.C % 8 == 0, "implicit conv needs channels % 8 == 0"
    # the kernel's fp32-reciprocal index division is exact below 2^24
    assert g.N * g.P * g.Q < (1 << 24) and g.N * g.H * g.W < (1 << 24), "conv too large for one launch"
    s = _lib.SnOperand(op.x.data_ptr(), 0, op.gstride, g.c_struct())
    return s, 0 if op.kcontig else 1, OP_IM2COL


TILES = {0: (128, 128), 1: (256, 64)}


def choose_tile(M: int, N: int) -> int:
    """256x64 for skinny N (<= 64 per group, e.g. 48-channel grouped dgrad), else 128x128."""
    return 1 if N <= 64 and M >= 256 else 0


def choose_splits(M: int, N: int, K: int, groups: int = 1, tile: int = 0) -> tuple[int, int]:
    bm, bn = TILES[tile]
    tiles = -(-M // bm) * -(-N // bn) * groups
    splits = 1
    if tiles < TARGET_BLOCKS and K > 4 * BK:
        ws_cap = max(1, (256 << 20) // max(1, 4 * M * N * groups))  # fp32 partial slabs <= 256 MB
        splits = max(1, min(-(-TARGET_BLOCKS // tiles), K // (4 * BK), 256, ws_cap))
    kchunk = -(-K // splits)
    kchunk = -(-kchunk // BK) * BK
    splits = -(-K // kchunk)
    return splits, kchunk


def gemm(M: int, N: int, K: int, A, B, out: torch.Tensor, ldc: int, *, epi: int,
         groups: int = 1, c_gstride: int = 0, bias: torch.Tensor | None = None, relu: bool = False,
         splits: int | None = None) -> None:
    """Run one (possibly grouped, split-K) GEMM.  ``epi``: EPI_BF16 (store bf16 with
    bias/ReLU), EPI_F32 (store), EPI_F32_ACC (accumulate into an fp32 output)."""
    if M == 0 or N == 0:
        return
    sa, a_mc, a_mode = _operand(A)
    sb, b_mc, b_mode = _operand(B)
    tile = choose_tile(M, N)
    if splits is None:
        splits, kchunk = choose_splits(M, N, K, groups, tile)
    else:
        kchunk = -(-(-(-K // splits)) // BK) * BK
        splits = max(1, -(-K // kchunk))
    if bias is not None:
        assert bias.dtype == torch.float32 and bias.is_contiguous()
    if splits == 1:
        args = _lib.SnGemmArgs(M, N, K, groups, 1, max(kchunk, BK), a_mc, a_mode, b_mc, b_mode, epi,
                               sa, sb, out.data_ptr(), ldc, c_gstride, 0,
                               bias.data_ptr() if bias is not None else 0, int(relu), tile)
        _lib.check(_lib.kernels().sn_gemm(C.byref(args), C.c_void_p(_lib.stream_ptr())), "gemm")
        return
    ws = torch.empty((groups, splits, M, N), dtype=torch.float32, device=out.device)
    args = _lib.SnGemmArgs(M, N, K, groups, splits, kchunk, a_mc, a_mode, b_mc, b_mode, EPI_F32,
                           sa, sb, ws.data_ptr(), N, splits * M * N, M * N, 0, 0, tile)
    _lib.check(_lib.kernels().sn_gemm(C.byref(args), C.c_void_p(_lib.stream_ptr())), "gemm")
    mode = {EPI_BF16: 0, EPI_F32: 1, EPI_F32_ACC: 2}[epi]
    _lib.call("splitk_reduce", ws, splits, M * N, M, N, N, out, ldc, mode, bias, int(relu),
              groups, splits * M * N, c_gstride)


# --- dense helpers ---------------------------------------------------------------------

def _pad8(t: torch.Tensor, dim: int) -> torch.Tensor:
    n = t.shape[dim]
    if n % 8 == 0 and t.is_contiguous() and t.data_ptr() % 16 == 0:
        return t
    pad = (-n) % 8
    shape = list(t.shape)
    shape[dim] = n + pad
    out = torch.zeros(shape, dtype=t.dtype, device=t.device)
    out.narrow(dim, 0, n).copy_(t)
    return out


def linear_fwd(x: torch.Tensor, w: torch.Tensor, bias: torch.Tensor | None = None,
               relu: bool = False, out: torch.Tensor | None = None) -> torch.Tensor:
    """y[M,N] = x[M,K] @ w[N,K]^T (+bias, ReLU) in bf16."""
    M, K = x.shape
    N = w.shape[0]
    xp, wp = _pad8(x, 1), _pad8(w, 1)
    Kp = xp.shape[1]
    if out is None:
        out = torch.empty((M, N), dtype=torch.bfloat16, device=x.device)
    gemm(M, N, Kp, Dense(xp, Kp, True), Dense(wp, Kp, True), out, out.stride(0), epi=EPI_BF16,
         bias=bias, relu=relu)
    return out


def linear_dgrad(dy: torch.Tensor, w: torch.Tensor, out: torch.Tensor | None = None) -> torch.Tensor:
    """dx[M,K] = dy[M,N] @ w[N,K] in bf16 (B operand read transposed from LDS)."""
    M, N = dy.shape
    K = w.shape[1]
    dyp = _pad8(dy, 1)
    Np = dyp.shape[1]
    wp = w
    if Np != N or K % 8 or not w.is_contiguous():
        wp = torch.zeros((Np, -(-K // 8) * 8), dtype=w.dtype, device=w.device)
        wp[:N, :K].copy_(w)
    Kp = wp.shape[1]
    if out is None or Kp != K:
        o = torch.empty((M, Kp), dtype=torch.bfloat16, device=dy.device)
    else:
        o = out
    gemm(M, Kp, Np, Dense(dyp, Np, True), Dense(wp, Kp, False), o, o.stride(0), epi=EPI_BF16)
    if o is not out:
        o = o[:, :K]
        if out is not None:
            out.copy_(o)
            return out
    return o


def linear_wgrad(dy: torch.Tensor, x: torch.Tensor, dw: torch.Tensor, accumulate: bool = True) -> None:
    """dw[N,K] (+)= dy[M,N]^T @ x[M,K], fp32 output; both operands read along M."""
    M, N = dy.shape
    K = x.shape[1]
    dyp, xp = _pad8(dy, 1), _pad8(x, 1)
    Np, Kp = dyp.shape[1], xp.shape[1]
    if Np == N and Kp == K and dw.is_contiguous():
        gemm(N, K, M, Dense(dyp, Np, False), Dense(xp, Kp, False), dw, K,
             epi=EPI_F32_ACC if accumulate else EPI_F32)
        return
    tmp = torch.zeros((Np, Kp), dtype=torch.float32, device=dw.device)
    gemm(Np, Kp, M, Dense(dyp, Np, False), Dense(xp, Kp, False), tmp, Kp, epi=EPI_F32)
    if accumulate:
        dw.add_(tmp[:N, :K])
    else:
        dw.copy_(tmp[:N, :K])


def colsum(x: torch.Tensor, out: torch.Tensor, accumulate: bool = True) -> None:
    """out[N] (+)= sum over rows of a bf16 [M, N] matrix (bias gradient)."""
    M, N = x.shape
    nparts = max(1, min(1024, M // 64))
    part = torch.empty((nparts, N), dtype=torch.float32, device=x.device)
    _lib.call("colsum_bf16", x, M, N, x.stride(0), part, nparts, out, int(accumulate))
