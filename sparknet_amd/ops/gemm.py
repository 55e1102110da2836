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

import ast
import contextlib
import ctypes as C
import json
import os
from dataclasses import dataclass

import torch

from . import _lib
from ..utils import features

OP_DENSE, OP_IM2COL, OP_FLIPW = 0, 1, 2
EPI_BF16, EPI_F32, EPI_F32_ACC, EPI_SGD, EPI_BF16_DROP = 0, 1, 2, 3, 4
BM = BN = 128
BK = 64


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


@dataclass
class FlipW:
    """Conv weights w [K][R][S][Cg] (bf16) read as the dgrad B operand:
    B_g(n = c, k = tap * Kg + kout) = w[g*Kg + kout][R-1-r][S-1-s][c]  (MC layout)."""
    w: torch.Tensor
    Kg: int
    R: int
    S: int
    Cg: int


FP8 = torch.uint8  # e4m3 bytes (torch.float8_e4m3fn tensors are viewed as uint8)


def _operand(op, fp8: bool = False) -> tuple[_lib.SnOperand, int, int]:
    elt = FP8 if fp8 else torch.bfloat16
    if isinstance(op, FlipW):
        assert op.w.dtype == torch.bfloat16 and op.w.is_contiguous() and op.Cg % 8 == 0
        g = _lib.SnConvGeom(0, 0, 0, op.Kg, 1, 1, op.R, op.S, 1, 1, 0, 0, 1, 1, op.Cg)
        s = _lib.SnOperand(op.w.data_ptr(), 0, op.Kg * op.R * op.S * op.Cg, g)
        return s, 1, OP_FLIPW
    if isinstance(op, Dense):
        assert op.t.dtype == elt, (op.t.dtype, elt)
        assert op.t.data_ptr() % 16 == 0 and (op.ld * op.t.element_size()) % 16 == 0, \
            "dense operand must be 16-B aligned"
        s = _lib.SnOperand(op.t.data_ptr(), op.ld, op.gstride, _lib.SnConvGeom())
        return s, 0 if op.kcontig else 1, OP_DENSE
    g = op.geom
    # contiguous NHWC, or a channel slice of a wider NHWC tensor whose pixel stride is g.C
    assert op.x.dtype == elt and (op.x.is_contiguous() or (
        op.x.dim() == 4 and op.x.stride(-1) == 1 and op.x.stride(2) == g.C and op.x.shape[-1] <= g.C)), \
        "implicit conv operand must be NHWC (contiguous or a channel slice with pixel stride C)"
    cm = 16 if fp8 else 8
    assert g.Cg % cm == 0 and g.C % cm == 0, f"implicit conv needs channels % {cm} == 0"
    # the kernel's fp32-reciprocal index division is exact below 2^24
    assert g.N * g.P * g.Q < (1 << 24) and g.N * g.H * g.W < (1 << 24), "conv too large for one launch"
    assert g.N * g.H * g.W * g.C < (1 << 31), "implicit conv uses 32-bit element offsets"
    assert op.x.data_ptr() % 16 == 0, "implicit conv operand must be 16-B aligned"
    s = _lib.SnOperand(op.x.data_ptr(), 0, op.gstride, g.c_struct())
    return s, 0 if op.kcontig else 1, OP_IM2COL


TILES = {0: (128, 128), 1: (256, 64), 2: (256, 128), 3: (128, 256), 4: (128, 96), 5: (256, 48),
         6: (256, 256), 7: (256, 128), 10: (128, 64),
         11: (256, 256), 12: (256, 128), 13: (256, 128), 14: (256, 192), 15: (128, 192), 16: (192, 128),
         17: (192, 96), 18: (192, 64), 19: (128, 128), 20: (128, 64), 21: (64, 256), 22: (64, 128)}
# (round 6 removed the measured-and-rejected families: the v_mfma 32x32x16 twins 23-28, the
# persistent ring tiles 30-39, the 4- and 8-phase gemm256 schedules 8 / 9 / 40 / 41 —
# docs/PERF_NOTES.md rounds 4-5)
# gemm256_kernel tiles (6, 7) and the 8-wave 2-stage gemm_kernel tiles (11-14) run one
# 512-thread block per CU
_SLOTS = {6: 256, 7: 256, 10: 768, 11: 256, 12: 256, 13: 256, 14: 256, 19: 256, 20: 512, 21: 512, 22: 768}
_KTILE_US = {6: 2.0, 7: 1.1, 11: 2.0, 12: 1.1, 13: 1.1, 14: 1.55}
_FORCE_TILE = int(os.environ.get("SN_GEMM_TILE", "-1"))  # tuning / A-B experiments only


def choose_tile(M: int, N: int, b_kcontig: bool = False) -> int:
    """256x64 for skinny N (<= 64 per group; 256x48 when N is 48: AlexNet conv2's dgrad has
    48 channels per group); 128x96 when N
    is a multiple of 96 that 128-wide tiles would pad by a third (AlexNet conv1's 96
    filters, conv4's 192 per group; K-contiguous B only); else 128x128."""
    if N <= 64 and M >= 256:
        return 5 if N % 48 == 0 and N % 64 != 0 else 1
    if b_kcontig and N % 96 == 0 and N % 128 != 0 and M >= 128:
        return 4
    return 0


SLOTS = 512          # resident blocks: 2 per CU (64 KB of LDS each) x 256 CUs
KTILE_US = 1.25      # measured: one 128x128x64 k-step of one block at full occupancy
BLOCK_OVERHEAD = 4   # prologue + epilogue of a block, in k-steps
REDUCE_BW = 5e12     # split-K slab read+write, bytes/s effective (+ one launch)


def _cost(tiles: int, ktiles: int, s: int, out_elems: int, tile: int = 0) -> float:
    """Modelled microseconds of a GEMM split s ways: whole waves of SLOTS blocks (a wave
    that is 1 % full costs a full block time) plus the slab reduction."""
    kt = -(-ktiles // s)
    t = -(-tiles * s // _SLOTS.get(tile, SLOTS)) * (kt + BLOCK_OVERHEAD) * _KTILE_US.get(tile, KTILE_US)
    if s > 1:
        t += (out_elems * 4.0 * (s + 1)) / REDUCE_BW * 1e6 + 3.0
    return t


def choose_splits(M: int, N: int, K: int, groups: int = 1, tile: int = 0) -> tuple[int, int]:
    """Split-K factor minimising the wave-quantised cost model above: e.g. 54 tiles x 10
    splits = 540 blocks would run a second, nearly empty wave; 9 splits fits in one."""
    bm, bn = TILES[tile]
    tiles = -(-M // bm) * -(-N // bn) * groups
    ktiles = -(-K // BK)
    ws_cap = max(1, (256 << 20) // max(1, 4 * M * N * groups))  # fp32 partial slabs <= 256 MB
    smax = max(1, min(256, ktiles // 4, ws_cap))
    best, best_t = 1, _cost(tiles, ktiles, 1, M * N * groups, tile)
    for s in range(2, smax + 1):
        t = _cost(tiles, ktiles, s, M * N * groups, tile)
        if t < best_t * 0.98:
            best, best_t = s, t
    kchunk = -(-K // best)
    kchunk = -(-kchunk // BK) * BK
    splits = -(-K // kchunk)
    return splits, kchunk


def gemm(M: int, N: int, K: int, A, B, out: torch.Tensor, ldc: int, *, epi: int,
         groups: int = 1, c_gstride: int = 0, bias: torch.Tensor | None = None, relu: bool = False,
         splits: int | None = None, gate: torch.Tensor | None = None,
         deq: tuple[torch.Tensor, torch.Tensor] | None = None,
         bias_grad: torch.Tensor | None = None, bias_acc: bool = True, sgd: dict | None = None,
         dropout: tuple | None = None, gate_scale: float = 1.0) -> None:
    """Run one (possibly grouped, split-K) GEMM.  ``epi``: EPI_BF16 (store bf16 with
    bias/ReLU; ``gate``: a bf16 tensor laid out like ``out`` — outputs where gate <= 0
    are zeroed, i.e. a following slope-0 ReLU's backward), EPI_F32 (store), EPI_F32_ACC
    (accumulate into an fp32 output).

    ``bias_grad`` (fp32 [groups * M], weight-gradient products with an MC B operand and
    N % 8 == 0): also compute sum_k A_g(m, k) — the bias gradient — through a virtual
    ones column N of B, written (``bias_acc``: accumulated) into ``bias_grad[g*M + m]``.

    ``epi=EPI_SGD`` with ``sgd`` = {w, h, shadow, hyper, lr_mult, decay_mult, flags}:
    the product is the gradient of the fp32 master ``w`` (laid out like ``out``), and the
    epilogue applies the solver update to w / h / shadow instead of storing it.

    EPI_BF16 only: ``dropout`` = (rng_state, layer stream id, ratio) applies a Dropout
    forward (Philox keep mask over the output's element index, scaled by 1/(1-ratio))
    after bias / ReLU; ``gate_scale`` multiplies the values a ``gate`` lets through (a
    fused Dropout backward: the gate is the dropout output)."""
    if M == 0 or N == 0:
        return
    sg = (0, 0, 0, 0, 0.0, 0.0, 0)
    if epi == EPI_SGD:
        assert sgd is not None and groups == 1 and deq is None
        splits = 1
        sg = (sgd["w"].data_ptr(), sgd["h"].data_ptr(), sgd["shadow"].data_ptr(), sgd["hyper"].data_ptr(),
              float(sgd["lr_mult"]), float(sgd["decay_mult"]), int(sgd["flags"]))
    # fp8 operands; deq = (1/scale_A, 1/scale_B[, format]) device scalars, format 1 = e4m3 x e4m3
    # (default), 2 = e5m2 A x e4m3 B (SnGemmArgs.fp8)
    fp8 = deq is not None
    sa, a_mc, a_mode = _operand(A, fp8)
    sb, b_mc, b_mode = _operand(B, fp8)
    ones = -1
    if bias_grad is not None:
        assert epi in (EPI_F32, EPI_F32_ACC, EPI_SGD) and b_mc == 1 and b_mode != OP_FLIPW and N % 8 == 0
        assert not fp8 or (a_mc == 1 and N % 16 == 0)  # fp8: the MC weight-gradient products
        assert bias_grad.dtype == torch.float32 and bias_grad.is_contiguous() and bias_grad.numel() == groups * M
        ones, N = N, N + 1
    bk = 128 if fp8 else BK
    if bias is not None:
        assert bias.dtype == torch.float32 and bias.is_contiguous()
    if gate is not None:
        assert epi == EPI_BF16 and gate.dtype == torch.bfloat16
    xtra = (0, 0, 0.0, float(gate_scale))
    if dropout is not None:
        assert epi == EPI_BF16
        rng, dstream, ratio = dropout
        xtra = (rng.data_ptr(), int(dstream), float(ratio), float(gate_scale))
    ops = (sa, a_mc, a_mode, sb, b_mc, b_mode)
    if splits is not None or _FORCE_TILE >= 0:
        if fp8:
            tile = _FORCE_TILE if (_FORCE_TILE in _FP8_TILES and not (a_mc or b_mc)) else 0
        else:
            tile = _FORCE_TILE if _FORCE_TILE >= 0 else choose_tile(M, N, b_mc == 0 and b_mode == OP_DENSE)
        if epi == EPI_SGD and tile not in (0, 1, 2, 3):
            tile = 0
        if splits is None:
            splits, kchunk = choose_splits(M, N, K * BK // bk, groups, tile)
            kchunk = kchunk * bk // BK
        else:
            kchunk = -(-(-(-K // splits)) // bk) * bk
    else:
        tile, splits, kchunk = _tuned_config(M, N, K, groups, ops, epi, out, ldc, c_gstride, bias, relu, gate,
                                             bias_grad, bias_acc, ones, sg, xtra, deq)
    _launch(M, N, K, groups, ops, epi, out, ldc, c_gstride, bias, relu, gate, bias_grad, bias_acc, ones, sg,
            tile, splits, kchunk, deq, xtra)


_NO_XTRA = (0, 0, 0.0, 1.0)
# bf16 epilogues of the 4-wave tiles store through LDS as whole 16-B row chunks
# (SnGemmArgs.lds_store)
_LDS_EPI = True
_LDS_EPI_TILES = frozenset((0, 1, 4, 5, 10, 12, 13, 14, 15, 16, 17, 18, 19, 20))
def _drop_fields(xtra):
    """(drop_rng, drop_stream, drop_thr, drop_scale, gate_scale) of SnGemmArgs."""
    rng, dstream, ratio, gscale = xtra
    if not rng:
        return (0, 0, 0, 1.0, gscale)
    return (rng, dstream, int(4294967295 * ratio) & 0xffffffff, 1.0 / (1.0 - ratio), gscale)


def _launch(M, N, K, groups, ops, epi, out, ldc, c_gstride, bias, relu, gate, bias_grad, bias_acc, ones, sg,
            tile, splits, kchunk, deq=None, xtra=_NO_XTRA):
    """One GEMM launch (+ the split-K reduce) with an explicit tile / split choice."""
    sa, a_mc, a_mode, sb, b_mc, b_mode = ops
    fp8 = deq is not None
    bk = 128 if fp8 else BK
    splits = max(1, -(-K // kchunk))
    dq = (deq[0].data_ptr(), deq[1].data_ptr()) if fp8 else (0, 0)
    f8 = (deq[2] if len(deq) > 2 else 1) if fp8 else 0
    bm, bn = TILES[tile]
    tm_, tn_ = -(-M // bm), -(-N // bn)
    raster = int(1 < tn_ <= 8 and tm_ >= 8 * tn_)
    gp = gate.data_ptr() if gate is not None else 0
    bg = bias_grad.data_ptr() if bias_grad is not None else 0
    if splits == 1:
        e = EPI_BF16_DROP if (epi == EPI_BF16 and xtra[0]) else epi
        lds = int(_LDS_EPI and epi == EPI_BF16 and tile in _LDS_EPI_TILES and ldc % 8 == 0 and c_gstride % 8 == 0
                  and out.data_ptr() % 16 == 0)
        args = _lib.SnGemmArgs(M, N, K, groups, 1, max(kchunk, bk), a_mc, a_mode, b_mc, b_mode, e,
                               sa, sb, out.data_ptr(), ldc, c_gstride, 0,
                               bias.data_ptr() if bias is not None else 0, int(relu), tile, gp, f8, *dq, raster,
                               ones, bg, int(bias_acc), *sg, *_drop_fields(xtra), lds)
        side = _SIDE
        if side is not None and side.covers(out):
            q = _side_fields(side, out, ldc, c_gstride, N, tile, e, lds)
            if q is not None:
                args.q_out, args.q_ld, args.q_gstride, args.q_slot, args.q_e5m2, args.q_part = q
        _lib.check(_lib.kernels().sn_gemm(C.byref(args), C.c_void_p(_lib.stream_ptr())), "gemm")
        if _lib.DEBUG_SYNC:
            _lib.debug_sync("gemm")
        return
    if _SIDE is not None and _SIDE.covers(out):
        _SIDE.ok = False  # the split-K reduce writes the bf16 output
    ldw = -(-N // 4) * 4  # fp32 slabs keep 16-B rows (the ones column makes N odd)
    sink = _DEFER_SINK
    deferred = (sink is not None and epi == EPI_F32 and not fp8 and (bias_grad is None or not bias_acc)
                and sink.accepts(out, bias_grad))
    ws = (sink.slab(groups * splits * M * ldw, out.device).view(groups, splits, M, ldw) if deferred
          else torch.empty((groups, splits, M, ldw), dtype=torch.float32, device=out.device))
    args = _lib.SnGemmArgs(M, N, K, groups, splits, kchunk, a_mc, a_mode, b_mc, b_mode, EPI_F32,
                           sa, sb, ws.data_ptr(), ldw, splits * M * ldw, M * ldw, 0, 0, tile, 0, f8, *dq, raster,
                           ones, 0, 0, *sg, *_drop_fields(_NO_XTRA))
    _lib.check(_lib.kernels().sn_gemm(C.byref(args), C.c_void_p(_lib.stream_ptr())), "gemm")
    if deferred:
        # the solver update sums these slabs itself (engine.fuse_splitk_updates)
        sink.record(dict(ws=ws, splits=splits, M=M, N=N - (1 if ones >= 0 else 0), ldw=ldw, groups=groups,
                         ones=ones, ldc=ldc, c_gstride=c_gstride))
        return
    mode = {EPI_BF16: 0, EPI_F32: 1, EPI_F32_ACC: 2}[epi]
    rng, dstream, ratio, gscale = xtra
    _lib.call("splitk_reduce", ws, splits, M * ldw, M, N, ldw, out, ldc, mode, bias, int(relu),
              groups, splits * M * ldw, c_gstride, gate, bias_grad, ones, int(bias_acc), M,
              C.c_void_p(rng), int(dstream), float(ratio), float(gscale))


# --- fused fp8 side output ----------------------------------------------------------------
# A bf16 GEMM output that the next layer quantises for an fp8 product (its e4m3 input, or
# the e4m3 / e5m2 output gradient of the layer below) can be quantised by the producing
# GEMM's epilogue instead (SnGemmArgs.q_out): every launch under ``fp8_side_output(side)``
# whose output lies inside ``side.base`` also stores its fp8 bytes into ``side.q`` and
# folds the block |max| into the slot.  A launch that cannot (split-K, the 8-wave
# gemm256 tiles, ragged channel counts) marks the side incomplete and the consumer runs
# its own quantisation pass.  The slot must be an initialised delayed-scaling slot.


class Fp8Side:
    def __init__(self, base: torch.Tensor, slot: torch.Tensor, e5m2: bool = False, part: torch.Tensor | None = None):
        assert base.is_contiguous() and base.dtype == torch.bfloat16
        self.base = base
        self.q = torch.empty(base.shape, dtype=torch.uint8, device=base.device)
        self.slot = slot
        self.e5m2 = bool(e5m2)
        self.ok = True
        self.only = False  # the bf16 base was not written: the fp8 bytes are the only copy
        self.launches = 0
        # block |max| partials (zero between uses: the fold kernel clears them); pass a persistent
        # buffer so a captured graph does not re-zero a fresh one every replay
        self.part = part if part is not None else new_side_part(base.device)

    def finish(self) -> None:
        """Fold the launches' block |max| partials into the slot (one 256-thread block)."""
        if self.launches:
            _lib.call("fp8_fold_amax", self.part, self.slot)

    def covers(self, out: torch.Tensor) -> bool:
        b = self.base.data_ptr()
        return out.dtype == torch.bfloat16 and b <= out.data_ptr() < b + 2 * self.base.numel()

    @property
    def complete(self) -> bool:
        return self.ok and self.launches > 0

    def matches(self, x: torch.Tensor) -> bool:
        return self.complete and x.data_ptr() == self.base.data_ptr() and x.numel() == self.base.numel()


def new_side_part(device) -> torch.Tensor:
    return torch.zeros(256 * 32, dtype=torch.float32, device=device)


_SIDE = None
# the per-fragment epilogue stores side outputs too (SN_FEATURES=fp8_side_frag=0: LDS-staged launches only;
# VGG-16 b2048 8.98k / 8.97k with vs 8.96k / 8.94k img/s without, profiles/r3_fp8_dgrad.txt)
_SIDE_FRAG = features.enabled("fp8_side_frag")
SIDE_STATS = {"used": 0, "missed": 0}  # consumer lookups of a side output (tests, probes)


def side_bytes(side, x: torch.Tensor, e5m2: bool = False):
    """The fp8 bytes of ``x`` stored by its producer's epilogue, or None (quantise it)."""
    if side is None:
        return None
    if side.matches(x) and side.e5m2 == bool(e5m2):
        SIDE_STATS["used"] += 1
        return side.q
    SIDE_STATS["missed"] += 1
    return None


@contextlib.contextmanager
def fp8_side_output(side):
    global _SIDE
    prev, _SIDE = _SIDE, side
    try:
        yield side
    finally:
        _SIDE = prev
    side.finish()


def _side_fields(side, out, ldc, c_gstride, N, tile, epi, lds):
    """(q_out, q_ld, q_gstride, q_slot, q_e5m2) of one unsplit launch, or None when this
    launch cannot store the side output (the side is then marked incomplete)."""
    off = (out.data_ptr() - side.base.data_ptr()) // 2
    qp = side.q.data_ptr() + off
    if ((not lds and not _SIDE_FRAG) or epi not in (EPI_BF16, EPI_BF16_DROP) or tile in (6, 7)
            or N % 8 or ldc % 8
            or c_gstride % 8 or qp % 8):
        side.ok = False
        return None
    side.launches += 1
    return (qp, ldc, c_gstride, side.slot.data_ptr(), int(side.e5m2), side.part.data_ptr())


# --- deferred split-K reduction ---------------------------------------------------------
# A weight-gradient product run under ``defer_reduce(sink)`` (a single, overwriting
# contribution to a parameter's gradient) leaves its fp32 split-K slabs in a persistent
# buffer owned by ``sink`` instead of reducing them into the gradient; the solver's update
# kernel then sums the slabs in split order itself (engine.fuse_splitk_updates).  A
# product that is not split (or accumulates) runs normally and the sink records None.
_DEFER_SINK = None


class defer_reduce:
    def __init__(self, sink):
        self.sink = sink

    def __enter__(self):
        global _DEFER_SINK
        self.prev, _DEFER_SINK = _DEFER_SINK, self.sink
        self.sink.begin()
        return self.sink

    def __exit__(self, *exc):
        global _DEFER_SINK
        _DEFER_SINK = self.prev
        self.sink.end()
        return False


# --- per-shape autotuning ----------------------------------------------------------------
# The cost model picks a tile and split-K factor from the shape alone; the first eager
# call of every distinct GEMM (shape, operand kinds and geometry, epilogue) instead times
# the candidate tiles x split factors on scratch outputs and caches the fastest.  Graph
# captures replay the cached choice.
# OFF by default (SN_GEMM_AUTOTUNE=1 turns it on, e.g. to build the database): first-call
# timing is noisy, so two processes on one box could pick different tiles for one product
# and train on different summation orders (profiles/r5_fp8_fidelity_lr.txt), and N ranks
# tuning independently would each replay their own kernels (the slowest sets the job's
# rate).  The production path is the committed database plus the cost model for anything
# it lacks (recorded in _MISSES; tests/test_tune_db_gpu.py keeps the zoo models covered),
# and a tuned run with N > 1 ranks adopts rank 0's choices before capture (sync_tuned).
_AUTOTUNE = os.environ.get("SN_GEMM_AUTOTUNE", "0") == "1"
_TUNED: dict = {}
_MISSES: set = set()  # database misses served by the cost model (keys)
_TUNE_LOG = os.environ.get("SN_GEMM_TUNE_LOG", "0") == "1"
_TUNE_PASSES = 3
# The 64-row tiles (21, 22) are autotune candidates for products with M <= 64, or whose M they
# pad less than 128-row tiles do.
# Round 4 made the tiles opt-in after cifar10_quick stopped learning when its conv1 weight
# gradient (M 32, N 201 with the bias column, K 102400) picked tile 22 at 229-way split-K.
# Root cause (round 5, docs/PERF_NOTES.md "thin tiles"): not the tile.  Tiles 0, 10, 21 and 22
# give bitwise-identical products at equal split-K (tests/test_gemm_gpu.py::
# test_thin_tiles_bitwise_equal_at_same_split); the same failure reproduces with tile 0 or 10
# at 229 splits, and the fp32 CPU engine spikes too: at the reference solver's lr 0.001 that
# synthetic-pattern training is unstable under ANY summation order (tests/test_training_gpu.py).
_THIN = True
# Tuning database: choices measured offline on an MI355X (scripts/build_tune_db.sh, many
# more timing passes than a first-call tune) are loaded at import so the production
# models run a fixed, reproducible tile / split-K per GEMM; first-call timing only fills
# in products the database does not cover.  SN_GEMM_TUNE_DB=0 disables it, a path
# overrides the packaged file.
_DB_PATH = os.environ.get("SN_GEMM_TUNE_DB", os.path.join(os.path.dirname(os.path.abspath(__file__)),
                                                          "gemm_tuned.json"))


def _key_to_str(key) -> str:
    return repr(key[:-1] + (str(key[-1]).replace("torch.", ""),))


def _key_from_str(s: str):
    k = ast.literal_eval(s)
    return k[:-1] + (getattr(torch, k[-1]),)


def load_tune_db(path: str | None = None) -> int:
    """Merge a tuning database (JSON {key: [tile, splits, kchunk]}) into the cache."""
    path = path or _DB_PATH
    if not path or path == "0" or not os.path.exists(path):
        return 0
    with open(path) as f:
        db = json.load(f)
    for k, v in db.items():
        _TUNED[_key_from_str(k)] = tuple(int(x) for x in v)
    return len(db)


def save_tune_db(path: str) -> int:
    """Write every cached choice (database entries and first-call tunes) to ``path``,
    merged over what the file already holds."""
    db = {}
    if os.path.exists(path):
        with open(path) as f:
            db = json.load(f)
    db.update({_key_to_str(k): list(v) for k, v in _TUNED.items()})
    with open(path, "w") as f:
        json.dump(dict(sorted(db.items())), f, indent=0)
    return len(db)


load_tune_db()


def _geom_key(s) -> tuple:
    return (s.ld, s.gstride) + tuple(getattr(s.g, f) for f, _ in s.g._fields_)


def _candidates(M, N, K, groups, b_kc_dense, epi):
    tiles = [0, 1, 2]
    if N >= 256:
        tiles.append(3)
    if epi != EPI_SGD and M >= 256:
        tiles.append(7)
        if N > 128:
            tiles.append(6)
    if epi != EPI_SGD and M >= 256 and N > 64:
        tiles += [12, 13]
        if N > 128:
            tiles.append(11)
        if N > 128 and (b_kc_dense or N % 192 == 0):
            tiles.append(14)
    if epi != EPI_SGD and N > 64:
        tiles.append(16)
        if b_kc_dense and N > 128:
            tiles.append(15)
    if epi != EPI_SGD and M >= 192:
        tiles.append(18)
        if b_kc_dense and N % 96 == 0:
            tiles.append(17)
    if epi != EPI_SGD and N >= 64:
        tiles.append(20)  # 3-stage 128x64: dense NT / NN (InnerProduct fwd / dgrad), MC x MC (weight gradients)
    if _THIN and (M <= 64 or -(-M // 64) * 64 < -(-M // 128) * 128):
        # 64-row tiles: thin weight gradients (64-channel convs, Inception reduce layers), and
        # any M that 64-row tiles pad less than 128-row ones (M = 192: 3 x 64 rows instead of
        # 2 x 128, a quarter of every MFMA idle — AlexNet conv4's grouped weight gradient,
        # GoogLeNet's 192-, 160-, 320-channel convs)
        tiles += [21, 22]
    if epi != EPI_SGD:
        tiles.append(10)
        if b_kc_dense and N % 96 == 0:
            tiles.append(4)
        if N % 48 == 0 and N <= 96 and M >= 256:
            tiles.append(5)
    out = []
    for t in tiles:
        s, kc = choose_splits(M, N, K, groups, t)
        out.append((t, s, kc))
        if epi == EPI_SGD:
            continue
        for s2 in {1, 2 * s} - {s}:
            kc2 = -(-(-(-K // s2)) // BK) * BK
            s2 = max(1, -(-K // kc2))
            if s2 * M * N * groups * 4 <= (256 << 20):
                out.append((t, s2, kc2))
    return list(dict.fromkeys(out))


# e4m3 forward products: the 128x128 tile (gemm.hip launch_fp8) and the large tiles of
# gemm_fp8big.hip (bf16 / fp32 epilogues; the fused-dropout epilogue only on 128x128)
_FP8_TILES = (0, 11, 16)


def _candidates_fp8(M, N, K, groups, epi, xtra, mc=False):
    out = []
    for t in ((0,) if mc else _FP8_TILES):  # fp8 MC operands (weight gradients): 128x128 only
        if t != 0 and (xtra[0] or epi not in (EPI_BF16, EPI_F32)):
            continue
        s, kc = choose_splits(M, N, K // 2, groups, t)
        for s2 in dict.fromkeys((s, 1)):
            kc2 = -(-(-(-K // s2)) // 128) * 128
            s2 = max(1, -(-K // kc2))
            if s2 == 1 or s2 * M * N * groups * 4 <= (256 << 20):  # fp32 slabs only when split
                out.append((t, s2, kc2))
    return list(dict.fromkeys(out))


def _tuned_config(M, N, K, groups, ops, epi, out, ldc, c_gstride, bias, relu, gate, bias_grad, bias_acc,
                  ones, sg, xtra=_NO_XTRA, deq=None):
    # (split-K caps were measured neutral or slower, docs/PERF_NOTES.md round 2; removed)
    return _tuned_config_raw(M, N, K, groups, ops, epi, out, ldc, c_gstride, bias, relu, gate, bias_grad,
                             bias_acc, ones, sg, xtra, deq)


def _tuned_config_raw(M, N, K, groups, ops, epi, out, ldc, c_gstride, bias, relu, gate, bias_grad, bias_acc,
                      ones, sg, xtra=_NO_XTRA, deq=None):
    sa, a_mc, a_mode, sb, b_mc, b_mode = ops
    b_kc_dense = b_mc == 0 and b_mode == OP_DENSE
    fp8 = deq is not None
    key = (M, N, K, groups, a_mc, a_mode, b_mc, b_mode, epi, gate is not None, bias_grad is not None, bool(xtra[0]),
           _geom_key(sa), _geom_key(sb)) + ((("fp8",) if len(deq) < 3 or deq[2] == 1 else ("fp8", deq[2])) if fp8 else ()) + (out.dtype,)
    hit = _TUNED.get(key)
    if hit is None and not _AUTOTUNE and epi != EPI_SGD:
        _MISSES.add(key)
    if hit is not None:
        return hit
    tile = 0 if fp8 else choose_tile(M, N, b_kc_dense)
    if epi == EPI_SGD and tile not in (0, 1, 2, 3):
        tile = 0
    if fp8:  # K counts e4m3 elements, 128 per K-step; the cost model counts bf16 K-steps
        splits, kchunk = choose_splits(M, N, K // 2, groups, tile)
        kchunk *= 2
        splits = -(-K // kchunk)
    else:
        splits, kchunk = choose_splits(M, N, K, groups, tile)
    default = (tile, splits, kchunk)
    extent = (groups - 1) * c_gstride + (M - 1) * ldc + (N - (1 if ones >= 0 else 0))
    if (not _AUTOTUNE or epi == EPI_SGD or not out.is_cuda or torch.cuda.is_current_stream_capturing()
            or (out.is_contiguous() and extent > out.numel())):
        return default
    # a strided output (a channel slice of a zero-copy concat) is timed on a flat scratch
    scratch = torch.empty_like(out) if out.is_contiguous() else torch.empty(extent, dtype=out.dtype, device=out.device)
    bscratch = torch.zeros_like(bias_grad) if bias_grad is not None else None
    runs = []
    cands = (_candidates_fp8(M, N, K, groups, epi, xtra, bool(a_mc or b_mc)) if fp8
             else _candidates(M, N, K, groups, b_kc_dense, epi))
    for cand in cands:
        t, s, kc = cand

        def run(t=t, s=s, kc=kc):
            _launch(M, N, K, groups, ops, epi, scratch, ldc, c_gstride, bias, relu, gate, bscratch, bias_acc,
                    ones, sg, t, s, kc, deq, xtra)
        try:
            run()
        except RuntimeError as e:  # a tile this operand combination has no instance for
            if _TUNE_LOG:
                print(f"[gemm-tune] candidate {cand} skipped: {e}", flush=True)
            continue
        runs.append((cand, run))
    # Each candidate is timed over 4 back-to-back launches queued behind a GPU spin (so small
    # GEMMs are timed as a graph replays them, not at the host's launch rate), in 3
    # interleaved passes; the minimum per candidate counts.  A candidate must beat the cost
    # model's pick by 3% to replace it, so timing noise cannot flip a choice.
    times = {c: float("inf") for c, _ in runs}
    # Drain every stream of the device first: inside a warm-up step with branch streams the
    # other towers' kernels would otherwise share the CUs with the candidates being timed —
    # GoogLeNet's database held choices up to 1.6x off the isolated best that way
    # (profiles/r5_retune_isolated_googlenet.txt).
    torch.cuda.synchronize(out.device)
    # enough back-to-back launches per timed window that it spans >= ~150 us
    est = _cost(-(-M // TILES[tile][0]) * -(-N // TILES[tile][1]) * groups, -(-K // BK), splits, M * N * groups, tile)
    reps = max(4, min(32, int(150.0 / max(est, 1.0))))
    for _ in range(_TUNE_PASSES):
        for cand, run in runs:
            torch.cuda._sleep(1 << 19)
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record()
            for _ in range(reps):
                run()
            e1.record()
            e1.synchronize()
            times[cand] = min(times[cand], e0.elapsed_time(e1))
    best = min(times, key=times.get) if times else default
    if default in times and times[best] > 0.97 * times[default]:
        best = default
    if _TUNE_LOG:
        print(f"[gemm-tune] M={M} N={N} K={K} g={groups} modes={ops[1:3]}/{ops[4:]} epi={epi} "
              f"default={default} best={best} " +
              " ".join(f"{c[0]}/{c[1]}:{v * 1000 / reps:.1f}" for c, v in sorted(times.items())), flush=True)
    _TUNED[key] = best
    return best


def set_autotune(on: bool) -> None:
    """Enable / disable first-call timing of products the database does not cover."""
    global _AUTOTUNE
    _AUTOTUNE = bool(on)


def tune_misses() -> list:
    """Products (database keys) this process ran on the cost model's choice because the
    tuning database has no entry for them (autotune off)."""
    return sorted(_MISSES, key=repr)


def sync_tuned(comm) -> int:
    """Adopt rank 0's tile / split-K choices on every rank (a tuned run at N > 1: each rank's
    first-call timings differ, so without this the ranks would capture different kernels for
    one product).  Call after the eager warm-up iterations and before graph capture.
    Returns the number of entries rank 0 sent."""
    import torch.distributed as dist
    if (comm is None or not getattr(comm, "active", False) or comm.world_size <= 1
            or not (dist.is_available() and dist.is_initialized())):
        return 0  # (a stand-in communicator without a process group: nothing to agree with)
    payload = [{_key_to_str(k): list(v) for k, v in _TUNED.items()} if comm.rank == 0 else None]
    dist.broadcast_object_list(payload, src=0)
    for ks, v in payload[0].items():
        _TUNED[_key_from_str(ks)] = tuple(v)
    return len(payload[0])


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
               relu: bool = False, out: torch.Tensor | None = None, dropout: tuple | None = None) -> torch.Tensor:
    """y[M,N] = x[M,K] @ w[N,K]^T (+bias, ReLU, fused Dropout forward) in bf16."""
    M, K = x.shape
    N = w.shape[0]
    xp, wp = _pad8(x, 1), _pad8(w, 1)
    Kp = xp.shape[1]
    if out is None:
        out = torch.empty((M, N), dtype=torch.bfloat16, device=x.device)
    if dropout is not None:
        assert out.is_contiguous()  # the mask is drawn over the blob's element index
    gemm(M, N, Kp, Dense(xp, Kp, True), Dense(wp, Kp, True), out, out.stride(0), epi=EPI_BF16,
         bias=bias, relu=relu, dropout=dropout)
    return out


def linear_dgrad(dy: torch.Tensor, w: torch.Tensor, out: torch.Tensor | None = None,
                 gate: torch.Tensor | None = None, gate_scale: float = 1.0) -> torch.Tensor:
    """dx[M,K] = dy[M,N] @ w[N,K] in bf16 (B operand read transposed from LDS);
    ``gate`` [M,K]: zero dx where gate <= 0 (fused ReLU backward)."""
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
    if gate is not None and (Kp != K or not gate.is_contiguous()):
        gemm(M, Kp, Np, Dense(dyp, Np, True), Dense(wp, Kp, False), o, o.stride(0), epi=EPI_BF16)
        o = o[:, :K] * (gate > 0).to(o.dtype) * gate_scale
        if out is not None:
            out.copy_(o)
            return out
        return o
    gemm(M, Kp, Np, Dense(dyp, Np, True), Dense(wp, Kp, False), o, o.stride(0), epi=EPI_BF16, gate=gate,
         gate_scale=gate_scale)
    if o is not out:
        o = o[:, :K]
        if out is not None:
            out.copy_(o)
            return out
    return o


def linear_wgrad(dy: torch.Tensor, x: torch.Tensor, dw: torch.Tensor, accumulate: bool = True,
                 db: torch.Tensor | None = None, db_acc: bool = True) -> bool:
    """dw[N,K] (+)= dy[M,N]^T @ x[M,K], fp32 output; both operands read along M.  With
    ``db`` the bias gradient db[N] (+)= sum_m dy[m, :] comes out of the same GEMM when the
    shapes allow it; returns whether db was written."""
    M, N = dy.shape
    K = x.shape[1]
    dyp, xp = _pad8(dy, 1), _pad8(x, 1)
    Np, Kp = dyp.shape[1], xp.shape[1]
    if Np == N and Kp == K and dw.is_contiguous():
        fuse = db is not None and db.is_contiguous() and db.dtype == torch.float32
        gemm(N, K, M, Dense(dyp, Np, False), Dense(xp, Kp, False), dw, K,
             epi=EPI_F32_ACC if accumulate else EPI_F32, bias_grad=db if fuse else None, bias_acc=db_acc)
        return fuse
    tmp = torch.zeros((Np, Kp), dtype=torch.float32, device=dw.device)
    gemm(Np, Kp, M, Dense(dyp, Np, False), Dense(xp, Kp, False), tmp, Kp, epi=EPI_F32)
    if accumulate:
        dw.add_(tmp[:N, :K])
    else:
        dw.copy_(tmp[:N, :K])
    return False


def linear_wgrad_sgd(dy: torch.Tensor, x: torch.Tensor, sgd: dict, db: torch.Tensor | None = None,
                     db_acc: bool = True) -> bool:
    """The InnerProduct weight gradient dy^T @ x consumed in the GEMM epilogue by the
    solver update of sgd["w"] / ["h"] / ["shadow"] (EPI_SGD; the gradient is never
    stored).  Needs N, K % 8 == 0.  Returns whether db (the bias gradient) was written."""
    M, N = dy.shape
    K = x.shape[1]
    assert N % 8 == 0 and K % 8 == 0 and dy.is_contiguous() and x.is_contiguous()
    fuse = db is not None and db.is_contiguous() and db.dtype == torch.float32
    w = sgd["w"]
    gemm(N, K, M, Dense(dy, N, False), Dense(x, K, False), w, K, epi=EPI_SGD, sgd=sgd,
         bias_grad=db if fuse else None, bias_acc=db_acc)
    return fuse


def colsum(x: torch.Tensor, out: torch.Tensor, accumulate: bool = True) -> None:
    """out[N] (+)= sum over rows of a bf16 [M, N] matrix (bias gradient)."""
    M, N = x.shape
    c8 = -(-N // 8)
    cl = 1
    while cl < c8 and cl < 64:
        cl *= 2
    cblocks = -(-c8 // cl)
    rl = 256 // cl
    # ~1024 blocks in pass 1, at least two rows per row lane
    nparts = max(1, min(max(1, 1024 // cblocks), -(-M // (2 * rl))))
    part = torch.empty((nparts, N), dtype=torch.float32, device=x.device)
    _lib.call("colsum_bf16", x, M, N, x.stride(0), part, nparts, out, int(accumulate))
