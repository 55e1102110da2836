// Implementation of the MFMA GEMM engine shared by the gemm*.hip translation units
// (kernels, operand stagers, epilogues and templated launchers).  Split over several
// TUs only so the hundreds of tile x operand x epilogue instantiations compile in
// parallel; see gemm.hip for the design notes and the sn_gemm dispatcher.
#pragma once
#include "common.h"

#include <type_traits>

namespace {

constexpr int BK = 64, NTHR = 256;

// OP_FLIPW (MC only): the dgrad B operand read straight from conv weights W[K][R][S][Cg]:
// row k = tap * Kg + kout, col = c  ->  W[g*Kg + kout][R-1-r][S-1-s][c]  (flipped taps,
// transposed channels) with geometry fields R, S, Cg and C := Kg — no flip pass over W.
enum { OP_DENSE = 0, OP_IM2COL = 1, OP_FLIPW = 2 };
enum { EPI_BF16 = 0, EPI_F32 = 1, EPI_F32_ACC = 2, EPI_SGD = 3, EPI_BF16_DROP = 4 };
// EPI_BF16_DROP: EPI_BF16 + the fused Dropout forward (its own instantiations, so the
// Philox code does not weigh on every bf16 epilogue)
template <int EPI>
constexpr bool epi_bf16() { return EPI == EPI_BF16 || EPI == EPI_BF16_DROP; }

}  // namespace

extern "C" {

struct SnConvGeom {
  int N, H, W, C;  // input tensor (NHWC); C = channel stride of a pixel
  int P, Q;        // output spatial
  int R, S;        // kernel
  int sh, sw, ph, pw, dh, dw;
  int Cg;          // channels per group (multiple of 8)
};

struct SnOperand {
  const bf16_t* ptr;
  long long ld;       // row stride (elements) for DENSE
  long long gstride;  // per-group offset: elements (DENSE) / channels (IM2COL)
  SnConvGeom g;
};

struct SnGemmArgs {
  int M, N, K;
  int groups, splits, kchunk;  // kchunk: reduction length per split (multiple of 64)
  int a_mc, a_mode, b_mc, b_mode, epi;
  SnOperand A, B;
  void* C;
  long long ldc, c_gstride, c_split_stride;
  const float* bias;  // per output column n (offset by g*N), EPI_BF16 only
  int relu;
  int tile;           // 0: 128x128, 1: 256x64, 4: 128x96, 5: 256x48 (4 waves, 2 stages); 2: 256x128, 3: 128x256 (8 waves, 3 stages);
                      // 6: 256x256, 7: 256x128 (gemm256_kernel: 8 waves, half-tile phased pipeline);
                      // 10: 128x64 (4 waves, 3 blocks / CU); 11: 256x256, 12 / 13: 256x128, 14: 256x192
                      // (gemm_kernel, 8 waves, 2 stages, one block per CU)
  const bf16_t* gate; // EPI_BF16: zero outputs where gate (same layout as C) <= 0 (fused ReLU backward)
  int fp8;            // operands are fp8 bytes (K-contiguous only; k counts fp8 elements): 1 = e4m3 x e4m3,
                      // 2 = A e5m2 (bf8: output gradients of the fp8 data-gradient products) x B e4m3
  const float* deq_a; // fp8: dequantisation factors (1 / quantisation scale) of A and B, device scalars
  const float* deq_b;
  int raster_n;       // N-fastest tile order (see gemm_kernel)
  // Bias gradient folded into a weight-gradient product (MC B operand only): B column
  // `ones_col` is a virtual column of ones (for every reduction row < K), so output column
  // ones_col of C is sum_k A(m, k) = the bias gradient of output channel m.  With
  // bias_out set (unsplit launch) that column goes to bias_out[grp * M + m] (+= when
  // bias_acc) instead of C; split-K launches keep it in the fp32 slabs for the reduce.
  int ones_col;       // -1: none
  float* bias_out;
  int bias_acc;
  // EPI_SGD (InnerProduct weight gradient, unsplit TN product): instead of storing the
  // gradient, apply the solver update to it in the epilogue — Caffe's ComputeUpdateValue
  // + Blob::Update (sgd_solver.cpp:207-239, nesterov_solver.cpp:8-69) on the fp32 master
  // w[m*ldc + n], history h, and the bf16 compute shadow; hyper-parameters are read from
  // the solver's device tensor (same layout as solver.hip).  sgd_flags: 1 Nesterov, 2 L1.
  float* sgd_w;
  float* sgd_h;
  bf16_t* sgd_shadow;
  const float* sgd_hyper;
  float sgd_lr_mult, sgd_decay_mult;
  int sgd_flags;
  // EPI_BF16 extras: fused Dropout forward (Philox keep mask of element index
  // grp * c_gstride + m * ldc + n — the same mask dropout_kernel draws for that blob, so the
  // standalone backward could regenerate it) applied after bias / ReLU, and a scale on the
  // gated values (a fused Dropout backward: gate = the dropout output, > 0 exactly where
  // the ReLU passed and the element was kept, times 1 / (1 - ratio)).
  const long long* drop_rng;  // null: no dropout
  int drop_stream;
  unsigned drop_thr;
  float drop_scale;
  float gate_scale;
  // bf16 epilogues of unsplit 4-wave tiles: stage the finished tile through the idle LDS
  // stages and store it as whole 16-B row chunks (host: ldc % 8 == 0, 16-B aligned C)
  int lds_store;
  // bf16 epilogues of gemm_kernel, unsplit: also store the finished (bf16-rounded) output as
  // fp8 bytes q_out[grp * q_gstride + m * q_ld + n] = sat(v * q_slot[0]) and fold its |max|
  // into q_slot[1] — the quantisation pass of the fp8 product that consumes this output
  // (the next conv's e4m3 input, or the next lower conv's output gradient) fused into its
  // producer (engine.fuse_fp8_quant).  q_slot is an initialised delayed-scaling slot
  // (csrc/kernels/fp8.hip), so the bytes equal what the separate pass would write.
  unsigned char* q_out;
  long long q_ld, q_gstride;
  float* q_slot;
  int q_e5m2;
  // block |max| partials: one atomicMax per block on q_part[(block & 255) * 32] (128-B apart;
  // a single address serialises ~10^5 block atomics), folded into q_slot[1] afterwards by
  // sn_fp8_fold_amax
  float* q_part;
};

}  // extern "C"

namespace {

// a * b + c on the full-rate 24-bit multiplier (a, b < 2^24; the low 32 bits of the sum).
// Inline asm: the compiler otherwise forms quarter-rate v_mad_u64_u32 from __umul24 + add.
SN_DEV unsigned mad24(unsigned a, unsigned b, unsigned c) {
  unsigned d;
  asm("v_mad_u32_u24 %0, %1, %2, %3" : "=v"(d) : "v"(a), "v"(b), "v"(c));
  return d;
}

// KC tile: [TILE rows][64 k] bf16, 128-B rows, 16-B chunk index XOR (row>>1)&7.
SN_DEV int kc_off(int row, int kc) { return row * 128 + ((kc ^ ((row >> 1) & 7)) << 4); }

// MC tile: [64 k rows][TILE cols] bf16 (TILE*2-byte rows).  32-B granules XOR-swizzled
// so the 8 rows a half-wave tr-reads land in 8 distinct granules of the 256-B bank row.
template <int TILE>
SN_DEV int swz_mc(int k) {
  if (TILE >= 128) return (((k & 3) | (((k >> 3) & 1) << 2)) << 5);
  return ((((k >> 1) & 1) | (((k >> 3) & 1) << 1)) << 5);  // 128-B rows: 2 rows per bank row
}
template <int TILE>
SN_DEV int mc_off(int k, int mc) { return k * (TILE * 2) + ((mc << 4) ^ swz_mc<TILE>(k)); }

// fp8 MC tile: [128 k rows][128 cols] bytes (128-B rows).  16-B chunk index XOR f(k) so the
// 16 rows {8r+q, 32+8r+q} a 32-lane half reads with ds_read_b64_tr_b8 (read_frag8_mc)
// cover all 64 banks once: f(k) = ((k >> 1) & 3) | (((k >> 5) & 1) << 2).
SN_DEV int swz_mc8(int k) { return ((k >> 1) & 3) | (((k >> 5) & 1) << 2); }

// Zero source for LDS-DMA lanes that fall outside the matrix (padding, ragged edges), and
// the ones page of the bias-gradient column (bf16 1.0 then seven zeros).
__device__ __attribute__((aligned(16))) uint4 g_zero16[1];
__device__ __attribute__((aligned(16))) uint32_t g_one16[4] = {0x3F80u, 0u, 0u, 0u};
// the same for fp8 operands: e4m3 1.0 (0x38) then fifteen zero bytes
__device__ __attribute__((aligned(16))) uint32_t g_one16_f8[4] = {0x38u, 0u, 0u, 0u};

typedef __attribute__((address_space(3))) void lds_void;
typedef int i32x4 __attribute__((ext_vector_type(4)));

// Global->LDS staging of one operand tile with global_load_lds_dwordx4 (LDS-DMA, no VGPR
// round trip and no ds_write pass).  One wave-instruction writes 1 KB of LDS linearly
// (lane l -> byte 16 l), so the XOR swizzle of the LDS image is applied on the SOURCE
// side: lane l of instruction j of wave w fills LDS row r = (w*NI + j)*RPI + l/CPL at
// physical 16-B slot l%CPL, and therefore fetches the LOGICAL chunk that the swizzle
// maps to that slot.  Lanes outside the matrix read a zero page.
//   KC: [TILE rows][64 k], 8 chunks per row, 8 rows per instruction.
//   MC: [64 k rows][TILE cols], TILE/8 chunks per row.
template <int MC, int MODE, int TILE, int NW, int ES = 2>
struct GStager {
  static constexpr int NI = TILE / (8 * NW);      // wave-instructions per wave per tile
  static constexpr int CPL = MC ? TILE * ES / 16 : 8;  // 16-B chunks per LDS row
  static constexpr int RPI = 64 / CPL;            // LDS rows per wave-instruction
  static constexpr int EPC = 16 / ES;             // elements per 16-B chunk (8 bf16, 16 fp8)
  static constexpr int BKE = 128 / ES;            // reduction elements per K-step (64 bf16, 128 fp8)
  static_assert(NI >= 1 && NI * 8 * NW == TILE, "whole wave-instructions per tile");
  // KC im2col: the chunk pattern of instruction j repeats with period 2 in j (row parity of
  // (wave * NI + j) differs between j and j' iff j - j' is odd), so instructions 0 and 1
  // describe all of them — for any NI >= 2, odd NI included
  static_assert(MC || MODE != OP_IM2COL || NI >= 2, "KC im2col: at least two instructions per wave");
  static_assert(ES == 2 || !MC || (TILE == 128 && MODE != OP_FLIPW), "fp8 MC images: 128 x 128-B rows");
  static_assert(!MC || RPI * CPL == 64, "MC images: whole rows per wave-instruction");
  const char* base;  // element offsets below are scaled by ES
  long long ld;
  SnConvGeom g;
  int coff;
  int ones_col;  // MC operands: column index of the virtual ones column (-1: none)
  int rr[NI];  // tile-relative LDS row of this lane in instruction j
  int ch[NI];  // logical 16-B chunk this lane fetches in instruction j
  int rowoff[NI], ph[NI], pw[NI];  // KC+IM2COL: pixel decode (rows fixed across k); rowoff =
  bool pv[NI];                     // element offset of the (h=ph, w=pw) corner, may be < 0
  int cr[NI], cs[NI], cc[NI];  // MC+IM2COL: column decode (cols fixed across k)
  bool cv[NI], co[NI];         //   column valid / column is the ones column
  float invPQ, invQ, invCg, invS, invKg;
  // KC+IM2COL: (tap row, tap col, channel) of the NEXT tile to issue — tiles are issued in
  // order, so the decode advances by one K-step per issue (wave-uniform, scalar) instead
  // of dividing k_tile by Cg and S every time; and a raw buffer resource over the input
  // tensor, so the DMA takes a 32-bit byte offset and a lane outside the image reads
  // offset 0xffffffff, which the buffer range check turns into zeros (no zero-page select,
  // no 64-bit address arithmetic per lane).
  int nr, ns, nc;
  i32x4 rsrc;
  // MC+IM2COL (weight gradients: rows = output pixels, the reduction): every lane keeps, per
  // instruction j, the state of ITS pixel row for the NEXT tile to issue — hc / wc = the input
  // row / column its tap reads (p*sh - ph + r*dh, q*sw - pw + s*dw) and mofs = the byte offset
  // of its 16-B source chunk — and advances it by BKE pixels per issue with at most one carry
  // into p and one into n (BKE % (P*Q) < P*Q): ~14 full-rate VALU per instruction, where the
  // former per-instruction (n, p, q) walk ran divergent carry loops and quarter-rate
  // 64-bit multiply-adds (~28 VALU cycles per MFMA on the 128x128 tile, more than the
  // MFMA's free issue slots: the implicit weight gradient ran 1.4-1.75x the dense product
  // of an explicit im2col matrix, scripts/wgrad_probe.py, profiles/r6_wgrad_stager.txt).
  // A column outside the matrix gets hc = -2^29: never inside the image, never carries.
  static constexpr int NJ = (MC && MODE == OP_IM2COL) ? NI : 1;
  int cdh[NJ], cdw[NJ], colo[NJ];  // the column's tap shift and source offset (init only)
  int hc[NJ], wc[NJ], hlim[NJ], wlim[NJ];
  unsigned mofs[NJ];
  int s_dq, s_qsw, s_dp, s_sh, s_psh;  // per-issue advance (scalars)
  unsigned s_d0, s_d1, s_d2;           // byte offset advance: none / q carry / p carry
  bool wave_has_one;  // a ones-column lane in this wave: stage through global loads
  // Low-VALU address paths (all decisions wave-uniform, taken once at init):
  //  KC+IM2COL: kcmode 1 = every K-step lies inside ONE filter tap (Cg % (8*EPC) == 0), so
  //   the tap offset and its (dh, dw) shift are scalars and a lane's DMA offset is
  //   rowb[j] + scalar with a two-compare bounds test; kcmode 2 = a K-step straddles at
  //   most one tap boundary (Cg >= 8*EPC), resolved by one per-lane select per chunk
  //   parity; kcmode 0 = the general per-lane decode.  rowb[j] = byte offset of the
  //   lane's pixel corner + its chunk (pixels past the matrix get ph = -2^28: never valid).
  //  DENSE (KC and MC): fast = the operand spans < 2^31 bytes, so each lane keeps a fixed
  //   32-bit voffset (its row / column and chunk, or 0x80000000 when outside the matrix)
  //   and the K advance is the instruction's scalar soffset: no VALU per DMA outside the
  //   K tail.
  int kcmode;
  bool fast;
  unsigned rowb[NI];  // modular byte arithmetic: operands up to 4 GB (the resource's range)
  int kch[NI], voff[NI];
  // kcmode 1: the lane's valid filter taps, bit r (h = ph + r*dh inside the image) and bit
  // 16 + s (w = pw + s*dw inside), 0 for rows past the matrix: a DMA is valid iff both bits
  // of its tap are set — one v_and + v_cmp instead of two adds and two range compares
  unsigned vrs[NI];

  SN_DEV void init(const SnOperand& op, int grp, int wave, int lane, int tile_row0, int rows_lim,
                   int tile_col0, int cols_lim, int ones = -1, int k_start = 0, int k_lim_hint = 0) {
    ld = op.ld;
    g = op.g;
    ones_col = ones;
    if (MODE == OP_IM2COL) {
      const unsigned long long a = reinterpret_cast<unsigned long long>(op.ptr);
      const unsigned nbytes = (unsigned)((unsigned long long)g.N * g.H * g.W * g.C * ES);
      rsrc[0] = __builtin_amdgcn_readfirstlane((int)(unsigned)a);
      rsrc[1] = __builtin_amdgcn_readfirstlane((int)((a >> 32) & 0xffffu));
      rsrc[2] = __builtin_amdgcn_readfirstlane((int)nbytes);
      rsrc[3] = 0x00020000;
    }
    if (MODE == OP_IM2COL && !MC) {
      const int tap = k_start / g.Cg;
      nc = k_start - tap * g.Cg;
      nr = tap / g.S;
      ns = tap - nr * g.S;
    }
    if (MODE != OP_IM2COL) {
      base = reinterpret_cast<const char*>(op.ptr) + (long long)grp * op.gstride * ES;
      coff = 0;
    } else {
      base = reinterpret_cast<const char*>(op.ptr);
      coff = (int)(grp * op.gstride);
    }
    invKg = MODE == OP_FLIPW ? 1.f / (float)g.C : 0.f;
    invPQ = 1.f / (float)(g.P * g.Q);
    invQ = 1.f / (float)g.Q;
    invCg = 1.f / (float)g.Cg;
    invS = 1.f / (float)g.S;
#pragma unroll
    for (int j = 0; j < NI; ++j) {
      const int row = (wave * NI + j) * RPI + lane / CPL, pos = lane % CPL;
      rr[j] = row;
      ch[j] = MC ? (pos ^ (ES == 1 ? swz_mc8(row) : (swz_mc<TILE>(row) >> 4))) : (pos ^ ((row >> 1) & 7));
      if (MODE == OP_IM2COL && !MC) {
        const int PQ = g.P * g.Q;
        int pix = tile_row0 + row;
        pv[j] = pix < rows_lim;
        int n = fdiv(pix, PQ, invPQ), pq = pix - n * PQ;
        int p = fdiv(pq, g.Q, invQ), q = pq - p * g.Q;
        ph[j] = p * g.sh - g.ph;
        pw[j] = q * g.sw - g.pw;
        rowoff[j] = ((n * g.H + ph[j]) * g.W + pw[j]) * g.C + coff;  // host guarantees < 2^31 elements
      }
      if (MODE == OP_IM2COL && MC) {
        int col = tile_col0 + ch[j] * EPC;
        co[j] = col == ones_col && col < cols_lim;
        cv[j] = col < cols_lim && col != ones_col;
        int tap = col / g.Cg;
        cc[j] = col - tap * g.Cg;
        cr[j] = tap / g.S;
        cs[j] = tap - cr[j] * g.S;
        cdh[j] = cr[j] * g.dh;
        cdw[j] = cs[j] * g.dw;
        colo[j] = (cdh[j] * g.W + cdw[j]) * g.C + coff + cc[j];
      }
    }
    kcmode = 0;
    fast = false;
    if (MODE == OP_IM2COL && !MC) {
      kcmode = __builtin_amdgcn_readfirstlane((g.Cg % (8 * EPC)) == 0 ? 1 : (g.Cg >= 8 * EPC ? 2 : 0));
      if (kcmode == 1 && (g.R > 16 || g.S > 16)) kcmode = 2;  // the tap masks hold 16 rows / cols
#pragma unroll
      for (int j = 0; j < NI; ++j) {
        kch[j] = ch[j] * EPC;
        rowb[j] = (unsigned)(rowoff[j] + kch[j]) * (unsigned)ES;
        if (!pv[j]) ph[j] = -(1 << 28);
        unsigned m = 0;
        if (kcmode == 1 && pv[j]) {
          for (int r = 0; r < g.R; ++r) m |= (unsigned)((unsigned)(ph[j] + r * g.dh) < (unsigned)g.H) << r;
          for (int t = 0; t < g.S; ++t) m |= (unsigned)((unsigned)(pw[j] + t * g.dw) < (unsigned)g.W) << (16 + t);
        }
        vrs[j] = m;
      }
    }
    if (MODE == OP_DENSE) {
      // element extent of the operand for this group: KC rows x ld, MC (k rows) x ld
      const long long extent = MC ? (long long)k_lim_hint * ld : (long long)rows_lim * ld;
      fast = __builtin_amdgcn_readfirstlane((int)(extent * ES < (1ll << 31) && (!MC || ones_col < 0))) != 0;
      // built unconditionally from wave-uniform values so it stays in SGPRs
      const unsigned long long a = reinterpret_cast<unsigned long long>(base);
      rsrc[0] = __builtin_amdgcn_readfirstlane((int)(unsigned)a);
      rsrc[1] = __builtin_amdgcn_readfirstlane((int)((a >> 32) & 0xffffu));
      rsrc[2] = (int)0x80000000u;  // num_records: every valid offset is below 2^31
      rsrc[3] = 0x00020000;
      if (fast) {
#pragma unroll
        for (int j = 0; j < NI; ++j) {
          if (!MC) {
            const int row = tile_row0 + rr[j];
            kch[j] = ch[j] * EPC;
            voff[j] = row < rows_lim ? (int)(((long long)row * ld + kch[j]) * ES) : (int)0x80000000u;
          } else {
            const int col = tile_col0 + ch[j] * EPC;
            kch[j] = rr[j];
            voff[j] = col < cols_lim ? (int)(((long long)rr[j] * ld + col) * ES) : (int)0x80000000u;
          }
        }
      }
    }
    if (MODE == OP_IM2COL && MC) {
      const int PQ = g.P * g.Q;
      bool any = false;
#pragma unroll
      for (int j = 0; j < NI; ++j) {
        const int pix = k_start + rr[j];
        const int n = fdiv(pix, PQ, invPQ), pq = pix - n * PQ;
        const int p = fdiv(pq, g.Q, invQ), q = pq - p * g.Q;
        const int hrow = p * g.sh - g.ph, wrow = q * g.sw - g.pw;
        hc[j] = cv[j] ? hrow + cdh[j] : -(1 << 29);
        wc[j] = wrow + cdw[j];
        hlim[j] = g.P * g.sh - g.ph + cdh[j];
        wlim[j] = g.Q * g.sw - g.pw + cdw[j];
        mofs[j] = (unsigned)((n * g.H + hrow) * g.W + wrow) * (unsigned)g.C * (unsigned)ES +
                  (unsigned)colo[j] * (unsigned)ES;  // modular: < 2^32 where valid (host)
        any = any || co[j];
      }
      wave_has_one = __ballot(any) != 0ull;
      const int dn = BKE / PQ, rem = BKE - dn * PQ, dp = rem / g.Q, dq = rem - dp * g.Q;
      s_dq = __builtin_amdgcn_readfirstlane(dq * g.sw);
      s_qsw = __builtin_amdgcn_readfirstlane(g.Q * g.sw);
      s_dp = __builtin_amdgcn_readfirstlane(dp * g.sh);
      s_sh = __builtin_amdgcn_readfirstlane(g.sh);
      s_psh = __builtin_amdgcn_readfirstlane(g.P * g.sh);
      const unsigned cb = (unsigned)g.C * (unsigned)ES;
      s_d0 = __builtin_amdgcn_readfirstlane((unsigned)((dn * g.H + dp * g.sh) * g.W + dq * g.sw) * cb);
      s_d1 = __builtin_amdgcn_readfirstlane((unsigned)(g.sh * g.W - g.Q * g.sw) * cb);
      s_d2 = __builtin_amdgcn_readfirstlane((unsigned)((g.H - g.P * g.sh) * g.W) * cb);
    }
  }

  // M0 of an LDS-DMA: the LDS byte address of the destination.  The low 32 bits of a generic
  // pointer into LDS are that address (shared aperture), so no address-space cast (whose
  // null check costs two SALU per DMA).
  static SN_DEV uint32_t lds_m0(const char* lds) {
    return __builtin_amdgcn_readfirstlane((uint32_t)reinterpret_cast<uintptr_t>(lds));
  }
  // The DMA is issued from inline asm so the compiler's wait-count pass does not see an
  // LDS write it cannot disambiguate (it would drain vmcnt(0) before the next ds_read);
  // every wait on these DMAs is explicit in the K-loop (counted vmcnt + barrier).
  SN_DEV void dma(const char* src, bool valid, char* lds, bool one = false) {
    const void* s = valid ? (const void*)src
                          : (one ? (ES == 1 ? (const void*)g_one16_f8 : (const void*)g_one16) : (const void*)g_zero16);
    const uint32_t m0 = lds_m0(lds);
    asm volatile("s_mov_b32 m0, %0\n\ts_nop 0\n\tglobal_load_lds_dwordx4 %1, off" ::"s"(m0), "v"(s) : "memory");
  }
  // LDS-DMA through the buffer resource: byte offset off (0xffffffff: out of range -> 0)
  SN_DEV void dma_buf(unsigned off, char* lds) {
    const uint32_t m0 = lds_m0(lds);
    asm volatile("s_mov_b32 m0, %0\n\ts_nop 0\n\tbuffer_load_dwordx4 %1, %2, 0 offen lds" ::"s"(m0), "v"(off),
                 "s"(rsrc)
                 : "memory");
  }
  // ... with a wave-uniform byte offset `so` in the instruction's SGPR offset field
  // (the per-lane voffset carries the out-of-range marker 0x80000000)
  SN_DEV void dma_buf_so(unsigned off, unsigned so, char* lds) {
    const uint32_t m0 = lds_m0(lds);
    asm volatile("s_mov_b32 m0, %0\n\ts_nop 0\n\tbuffer_load_dwordx4 %1, %2, %3 offen lds" ::"s"(m0), "v"(off),
                 "s"(rsrc), "s"(so)
                 : "memory");
  }

  // Issue the LDS-DMA of the tile whose first reduction index is k_tile into `lds`.
  SN_DEV void issue(char* lds, int wave, int k_tile, int k_lim, int tile_rc0, int rc_lim) {
    char* dst = lds + wave * NI * 1024;
    if (!MC) {
      if (MODE == OP_DENSE) {
        if (fast) {
          const unsigned so = __builtin_amdgcn_readfirstlane((unsigned)(k_tile * ES));
          if (k_tile + 8 * EPC <= k_lim) {  // no K tail: fixed per-lane offsets, no VALU
#pragma unroll
            for (int j = 0; j < NI; ++j) dma_buf_so((unsigned)voff[j], so, dst + j * 1024);
            return;
          }
#pragma unroll
          for (int j = 0; j < NI; ++j)
            dma_buf_so(k_tile + kch[j] >= k_lim ? 0x80000000u : (unsigned)voff[j], so, dst + j * 1024);
          return;
        }
#pragma unroll
        for (int j = 0; j < NI; ++j) {
          int row = tile_rc0 + rr[j], k = k_tile + ch[j] * EPC;
          dma(base + ((long long)row * ld + k) * ES, row < rc_lim && k < k_lim, dst + j * 1024);
        }
      } else {
        // k = (tap, c), c innermost.  (r0, s0, c0) is the running scalar decode of k_tile;
        // each lane adds its chunk (< 8*EPC channels), which crosses at most one tap
        // boundary when Cg >= 8*EPC — no per-lane division on the fast path.
        const int c0 = nc, r0 = nr, s0 = ns;
        nc += 8 * EPC;
        while (nc >= g.Cg) {
          nc -= g.Cg;
          if (++ns == g.S) {
            ns = 0;
            ++nr;
          }
        }
        if (kcmode == 1) {
          // one tap per K-step: scalar tap offset and tap mask; per DMA v_and + v_cmp (tap
          // inside the image), v_add + v_cndmask (offset, or out of range -> zeros)
          const unsigned tb0 = (unsigned)(((r0 * g.dh) * g.W + s0 * g.dw) * g.C + c0) * (unsigned)ES;
          const unsigned msk = (1u << r0) | (1u << (16 + s0));
          if (k_tile + 8 * EPC <= k_lim) {
#pragma unroll
            for (int j = 0; j < NI; ++j) dma_buf((vrs[j] & msk) == msk ? rowb[j] + tb0 : 0xffffffffu, dst + j * 1024);
            return;
          }
#pragma unroll
          for (int j = 0; j < NI; ++j)
            dma_buf((vrs[j] & msk) == msk && k_tile + kch[j] < k_lim ? rowb[j] + tb0 : 0xffffffffu, dst + j * 1024);
          return;
        }
        if (kcmode != 0) {
          const bool tail = k_tile + 8 * EPC > k_lim;
          const int hr0 = r0 * g.dh, ws0 = s0 * g.dw;
          const unsigned tb0 = (unsigned)((hr0 * g.W + ws0) * g.C + c0) * (unsigned)ES;
          int hre[2], wse[2];
          unsigned tbe[2];
          if (kcmode == 1) {
            hre[0] = hre[1] = hr0;
            wse[0] = wse[1] = ws0;
            tbe[0] = tbe[1] = tb0;
          } else {
            // chunks past the tap's last channel belong to the next tap (scalar decode)
            int r1 = r0, s1 = s0 + 1;
            if (s1 == g.S) {
              s1 = 0;
              ++r1;
            }
            const int hr1 = r1 * g.dh, ws1 = s1 * g.dw;
            const unsigned tb1 = (unsigned)((hr1 * g.W + ws1) * g.C + c0 - g.Cg) * (unsigned)ES;
#pragma unroll
            for (int e = 0; e < 2; ++e) {
              const bool x = c0 + kch[e] >= g.Cg;
              hre[e] = x ? hr1 : hr0;
              wse[e] = x ? ws1 : ws0;
              tbe[e] = x ? tb1 : tb0;
            }
          }
#pragma unroll
          for (int j = 0; j < NI; ++j) {
            const int e = j & 1;
            const int h = ph[j] + hre[e], w = pw[j] + wse[e];
            bool v = (unsigned)h < (unsigned)g.H && (unsigned)w < (unsigned)g.W;
            if (tail) v = v && k_tile + kch[j] < k_lim;
            dma_buf(v ? rowb[j] + tbe[e] : 0xffffffffu, dst + j * 1024);
          }
          return;
        }
        int kv[2], dh[2], dw[2], toff[2];
#pragma unroll
        for (int e = 0; e < 2; ++e) {
          int c = c0 + ch[e] * EPC, r = r0, s = s0;
          if (g.Cg >= 8 * EPC) {
            if (c >= g.Cg) {
              c -= g.Cg;
              s += 1;
              if (s == g.S) {
                s = 0;
                r += 1;
              }
            }
          } else if (g.Cg > 2 * EPC && g.S >= 2) {
            // Cg in (16, 64) bf16 channels (AlexNet conv2's 48 per group, GoogLeNet's reduce
            // widths): c < Cg + 6 EPC < 4 Cg, so the chunk crosses at most three tap boundaries
            // and the tap column wraps at most twice — compares and selects, not a per-lane
            // (divergent) carry loop
            const int d = (c >= g.Cg) + (c >= 2 * g.Cg) + (c >= 3 * g.Cg);
            c -= (int)__umul24((unsigned)d, (unsigned)g.Cg);
            s += d;
            const bool ws = s >= g.S;
            s -= ws ? g.S : 0;
            r += ws;
            if (s >= g.S) {  // S == 2 and three crossings
              s -= g.S;
              ++r;
            }
          } else if (g.Cg >= 2 * EPC) {
            // narrower channel runs (fp8 with 64 channels: VGG conv1_2): the chunk may cross
            // up to 8 * EPC / Cg taps — a short carry loop instead of two divisions
            while (c >= g.Cg) {
              c -= g.Cg;
              if (++s == g.S) {
                s = 0;
                ++r;
              }
            }
          } else {
            const int kk = k_tile + ch[e] * EPC;
            const int tap = fdiv(kk, g.Cg, invCg);
            c = kk - tap * g.Cg;
            r = fdiv(tap, g.S, invS);
            s = tap - r * g.S;
          }
          kv[e] = k_tile + ch[e] * EPC < k_lim;
          dh[e] = (int)__umul24((unsigned)r, (unsigned)g.dh);
          dw[e] = (int)__umul24((unsigned)s, (unsigned)g.dw);
          toff[e] = (int)mad24(mad24((unsigned)dh[e], (unsigned)g.W, (unsigned)dw[e]), (unsigned)g.C, (unsigned)c);
        }
#pragma unroll
        for (int j = 0; j < NI; ++j) {
          const int e = j & 1;
          const int h = ph[j] + dh[e], w = pw[j] + dw[e];
          const bool v = kv[e] && pv[j] && (unsigned)h < (unsigned)g.H && (unsigned)w < (unsigned)g.W;
          dma_buf(v ? (unsigned)(rowoff[j] + toff[e]) * (unsigned)ES : 0xffffffffu, dst + j * 1024);
        }
      }
    } else {
      if (MODE == OP_DENSE && fast) {
        const unsigned so = __builtin_amdgcn_readfirstlane((unsigned)((long long)k_tile * ld * ES));
        if (k_tile + BKE <= k_lim) {
#pragma unroll
          for (int j = 0; j < NI; ++j) dma_buf_so((unsigned)voff[j], so, dst + j * 1024);
        } else {
#pragma unroll
          for (int j = 0; j < NI; ++j)
            dma_buf_so(k_tile + kch[j] >= k_lim ? 0x80000000u : (unsigned)voff[j], so, dst + j * 1024);
        }
      } else if (MODE == OP_DENSE) {
#pragma unroll
        for (int j = 0; j < NI; ++j) {
          int k = k_tile + rr[j], col = tile_rc0 + ch[j] * EPC;
          const bool one = col == ones_col && col < rc_lim && k < k_lim;
          dma(base + ((long long)k * ld + col) * ES, k < k_lim && col < rc_lim && col != ones_col, dst + j * 1024,
              one);
        }
      } else if (MODE == OP_FLIPW) {
        const int RS = g.R * g.S;
        const long long rowlen = (long long)RS * g.Cg;
#pragma unroll
        for (int j = 0; j < NI; ++j) {
          int k = k_tile + rr[j], col = tile_rc0 + ch[j] * 8;
          int tap = fdiv(k, g.C, invKg), kout = k - tap * g.C;
          bool v = k < k_lim && col < rc_lim;
          long long off = v ? (long long)kout * rowlen + (long long)(RS - 1 - tap) * g.Cg + col : 0;
          dma(base + off * 2, v, dst + j * 1024);
        }
      } else {
        // rows = pixels, incremental per-lane state (see the members); rows at or past k_lim
        // (the split's / the product's end) read zeros: one compare against a scalar
        const int krem = __builtin_amdgcn_readfirstlane(k_lim - k_tile);
        if (!wave_has_one) {
#pragma unroll
          for (int j = 0; j < NI; ++j) {
            const bool v = ((unsigned)hc[j] < (unsigned)g.H) & ((unsigned)wc[j] < (unsigned)g.W) & (rr[j] < krem);
            dma_buf(v ? mofs[j] : 0xffffffffu, dst + j * 1024);
          }
        } else {
#pragma unroll
          for (int j = 0; j < NI; ++j) {
            const bool kin = rr[j] < krem;
            const bool v = kin && (unsigned)hc[j] < (unsigned)g.H && (unsigned)wc[j] < (unsigned)g.W;
            dma(base + mofs[j], v, dst + j * 1024, co[j] && kin);
          }
        }
        // next tile: BKE pixels on (q carry c1, then p carry c2)
#pragma unroll
        for (int j = 0; j < NI; ++j) {
          int w = wc[j] + s_dq;
          const bool c1 = w >= wlim[j];
          w -= c1 ? s_qsw : 0;
          int h = hc[j] + s_dp + (c1 ? s_sh : 0);
          const bool c2 = h >= hlim[j];
          h -= c2 ? s_psh : 0;
          mofs[j] += s_d0 + (c1 ? s_d1 : 0u) + (c2 ? s_d2 : 0u);
          wc[j] = w;
          hc[j] = h;
        }
      }
    }
  }
};

// Fragment of a 16-row subtile (rows x0..x0+15 of the operand's M/N axis) for k-step s
// (32 reduction elements), laid out as the 16x16x32 MFMA operand: lane l holds
// X[x0 + (l&15)][32s + 8(l>>4) + j], j = 0..7.
template <int MC, int TILE>
SN_DEV bf16x8_t read_frag(const char* lds, int x0, int s, int lane) {
  if (!MC) {
    int row = x0 + (lane & 15);
    int kc = s * 4 + (lane >> 4);
    uint4 v = *reinterpret_cast<const uint4*>(lds + kc_off(row, kc));
    return __builtin_bit_cast(bf16x8_t, v);
  } else {
    // ds_read_b64_tr_b16: lane 4q+p of each 16-lane group addresses row q, cols 4p..4p+3
    // of a 4x16 block; lane i receives column i of the 4 rows.  Two reads = 8 k values.
    int gq = lane >> 4, li = lane & 15, q = li >> 2, p = li & 3;
    int col_b = (x0 + 4 * p) * 2;
    int k0 = s * 32 + gq * 8 + q;
    int k1 = k0 + 4;
    typedef __attribute__((address_space(3))) s16x4 lds_s16x4;
    const char* a0 = lds + k0 * (TILE * 2) + (col_b ^ swz_mc<TILE>(k0));
    const char* a1 = lds + k1 * (TILE * 2) + (col_b ^ swz_mc<TILE>(k1));
    s16x4 lo = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_s16x4*)a0);
    s16x4 hi = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_s16x4*)a1);
    s16x8 r = {lo[0], lo[1], lo[2], lo[3], hi[0], hi[1], hi[2], hi[3]};
    return __builtin_bit_cast(bf16x8_t, r);
  }
}

// s_waitcnt immediate (gfx9 encoding) that waits for vmcnt <= N only.
constexpr int waitcnt_vm(int n) { return (n & 15) | (7 << 4) | (15 << 8) | (((n >> 4) & 3) << 14); }

// NW waves (4 or 8), each owning a 64x64 output sub-tile; NS LDS stages (2 or 3).
//   NS = 2: one barrier per K-step, DMA of tile k+1 under the MFMAs of tile k (vmcnt(0)).
//   NS = 3: two tiles in flight; each K-step waits with a COUNTED vmcnt for its own tile
//           only and uses a raw s_barrier (no fence), so the DMA of tile k+1 keeps
//           flying across the barrier while tile k+2 is issued (cdna_hip_programming
//           "Pipelining across barriers").
// fp8 (e4m3) fragment of a 16-row subtile for v_mfma_scale_f32_16x16x128_f8f6f4: lane l
// holds X[x0 + (l&15)][32(l>>4) + j], j = 0..31 — two 16-B chunks of the 128-B KC row.
typedef __attribute__((ext_vector_type(8))) int i32x8;
SN_DEV i32x8 read_frag8(const char* lds, int x0, int lane) {
  const int row = x0 + (lane & 15), kc = 2 * (lane >> 4);
  const uint4 v0 = *reinterpret_cast<const uint4*>(lds + kc_off(row, kc));
  const uint4 v1 = *reinterpret_cast<const uint4*>(lds + kc_off(row, kc + 1));
  i32x8 r = {(int)v0.x, (int)v0.y, (int)v0.z, (int)v0.w, (int)v1.x, (int)v1.y, (int)v1.z, (int)v1.w};
  return r;
}

// fp8 fragment of a 16-column subtile (columns x0..x0+15, x0 % 16 == 0) of an MC image
// ([128 k][128 cols] bytes, swz_mc8): lane l needs X[k = 32(l>>4) + j][x0 + (l&15)],
// j = 0..31, i.e. one column down 32 rows.  ds_read_b64_tr_b8 transposes an 8-row x 16-byte
// block per 16-lane group (lane 2q+p addresses row q, bytes 8p..8p+7; lane i receives column
// i of the 8 rows: tests/test_gemm_fp8_mc_gpu.py pins this), so four reads = 32 k values.
SN_DEV i32x8 read_frag8_mc(const char* lds, int x0, int lane) {
  typedef int v2i __attribute__((ext_vector_type(2)));
  typedef __attribute__((address_space(3))) v2i lds_v2i;
  const int g = lane >> 4, i = lane & 15, q = i >> 1, p = i & 1, c = x0 >> 4;
  i32x8 r;
#pragma unroll
  for (int rr = 0; rr < 4; ++rr) {
    const int k = 32 * g + 8 * rr + q;
    const char* a = lds + k * 128 + ((c ^ swz_mc8(k)) << 4) + 8 * p;
    const v2i v = __builtin_amdgcn_ds_read_tr8_b64_v2i32((lds_v2i*)a);
    r[2 * rr] = v[0];
    r[2 * rr + 1] = v[1];
  }
  return r;
}
template <int MC>
SN_DEV i32x8 read_frag8x(const char* lds, int x0, int lane) {
  if constexpr (MC)
    return read_frag8_mc(lds, x0, lane);
  else
    return read_frag8(lds, x0, lane);
}

// fused fp8 side output (SnGemmArgs.q_out): 4 bf16-rounded values -> 4 fp8 bytes
SN_DEV uint32_t q_pack4(const SnGemmArgs& args, float sc, const float* v, float& qmax) {
  const float fmax = args.q_e5m2 ? 57344.f : 448.f;
  float f[4];
#pragma unroll
  for (int r = 0; r < 4; ++r) {
    const float b = bf2f(f2bf(v[r]));  // the bf16 value the separate pass would read
    qmax = fmaxf(qmax, fabsf(b));
    f[r] = fminf(fmaxf(b * sc, -fmax), fmax);
  }
  int w = 0;
  if (args.q_e5m2) {
    w = __builtin_amdgcn_cvt_pk_bf8_f32(f[0], f[1], w, false);
    w = __builtin_amdgcn_cvt_pk_bf8_f32(f[2], f[3], w, true);
  } else {
    w = __builtin_amdgcn_cvt_pk_fp8_f32(f[0], f[1], w, false);
    w = __builtin_amdgcn_cvt_pk_fp8_f32(f[2], f[3], w, true);
  }
  return (uint32_t)w;
}

// block |max| of the fp8 side output -> one atomicMax on q_slot[1] (every thread calls it).
// The 32-B scratch is the start of an idle LDS stage, NOT a __shared__ array of its own:
// the 2-block-per-CU tiles use exactly 160 KB of LDS, one more byte halves their occupancy.
SN_DEV void q_amax_flush(const SnGemmArgs& args, float qmax, char* lds_scratch) {
  float* qred = reinterpret_cast<float*>(lds_scratch);
  qmax = wave_max(qmax);
  const int w = threadIdx.x >> 6;
  __syncthreads();  // every wave is done with the stage (fragment reads / staged stores)
  if ((threadIdx.x & 63) == 0) qred[w] = qmax;
  __syncthreads();
  if (threadIdx.x == 0) {
    float m = 0.f;
    for (int i = 0; i < (int)(blockDim.x >> 6); ++i) m = fmaxf(m, qred[i]);
    if (m > 0.f) atomicMax(reinterpret_cast<unsigned int*>(args.q_part + (blockIdx.x & 255) * 32), __float_as_uint(m));
  }
}

// bias / ReLU / ReLU-backward gate / dropout of one 4-column bf16 output fragment
template <int EPI, bool FP8>
SN_DEV void epi_bf16_math(const SnGemmArgs& args, int grp, int m, int n, f32x4 v, int c_cols, float* o) {
  const bool full = (n + 3 < c_cols) && ((args.ldc & 3) == 0);
  if (FP8) v = v * (args.deq_a[0] * args.deq_b[0]);  // per-tensor fp8 scales
  o[0] = v[0];
  o[1] = v[1];
  o[2] = v[2];
  o[3] = v[3];
  {
    if (args.bias) {
      const float* bz = args.bias + (long long)grp * args.N;
#pragma unroll
      for (int r = 0; r < 4; ++r) o[r] += (n + r < args.N) ? bz[n + r] : 0.f;
    }
    if (args.relu) {
#pragma unroll
      for (int r = 0; r < 4; ++r) o[r] = fmaxf(o[r], 0.f);
    }
    if (args.gate) {
      const bf16_t* gp = args.gate + grp * args.c_gstride + (long long)m * args.ldc + n;
      float gv[4];
      if (full && (args.c_gstride & 3) == 0) {
        const uint2 u = *reinterpret_cast<const uint2*>(gp);
        gv[0] = __uint_as_float(u.x << 16);
        gv[1] = __uint_as_float(u.x & 0xffff0000u);
        gv[2] = __uint_as_float(u.y << 16);
        gv[3] = __uint_as_float(u.y & 0xffff0000u);
      } else {
#pragma unroll
        for (int r = 0; r < 4; ++r) gv[r] = (n + r < args.N) ? bf2f(gp[r]) : 0.f;
      }
#pragma unroll
      for (int r = 0; r < 4; ++r) o[r] = gv[r] > 0.f ? o[r] * args.gate_scale : 0.f;
    }
    if (EPI == EPI_BF16_DROP) {
      const long long e0 = grp * args.c_gstride + (long long)m * args.ldc + n;
      if ((e0 & 3) == 0) {  // the usual case: the 4 columns are one Philox draw
        const uint4 u = dropout_bits4(args.drop_rng, args.drop_stream, (unsigned long long)e0 >> 2);
        o[0] = u.x > args.drop_thr ? o[0] * args.drop_scale : 0.f;
        o[1] = u.y > args.drop_thr ? o[1] * args.drop_scale : 0.f;
        o[2] = u.z > args.drop_thr ? o[2] * args.drop_scale : 0.f;
        o[3] = u.w > args.drop_thr ? o[3] * args.drop_scale : 0.f;
      } else {
#pragma unroll
        for (int r = 0; r < 4; ++r)
          o[r] = dropout_keep(args.drop_rng, args.drop_stream, args.drop_thr, e0 + r) ? o[r] * args.drop_scale : 0.f;
      }
    }
  }
}

// Store one 4-column output fragment v = C[m][n..n+3] (the caller checked m < M, n < N):
// bias / ReLU / ReLU-backward gate for bf16 outputs, fp32 store / accumulate (+ the
// bias-gradient column routed to bias_out), or the fused solver update (EPI_SGD).
template <int EPI, bool FP8>
SN_DEV void epi_store(const SnGemmArgs& args, int grp, int split, int m, int n, f32x4 v, int c_cols,
                      float* qmax = nullptr) {
  const bool full = (n + 3 < c_cols) && ((args.ldc & 3) == 0);
  if (epi_bf16<EPI>()) {
    bf16_t* C = reinterpret_cast<bf16_t*>(args.C) + grp * args.c_gstride + (long long)m * args.ldc;
    float o[4];
    epi_bf16_math<EPI, FP8>(args, grp, m, n, v, c_cols, o);
    if (qmax && args.q_out) {  // host: q_ld % 4 == 0, N % 4 == 0 (whole 4-byte fragments)
      const uint32_t w = q_pack4(args, args.q_slot[0], o, *qmax);
      *reinterpret_cast<uint32_t*>(args.q_out + grp * args.q_gstride + (long long)m * args.q_ld + n) = w;
    }
    if (full) {
      uint2 pk = make_uint2(pack2(o[0], o[1]), pack2(o[2], o[3]));
      *reinterpret_cast<uint2*>(C + n) = pk;
    } else {
#pragma unroll
      for (int r = 0; r < 4; ++r)
        if (n + r < args.N) C[n + r] = f2bf(o[r]);
    }
  } else {
    if (FP8) {
      // per-tensor fp8 scales; the virtual ones column (bias gradient of an fp8 weight
      // gradient) holds an UNSCALED e4m3 1.0, so it takes A's dequantisation only
      const float dab = args.deq_a[0] * args.deq_b[0], da = args.deq_a[0];
#pragma unroll
      for (int r = 0; r < 4; ++r) v[r] *= (n + r == args.ones_col) ? da : dab;
    }
    if (args.bias_out && n <= args.ones_col && args.ones_col < n + 4) {
      const int r = args.ones_col - n;
      const float bv = r == 0 ? v[0] : (r == 1 ? v[1] : (r == 2 ? v[2] : v[3]));
      float* bp = args.bias_out + (long long)grp * args.M + m;
      *bp = args.bias_acc ? *bp + bv : bv;
    }
    if (n >= c_cols) return;
    if (EPI == EPI_SGD) {
      // H_LR = 0, H_MOM = 1, H_WD = 2, H_NORM = 4 (solver.hip); same op order as
      // solver_update_kernel KIND 0 / 1 so both paths give identical weights
      const float* hy = args.sgd_hyper;
      const float rate = hy[0] * args.sgd_lr_mult, mom = hy[1], decay = hy[2] * args.sgd_decay_mult;
      const float gscale = hy[4];
      const long long o = grp * args.c_gstride + (long long)m * args.ldc + n;
      const bool vec = (n + 3 < c_cols) && ((args.ldc & 3) == 0) && ((o & 3) == 0);
      float W[4], A[4];
      if (vec) {
        const float4 w4 = *reinterpret_cast<const float4*>(args.sgd_w + o);
        const float4 a4 = *reinterpret_cast<const float4*>(args.sgd_h + o);
        W[0] = w4.x; W[1] = w4.y; W[2] = w4.z; W[3] = w4.w;
        A[0] = a4.x; A[1] = a4.y; A[2] = a4.z; A[3] = a4.w;
      } else {
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          W[r] = n + r < c_cols ? args.sgd_w[o + r] : 0.f;
          A[r] = n + r < c_cols ? args.sgd_h[o + r] : 0.f;
        }
      }
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        float gg = v[r] * gscale;
        gg += decay * ((args.sgd_flags & 2) ? (float)((W[r] > 0.f) - (W[r] < 0.f)) : W[r]);
        const float prev = A[r];
        A[r] = mom * A[r] + rate * gg;
        W[r] -= (args.sgd_flags & 1) ? (1.f + mom) * A[r] - mom * prev : A[r];
      }
      if (vec) {
        *reinterpret_cast<float4*>(args.sgd_w + o) = make_float4(W[0], W[1], W[2], W[3]);
        *reinterpret_cast<float4*>(args.sgd_h + o) = make_float4(A[0], A[1], A[2], A[3]);
        *reinterpret_cast<uint2*>(args.sgd_shadow + o) = make_uint2(pack2(W[0], W[1]), pack2(W[2], W[3]));
      } else {
#pragma unroll
        for (int r = 0; r < 4; ++r)
          if (n + r < c_cols) {
            args.sgd_w[o + r] = W[r];
            args.sgd_h[o + r] = A[r];
            args.sgd_shadow[o + r] = f2bf(W[r]);
          }
      }
      return;
    }
    float* C = reinterpret_cast<float*>(args.C) + split * args.c_split_stride + grp * args.c_gstride +
               (long long)m * args.ldc;
    if (full) {
      float4* p = reinterpret_cast<float4*>(C + n);
      if (EPI == EPI_F32_ACC) {
        float4 o = *p;
        *p = make_float4(o.x + v[0], o.y + v[1], o.z + v[2], o.w + v[3]);
      } else {
        *p = make_float4(v[0], v[1], v[2], v[3]);
      }
    } else {
#pragma unroll
      for (int r = 0; r < 4; ++r)
        if (n + r < c_cols) {
          if (EPI == EPI_F32_ACC)
            C[n + r] += v[r];
          else
            C[n + r] = v[r];
        }
    }
  }
}

// (v_mfma_f32_32x32x16_bf16 twins of these tiles measured slower on every conv product,
// docs/PERF_NOTES.md round 5, and were removed in round 6)
template <int AMC, int AMODE, int BMC, int BMODE, int EPI, int BM, int BN, int NW, int NS, int FP8 = 0,
          int NFR = 4, int MFR = 4>
__global__ void __launch_bounds__(NW * 64, NW == 4 ? (BM * BN <= 128 * 64 ? 3 : 2) : 1) gemm_kernel(SnGemmArgs args) {
  // LDS rows are 128 B in both precisions: BK = 64 bf16 or 128 fp8 reduction elements
  constexpr int ES = FP8 ? 1 : 2, BKE = FP8 ? 128 : BK;
  // MFMA operand formats: src A of the instruction is our B fragment (cbsz), src B our A
  // fragment (blgp); 0 = e4m3, 1 = e5m2
  constexpr int FMT_A = FP8 == 2 ? 1 : 0;
  // B's LDS image holds BNL >= BN rows: whole wave-instructions per wave (a 48-wide tile
  // stages 64 rows, the 16 beyond the tile read the zero page)
  constexpr int BNL = ((BN / 8) % NW == 0) ? BN : (BN + 63) / 64 * 64;
  constexpr int A_BYTES = BM * 128, B_BYTES = BNL * 128, STAGE = A_BYTES + B_BYTES;
  // waves along N / M; each wave owns (16*MFR) rows x (16*NFR) columns: 64 x 64 (NFR = 4, or
  // 3 for 96-wide tiles), or 128 x (16*NFR) for the 8-wave 256-row tiles (MFR = 8)
  constexpr int WN = BN / (16 * NFR), WM = NW / WN;
  static_assert(WN * 16 * NFR == BN && WM * 16 * MFR == BM && WM * WN == NW, "tile/wave layout mismatch");
  static_assert(NS == 2 || NS == 3, "2 or 3 LDS stages");
  // Distinct LDS objects (one per stage): the compiler's alias scopes then prove that
  // the ds_reads of one stage do not depend on the DMA in flight into another, so it
  // does not drain vmcnt before every k-step's first ds_read.
  __shared__ __attribute__((aligned(16))) char smem0[STAGE];
  __shared__ __attribute__((aligned(16))) char smem1[STAGE];
  __shared__ __attribute__((aligned(16))) char smem2[NS == 3 ? STAGE : 16];
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int tiles_m = (args.M + BM - 1) / BM;

  // XCD-aware bijective remap: blocks that share an XCD (same bid % 8) get a
  // contiguous range of tile ids, so tiles sharing an operand panel share an L2.
  int bid = blockIdx.x;
  const int nwg = gridDim.x;
  if (nwg >= 16) {
    int xcd = bid & 7, qq = nwg >> 3, rr = nwg & 7;
    bid = (xcd < rr ? xcd * (qq + 1) : rr * (qq + 1) + (xcd - rr) * qq) + (bid >> 3);
  }
  // raster: M-fastest by default; N-fastest (args.raster_n) when a few N tiles share a tall A
  // panel (conv fwd / dgrad: pixels x channels) so its N tiles run together and the panel
  // is read from HBM once and from L2 for the others.
  // The grid is 1-D over (tile, split, group), tile fastest: after the remap the tiles of
  // one split / group (which share the A panel of that K range, e.g. a weight gradient's
  // dy chunk read by every N tile) are contiguous and so run on one XCD and its L2.
  const int tiles_n = (args.N + BN - 1) / BN;
  const int tiles = tiles_m * tiles_n;
  const int tile = bid % tiles, rest = bid / tiles;
  const int split = rest % args.splits, grp = rest / args.splits;
  const int tm = args.raster_n ? tile / tiles_n : tile % tiles_m;
  const int tn = args.raster_n ? tile % tiles_n : tile / tiles_m;
  const int m_blk = tm * BM, n_blk = tn * BN;
  const int k0 = split * args.kchunk;
  const int k1 = min(args.K, k0 + args.kchunk);

  const int wv = __builtin_amdgcn_readfirstlane(wave);
  using SA = GStager<AMC, AMODE, BM, NW, ES>;
  using SB = GStager<BMC, BMODE, BNL, NW, ES>;
  SA sa;
  SB sb;
  sa.init(args.A, grp, wv, lane, m_blk, args.M, m_blk, args.M, -1, split * args.kchunk, args.K);
  const int n_lim = min(args.N, n_blk + BN);
  sb.init(args.B, grp, wv, lane, n_blk, n_lim, n_blk, n_lim, BMC ? args.ones_col : -1, split * args.kchunk, args.K);

  f32x4 acc[NFR][MFR];
#pragma unroll
  for (int i = 0; i < NFR; ++i)
#pragma unroll
    for (int j = 0; j < MFR; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};

  const int wm0 = (wave % WM) * (16 * MFR), wn0 = (wave / WM) * (16 * NFR);
  const int nk = k1 > k0 ? (k1 - k0 + BKE - 1) / BKE : 0;

  auto compute = [&](const char* la) __attribute__((always_inline)) {
    const char* lb = la + A_BYTES;
    if constexpr (FP8 && MFR * NFR > 16) {
      // large fp8 tiles (gemm_fp8big.hip): B fragments held, A fragments streamed per row
      // group, so at most NFR + 1 fragments (8 VGPRs each) live beside the accumulators
      i32x8 fb8[NFR];
#pragma unroll
      for (int i = 0; i < NFR; ++i) fb8[i] = read_frag8x<BMC>(lb, wn0 + 16 * i, lane);
      __builtin_amdgcn_s_setprio(1);
#pragma unroll
      for (int j = 0; j < MFR; ++j) {
        const i32x8 fa = read_frag8x<AMC>(la, wm0 + 16 * j, lane);
#pragma unroll
        for (int i = 0; i < NFR; ++i)
          acc[i][j] = __builtin_amdgcn_mfma_scale_f32_16x16x128_f8f6f4(fb8[i], fa, acc[i][j], 0, FMT_A, 0, 127, 0, 127);
      }
      __builtin_amdgcn_s_setprio(0);
      return;
    } else if constexpr (FP8) {
      i32x8 fa8[MFR], fb8[NFR];
#pragma unroll
      for (int i = 0; i < NFR; ++i) fb8[i] = read_frag8x<BMC>(lb, wn0 + 16 * i, lane);
#pragma unroll
      for (int i = 0; i < MFR; ++i) fa8[i] = read_frag8x<AMC>(la, wm0 + 16 * i, lane);
      __builtin_amdgcn_s_setprio(1);
#pragma unroll
      for (int i = 0; i < NFR; ++i)
#pragma unroll
        for (int j = 0; j < MFR; ++j)  // formats e4m3 (B) x e4m3 / e5m2 (A), block scales 2^0 (E8M0 127)
          acc[i][j] = __builtin_amdgcn_mfma_scale_f32_16x16x128_f8f6f4(fb8[i], fa8[j], acc[i][j], 0, FMT_A, 0, 127, 0,
                                                                        127);
      __builtin_amdgcn_s_setprio(0);
      return;
    }
    if constexpr (MFR * NFR > 16 || (EPI == EPI_SGD && BM == 128 && BN == 128 && NW == 4 && NS == 2)) {
      // 128-row wave tiles: fragments of one 32-deep k-substep at a time (the accumulators
      // already take 4 * MFR * NFR VGPRs); EPI_SGD: the prefetched master / history rows do
#pragma unroll
      for (int s = 0; s < 2; ++s) {
        bf16x8_t fa[MFR], fb[NFR];
#pragma unroll
        for (int i = 0; i < NFR; ++i) fb[i] = read_frag<BMC, BNL>(lb, wn0 + 16 * i, s, lane);
#pragma unroll
        for (int i = 0; i < MFR; ++i) fa[i] = read_frag<AMC, BM>(la, wm0 + 16 * i, s, lane);
        __builtin_amdgcn_s_setprio(1);
#pragma unroll
        for (int i = 0; i < NFR; ++i)
#pragma unroll
          for (int j = 0; j < MFR; ++j)
            acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(fb[i], fa[j], acc[i][j], 0, 0, 0);
        __builtin_amdgcn_s_setprio(0);
      }
      return;
    }
    bf16x8_t fa[2][MFR], fb[2][NFR];
#pragma unroll
    for (int s = 0; s < 2; ++s) {
#pragma unroll
      for (int i = 0; i < NFR; ++i) fb[s][i] = read_frag<BMC, BNL>(lb, wn0 + 16 * i, s, lane);
#pragma unroll
      for (int i = 0; i < MFR; ++i) fa[s][i] = read_frag<AMC, BM>(la, wm0 + 16 * i, s, lane);
    }
    __builtin_amdgcn_s_setprio(1);
#pragma unroll
    for (int s = 0; s < 2; ++s)
#pragma unroll
      for (int i = 0; i < NFR; ++i)
#pragma unroll
        for (int j = 0; j < MFR; ++j)
          acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(fb[s][i], fa[s][j], acc[i][j], 0, 0, 0);
    __builtin_amdgcn_s_setprio(0);
  };
  auto issue = [&](char* st, int kt) __attribute__((always_inline)) {
    sa.issue(st, wv, k0 + kt * BKE, k1, m_blk, args.M);
    sb.issue(st + A_BYTES, wv, k0 + kt * BKE, k1, n_blk, n_lim);
  };
  // EPI_SGD on 128x128 tiles (InnerProduct weight gradient + solver update; K = the batch,
  // a few K-steps, so the kernel is bound by the 18 B/param update traffic): the interior
  // tile's master / history loads do not depend on the product, so they are issued before
  // the K-loop and their HBM latency overlaps the first tile's DMA instead of following
  // the MFMAs (the first K-step's vmcnt(0) retires both).
  constexpr bool SGD_PF = EPI == EPI_SGD && BM == 128 && BN == 128 && NW == 4 && NFR == 4 && MFR == 4 && NS == 2 &&
                          !FP8;
  constexpr int PF = 8;  // of the 16 row groups: all 16 (128 VGPRs) spill beside the accumulators
  float4 Wv[SGD_PF ? 16 : 1], Av[SGD_PF ? 16 : 1];
  bool sgd_interior = false;
  if constexpr (SGD_PF) {
    const int cc0 = args.bias_out ? args.ones_col : args.N;
    sgd_interior = m_blk + BM <= args.M && n_blk + BN <= cc0 && (args.ldc & 3) == 0 && ((grp * args.c_gstride) & 3) == 0;
    if (sgd_interior) {
      const long long ob = grp * args.c_gstride + (long long)m_blk * args.ldc + n_blk + (tid & 31) * 4;
#pragma unroll
      for (int it = 0; it < PF; ++it) {
        const long long o = ob + (long long)(it * 8 + (tid >> 5)) * args.ldc;
        Wv[it] = *reinterpret_cast<const float4*>(args.sgd_w + o);
        Av[it] = *reinterpret_cast<const float4*>(args.sgd_h + o);
      }
    }
  }
  if (NS == 2) {
    // One barrier per K-step: retire this wave's DMA of tile kt, barrier (all waves' DMAs
    // landed AND all reads of the other stage from step kt-1 are done), then start the
    // DMA of tile kt+1 into the other stage and run the MFMAs of tile kt under it.
    auto step = [&](char* cur, char* nxt, int kt) __attribute__((always_inline)) {
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
      __syncthreads();
      if (kt + 1 < nk) issue(nxt, kt + 1);
      compute(cur);
    };
    if (nk > 0) issue(smem0, 0);
    for (int kt = 0; kt < nk; kt += 2) {
      step(smem0, smem1, kt);
      if (kt + 1 < nk) step(smem1, smem0, kt + 1);
    }
  } else {
    constexpr int PER_TILE = SA::NI + SB::NI;  // LDS-DMA instructions per wave per tile
    auto step = [&](char* cur, char* nxt2, int kt) __attribute__((always_inline)) {
      // retire tile kt; tile kt+1 (if any) stays in flight
      if (kt + 1 < nk)
        __builtin_amdgcn_s_waitcnt(waitcnt_vm(PER_TILE));
      else
        __builtin_amdgcn_s_waitcnt(waitcnt_vm(0));
      asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
      __builtin_amdgcn_s_barrier();  // all waves: tile kt landed, stage of tile kt-1 free
      if (kt + 2 < nk) issue(nxt2, kt + 2);
      compute(cur);
    };
    if (nk > 0) issue(smem0, 0);
    if (nk > 1) issue(smem1, 1);
    for (int kt = 0; kt < nk; kt += 3) {
      step(smem0, smem2, kt);
      if (kt + 1 < nk) step(smem1, smem0, kt + 1);
      if (kt + 2 < nk) step(smem2, smem1, kt + 2);
    }
  }

  // Epilogue.  acc[i][j] holds D[n][m] with m = lane&15 (+16j), n = 4(lane>>4)+r (+16i):
  // each lane owns 4 consecutive output columns of one output row.
  // wave-relative row (m) of fragment row j, and column (n) of fragment (i, j), of this lane
  auto wave_m = [&](int j) __attribute__((always_inline)) { return 16 * j + (lane & 15); };
  auto wave_n = [&](int i, int j) __attribute__((always_inline)) { return 16 * i + 4 * (lane >> 4); };
  const int esplit = split;  // the fp32 slab the epilogue stores into (split-K)
  // fp32 outputs: the bias-gradient column (when routed to bias_out) is not part of C
  const int c_cols = (!epi_bf16<EPI>() && args.bias_out) ? args.ones_col : args.N;
  if constexpr (EPI == EPI_SGD) {
    // Interior tiles: issue every master-weight / history load of the wave's 64x64 sub-tile
    // first (32 x 16 B per lane in flight), then update and store — a load -> update ->
    // store chain per fragment would expose the HBM latency 16 times.  Edge tiles and
    // the bias column take the per-fragment path below.
    const bool interior = m_blk + BM <= args.M && n_blk + BN <= c_cols && (args.ldc & 3) == 0 &&
                          ((grp * args.c_gstride) & 3) == 0;
    if constexpr (BM == 128 && BN == 128 && NW == 4 && NFR == 4 && MFR == 4 && NS == 2 && !FP8) {
      // LDS-transposed update (128x128 tiles): the MFMA layout gives each wave-instruction
      // 16 rows x 64 B, which the HBM streams of w / h / shadow serve at ~3.7 TB/s; the
      // gradient tile is instead staged through the (now idle) LDS stages as fp32 row-major
      // (rows 0-63 in smem0, 64-127 in smem1, 16-B chunks XOR-swizzled by row) and every
      // 32 lanes then update one contiguous 512-B row segment.  The master / history loads
      // are all issued (32 x 16 B per lane in flight) before the exchange barrier.
      if (interior) {
        const float* hy = args.sgd_hyper;
        const float rate = hy[0] * args.sgd_lr_mult, mom = hy[1], decay = hy[2] * args.sgd_decay_mult;
        const float gscale = hy[4];
        const int cq = tid & 31, r0 = tid >> 5;
        const long long ob = grp * args.c_gstride + (long long)m_blk * args.ldc + n_blk + cq * 4;
        __builtin_amdgcn_s_barrier();  // every wave is past its last fragment read of the stages
        char* wbuf = (wave % WM) == 0 ? smem0 : smem1;
#pragma unroll
        for (int j = 0; j < 4; ++j) {
          const int lr = wave_m(j);
#pragma unroll
          for (int i = 0; i < NFR; ++i) {
            const int ch = (wn0 + wave_n(i, j)) >> 2;
            *reinterpret_cast<f32x4*>(wbuf + lr * 512 + ((ch ^ (lr & 15)) << 4)) = acc[i][j];
          }
        }
        // the first PF master / history row groups were loaded before the K-loop
#pragma unroll
        for (int it = PF; it < 16; ++it) {
          const long long o = ob + (long long)(it * 8 + r0) * args.ldc;
          Wv[it] = *reinterpret_cast<const float4*>(args.sgd_w + o);
          Av[it] = *reinterpret_cast<const float4*>(args.sgd_h + o);
        }
        asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
        __builtin_amdgcn_s_barrier();
#pragma unroll
        for (int it = 0; it < 16; ++it) {
          const int r = it * 8 + r0, lr = r & 63;
          const char* rbuf = r < 64 ? smem0 : smem1;
          const f32x4 v = *reinterpret_cast<const f32x4*>(rbuf + lr * 512 + ((cq ^ (lr & 15)) << 4));
          float W[4] = {Wv[it].x, Wv[it].y, Wv[it].z, Wv[it].w};
          float A[4] = {Av[it].x, Av[it].y, Av[it].z, Av[it].w};
#pragma unroll
          for (int q = 0; q < 4; ++q) {
            float gg = v[q] * gscale;
            gg += decay * ((args.sgd_flags & 2) ? (float)((W[q] > 0.f) - (W[q] < 0.f)) : W[q]);
            const float prev = A[q];
            A[q] = mom * A[q] + rate * gg;
            W[q] -= (args.sgd_flags & 1) ? (1.f + mom) * A[q] - mom * prev : A[q];
          }
          const long long o = ob + (long long)r * args.ldc;
          *reinterpret_cast<float4*>(args.sgd_w + o) = make_float4(W[0], W[1], W[2], W[3]);
          *reinterpret_cast<float4*>(args.sgd_h + o) = make_float4(A[0], A[1], A[2], A[3]);
          *reinterpret_cast<uint2*>(args.sgd_shadow + o) = make_uint2(pack2(W[0], W[1]), pack2(W[2], W[3]));
        }
        return;
      }
    }
    if (interior) {
      const float* hy = args.sgd_hyper;
      const float rate = hy[0] * args.sgd_lr_mult, mom = hy[1], decay = hy[2] * args.sgd_decay_mult;
      const float gscale = hy[4];
      float4 Wv[MFR][NFR], Av[MFR][NFR];
#pragma unroll
      for (int j = 0; j < MFR; ++j)
#pragma unroll
        for (int i = 0; i < NFR; ++i) {
          const long long o = grp * args.c_gstride + (long long)(m_blk + wm0 + wave_m(j)) * args.ldc +
                              n_blk + wn0 + wave_n(i, j);
          Wv[j][i] = *reinterpret_cast<const float4*>(args.sgd_w + o);
          Av[j][i] = *reinterpret_cast<const float4*>(args.sgd_h + o);
        }
#pragma unroll
      for (int j = 0; j < MFR; ++j)
#pragma unroll
        for (int i = 0; i < NFR; ++i) {
          const long long o = grp * args.c_gstride + (long long)(m_blk + wm0 + wave_m(j)) * args.ldc +
                              n_blk + wn0 + wave_n(i, j);
          float W[4] = {Wv[j][i].x, Wv[j][i].y, Wv[j][i].z, Wv[j][i].w};
          float A[4] = {Av[j][i].x, Av[j][i].y, Av[j][i].z, Av[j][i].w};
          const f32x4 v = acc[i][j];
#pragma unroll
          for (int r = 0; r < 4; ++r) {
            float gg = v[r] * gscale;
            gg += decay * ((args.sgd_flags & 2) ? (float)((W[r] > 0.f) - (W[r] < 0.f)) : W[r]);
            const float prev = A[r];
            A[r] = mom * A[r] + rate * gg;
            W[r] -= (args.sgd_flags & 1) ? (1.f + mom) * A[r] - mom * prev : A[r];
          }
          *reinterpret_cast<float4*>(args.sgd_w + o) = make_float4(W[0], W[1], W[2], W[3]);
          *reinterpret_cast<float4*>(args.sgd_h + o) = make_float4(A[0], A[1], A[2], A[3]);
          *reinterpret_cast<uint2*>(args.sgd_shadow + o) = make_uint2(pack2(W[0], W[1]), pack2(W[2], W[3]));
        }
      return;
    }
  }
  if constexpr (epi_bf16<EPI>() && NS == 2 && (BM / 2) * (BN * 2 + 16) <= STAGE) {
    if (args.lds_store) {
      // The MFMA layout stores 16 rows x 8 B per lane group (32-B row pieces per
      // wave-instruction); instead stage the finished bf16 tile in the idle LDS stages
      // (rows of the first M half in smem0, the second in smem1; 16-B row padding keeps
      // the 8-B fragment writes of 16 consecutive rows on distinct banks) and store it as
      // whole 16-B chunks, each wave-instruction covering 1 KB of consecutive rows.
      constexpr int PITCH = BN * 2 + 16, HALF = BM / 2, CPR = BN / 8;
      static_assert(HALF * PITCH <= STAGE, "staged epilogue half-tile must fit one LDS stage");
      __builtin_amdgcn_s_barrier();  // every wave is past its last fragment read of the stages
      char* wbuf = wm0 < HALF ? smem0 : smem1;
#pragma unroll
      for (int j = 0; j < MFR; ++j) {
        const int lr = wm0 + wave_m(j), m = m_blk + lr;
#pragma unroll
        for (int i = 0; i < NFR; ++i) {
          const int nl = wn0 + wave_n(i, j), n = n_blk + nl;
          float o[4] = {0.f, 0.f, 0.f, 0.f};
          if (m < args.M && n < args.N) epi_bf16_math<EPI, (FP8 != 0)>(args, grp, m, n, acc[i][j], args.N, o);
          *reinterpret_cast<uint2*>(wbuf + (lr % HALF) * PITCH + nl * 2) =
              make_uint2(pack2(o[0], o[1]), pack2(o[2], o[3]));
        }
      }
      asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
      __builtin_amdgcn_s_barrier();
      bf16_t* Cb = reinterpret_cast<bf16_t*>(args.C) + grp * args.c_gstride;
      float qmax = 0.f;
      const float qsc = args.q_out ? args.q_slot[0] : 0.f;
      for (int q = tid; q < BM * CPR; q += NW * 64) {
        const int lr = q / CPR, c = q - lr * CPR;
        const int m = m_blk + lr, n = n_blk + c * 8;
        if (m >= args.M || n >= args.N) continue;
        const uint4 v = *reinterpret_cast<const uint4*>((lr < HALF ? smem0 : smem1) + (lr % HALF) * PITCH + c * 16);
        bf16_t* dst = Cb + (long long)m * args.ldc + n;
        if (args.q_out) {  // host: N % 8 == 0 with a side output, so the chunk is whole
          float f[8];
          unpack8(v, f);
          const uint2 w = make_uint2(q_pack4(args, qsc, f, qmax), q_pack4(args, qsc, f + 4, qmax));
          *reinterpret_cast<uint2*>(args.q_out + grp * args.q_gstride + (long long)m * args.q_ld + n) = w;
        }
        if (n + 8 <= args.N) {
          *reinterpret_cast<uint4*>(dst) = v;
        } else {
          const uint32_t w[4] = {v.x, v.y, v.z, v.w};
#pragma unroll
          for (int k = 0; k < 8; ++k)
            if (k < args.N - n) dst[k] = (bf16_t)(w[k >> 1] >> (16 * (k & 1)));
        }
      }
      if (args.q_out) q_amax_flush(args, qmax, smem0);
      return;
    }
  }
  float qmax = 0.f;
#pragma unroll
  for (int j = 0; j < MFR; ++j) {
    const int m = m_blk + wm0 + wave_m(j);
    if (m >= args.M) continue;
#pragma unroll
    for (int i = 0; i < NFR; ++i) {
      const int n = n_blk + wn0 + wave_n(i, j);
      if (n >= args.N) continue;
      epi_store<EPI, (FP8 != 0)>(args, grp, esplit, m, n, acc[i][j], c_cols, epi_bf16<EPI>() ? &qmax : nullptr);
    }
  }
  if (epi_bf16<EPI>() && args.q_out) q_amax_flush(args, qmax, smem0);
}

// ---------------------------------------------------------------------------------------
// gemm256_kernel: 256 x BN block tile (BN = 256 or 128), 8 waves (512 threads), one
// block per CU, phased LDS-DMA pipeline with loads in flight ACROSS barriers.
//
// Each operand tile of a K-step (BK = 64) is staged as two halves (A: rows 0-127 /
// 128-255, B: rows or columns 0..BN/2-1 / BN/2..BN-1), each its own swizzled LDS image
// (same images and reads as gemm_kernel, at TILE = the half size).  A wave owns a
// (2 x MF frags) x (2 x NF frags) sub-tile whose row / column halves come from the two
// LDS halves, so one K-step is four phases over the quadrants (lo,lo) (lo,hi) (hi,hi)
// (hi,lo): the A_lo / B_lo halves are read only in phase 1, B_hi only in phase 2 and
// A_hi only in phase 3, and each half is re-filled (for the K-step two ahead) as soon as
// every wave is past its last read.  The DMA issue stream is one half per phase:
//      P1(t): A_hi(t+1)   P2(t): A_lo(t+2)   P3(t): B_lo(t+2)   P4(t): B_hi(t+2)
// so every half is issued ~6 phases (1.5 K-steps of MFMA) before it is read, and each
// phase waits with a COUNTED vmcnt for exactly the halves it reads (raw s_barrier, no
// vmcnt(0) in the loop: cdna_hip_programming.md §5 "Pipelining across barriers", the
// 256² template of §5).  Phase 4 reads nothing new and needs no barrier.  DMAs past the
// last K-step read the zero page, which keeps the vmcnt arithmetic uniform.
// ---------------------------------------------------------------------------------------
// The four phases are merged pairwise: X = (lo,lo)+(lo,hi) reading A_lo, B_lo, B_hi and
// Y = (hi,hi)+(hi,lo) reading A_hi; DMA stream X(t): A_hi(t+1), Y(t): A_lo, B_lo, B_hi of
// t+2 — two barriers per K-step and twice the MFMAs behind each read burst.  (The unmerged
// 4-phase form and the 8-phase template schedule measured slower on every shape, round 4;
// removed in round 6.)
template <int AMC, int AMODE, int BMC, int BMODE, int EPI, int BN>
__global__ void __launch_bounds__(512, 1) gemm256_kernel(SnGemmArgs args) {
  constexpr int BM = 256, HA = 128, HB = BN / 2, NW = 8;
  constexpr int WM = BN == 256 ? 2 : 4, WN = NW / WM;
  constexpr int MF = HA / (16 * WM), NF = HB / (16 * WN);  // 16-row frags per half
  constexpr int A_HALF = HA * 128, B_HALF = HB * 128;     // bytes (KC and MC images alike)
  constexpr int STAGE = 2 * A_HALF + 2 * B_HALF;
  using SA = GStager<AMC, AMODE, HA, NW>;
  using SB = GStager<BMC, BMODE, HB, NW>;
  constexpr int H_A = SA::NI, H_B = SB::NI;  // DMA instructions per wave per half
  static_assert(MF >= 1 && NF >= 1 && MF * 16 * WM == HA && NF * 16 * WN == HB, "wave layout");
  static_assert(2 * STAGE <= 160 * 1024, "LDS");

  __shared__ __attribute__((aligned(16))) char smem[2 * STAGE];
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int wv = __builtin_amdgcn_readfirstlane(wave);
  const int wr = wv % WM, wc = wv / WM;

  int bid = blockIdx.x;
  const int nwg = gridDim.x;
  if (nwg >= 16) {
    int xcd = bid & 7, qq = nwg >> 3, rr = nwg & 7;
    bid = (xcd < rr ? xcd * (qq + 1) : rr * (qq + 1) + (xcd - rr) * qq) + (bid >> 3);
  }
  const int tiles_m = (args.M + BM - 1) / BM, tiles_n = (args.N + BN - 1) / BN;
  const int tiles = tiles_m * tiles_n;  // 1-D grid over (tile, split, group), as gemm_kernel
  const int tile = bid % tiles, rest = bid / tiles;
  const int split = rest % args.splits, grp = rest / args.splits;
  const int tm = args.raster_n ? tile / tiles_n : tile % tiles_m;
  const int tn = args.raster_n ? tile % tiles_n : tile / tiles_m;
  const int m_blk = tm * BM, n_blk = tn * BN;
  const int k0 = split * args.kchunk, k1 = min(args.K, k0 + args.kchunk);
  const int nk = k1 > k0 ? (k1 - k0 + BK - 1) / BK : 0;
  const int n_lim = min(args.N, n_blk + BN);
  const int ones = BMC ? args.ones_col : -1;

  SA sa_lo, sa_hi;
  SB sb_lo, sb_hi;
  sa_lo.init(args.A, grp, wv, lane, m_blk, args.M, m_blk, args.M, -1, k0, args.K);
  sa_hi.init(args.A, grp, wv, lane, m_blk + HA, args.M, m_blk + HA, args.M, -1, k0, args.K);
  sb_lo.init(args.B, grp, wv, lane, n_blk, n_lim, n_blk, n_lim, ones, k0, args.K);
  sb_hi.init(args.B, grp, wv, lane, n_blk + HB, n_lim, n_blk + HB, n_lim, ones, k0, args.K);

  auto A_lo = [&](int b) { return smem + b * STAGE; };
  auto A_hi = [&](int b) { return smem + b * STAGE + A_HALF; };
  auto B_lo = [&](int b) { return smem + b * STAGE + 2 * A_HALF; };
  auto B_hi = [&](int b) { return smem + b * STAGE + 2 * A_HALF + B_HALF; };
  auto kt = [&](int t) { return k0 + t * BK; };
  auto dma_a_lo = [&](int t) { sa_lo.issue(A_lo(t & 1), wv, kt(t), k1, m_blk, args.M); };
  auto dma_a_hi = [&](int t) { sa_hi.issue(A_hi(t & 1), wv, kt(t), k1, m_blk + HA, args.M); };
  auto dma_b_lo = [&](int t) { sb_lo.issue(B_lo(t & 1), wv, kt(t), k1, n_blk, n_lim); };
  auto dma_b_hi = [&](int t) { sb_hi.issue(B_hi(t & 1), wv, kt(t), k1, n_blk + HB, n_lim); };

  f32x4 acc[2][2][NF][MF];
#pragma unroll
  for (int a = 0; a < 2; ++a)
#pragma unroll
    for (int b = 0; b < 2; ++b)
#pragma unroll
      for (int i = 0; i < NF; ++i)
#pragma unroll
        for (int j = 0; j < MF; ++j) acc[a][b][i][j] = f32x4{0.f, 0.f, 0.f, 0.f};

  bf16x8_t fa[2][MF], fbl[2][NF], fbh[2][NF];
  auto read_a = [&](const char* base) {
#pragma unroll
    for (int s = 0; s < 2; ++s)
#pragma unroll
      for (int j = 0; j < MF; ++j) fa[s][j] = read_frag<AMC, HA>(base, wr * (MF * 16) + 16 * j, s, lane);
  };
  auto read_b = [&](bf16x8_t (&fb)[2][NF], const char* base) {
#pragma unroll
    for (int s = 0; s < 2; ++s)
#pragma unroll
      for (int i = 0; i < NF; ++i) fb[s][i] = read_frag<BMC, HB>(base, wc * (NF * 16) + 16 * i, s, lane);
  };
  auto mma = [&](f32x4 (&c)[NF][MF], const bf16x8_t (&fb)[2][NF]) {
    __builtin_amdgcn_s_setprio(1);
#pragma unroll
    for (int s = 0; s < 2; ++s)
#pragma unroll
      for (int i = 0; i < NF; ++i)
#pragma unroll
        for (int j = 0; j < MF; ++j) c[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(fb[s][i], fa[s][j], c[i][j], 0, 0, 0);
    __builtin_amdgcn_s_setprio(0);
  };

  if (nk > 0) {
    // prologue: K-step 0 whole, K-step 1 without A_hi (issued in P1(0))
    dma_a_lo(0);
    dma_b_lo(0);
    dma_b_hi(0);
    dma_a_hi(0);
    dma_a_lo(1);
    dma_b_lo(1);
    dma_b_hi(1);
    {
      constexpr int VMX = 2 * H_A + 2 * H_B;
      // prologue above also issued B_hi(1) and A_hi(0): the stream matches X/Y's
      for (int t = 0; t < nk; ++t) {
        const int b = t & 1;
        // X: needs A_lo(t), B_lo(t), B_hi(t)
        __builtin_amdgcn_s_waitcnt(waitcnt_vm(VMX));
        asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
        __builtin_amdgcn_s_barrier();
        dma_a_hi(t + 1);
        read_a(A_lo(b));
        read_b(fbl, B_lo(b));
        read_b(fbh, B_hi(b));
        mma(acc[0][0], fbl);
        mma(acc[0][1], fbh);
        // Y: needs A_hi(t); A_lo / B_lo / B_hi of buffer b are free after this barrier
        __builtin_amdgcn_s_waitcnt(waitcnt_vm(VMX));
        asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
        __builtin_amdgcn_s_barrier();
        dma_a_lo(t + 2);
        dma_b_lo(t + 2);
        dma_b_hi(t + 2);
        read_a(A_hi(b));
        mma(acc[1][1], fbh);
        mma(acc[1][0], fbl);
      }
    }
    // no LDS-DMA may still be landing when the workgroup retires
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  }

  const int mrow_l = lane & 15, ncol_l = (lane >> 4) * 4;
  const int c_cols = (!epi_bf16<EPI>() && args.bias_out) ? args.ones_col : args.N;
#pragma unroll
  for (int mh = 0; mh < 2; ++mh)
#pragma unroll
    for (int j = 0; j < MF; ++j) {
      const int m = m_blk + mh * HA + wr * (MF * 16) + 16 * j + mrow_l;
      if (m >= args.M) continue;
#pragma unroll
      for (int nh = 0; nh < 2; ++nh)
#pragma unroll
        for (int i = 0; i < NF; ++i) {
          const int n = n_blk + nh * HB + wc * (NF * 16) + 16 * i + ncol_l;
          if (n >= args.N) continue;
          epi_store<EPI, false>(args, grp, split, m, n, acc[mh][nh][i][j], c_cols);
        }
    }
}

template <int AMC, int AMODE, int BMC, int BMODE, int BN>
int launch256_epi(const SnGemmArgs& a, dim3 grid, hipStream_t st) {
  switch (a.epi) {
    case EPI_BF16:
      hipLaunchKernelGGL((gemm256_kernel<AMC, AMODE, BMC, BMODE, EPI_BF16, BN>), grid, dim3(512), 0, st, a);
      break;
    case EPI_F32:
      hipLaunchKernelGGL((gemm256_kernel<AMC, AMODE, BMC, BMODE, EPI_F32, BN>), grid, dim3(512), 0, st, a);
      break;
    case EPI_F32_ACC:
      hipLaunchKernelGGL((gemm256_kernel<AMC, AMODE, BMC, BMODE, EPI_F32_ACC, BN>), grid, dim3(512), 0, st, a);
      break;
    default:
      return 2;
  }
  return SN_CHECK_LAUNCH();
}

template <int BN>
int launch256(const SnGemmArgs& a, hipStream_t stream) {
  const int tiles = ((a.M + 255) / 256) * ((a.N + BN - 1) / BN);
  dim3 grid(tiles * a.splits * a.groups);
  const int key = (a.a_mc << 3) | (a.a_mode << 2) | (a.b_mc << 1) | a.b_mode;
  switch (key) {
    case 0b0000: return launch256_epi<0, OP_DENSE, 0, OP_DENSE, BN>(a, grid, stream);   // NT dense
    case 0b0100: return launch256_epi<0, OP_IM2COL, 0, OP_DENSE, BN>(a, grid, stream);  // conv fwd / dgrad
    case 0b0010: return launch256_epi<0, OP_DENSE, 1, OP_DENSE, BN>(a, grid, stream);   // NN dense
    case 0b1010: return launch256_epi<1, OP_DENSE, 1, OP_DENSE, BN>(a, grid, stream);   // TN dense
    case 0b1011: return launch256_epi<1, OP_DENSE, 1, OP_IM2COL, BN>(a, grid, stream);  // conv wgrad
    default: break;
  }
  return 4;
}

template <int AMC, int AMODE, int BMC, int BMODE, int BM, int BN, int NW, int NS, int NFR = 4, int MFR = 4>
int launch_epi(const SnGemmArgs& a, dim3 grid, hipStream_t st) {
  switch (a.epi) {
    case EPI_BF16:
      hipLaunchKernelGGL((gemm_kernel<AMC, AMODE, BMC, BMODE, EPI_BF16, BM, BN, NW, NS, false, NFR, MFR>), grid,
                         dim3(NW * 64), 0, st, a);
      break;
    case EPI_BF16_DROP:  // InnerProduct forward only (dense NT)
      if (AMC || AMODE != OP_DENSE || BMC || BMODE != OP_DENSE) return 4;
      hipLaunchKernelGGL((gemm_kernel<0, OP_DENSE, 0, OP_DENSE, EPI_BF16_DROP, BM, BN, NW, NS, false, NFR, MFR>),
                         grid, dim3(NW * 64), 0, st, a);
      break;
    case EPI_F32:
      hipLaunchKernelGGL((gemm_kernel<AMC, AMODE, BMC, BMODE, EPI_F32, BM, BN, NW, NS, false, NFR, MFR>), grid,
                         dim3(NW * 64), 0, st, a);
      break;
    case EPI_F32_ACC:
      hipLaunchKernelGGL((gemm_kernel<AMC, AMODE, BMC, BMODE, EPI_F32_ACC, BM, BN, NW, NS, false, NFR, MFR>),
                         grid, dim3(NW * 64), 0, st, a);
      break;
    default:
      return 2;
  }
  return SN_CHECK_LAUNCH();
}

template <int BM, int BN, int NW, int NS>
int launch_tile(const SnGemmArgs& a, hipStream_t stream) {
  const int tiles = ((a.M + BM - 1) / BM) * ((a.N + BN - 1) / BN);
  dim3 grid(tiles * a.splits * a.groups);
  const int key = (a.a_mc << 3) | (a.a_mode << 2) | (a.b_mc << 1) | a.b_mode;
  if (a.epi == EPI_SGD) {  // fused solver update: InnerProduct weight gradient (TN dense) only
    if (key != 0b1010 || a.splits != 1 || !a.sgd_w || !a.sgd_h || !a.sgd_shadow || !a.sgd_hyper) return 6;
    hipLaunchKernelGGL((gemm_kernel<1, OP_DENSE, 1, OP_DENSE, EPI_SGD, BM, BN, NW, NS>), grid, dim3(NW * 64), 0, stream,
                       a);
    return SN_CHECK_LAUNCH();
  }
  switch (key) {
    case 0b0000: return launch_epi<0, OP_DENSE, 0, OP_DENSE, BM, BN, NW, NS>(a, grid, stream);   // NT dense
    case 0b0100: return launch_epi<0, OP_IM2COL, 0, OP_DENSE, BM, BN, NW, NS>(a, grid, stream);  // conv fwd/dgrad
    case 0b0010: return launch_epi<0, OP_DENSE, 1, OP_DENSE, BM, BN, NW, NS>(a, grid, stream);   // NN dense
    case 0b1010: return launch_epi<1, OP_DENSE, 1, OP_DENSE, BM, BN, NW, NS>(a, grid, stream);   // TN dense
    case 0b1011: return launch_epi<1, OP_DENSE, 1, OP_IM2COL, BM, BN, NW, NS>(a, grid, stream);  // conv wgrad
    case 0b1000: return launch_epi<1, OP_DENSE, 0, OP_DENSE, BM, BN, NW, NS>(a, grid, stream);
    default: break;
  }
  if (a.a_mc == 0 && a.a_mode == OP_IM2COL && a.b_mc == 1 && a.b_mode == OP_FLIPW)  // conv dgrad
    return launch_epi<0, OP_IM2COL, 1, OP_FLIPW, BM, BN, NW, NS>(a, grid, stream);
  return 4;
}

// 8-wave tiles with 256 rows, 2 LDS stages, one block per CU (tiles 11-14): the block
// tile halves (256x256) or cuts by a quarter to a third (256x128, 256x192) the L2 -> LDS
// bytes and LDS-DMA instructions per MFMA of the 128x128 tile, whose operand traffic (not
// its MFMA rate) bounds it on the implicit-conv products.
template <int BM, int BN, int MFR, int NFR, int NW = 8>
int launch_big(const SnGemmArgs& a, hipStream_t stream) {
  const int tiles = ((a.M + BM - 1) / BM) * ((a.N + BN - 1) / BN);
  dim3 grid(tiles * a.splits * a.groups);
  const int key = (a.a_mc << 3) | (a.a_mode << 2) | (a.b_mc << 1) | a.b_mode;
  constexpr bool mc_b_ok = (BN / 8) == 8 || (BN / 8) == 16 || (BN / 8) == 32;  // MC images: 64 % chunks per row == 0
  constexpr bool mc_a_ok = (BM / 8) == 8 || (BM / 8) == 16 || (BM / 8) == 32;
  switch (key) {
    case 0b0000: return launch_epi<0, OP_DENSE, 0, OP_DENSE, BM, BN, NW, 2, NFR, MFR>(a, grid, stream);   // NT dense
    case 0b0100: return launch_epi<0, OP_IM2COL, 0, OP_DENSE, BM, BN, NW, 2, NFR, MFR>(a, grid, stream);  // conv fwd/dgrad
    default: break;
  }
  if constexpr (mc_b_ok) {
    switch (key) {
      case 0b0010: return launch_epi<0, OP_DENSE, 1, OP_DENSE, BM, BN, NW, 2, NFR, MFR>(a, grid, stream);   // NN dense
      default: break;
    }
    if constexpr (mc_a_ok) {
      switch (key) {
        case 0b1010: return launch_epi<1, OP_DENSE, 1, OP_DENSE, BM, BN, NW, 2, NFR, MFR>(a, grid, stream);   // TN dense
        case 0b1011: return launch_epi<1, OP_DENSE, 1, OP_IM2COL, BM, BN, NW, 2, NFR, MFR>(a, grid, stream);  // conv wgrad
        default: break;
      }
    }
  }
  return 4;
}


}  // namespace

// tile families compiled in their own translation units
int sn_gemm_tiles_b(const SnGemmArgs& a, hipStream_t stream);
int sn_gemm_t256(const SnGemmArgs& a, hipStream_t stream);
int sn_gemm_big8(const SnGemmArgs& a, hipStream_t stream);
int sn_gemm_big4(const SnGemmArgs& a, hipStream_t stream);
int sn_gemm_fp8_big(const SnGemmArgs& a, hipStream_t stream);
int sn_gemm_tiles_c(const SnGemmArgs& a, hipStream_t stream);
