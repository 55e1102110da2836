// Persistent, ring-pipelined MFMA GEMM (tiles 30-37): the round-4 mainloop.
//
// Why a second kernel family: the one-shot tiles of gemm_impl.h prefetch ONE K-step
// (two LDS stages) per block and pay a full DMA round trip per output tile (prologue),
// which leaves the conv products latency-bound at ~35 % MFMA busy
// (profiles/r3_pmc_conv3_fwd.txt).  Here
//   * one 512-thread block per CU loops over its share of the output tiles (persistent);
//   * the LDS holds an NS-slot ring of K-step stages (BK = 64, same swizzled images and
//     fragment reads as gemm_impl.h) and the loader runs NS-1 stages ahead of the MFMAs
//     as ONE flat stream over (tile, k-step): the first stages of the next tile are in
//     flight during the current tile's last K-steps and its epilogue;
//   * every wait is a counted vmcnt followed by a raw s_barrier (no vmcnt(0) in the
//     loop: cdna_hip_programming.md §5 "Pipelining across barriers");
//   * the 32 blocks of one XCD stride through a contiguous share of the tile order, so the
//     tiles in flight on an XCD at any time are neighbours that share operand panels in its
//     L2 (a contiguous run PER BLOCK measured 10-40 % slower: 32 distant panels per L2);
//   * the fragments of the next K-step's first half are read from LDS right after its
//     barrier, while the MFMAs of the current K-step's second half are in the pipe: the
//     two waves of a SIMD belong to the same block and would otherwise both sit in the
//     read phase with the matrix pipe idle.
// The reference runs these products as per-image im2col + SGEMM
// (caffe/src/caffe/layers/base_conv_layer.cpp:312-376, conv_layer.cu:14-56,
//  inner_product_layer.cu:22-54).
#pragma once
#include "gemm_impl.h"

namespace {

// wait until at most `after` stages of P DMA instructions each are still outstanding
template <int P>
SN_DEV void pk_wait_stages(int after) {
  if (after <= 0)
    __builtin_amdgcn_s_waitcnt(waitcnt_vm(0));
  else if (after == 1)
    __builtin_amdgcn_s_waitcnt(waitcnt_vm(P));
  else if (after == 2)
    __builtin_amdgcn_s_waitcnt(waitcnt_vm(2 * P));
  else
    __builtin_amdgcn_s_waitcnt(waitcnt_vm(3 * P));
}

struct PkItem {
  int m_blk, n_blk, n_lim, grp, split, k0, k1, nk;
};

SN_DEV PkItem pk_decode(const SnGemmArgs& a, int it, int BMv, int BNv) {
  const int tiles_m = (a.M + BMv - 1) / BMv, tiles_n = (a.N + BNv - 1) / BNv;
  const int tiles = tiles_m * tiles_n;
  const int tile = it % tiles, rest = it / tiles;
  PkItem r;
  r.split = rest % a.splits;
  r.grp = rest / a.splits;
  const int tm = a.raster_n ? tile / tiles_n : tile % tiles_m;
  const int tn = a.raster_n ? tile % tiles_n : tile / tiles_m;
  r.m_blk = tm * BMv;
  r.n_blk = tn * BNv;
  r.n_lim = min(a.N, r.n_blk + BNv);
  r.k0 = r.split * a.kchunk;
  r.k1 = min(a.K, r.k0 + a.kchunk);
  r.nk = r.k1 > r.k0 ? (r.k1 - r.k0 + BK - 1) / BK : 0;
  return r;
}

// BM x BN block tile, 8 waves laid out WM (along M) x 8/WM (along N), each wave owning
// (16 MFR) x (16 NFR) outputs; NS LDS stages of (BM + BNL) x 128 B.
// LOOP 0: two wave groups staggered by one barrier (below); 1: one barrier per K-step,
// fragments of the whole K-step read, then its MFMAs (A/B probe of the stagger)
template <int AMC, int AMODE, int BMC, int BMODE, int EPI, int BM, int BN, int WM, int MFR, int NFR, int NS,
          int LOOP = 0>
__global__ void __launch_bounds__(512, 1) gemm_pk_kernel(SnGemmArgs args) {
  constexpr int NW = 8, WN = NW / WM;
  constexpr int BNL = (BN + 63) / 64 * 64;
  constexpr int A_BYTES = BM * 128, B_BYTES = BNL * 128, STAGE = A_BYTES + B_BYTES;
  static_assert(WM * WN == NW && WM * 16 * MFR == BM && WN * 16 * NFR == BN, "tile / wave layout");
  static_assert(NS >= 2 && NS <= 5 && NS * STAGE <= 160 * 1024, "LDS ring");
  using SA = GStager<AMC, AMODE, BM, NW>;
  using SB = GStager<BMC, BMODE, BNL, NW>;
  constexpr int P = SA::NI + SB::NI;  // LDS-DMA instructions per wave per stage
  constexpr int D = NS - 1;           // stages in flight ahead of the one being computed
  static_assert(3 * P < 64, "vmcnt range");

  __shared__ __attribute__((aligned(16))) char smem[NS * STAGE];
  const int tid = threadIdx.x, lane = tid & 63;
  const int wv = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int wm0 = (wv % WM) * (16 * MFR), wn0 = (wv / WM) * (16 * NFR);

  // this block's items: a contiguous run of its XCD's share of the item order (blocks b and
  // b + 8 share an XCD under round-robin dispatch; speed only, any placement is correct)
  const int tiles = ((args.M + BM - 1) / BM) * ((args.N + BN - 1) / BN);
  const int total = tiles * args.splits * args.groups;
  const int G = gridDim.x;
  int first, stride, count;
  if (G >= 16 && (G & 7) == 0) {
    const int xcd = blockIdx.x & 7, loc = blockIdx.x >> 3, nloc = G >> 3;
    const int q = total >> 3, r = total & 7;
    const int cstart = xcd < r ? xcd * (q + 1) : r * (q + 1) + (xcd - r) * q;
    const int csize = q + (xcd < r ? 1 : 0);
    first = cstart + loc;
    stride = nloc;
    count = loc < csize ? (csize - loc + nloc - 1) / nloc : 0;
  } else {
    first = blockIdx.x;
    stride = G;
    count = first < total ? (total - first + G - 1) / G : 0;
  }
  first = __builtin_amdgcn_readfirstlane(first);
  count = __builtin_amdgcn_readfirstlane(count);
  if (count <= 0) return;

  // ---- loader: one flat stream of K-step stages over this block's items ----
  SA sa;
  SB sb;
  int l_ord = 0, l_k = 0;
  PkItem L = pk_decode(args, first, BM, BN);
  const int ones = BMC ? args.ones_col : -1;
  auto loader_init = [&]() {
    sa.init(args.A, L.grp, wv, lane, L.m_blk, args.M, L.m_blk, args.M, -1, L.k0, args.K, args.addr_legacy);
    sb.init(args.B, L.grp, wv, lane, L.n_blk, L.n_lim, L.n_blk, L.n_lim, ones, L.k0, args.K, args.addr_legacy);
  };
  loader_init();
  auto issue_next = [&](char* st) -> int {
    if (l_ord >= count) return 0;
    const int kt = L.k0 + l_k * BK;
    sa.issue(st, wv, kt, L.k1, L.m_blk, args.M);
    sb.issue(st + A_BYTES, wv, kt, L.k1, L.n_blk, L.n_lim);
    if (++l_k >= L.nk) {
      l_k = 0;
      if (++l_ord < count) {
        L = pk_decode(args, first + l_ord * stride, BM, BN);
        loader_init();
      }
    }
    return 1;
  };

  f32x4 acc[NFR][MFR];
#pragma unroll
  for (int i = 0; i < NFR; ++i)
#pragma unroll
    for (int j = 0; j < MFR; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};

  // fragments of one 32-deep k-substep: F[0] = A (MFR), F[1..] = B (NFR)
  struct Frags {
    bf16x8_t a[MFR], b[NFR];
  };
  auto read_sub = [&](Frags& f, const char* la, int sub) {
    const char* lb = la + A_BYTES;
#pragma unroll
    for (int i = 0; i < NFR; ++i) f.b[i] = read_frag<BMC, BNL>(lb, wn0 + 16 * i, sub, lane);
#pragma unroll
    for (int i = 0; i < MFR; ++i) f.a[i] = read_frag<AMC, BM>(la, wm0 + 16 * i, sub, lane);
  };
  auto mma_sub = [&](const Frags& f) {
    __builtin_amdgcn_s_setprio(1);
#pragma unroll
    for (int i = 0; i < NFR; ++i)
#pragma unroll
      for (int j = 0; j < MFR; ++j) acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(f.b[i], f.a[j], acc[i][j], 0, 0, 0);
    __builtin_amdgcn_s_setprio(0);
  };

  // ---- compute: consume the ring in order ----
  int issued = 0;
#pragma unroll
  for (int d = 0; d < D; ++d) issued += issue_next(smem + d * STAGE);

  int c_ord = 0, c_k = 0, step = 0;
  PkItem Cc = pk_decode(args, first, BM, BN);
  const int mrow_l = lane & 15, ncol_l = (lane >> 4) * 4;
  const int c_cols = (!epi_bf16<EPI>() && args.bias_out) ? args.ones_col : args.N;
  auto epilogue = [&]() {
#pragma unroll
    for (int j = 0; j < MFR; ++j) {
      const int m = Cc.m_blk + wm0 + 16 * j + mrow_l;
      if (m >= args.M) continue;
#pragma unroll
      for (int i = 0; i < NFR; ++i) {
        const int n = Cc.n_blk + wn0 + 16 * i + ncol_l;
        if (n >= args.N) continue;
        epi_store<EPI, false>(args, Cc.grp, Cc.split, m, n, acc[i][j], c_cols);
      }
    }
#pragma unroll
    for (int i = 0; i < NFR; ++i)
#pragma unroll
      for (int j = 0; j < MFR; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};
  };

  // Two wave groups staggered by one barrier (cdna_hip_programming.md §5, the 256^2
  // template's `if (wr == 1) s_barrier`; MI355X_MICROARCH.md "Two waves per SIMD", item 9):
  // waves 0-3 and 4-7 sit on different SIMDs in pairs, and every K-step is two phases per
  // k-substep, R (fragment reads [+ the ring refill]) | barrier | C (MFMAs) | barrier.  With
  // group B one barrier behind, each SIMD runs group A's C beside group B's R and vice
  // versa, so the matrix pipe is not idle while fragments are read.
  //   stage k is read in phases 2k, 2k+1; group A's first read of it follows global barrier
  //   4k+1, so EVERY wave retires its own DMAs of stage k before arriving there: group A at
  //   the end of C(2k-1), group B at the end of R(2k-1).  The refill of stage k's slot
  //   (stage k + NS) is issued in the R phase of step k+1, after group B's last read of
  //   stage k (R(2k+1)) has passed a barrier.
  if constexpr (LOOP == 1) {
    Frags g0, g1;
    while (c_ord < count) {
      pk_wait_stages<P>(issued - step - 1);
      asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
      __builtin_amdgcn_s_barrier();
      {
        const int ns = step % NS == 0 ? NS - 1 : step % NS - 1;  // (step + D) % NS
        issued += issue_next(smem + ns * STAGE);
      }
      const char* cur = smem + (step % NS) * STAGE;
      read_sub(g0, cur, 0);
      read_sub(g1, cur, 1);
      mma_sub(g0);
      mma_sub(g1);
      ++step;
      if (++c_k >= Cc.nk) {
        epilogue();
        c_k = 0;
        if (++c_ord < count) Cc = pk_decode(args, first + c_ord * stride, BM, BN);
      }
    }
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    return;
  }
  const bool gB = wv >= 4;
  Frags f;
  pk_wait_stages<P>(issued - 1);
  asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
  __builtin_amdgcn_s_barrier();  // stage 0 landed for every wave
  if (gB) __builtin_amdgcn_s_barrier();  // the stagger
  int slot = 0, pslot = NS - 1;  // ring slots of `step` and of step - 1
  while (true) {
    const char* cur = smem + slot * STAGE;
    const bool last_k = c_k + 1 >= Cc.nk;
    const bool more = !last_k || c_ord + 1 < count;
    // ---- k-substep 0 ----
    issued += issue_next(smem + pslot * STAGE);  // stage step + NS - 1 into step - 1's slot
    read_sub(f, cur, 0);
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    __builtin_amdgcn_s_barrier();
    mma_sub(f);
    __builtin_amdgcn_s_barrier();
    // ---- k-substep 1 ----
    read_sub(f, cur, 1);
    if (gB) pk_wait_stages<P>(issued - step - 2);  // stage step + 1 (group B: end of R)
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    __builtin_amdgcn_s_barrier();
    mma_sub(f);
    if (!gB) pk_wait_stages<P>(issued - step - 2);  // stage step + 1 (group A: end of C)
    __builtin_amdgcn_s_barrier();
    if (last_k) {
      epilogue();  // item c_ord; the next items' first stages are already in flight
      c_k = 0;
      if (++c_ord < count) Cc = pk_decode(args, first + c_ord * stride, BM, BN);
    } else {
      ++c_k;
    }
    if (!more) break;
    ++step;
    pslot = slot;
    slot = slot == NS - 1 ? 0 : slot + 1;
  }
  if (!gB) __builtin_amdgcn_s_barrier();  // both groups execute the same number of barriers
  // nothing may still be landing in LDS when the workgroup retires
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
}

int pk_grid_cap() {
  static int cus = 0;
  if (cus == 0) {
    int dev = 0, n = 0;
    if (hipGetDevice(&dev) == hipSuccess && hipDeviceGetAttribute(&n, hipDeviceAttributeMultiprocessorCount, dev) == hipSuccess && n > 0)
      cus = n;
    else
      cus = 256;
  }
  return cus;
}

template <int AMC, int AMODE, int BMC, int BMODE, int BM, int BN, int WM, int MFR, int NFR, int NS, int LOOP = 0>
int pk_launch_epi(const SnGemmArgs& a, hipStream_t st) {
  const long long tiles = (long long)((a.M + BM - 1) / BM) * ((a.N + BN - 1) / BN);
  const long long total = tiles * a.splits * a.groups;
  if (total <= 0 || total >= (1ll << 31)) return 3;
  const int cap = pk_grid_cap();
  const dim3 grid((unsigned)(total < cap ? total : cap));
  switch (a.epi) {
    case EPI_BF16:
      hipLaunchKernelGGL((gemm_pk_kernel<AMC, AMODE, BMC, BMODE, EPI_BF16, BM, BN, WM, MFR, NFR, NS, LOOP>), grid, dim3(512),
                         0, st, a);
      break;
    case EPI_F32:
      hipLaunchKernelGGL((gemm_pk_kernel<AMC, AMODE, BMC, BMODE, EPI_F32, BM, BN, WM, MFR, NFR, NS, LOOP>), grid, dim3(512),
                         0, st, a);
      break;
    case EPI_F32_ACC:
      hipLaunchKernelGGL((gemm_pk_kernel<AMC, AMODE, BMC, BMODE, EPI_F32_ACC, BM, BN, WM, MFR, NFR, NS, LOOP>), grid,
                         dim3(512), 0, st, a);
      break;
    case EPI_BF16_DROP:  // InnerProduct forward only (dense NT)
      if constexpr (AMC == 0 && AMODE == OP_DENSE && BMC == 0 && BMODE == OP_DENSE) {
        hipLaunchKernelGGL((gemm_pk_kernel<0, OP_DENSE, 0, OP_DENSE, EPI_BF16_DROP, BM, BN, WM, MFR, NFR, NS, LOOP>), grid,
                           dim3(512), 0, st, a);
        break;
      }
      return 4;
    default:
      return 2;
  }
  return SN_CHECK_LAUNCH();
}

// LOOP 1 probe instances: NT dense and conv fwd only
template <int BM, int BN, int WM, int MFR, int NFR, int NS>
int pk_launch_probe(const SnGemmArgs& a, hipStream_t stream) {
  const int key = (a.a_mc << 3) | (a.a_mode << 2) | (a.b_mc << 1) | a.b_mode;
  if (key == 0b0000) return pk_launch_epi<0, OP_DENSE, 0, OP_DENSE, BM, BN, WM, MFR, NFR, NS, 1>(a, stream);
  if (key == 0b0100) return pk_launch_epi<0, OP_IM2COL, 0, OP_DENSE, BM, BN, WM, MFR, NFR, NS, 1>(a, stream);
  return 4;
}

// operand combinations: NT dense, conv fwd / dgrad (implicit im2col A x K-contiguous
// weights), NN dense, TN dense, conv wgrad (dy^T x implicit im2col), conv dgrad with the
// flipped-weight B operand
template <int BM, int BN, int WM, int MFR, int NFR, int NS>
int pk_launch(const SnGemmArgs& a, hipStream_t stream) {
  const int key = (a.a_mc << 3) | (a.a_mode << 2) | (a.b_mc << 1) | a.b_mode;
  if (a.K <= 0) return 3;
  switch (key) {
    case 0b0000: return pk_launch_epi<0, OP_DENSE, 0, OP_DENSE, BM, BN, WM, MFR, NFR, NS>(a, stream);
    case 0b0100: return pk_launch_epi<0, OP_IM2COL, 0, OP_DENSE, BM, BN, WM, MFR, NFR, NS>(a, stream);
    default: break;
  }
  // MC (reduction-strided) images need whole LDS rows per DMA instruction
  constexpr int BNL = (BN + 63) / 64 * 64;
  constexpr bool mc_b = BNL == 64 || BNL == 128 || BNL == 256;
  constexpr bool mc_a = BM == 64 || BM == 128 || BM == 256;
  if constexpr (mc_b) {
    if (key == 0b0010) return pk_launch_epi<0, OP_DENSE, 1, OP_DENSE, BM, BN, WM, MFR, NFR, NS>(a, stream);
    if (a.a_mc == 0 && a.a_mode == OP_IM2COL && a.b_mc == 1 && a.b_mode == OP_FLIPW)
      return pk_launch_epi<0, OP_IM2COL, 1, OP_FLIPW, BM, BN, WM, MFR, NFR, NS>(a, stream);
    if constexpr (mc_a) {
      if (key == 0b1010) return pk_launch_epi<1, OP_DENSE, 1, OP_DENSE, BM, BN, WM, MFR, NFR, NS>(a, stream);
      if (key == 0b1011) return pk_launch_epi<1, OP_DENSE, 1, OP_IM2COL, BM, BN, WM, MFR, NFR, NS>(a, stream);
    }
  }
  return 4;
}

}  // namespace
