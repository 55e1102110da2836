// B-direct MFMA GEMM (tiles 21 / 22): 128x128 block tile, 4 waves of 64x64, for products
// whose B operand is a dense K-contiguous matrix — convolution forward (B = the filters
// W[K][R*S*C]) and the InnerProduct forward (B = the weights [N][K]).
//
// Why: in gemm_kernel every K-step's operands go global -> LDS (LDS-DMA) -> registers, and
// with 2 x 32 KB LDS stages per block only ONE K-step is in flight; the LDS-DMA takes
// longer to land than the 512 MFMA cycles of a K-step (PMC on conv3: MFMA busy 35 %,
// profiles/r3_pmc_conv3_fwd.txt).  Here B never touches LDS: each lane loads its own
// 16x16x32 B fragments (16 B = 8 consecutive k of one weight row) straight into VGPRs
// with buffer loads, NSA - 1 K-steps ahead, into a register ring; only A is staged through
// LDS (16 KB per stage), so NSA = 3 or 4 A stages still fit two blocks per CU and NSA - 1
// K-steps of both operands are in flight per block.  B rows read by the two waves along M
// are fetched twice (served by L1/L2); LDS traffic per MFMA halves.
//
// Waits: the A tile of step kt is retired with a counted vmcnt (every step issues the same
// 4 A + 8 B loads — steps past the end load zeros — so the count is a constant) before the
// barrier; the B loads are compiler-visible (__builtin_amdgcn_raw_buffer_load_b128), so the
// compiler's own wait before the MFMAs that read them is correct (it cannot see the A
// LDS-DMAs, which only makes its count conservative).
#include "gemm_impl.h"

namespace {

template <int AMODE, int EPI, int NSA>
__global__ void __launch_bounds__(256, 2) gemm_bdir_kernel(SnGemmArgs args) {
  constexpr int BM = 128, BN = 128, NW = 4, MFR = 4, NFR = 4, WM = 2;
  constexpr int A_BYTES = BM * 128;
  constexpr int D = NSA - 1;  // K-steps in flight ahead of the one being computed
  __shared__ __attribute__((aligned(16))) char smem0[A_BYTES];
  __shared__ __attribute__((aligned(16))) char smem1[A_BYTES];
  __shared__ __attribute__((aligned(16))) char smem2[A_BYTES];
  __shared__ __attribute__((aligned(16))) char smem3[NSA >= 4 ? A_BYTES : 16];
  char* const stages[4] = {smem0, smem1, smem2, smem3};
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int tiles_m = (args.M + BM - 1) / BM;
  int bid = blockIdx.x;
  const int nwg = gridDim.x;
  if (nwg >= 16) {  // XCD-aware bijective remap (gemm_kernel)
    int xcd = bid & 7, qq = nwg >> 3, rr = nwg & 7;
    bid = (xcd < rr ? xcd * (qq + 1) : rr * (qq + 1) + (xcd - rr) * qq) + (bid >> 3);
  }
  const int tiles_n = (args.N + BN - 1) / BN;
  const int tiles = tiles_m * tiles_n;
  const int tile = bid % tiles, rest = bid / tiles;
  const int split = rest % args.splits, grp = rest / args.splits;
  const int tm = args.raster_n ? tile / tiles_n : tile % tiles_m;
  const int tn = args.raster_n ? tile % tiles_n : tile / tiles_m;
  const int m_blk = tm * BM, n_blk = tn * BN;
  const int k0 = split * args.kchunk;
  const int k1 = min(args.K, k0 + args.kchunk);
  const int nk = k1 > k0 ? (k1 - k0 + BK - 1) / BK : 0;
  const int wv = __builtin_amdgcn_readfirstlane(wave);

  using SA = GStager<0, AMODE, BM, NW, 2>;
  SA sa;
  sa.init(args.A, grp, wv, lane, m_blk, args.M, m_blk, args.M, -1, k0, args.K, args.addr_legacy);

  const int wm0 = (wave % WM) * (16 * MFR), wn0 = (wave / WM) * (16 * NFR);
  const int n_lim = min(args.N, n_blk + BN);
  // B: lane (l & 15) of fragment i reads weight row n_blk + wn0 + 16 i + (l & 15), k chunk
  // 8 (l >> 4) (+ 32 s): a fixed byte offset per (lane, i), the K advance in soffset
  const char* bbase = reinterpret_cast<const char*>(args.B.ptr) + (long long)grp * args.B.gstride * 2;
  const __amdgpu_buffer_rsrc_t brs =
      __builtin_amdgcn_make_buffer_rsrc(const_cast<char*>(bbase), (short)0, 0x7fffffff, 0x00020000);
  constexpr unsigned OOB = 0x7fffffffu;
  unsigned boff[NFR];
  const int kl = 8 * (lane >> 4);
#pragma unroll
  for (int i = 0; i < NFR; ++i) {
    const int n = n_blk + wn0 + 16 * i + (lane & 15);
    boff[i] = n < n_lim ? (unsigned)(((long long)n * args.B.ld + kl) * 2) : OOB;
  }
  i32x4 breg[NSA][2][NFR];
  auto load_b = [&](auto SET, int kt) {
    constexpr int set = decltype(SET)::value;
    const int kb = k0 + kt * BK;
    const unsigned so = __builtin_amdgcn_readfirstlane((unsigned)kb * 2u);
    const bool tail = kb + BK > k1;
#pragma unroll
    for (int s = 0; s < 2; ++s)
#pragma unroll
      for (int i = 0; i < NFR; ++i) {
        unsigned o = boff[i] + 64u * s;
        if (tail && kb + 32 * s + kl >= k1) o = OOB;
        if (boff[i] == OOB) o = OOB;
        breg[set][s][i] = __builtin_amdgcn_raw_buffer_load_b128(brs, (int)o, (int)so, 0);
      }
  };

  f32x4 acc[NFR][MFR];
#pragma unroll
  for (int i = 0; i < NFR; ++i)
#pragma unroll
    for (int j = 0; j < MFR; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};

  // prologue: K-steps 0 .. D-1 (B then A per step: the compiler's conservative B wait then
  // over-waits only by the A loads it cannot see)
  load_b(std::integral_constant<int, 0>{}, 0);
  sa.issue(stages[0], wv, k0, k1, m_blk, args.M);
  load_b(std::integral_constant<int, 1>{}, 1);
  sa.issue(stages[1], wv, k0 + BK, k1, m_blk, args.M);
  if constexpr (D >= 3) {
    load_b(std::integral_constant<int, 2>{}, 2);
    sa.issue(stages[2], wv, k0 + 2 * BK, k1, m_blk, args.M);
  }

  constexpr int PER_STEP = SA::NI + 2 * NFR;  // VMEM instructions per wave per K-step
  auto step = [&](auto PP, int kt) {
    constexpr int p = decltype(PP)::value;  // kt % NSA
    constexpr int pn = (p + D) % NSA;       // ring slot of step kt + D
    // A(kt) landed for this wave (per step: B loads, then A): the D - 1 later steps'
    // loads may stay in flight
    __builtin_amdgcn_s_waitcnt(waitcnt_vm(PER_STEP * (D - 1)));
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    __builtin_amdgcn_s_barrier();  // A(kt) landed for every wave; slot pn (step kt-1) is free
    load_b(std::integral_constant<int, pn>{}, kt + D);
    sa.issue(stages[pn], wv, k0 + (kt + D) * BK, k1, m_blk, args.M);
    const char* la = stages[p];
    bf16x8_t fa[2][MFR];
#pragma unroll
    for (int s = 0; s < 2; ++s)
#pragma unroll
      for (int j = 0; j < MFR; ++j) fa[s][j] = read_frag<0, BM>(la, wm0 + 16 * j, s, lane);
    __builtin_amdgcn_s_setprio(1);
#pragma unroll
    for (int s = 0; s < 2; ++s)
#pragma unroll
      for (int i = 0; i < NFR; ++i)
#pragma unroll
        for (int j = 0; j < MFR; ++j)
          acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(__builtin_bit_cast(bf16x8_t, breg[p][s][i]), fa[s][j],
                                                              acc[i][j], 0, 0, 0);
    __builtin_amdgcn_s_setprio(0);
  };
  for (int kt = 0; kt < nk; kt += NSA) {
    step(std::integral_constant<int, 0>{}, kt);
    if (kt + 1 < nk) step(std::integral_constant<int, 1>{}, kt + 1);
    if (kt + 2 < nk) step(std::integral_constant<int, 2 % NSA>{}, kt + 2);
    if constexpr (NSA >= 4)
      if (kt + 3 < nk) step(std::integral_constant<int, 3 % NSA>{}, kt + 3);
  }
  // drain the loads issued past the end before the block exits (their LDS / registers die)
  __builtin_amdgcn_s_waitcnt(waitcnt_vm(0));

  const int mrow_l = lane & 15, ncol_l = (lane >> 4) * 4;
  const int c_cols = (!epi_bf16<EPI>() && args.bias_out) ? args.ones_col : args.N;
#pragma unroll
  for (int j = 0; j < MFR; ++j) {
    const int m = m_blk + wm0 + 16 * j + mrow_l;
    if (m >= args.M) continue;
#pragma unroll
    for (int i = 0; i < NFR; ++i) {
      const int n = n_blk + wn0 + 16 * i + ncol_l;
      if (n >= args.N) continue;
      epi_store<EPI, false>(args, grp, split, m, n, acc[i][j], c_cols);
    }
  }
}

template <int AMODE, int NSA>
int launch_bdir_epi(const SnGemmArgs& a, dim3 grid, hipStream_t st) {
  switch (a.epi) {
    case EPI_BF16: hipLaunchKernelGGL((gemm_bdir_kernel<AMODE, EPI_BF16, NSA>), grid, dim3(256), 0, st, a); break;
    case EPI_BF16_DROP:
      if (AMODE != OP_DENSE) return 4;
      hipLaunchKernelGGL((gemm_bdir_kernel<OP_DENSE, EPI_BF16_DROP, NSA>), grid, dim3(256), 0, st, a);
      break;
    case EPI_F32: hipLaunchKernelGGL((gemm_bdir_kernel<AMODE, EPI_F32, NSA>), grid, dim3(256), 0, st, a); break;
    case EPI_F32_ACC: hipLaunchKernelGGL((gemm_bdir_kernel<AMODE, EPI_F32_ACC, NSA>), grid, dim3(256), 0, st, a); break;
    default: return 2;
  }
  return SN_CHECK_LAUNCH();
}

}  // namespace

// tile 21: 3 A stages (48 KB), tile 22: 4 A stages (64 KB); K-contiguous dense B whose
// bytes fit the buffer range, A dense or implicit im2col (K-contiguous)
int sn_gemm_bdir(const SnGemmArgs& a, hipStream_t stream) {
  if (a.a_mc || a.b_mc || a.b_mode != OP_DENSE || a.fp8 || a.epi == EPI_SGD || a.ones_col >= 0) return 4;
  if (a.a_mode != OP_DENSE && a.a_mode != OP_IM2COL) return 4;
  // every valid B byte offset (+ the soffset K advance) below 2^31 - 16
  const long long extent = ((long long)(a.groups - 1) * a.B.gstride + (long long)a.N * a.B.ld) * 2;
  if (extent >= (1ll << 31) - 64 || (a.B.ld & 7)) return 4;
  const int tiles = ((a.M + 127) / 128) * ((a.N + 127) / 128);
  dim3 grid(tiles * a.splits * a.groups);
  if (a.tile == 21)
    return a.a_mode == OP_DENSE ? launch_bdir_epi<OP_DENSE, 3>(a, grid, stream)
                                : launch_bdir_epi<OP_IM2COL, 3>(a, grid, stream);
  return a.a_mode == OP_DENSE ? launch_bdir_epi<OP_DENSE, 4>(a, grid, stream)
                              : launch_bdir_epi<OP_IM2COL, 4>(a, grid, stream);
}
