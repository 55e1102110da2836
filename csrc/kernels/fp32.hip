// fp32 device mode (bench.py --dtype fp32, Net(dtype=torch.float32) on a ROCm device): the
// reference's numerics — Caffe computes in fp32 end to end (libccaffe/ccaffe.h:3 `#define
// DTYPE float`; SGEMM at caffe/src/caffe/util/math_functions.cu:14-28) — on the MI355X's
// exact-f32 matrix cores.
//
//   sn_gemm_f32:   C[m][n] (+)= sum_k A[m][k] * B[n][k] (+ bias[n], ReLU), every operand fp32,
//                  K-contiguous rows (the host transposes where a layout needs it)
//   sn_im2col_f32 / sn_col2im_f32: the NHWC patch matrix of a convolution group and its
//                  gather-form adjoint (no atomics: each input pixel sums the taps that read it)
//
// GEMM design: v_mfma_f32_16x16x4_f32 (f32 in, f32 accumulate, bit-for-bit a k-ordered fmaf
// chain; 64 FLOP/clk/SIMD = 1/16 of the bf16 rate).  128 x 128 block tile, 4 waves of
// 64 x 64 (4 x 4 MFMA tiles, 16 f32x4 accumulators), BK = 32 k per stage.  The next stage's
// global loads are issued into registers before the current stage's MFMAs (one stage of
// register double buffering) and written to the other LDS buffer after them; one barrier per
// stage.  LDS rows are 34 floats (136 B: 8-B aligned stores, and the 16 rows x 4 k a wave
// reads per operand fragment fall on 32 distinct banks).  A ds_read_b32 feeds a 32-cycle
// MFMA, so the loop is bound by the f32 matrix rate, not LDS.
#include "common.h"

namespace {

constexpr int F_BM = 128, F_BN = 128, F_BK = 32, F_LD = F_BK + 2, F_NT = 256;

struct F32Args {
  const float* A;
  const float* B;
  float* C;
  const float* bias;
  long long lda, ldb, ldc;
  int M, N, K, accumulate, relu;
  int kchunk;              // split-K: block row y of the grid reduces k in [y*kchunk, (y+1)*kchunk)
  long long c_split;       // ... into its own fp32 slab C + y * c_split (plain store; host sums)
};

__global__ void __launch_bounds__(F_NT, 2) gemm_f32_kernel(F32Args a) {
  __shared__ float sA[2][F_BM * F_LD];
  __shared__ float sB[2][F_BN * F_LD];
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int tiles_m = (a.M + F_BM - 1) / F_BM;
  const int bid = xcd_block(blockIdx.x, gridDim.x);
  const int m0 = (bid % tiles_m) * F_BM, n0 = (bid / tiles_m) * F_BN;
  const int kbeg = blockIdx.y * a.kchunk, kend = min(a.K, kbeg + a.kchunk);
  float* const Cs = a.C + blockIdx.y * a.c_split;
  const int wm = (wave & 1) * 64, wn = (wave >> 1) * 64;

  // staging: each thread moves 4 rows x 4 k (one float4 per row) of A and of B per stage
  const int lr = tid >> 3, lk = (tid & 7) * 4;  // rows lr + 32 j, k chunk lk
  const bool vec = (a.lda % 4) == 0 && (a.ldb % 4) == 0 && (reinterpret_cast<uintptr_t>(a.A) % 16) == 0 &&
                   (reinterpret_cast<uintptr_t>(a.B) % 16) == 0;
  float4 ra[4], rb[4];
  auto load = [&](int k0) __attribute__((always_inline)) {
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      const int m = m0 + lr + 32 * j, n = n0 + lr + 32 * j, k = k0 + lk;
      if (vec && k + 3 < kend) {
        ra[j] = m < a.M ? *reinterpret_cast<const float4*>(a.A + (long long)m * a.lda + k) : make_float4(0, 0, 0, 0);
        rb[j] = n < a.N ? *reinterpret_cast<const float4*>(a.B + (long long)n * a.ldb + k) : make_float4(0, 0, 0, 0);
      } else {
        float va[4], vb[4];
#pragma unroll
        for (int t = 0; t < 4; ++t) {
          va[t] = (m < a.M && k + t < kend) ? a.A[(long long)m * a.lda + k + t] : 0.f;
          vb[t] = (n < a.N && k + t < kend) ? a.B[(long long)n * a.ldb + k + t] : 0.f;
        }
        ra[j] = make_float4(va[0], va[1], va[2], va[3]);
        rb[j] = make_float4(vb[0], vb[1], vb[2], vb[3]);
      }
    }
  };
  auto store = [&](int b) __attribute__((always_inline)) {
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      float* pa = &sA[b][(lr + 32 * j) * F_LD + lk];
      float* pb = &sB[b][(lr + 32 * j) * F_LD + lk];
      *reinterpret_cast<float2*>(pa) = make_float2(ra[j].x, ra[j].y);
      *reinterpret_cast<float2*>(pa + 2) = make_float2(ra[j].z, ra[j].w);
      *reinterpret_cast<float2*>(pb) = make_float2(rb[j].x, rb[j].y);
      *reinterpret_cast<float2*>(pb + 2) = make_float2(rb[j].z, rb[j].w);
    }
  };

  f32x4 acc[4][4];
#pragma unroll
  for (int i = 0; i < 4; ++i)
#pragma unroll
    for (int j = 0; j < 4; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};

  const int nk = kend > kbeg ? (kend - kbeg + F_BK - 1) / F_BK : 0;
  const int fr = lane & 15, fk = lane >> 4;  // fragment row / k of this lane
  if (nk > 0) {
    load(kbeg);
    store(0);
  }
  __syncthreads();
  for (int kt = 0; kt < nk; ++kt) {
    const int b = kt & 1;
    if (kt + 1 < nk) load(kbeg + (kt + 1) * F_BK);  // in flight under this stage's MFMAs
    const float* la = sA[b];
    const float* lb = sB[b];
#pragma unroll
    for (int s = 0; s < F_BK / 4; ++s) {
      float fa[4], fb[4];
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        fa[i] = la[(wm + 16 * i + fr) * F_LD + 4 * s + fk];
        fb[i] = lb[(wn + 16 * i + fr) * F_LD + 4 * s + fk];
      }
#pragma unroll
      for (int i = 0; i < 4; ++i)
#pragma unroll
        for (int j = 0; j < 4; ++j) acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x4f32(fa[i], fb[j], acc[i][j], 0, 0, 0);
    }
    if (kt + 1 < nk) store(b ^ 1);  // the other buffer: last read one stage ago, behind the barrier below
    __syncthreads();
  }

  // D of MFMA (i, j): lane holds rows wm + 16 i + 4 (lane >> 4) + r, column wn + 16 j + (lane & 15)
#pragma unroll
  for (int i = 0; i < 4; ++i)
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      const int m = m0 + wm + 16 * i + 4 * (lane >> 4) + r;
      if (m >= a.M) continue;
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        const int n = n0 + wn + 16 * j + (lane & 15);
        if (n >= a.N) continue;
        float v = acc[i][j][r];
        float* c = Cs + (long long)m * a.ldc + n;
        if (a.accumulate) v += *c;
        if (a.bias) v += a.bias[n];
        if (a.relu) v = fmaxf(v, 0.f);
        *c = v;
      }
    }
}

struct F32Conv {
  int N, H, W, C, P, Q, R, S, sh, sw, ph, pw, dh, dw, Cg, coff;
};

// col[(n,p,q)][(r,s,c)] = x[n][p*sh-ph+r*dh][q*sw-pw+s*dw][coff+c] (0 outside the image)
__global__ void im2col_f32_k(const float* __restrict__ x, float* __restrict__ col, F32Conv g) {
  const int kred = g.R * g.S * g.Cg;
  const long long total = (long long)g.N * g.P * g.Q * kred;
  for (long long i = blockIdx.x * (long long)blockDim.x + threadIdx.x; i < total;
       i += (long long)gridDim.x * blockDim.x) {
    const int k = (int)(i % kred);
    const long long m = i / kred;
    const int q = (int)(m % g.Q), p = (int)((m / g.Q) % g.P), n = (int)(m / ((long long)g.Q * g.P));
    const int c = k % g.Cg, tap = k / g.Cg, s = tap % g.S, r = tap / g.S;
    const int h = p * g.sh - g.ph + r * g.dh, w = q * g.sw - g.pw + s * g.dw;
    col[i] = ((unsigned)h < (unsigned)g.H && (unsigned)w < (unsigned)g.W)
                 ? x[(((long long)n * g.H + h) * g.W + w) * g.C + g.coff + c]
                 : 0.f;
  }
}

// dx[n][h][w][coff+c] (=|+=) sum over the (p, q, r, s) that read (h, w) of dcol[(n,p,q)][(r,s,c)]
__global__ void col2im_f32_k(const float* __restrict__ dcol, float* __restrict__ dx, F32Conv g, int accumulate) {
  const int kred = g.R * g.S * g.Cg;
  const long long total = (long long)g.N * g.H * g.W * g.Cg;
  for (long long i = blockIdx.x * (long long)blockDim.x + threadIdx.x; i < total;
       i += (long long)gridDim.x * blockDim.x) {
    const int c = (int)(i % g.Cg);
    const long long pix = i / g.Cg;
    const int w = (int)(pix % g.W), h = (int)((pix / g.W) % g.H), n = (int)(pix / ((long long)g.W * g.H));
    float acc = 0.f;
    for (int r = 0; r < g.R; ++r) {
      const int hh = h + g.ph - r * g.dh;
      if (hh < 0 || hh % g.sh) continue;
      const int p = hh / g.sh;
      if (p >= g.P) continue;
      for (int s = 0; s < g.S; ++s) {
        const int ww = w + g.pw - s * g.dw;
        if (ww < 0 || ww % g.sw) continue;
        const int q = ww / g.sw;
        if (q >= g.Q) continue;
        acc += dcol[(((long long)n * g.P + p) * g.Q + q) * kred + (r * g.S + s) * g.Cg + c];
      }
    }
    float* o = dx + pix * g.C + g.coff + c;
    *o = accumulate ? *o + acc : acc;
  }
}

F32Conv mkf32conv(long long N, long long H, long long W, long long C, long long P, long long Q, long long R,
                  long long S, long long sh, long long sw, long long ph, long long pw, long long dh, long long dw,
                  long long Cg, long long coff) {
  F32Conv g;
  g.N = (int)N; g.H = (int)H; g.W = (int)W; g.C = (int)C; g.P = (int)P; g.Q = (int)Q; g.R = (int)R; g.S = (int)S;
  g.sh = (int)sh; g.sw = (int)sw; g.ph = (int)ph; g.pw = (int)pw; g.dh = (int)dh; g.dw = (int)dw;
  g.Cg = (int)Cg; g.coff = (int)coff;
  return g;
}

// Dropout on fp32 (forward, and backward with an optional slope-0 ReLU gate): the same
// device Philox keep mask as the bf16 dropout_kernel (eltwise.hip) draws for element e,
// so the mask is independent of the precision mode and never leaves the device.
__global__ void dropout_f32_k(const float* __restrict__ x, float* __restrict__ y, long long n,
                              const long long* __restrict__ rng, int stream, uint32_t thr, float scale,
                              const float* __restrict__ gate) {
  for (long long i = blockIdx.x * (long long)blockDim.x + threadIdx.x; i < (n + 3) / 4;
       i += (long long)gridDim.x * blockDim.x) {
    const uint4 u = dropout_bits4(rng, stream, (unsigned long long)i);
    const uint32_t b[4] = {u.x, u.y, u.z, u.w};
#pragma unroll
    for (int k = 0; k < 4; ++k) {
      const long long e = 4 * i + k;
      if (e >= n) break;
      float f = b[k] > thr ? x[e] * scale : 0.f;
      if (gate && !(gate[e] > 0.f)) f = 0.f;
      y[e] = f;
    }
  }
}

}  // namespace

extern "C" int sn_dropout_f32(const float* x, float* y, long long n, const long long* rng, long long stream,
                              float ratio, const float* gate, hipStream_t st) {
  const uint32_t thr = (uint32_t)((double)4294967295u * (double)ratio);
  const float scale = 1.f / (1.f - ratio);
  hipLaunchKernelGGL(dropout_f32_k, dim3(sn_blocks((n + 3) / 4, 256, 16384)), dim3(256), 0, st, x, y, n, rng,
                     (int)stream, thr, scale, gate);
  return SN_CHECK_LAUNCH();
}

// splits > 1: C is [splits][M][ldc] fp32 slabs written plainly (no bias / ReLU / accumulate);
// the host sums them in split order (deterministic).
extern "C" int sn_gemm_f32(const float* A, long long lda, const float* B, long long ldb, float* C, long long ldc,
                           long long M, long long N, long long K, const float* bias, long long accumulate,
                           long long relu, long long splits, long long kchunk, hipStream_t st) {
  if (M <= 0 || N <= 0) return 0;
  if (M >= (1ll << 31) || N >= (1ll << 31) || K >= (1ll << 31)) return 3;
  if (splits < 1 || (splits > 1 && (bias || accumulate || relu || kchunk % F_BK))) return 3;
  if (splits == 1) kchunk = K;
  F32Args a{A, B, C, bias, lda, ldb, ldc, (int)M, (int)N, (int)K, (int)accumulate, (int)relu, (int)kchunk,
            M * ldc};
  const long long tiles = ((M + F_BM - 1) / F_BM) * ((N + F_BN - 1) / F_BN);
  hipLaunchKernelGGL(gemm_f32_kernel, dim3((unsigned)tiles, (unsigned)splits), dim3(F_NT), 0, st, a);
  return SN_CHECK_LAUNCH();
}

extern "C" int sn_im2col_f32(const float* x, float* col, long long N, long long H, long long W, long long C,
                             long long P, long long Q, long long R, long long S, long long sh, long long sw,
                             long long ph, long long pw, long long dh, long long dw, long long Cg, long long coff,
                             hipStream_t st) {
  const F32Conv g = mkf32conv(N, H, W, C, P, Q, R, S, sh, sw, ph, pw, dh, dw, Cg, coff);
  const long long total = N * P * Q * R * S * Cg;
  hipLaunchKernelGGL(im2col_f32_k, dim3(sn_blocks(total, 256, 16384)), dim3(256), 0, st, x, col, g);
  return SN_CHECK_LAUNCH();
}

extern "C" int sn_col2im_f32(const float* dcol, float* dx, long long N, long long H, long long W, long long C,
                             long long P, long long Q, long long R, long long S, long long sh, long long sw,
                             long long ph, long long pw, long long dh, long long dw, long long Cg, long long coff,
                             long long accumulate, hipStream_t st) {
  const F32Conv g = mkf32conv(N, H, W, C, P, Q, R, S, sh, sw, ph, pw, dh, dw, Cg, coff);
  const long long total = N * H * W * Cg;
  hipLaunchKernelGGL(col2im_f32_k, dim3(sn_blocks(total, 256, 16384)), dim3(256), 0, st, dcol, dx, g,
                     (int)accumulate);
  return SN_CHECK_LAUNCH();
}
