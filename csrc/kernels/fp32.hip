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

// AT / BT: the operand is stored [K][M] / [K][N] (k-strided rows, e.g. the activations and
// output gradients of a weight gradient, or the weights of a data gradient) and is staged
// transposed into the same [row][k] LDS image, so no operand is ever copied to K-contiguous form.
template <bool AT, bool BT>
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

  // staging: a K-contiguous operand moves 4 rows x 4 k per thread and stage (one float4 along k
  // per row); a transposed one 4 k-rows x 4 rows (one float4 along the rows per k-row), written
  // to LDS transposed
  const int lr = tid >> 3, lk = (tid & 7) * 4;  // K-contiguous: rows lr + 32 j, k chunk lk
  const int tr = (tid & 31) * 4, tk = tid >> 5;  // transposed: rows tr..tr+3, k rows tk + 8 j
  const bool vec = (a.lda % 4) == 0 && (a.ldb % 4) == 0 && (reinterpret_cast<uintptr_t>(a.A) % 16) == 0 &&
                   (reinterpret_cast<uintptr_t>(a.B) % 16) == 0;
  float4 ra[4], rb[4];
  auto load_op = [&](const float* X, long long ld, int r0, int rows, bool trans, int k0, float4* rx)
                     __attribute__((always_inline)) {
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      if (!trans) {
        const int r = r0 + lr + 32 * j, k = k0 + lk;
        if (vec && k + 3 < kend) {
          rx[j] = r < rows ? *reinterpret_cast<const float4*>(X + (long long)r * ld + k) : make_float4(0, 0, 0, 0);
        } else {
          float v[4];
#pragma unroll
          for (int t = 0; t < 4; ++t) v[t] = (r < rows && k + t < kend) ? X[(long long)r * ld + k + t] : 0.f;
          rx[j] = make_float4(v[0], v[1], v[2], v[3]);
        }
      } else {
        const int r = r0 + tr, k = k0 + tk + 8 * j;
        if (k < kend && vec && r + 3 < rows) {
          rx[j] = *reinterpret_cast<const float4*>(X + (long long)k * ld + r);
        } else {
          float v[4];
#pragma unroll
          for (int t = 0; t < 4; ++t) v[t] = (k < kend && r + t < rows) ? X[(long long)k * ld + r + t] : 0.f;
          rx[j] = make_float4(v[0], v[1], v[2], v[3]);
        }
      }
    }
  };
  auto load = [&](int k0) __attribute__((always_inline)) {
    load_op(a.A, a.lda, m0, a.M, AT, k0, ra);
    load_op(a.B, a.ldb, n0, a.N, BT, k0, rb);
  };
  auto store_op = [&](float* sx, bool trans, const float4* rx) __attribute__((always_inline)) {
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      if (!trans) {
        float* p = &sx[(lr + 32 * j) * F_LD + lk];
        *reinterpret_cast<float2*>(p) = make_float2(rx[j].x, rx[j].y);
        *reinterpret_cast<float2*>(p + 2) = make_float2(rx[j].z, rx[j].w);
      } else {
        const int k = tk + 8 * j;
        sx[(tr + 0) * F_LD + k] = rx[j].x;
        sx[(tr + 1) * F_LD + k] = rx[j].y;
        sx[(tr + 2) * F_LD + k] = rx[j].z;
        sx[(tr + 3) * F_LD + k] = rx[j].w;
      }
    }
  };
  auto store = [&](int b) __attribute__((always_inline)) {
    store_op(sA[b], AT, ra);
    store_op(sB[b], BT, rb);
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

// col[(n,p,q)][(r,s,c)] = x[n][p*sh-ph+r*dh][q*sw-pw+s*dw][coff+c] (0 outside the image).
// A col row is the taps' channel runs back to back, so consecutive lanes take consecutive
// VW-channel chunks of it (float4 when the channel offsets allow): every wave-instruction
// stores one contiguous 1 KB (256 B scalar) piece of col and reads contiguous runs of x.
// IT = uint32_t decodes the index in 32 bits when the item count allows.
template <int VW, typename IT>
__global__ void im2col_f32_k(const float* __restrict__ x, float* __restrict__ col, F32Conv g) {
  const int cq = g.Cg / VW, taps = g.R * g.S;
  const IT items = (IT)g.N * g.P * g.Q * taps * cq;
  for (IT i = blockIdx.x * (IT)blockDim.x + threadIdx.x; i < items; i += (IT)gridDim.x * blockDim.x) {
    const IT t = i / cq;
    const int c = (int)(i - t * cq) * VW;
    const IT m = t / taps;
    const int tap = (int)(t - m * taps);
    const int pq = (int)(m % (IT)(g.P * g.Q)), n = (int)(m / (IT)(g.P * g.Q));
    const int p = pq / g.Q, q = pq - p * g.Q, r = tap / g.S, s = tap - r * g.S;
    const int h = p * g.sh - g.ph + r * g.dh, w = q * g.sw - g.pw + s * g.dw;
    const bool in = (unsigned)h < (unsigned)g.H && (unsigned)w < (unsigned)g.W;
    const float* src = x + (((long long)n * g.H + (in ? h : 0)) * g.W + (in ? w : 0)) * g.C + g.coff + c;
    float* dst = col + (long long)i * VW;
    if constexpr (VW == 4)
      *reinterpret_cast<float4*>(dst) = in ? *reinterpret_cast<const float4*>(src) : make_float4(0, 0, 0, 0);
    else
      *dst = in ? *src : 0.f;
  }
}

// dx[n][h][w][coff+c] (=|+=) sum over the (p, q, r, s) that read (h, w) of dcol[(n,p,q)][(r,s,c)]:
// one thread per (input pixel, 4-channel chunk) gathers its taps in (r, s) order
template <bool V4>
__global__ void col2im_f32_k(const float* __restrict__ dcol, float* __restrict__ dx, F32Conv g, int accumulate) {
  const int kred = g.R * g.S * g.Cg;
  constexpr int CW = V4 ? 4 : 1;
  const int chunks = g.Cg / CW;
  const long long total = (long long)g.N * g.H * g.W * chunks;
  for (long long i = blockIdx.x * (long long)blockDim.x + threadIdx.x; i < total;
       i += (long long)gridDim.x * blockDim.x) {
    const long long pix = i / chunks;
    const int c = (int)(i - pix * chunks) * CW;
    const int hw = (int)(pix % ((long long)g.H * g.W)), n = (int)(pix / ((long long)g.H * g.W));
    const int h = hw / g.W, w = hw - h * g.W;
    float acc[CW];
#pragma unroll
    for (int t = 0; t < CW; ++t) acc[t] = 0.f;
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
        const float* src = dcol + (((long long)n * g.P + p) * g.Q + q) * kred + (r * g.S + s) * g.Cg + c;
        if constexpr (V4) {
          const float4 v = *reinterpret_cast<const float4*>(src);
          acc[0] += v.x;
          acc[1] += v.y;
          acc[2] += v.z;
          acc[3] += v.w;
        } else {
          acc[0] += src[0];
        }
      }
    }
    float* o = dx + pix * g.C + g.coff + c;
#pragma unroll
    for (int t = 0; t < CW; ++t) o[t] = accumulate ? o[t] + acc[t] : acc[t];
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

// ---- pooling on NHWC fp32 (pooling_layer.cu semantics) ----
struct F32Pool {
  int N, H, W, C, P, Q, kh, kw, sh, sw, ph, pw;
};

// MAX: the first maximum of the window clipped to the image, in row-major scan order (strict >,
// from -FLT_MAX), and its flat index h * W + w (MaxPoolForward); AVE: the window sum over its
// image part divided by the size of the window clipped to the padded image (AvePoolForward)
template <bool MAX>
__global__ void pool_f32_fwd(const float* __restrict__ x, float* __restrict__ y, int* __restrict__ mask, F32Pool g) {
  const long long total = (long long)g.N * g.P * g.Q * g.C;
  for (long long i = blockIdx.x * (long long)blockDim.x + threadIdx.x; i < total;
       i += (long long)gridDim.x * blockDim.x) {
    const int c = (int)(i % g.C);
    const long long pix = i / g.C;
    const int q = (int)(pix % g.Q), p = (int)((pix / g.Q) % g.P), n = (int)(pix / ((long long)g.Q * g.P));
    int hs = p * g.sh - g.ph, ws = q * g.sw - g.pw;
    int he = min(hs + g.kh, MAX ? g.H : g.H + g.ph), we = min(ws + g.kw, MAX ? g.W : g.W + g.pw);
    const int pool_size = (he - hs) * (we - ws);
    hs = max(hs, 0);
    ws = max(ws, 0);
    he = min(he, g.H);
    we = min(we, g.W);
    const float* xn = x + (long long)n * g.H * g.W * g.C + c;
    if (MAX) {
      float best = -3.402823466e+38f;
      int arg = -1;
      for (int h = hs; h < he; ++h)
        for (int w = ws; w < we; ++w) {
          const float v = xn[((long long)h * g.W + w) * g.C];
          if (v > best) {
            best = v;
            arg = h * g.W + w;
          }
        }
      y[i] = best;
      mask[i] = arg;
    } else {
      float acc = 0.f;
      for (int h = hs; h < he; ++h)
        for (int w = ws; w < we; ++w) acc += xn[((long long)h * g.W + w) * g.C];
      y[i] = acc / (float)pool_size;
    }
  }
}

// the gather adjoint: each input element sums, in window order, the output gradients of the
// windows that selected it (MAX) or that cover it, divided by their sizes (AVE)
template <bool MAX>
__global__ void pool_f32_bwd(const float* __restrict__ dy, const int* __restrict__ mask, float* __restrict__ dx,
                             F32Pool g) {
  const long long total = (long long)g.N * g.H * g.W * g.C;
  for (long long i = blockIdx.x * (long long)blockDim.x + threadIdx.x; i < total;
       i += (long long)gridDim.x * blockDim.x) {
    const int c = (int)(i % g.C);
    const long long pix = i / g.C;
    const int w = (int)(pix % g.W), h = (int)((pix / g.W) % g.H), n = (int)(pix / ((long long)g.W * g.H));
    const int hp = h + g.ph, wp = w + g.pw;
    const int p0 = hp < g.kh ? 0 : (hp - g.kh) / g.sh + 1, p1 = min(hp / g.sh + 1, g.P);
    const int q0 = wp < g.kw ? 0 : (wp - g.kw) / g.sw + 1, q1 = min(wp / g.sw + 1, g.Q);
    const long long base = (long long)n * g.P * g.Q;
    float acc = 0.f;
    for (int p = p0; p < p1; ++p)
      for (int q = q0; q < q1; ++q) {
        const long long o = (base + (long long)p * g.Q + q) * g.C + c;
        if (MAX) {
          if (mask[o] == h * g.W + w) acc += dy[o];
        } else {
          const int hs = p * g.sh - g.ph, ws = q * g.sw - g.pw;
          const int he = min(hs + g.kh, g.H + g.ph), we = min(ws + g.kw, g.W + g.pw);
          acc += dy[o] / (float)((he - hs) * (we - ws));
        }
      }
    dx[i] = acc;
  }
}

// ReLU with negative slope (relu_layer.cu): y = x > 0 ? x : x * slope; dx = dy * (x > 0 ? 1 : slope),
// the reference formulas' own operations, one pass each
__global__ void relu_f32_fwd(const float* __restrict__ x, float* __restrict__ y, long long n, float slope) {
  for (long long i = blockIdx.x * (long long)blockDim.x + threadIdx.x; i < n; i += (long long)gridDim.x * blockDim.x) {
    const float v = x[i];
    y[i] = v > 0.f ? v : v * slope;
  }
}

__global__ void relu_f32_bwd(const float* __restrict__ dy, const float* __restrict__ x, float* __restrict__ dx,
                             long long n, float slope) {
  for (long long i = blockIdx.x * (long long)blockDim.x + threadIdx.x; i < n; i += (long long)gridDim.x * blockDim.x)
    dx[i] = dy[i] * (x[i] > 0.f ? 1.f : slope);
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
// trans: bit 0 = A stored [K][M], bit 1 = B stored [K][N] (lda / ldb are then the k-row strides)
extern "C" int sn_gemm_f32(const float* A, long long lda, const float* B, long long ldb, float* C, long long ldc,
                           long long M, long long N, long long K, const float* bias, long long accumulate,
                           long long relu, long long splits, long long kchunk, long long trans, hipStream_t st) {
  if (M <= 0 || N <= 0) return 0;
  if (M >= (1ll << 31) || N >= (1ll << 31) || K >= (1ll << 31)) return 3;
  if (splits < 1 || (splits > 1 && (bias || accumulate || relu || kchunk % F_BK))) return 3;
  if (splits == 1) kchunk = K;
  F32Args a{A, B, C, bias, lda, ldb, ldc, (int)M, (int)N, (int)K, (int)accumulate, (int)relu, (int)kchunk,
            M * ldc};
  const long long tiles = ((M + F_BM - 1) / F_BM) * ((N + F_BN - 1) / F_BN);
  const dim3 grid((unsigned)tiles, (unsigned)splits);
  switch (trans & 3) {
    case 0: hipLaunchKernelGGL((gemm_f32_kernel<false, false>), grid, dim3(F_NT), 0, st, a); break;
    case 1: hipLaunchKernelGGL((gemm_f32_kernel<true, false>), grid, dim3(F_NT), 0, st, a); break;
    case 2: hipLaunchKernelGGL((gemm_f32_kernel<false, true>), grid, dim3(F_NT), 0, st, a); break;
    default: hipLaunchKernelGGL((gemm_f32_kernel<true, true>), grid, dim3(F_NT), 0, st, a); break;
  }
  return SN_CHECK_LAUNCH();
}

extern "C" int sn_im2col_f32(const float* x, float* col, long long N, long long H, long long W, long long C,
                             long long P, long long Q, long long R, long long S, long long sh, long long sw,
                             long long ph, long long pw, long long dh, long long dw, long long Cg, long long coff,
                             hipStream_t st) {
  const F32Conv g = mkf32conv(N, H, W, C, P, Q, R, S, sh, sw, ph, pw, dh, dw, Cg, coff);
  const bool v4 = Cg % 4 == 0 && coff % 4 == 0 && C % 4 == 0 && reinterpret_cast<uintptr_t>(x) % 16 == 0 &&
                  reinterpret_cast<uintptr_t>(col) % 16 == 0;
  const long long items = N * P * Q * R * S * (v4 ? Cg / 4 : Cg);
  const dim3 grid(sn_blocks(items, 256, 16384));
  const bool i32 = items < (1ll << 31) - 256ll * 16384;
  if (v4 && i32) hipLaunchKernelGGL((im2col_f32_k<4, uint32_t>), grid, dim3(256), 0, st, x, col, g);
  else if (v4) hipLaunchKernelGGL((im2col_f32_k<4, long long>), grid, dim3(256), 0, st, x, col, g);
  else if (i32) hipLaunchKernelGGL((im2col_f32_k<1, uint32_t>), grid, dim3(256), 0, st, x, col, g);
  else hipLaunchKernelGGL((im2col_f32_k<1, long long>), grid, dim3(256), 0, st, x, col, g);
  return SN_CHECK_LAUNCH();
}

extern "C" int sn_col2im_f32(const float* dcol, float* dx, long long N, long long H, long long W, long long C,
                             long long P, long long Q, long long R, long long S, long long sh, long long sw,
                             long long ph, long long pw, long long dh, long long dw, long long Cg, long long coff,
                             long long accumulate, hipStream_t st) {
  const F32Conv g = mkf32conv(N, H, W, C, P, Q, R, S, sh, sw, ph, pw, dh, dw, Cg, coff);
  const bool v4 = Cg % 4 == 0 && coff % 4 == 0 && C % 4 == 0 && reinterpret_cast<uintptr_t>(dx) % 16 == 0 &&
                  reinterpret_cast<uintptr_t>(dcol) % 16 == 0;
  const long long total = N * H * W * (v4 ? Cg / 4 : Cg);
  if (v4)
    hipLaunchKernelGGL(col2im_f32_k<true>, dim3(sn_blocks(total, 256, 16384)), dim3(256), 0, st, dcol, dx, g,
                       (int)accumulate);
  else
    hipLaunchKernelGGL(col2im_f32_k<false>, dim3(sn_blocks(total, 256, 16384)), dim3(256), 0, st, dcol, dx, g,
                       (int)accumulate);
  return SN_CHECK_LAUNCH();
}

extern "C" int sn_pool_f32(const float* x, float* y, int* mask, long long N, long long H, long long W, long long C,
                           long long P, long long Q, long long kh, long long kw, long long sh, long long sw,
                           long long ph, long long pw, long long max_pool, hipStream_t st) {
  const F32Pool g{(int)N, (int)H, (int)W, (int)C, (int)P, (int)Q, (int)kh, (int)kw, (int)sh, (int)sw, (int)ph, (int)pw};
  const dim3 grid(sn_blocks(N * P * Q * C, 256, 16384));
  if (max_pool) hipLaunchKernelGGL(pool_f32_fwd<true>, grid, dim3(256), 0, st, x, y, mask, g);
  else hipLaunchKernelGGL(pool_f32_fwd<false>, grid, dim3(256), 0, st, x, y, mask, g);
  return SN_CHECK_LAUNCH();
}

extern "C" int sn_pool_f32_bwd(const float* dy, const int* mask, float* dx, long long N, long long H, long long W,
                               long long C, long long P, long long Q, long long kh, long long kw, long long sh,
                               long long sw, long long ph, long long pw, long long max_pool, hipStream_t st) {
  const F32Pool g{(int)N, (int)H, (int)W, (int)C, (int)P, (int)Q, (int)kh, (int)kw, (int)sh, (int)sw, (int)ph, (int)pw};
  const dim3 grid(sn_blocks(N * H * W * C, 256, 16384));
  if (max_pool) hipLaunchKernelGGL(pool_f32_bwd<true>, grid, dim3(256), 0, st, dy, mask, dx, g);
  else hipLaunchKernelGGL(pool_f32_bwd<false>, grid, dim3(256), 0, st, dy, mask, dx, g);
  return SN_CHECK_LAUNCH();
}

extern "C" int sn_relu_f32(const float* x, float* y, long long n, float slope, hipStream_t st) {
  hipLaunchKernelGGL(relu_f32_fwd, dim3(sn_blocks(n, 256, 16384)), dim3(256), 0, st, x, y, n, slope);
  return SN_CHECK_LAUNCH();
}

extern "C" int sn_relu_f32_bwd(const float* dy, const float* x, float* dx, long long n, float slope, hipStream_t st) {
  hipLaunchKernelGGL(relu_f32_bwd, dim3(sn_blocks(n, 256, 16384)), dim3(256), 0, st, dy, x, dx, n, slope);
  return SN_CHECK_LAUNCH();
}
