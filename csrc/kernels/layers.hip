// HIP kernels of the non-hot Caffe layer families (gfx950): neurons (Sigmoid, TanH, AbsVal,
// BNLL, Exp, Log, Power, Threshold, PReLU), Eltwise (PROD / SUM / MAX), BatchNorm / MVN
// statistics and normalisation, axis copies (Slice, Tile, generic Concat), NHWC <-> NCHW
// layout changes (Flatten / Reshape), row gathers and deterministic scatter-adds
// (BatchReindex, Filter, Embed), Reduction, ArgMax, Caffe-ordered Im2col and the loss
// family (Euclidean, Hinge, MultinomialLogistic, Infogain, SigmoidCrossEntropy,
// Contrastive).
//
// Reference kernels these replace (behaviour, not code): caffe/src/caffe/layers/
// {sigmoid,tanh,absval,bnll,exp,log,power,threshold,prelu,eltwise,batch_norm,mvn,slice,
// tile,concat,flatten,reshape,batch_reindex,filter,embed,reduction,argmax,im2col,
// euclidean_loss,hinge_loss,multinomial_logistic_loss,infogain_loss,
// sigmoid_cross_entropy_loss,contrastive_loss}_layer.{cpp,cu}.
//
// Conventions: a tensor argument is bf16 (dt = 0) or fp32 (dt = 1); arithmetic is fp32.
// Tensors are decomposed as [B][outer][A][inner] around the axis an op works on (A), in
// PHYSICAL (NHWC for 4-D blobs) order — the Python side computes the decomposition.
// Every reduction is deterministic: fixed-order partials in a workspace, then a fixed-
// order combine; no float atomics.  Elementwise kernels take an 8-wide vector path when
// the element count is a multiple of 8.
#include "common.h"

namespace {

enum { DT_BF16 = 0, DT_F32 = 1 };

SN_DEV float ldv(const void* p, long long i, int dt) {
  return dt ? reinterpret_cast<const float*>(p)[i] : bf2f(reinterpret_cast<const bf16_t*>(p)[i]);
}
SN_DEV void stv(void* p, long long i, int dt, float v) {
  if (dt)
    reinterpret_cast<float*>(p)[i] = v;
  else
    reinterpret_cast<bf16_t*>(p)[i] = f2bf(v);
}

SN_DEV void ld8(const void* p, long long i8, int dt, float* f) {
  if (dt) {
    const float4 a = reinterpret_cast<const float4*>(p)[2 * i8], b = reinterpret_cast<const float4*>(p)[2 * i8 + 1];
    f[0] = a.x; f[1] = a.y; f[2] = a.z; f[3] = a.w; f[4] = b.x; f[5] = b.y; f[6] = b.z; f[7] = b.w;
  } else {
    unpack8(reinterpret_cast<const uint4*>(p)[i8], f);
  }
}
SN_DEV void st8(void* p, long long i8, int dt, const float* f) {
  if (dt) {
    reinterpret_cast<float4*>(p)[2 * i8] = make_float4(f[0], f[1], f[2], f[3]);
    reinterpret_cast<float4*>(p)[2 * i8 + 1] = make_float4(f[4], f[5], f[6], f[7]);
  } else {
    reinterpret_cast<uint4*>(p)[i8] = pack8(f);
  }
}

inline int grid_for(long long n, int per = 256, int cap = 4096) {
  long long b = (n + per - 1) / per;
  return (int)(b < 1 ? 1 : (b > cap ? cap : b));
}

// ---------------------------------------------------------------------------------------
// Neurons
// ---------------------------------------------------------------------------------------
enum { NK_SIGMOID = 0, NK_TANH, NK_ABSVAL, NK_BNLL, NK_EXP, NK_LOG, NK_POWER, NK_THRESHOLD };

struct NP {
  float a, b, c;
};

// Exp: y = exp(a x + b) with a = ln(base) scale, b = ln(base) shift
// Log: y = c ln(b + a x) with a = scale, b = shift, c = 1 / ln(base)
// Power: y = (c + b x)^a with a = power, b = scale, c = shift
// Threshold: y = x > a
template <int K>
SN_DEV float nfwd(float x, NP p) {
  if (K == NK_SIGMOID) return 0.5f * tanhf(0.5f * x) + 0.5f;
  if (K == NK_TANH) return tanhf(x);
  if (K == NK_ABSVAL) return fabsf(x);
  if (K == NK_BNLL) return x > 0.f ? x + log1pf(expf(-x)) : log1pf(expf(x));
  if (K == NK_EXP) return expf(fmaf(p.a, x, p.b));
  if (K == NK_LOG) return p.c * logf(fmaf(p.a, x, p.b));
  if (K == NK_POWER) {
    const float v = fmaf(p.b, x, p.c);
    if (p.a == 1.f) return v;
    if (p.a == 2.f) return v * v;
    return powf(v, p.a);
  }
  return x > p.a ? 1.f : 0.f;
}

template <int K>
SN_DEV float nbwd(float x, float y, float dy, NP p) {
  if (K == NK_SIGMOID) return dy * y * (1.f - y);
  if (K == NK_TANH) return dy * (1.f - y * y);
  if (K == NK_ABSVAL) return dy * (float)((x > 0.f) - (x < 0.f));
  if (K == NK_BNLL) {
    const float e = expf(fminf(x, 50.f));  // kBNLL_THRESHOLD (bnll_layer.cu)
    return dy * e / (e + 1.f);
  }
  if (K == NK_EXP) return dy * y * p.a;
  if (K == NK_LOG) return dy * p.a * p.c / fmaf(p.a, x, p.b);
  if (K == NK_POWER) {
    if (p.a == 0.f || p.b == 0.f) return 0.f;
    const float v = fmaf(p.b, x, p.c);
    if (p.a == 1.f) return dy * p.b;
    if (p.a == 2.f) return dy * 2.f * p.b * v;
    return dy * p.a * p.b * powf(v, p.a - 1.f);
  }
  return 0.f;
}

template <int K>
__global__ void __launch_bounds__(256) neuron_fwd_k(const void* __restrict__ x, void* __restrict__ y, long long n,
                                                    int dtx, int dty, NP p) {
  const long long stride = (long long)gridDim.x * blockDim.x;
  if ((n & 7) == 0) {
    for (long long i = blockIdx.x * (long long)blockDim.x + threadIdx.x; i < n / 8; i += stride) {
      float f[8];
      ld8(x, i, dtx, f);
#pragma unroll
      for (int j = 0; j < 8; ++j) f[j] = nfwd<K>(f[j], p);
      st8(y, i, dty, f);
    }
    return;
  }
  for (long long i = blockIdx.x * (long long)blockDim.x + threadIdx.x; i < n; i += stride)
    stv(y, i, dty, nfwd<K>(ldv(x, i, dtx), p));
}

// x may be null (kinds that differentiate through y only), y may be null (kinds through x)
template <int K>
__global__ void __launch_bounds__(256) neuron_bwd_k(const void* __restrict__ x, const void* __restrict__ y,
                                                    const void* __restrict__ dy, void* __restrict__ dx, long long n,
                                                    int dtx, int dty, int dtd, NP p) {
  const long long stride = (long long)gridDim.x * blockDim.x;
  if ((n & 7) == 0) {
    for (long long i = blockIdx.x * (long long)blockDim.x + threadIdx.x; i < n / 8; i += stride) {
      float fx[8] = {0, 0, 0, 0, 0, 0, 0, 0}, fy[8] = {0, 0, 0, 0, 0, 0, 0, 0}, fd[8];
      if (x) ld8(x, i, dtx, fx);
      if (y) ld8(y, i, dty, fy);
      ld8(dy, i, dtd, fd);
#pragma unroll
      for (int j = 0; j < 8; ++j) fd[j] = nbwd<K>(fx[j], fy[j], fd[j], p);
      st8(dx, i, dtd, fd);
    }
    return;
  }
  for (long long i = blockIdx.x * (long long)blockDim.x + threadIdx.x; i < n; i += stride) {
    const float xv = x ? ldv(x, i, dtx) : 0.f, yv = y ? ldv(y, i, dty) : 0.f;
    stv(dx, i, dtd, nbwd<K>(xv, yv, ldv(dy, i, dtd), p));
  }
}

// PReLU over [outer][C][inner] (inner = 1 for NHWC images / [N, C] blobs); shared: C = 1
// x may be fp32 (a 2-D blob from an Input layer) while y / dy / dx are the compute dtype.
__global__ void __launch_bounds__(256) prelu_fwd_k(const void* __restrict__ x, const float* __restrict__ slope,
                                                   void* __restrict__ y, long long n, int C, long long inner, int dtx,
                                                   int dt) {
  const long long stride = (long long)gridDim.x * blockDim.x;
  for (long long i = blockIdx.x * (long long)blockDim.x + threadIdx.x; i < n; i += stride) {
    const float v = ldv(x, i, dtx);
    const int c = C == 1 ? 0 : (int)((i / inner) % C);
    stv(y, i, dt, v > 0.f ? v : v * slope[c]);
  }
}

__global__ void __launch_bounds__(256) prelu_bwd_k(const void* __restrict__ x, const void* __restrict__ dy,
                                                   const float* __restrict__ slope, void* __restrict__ dx, long long n,
                                                   int C, long long inner, int dtx, int dt) {
  const long long stride = (long long)gridDim.x * blockDim.x;
  for (long long i = blockIdx.x * (long long)blockDim.x + threadIdx.x; i < n; i += stride) {
    const float v = ldv(x, i, dtx), d = ldv(dy, i, dt);
    const int c = C == 1 ? 0 : (int)((i / inner) % C);
    stv(dx, i, dt, v > 0.f ? d : d * slope[c]);
  }
}

// ---------------------------------------------------------------------------------------
// Deterministic axis reduction: out[b][a] (+)= scale * sum_{o, i} f(p[b][o][a][i], q[...])
//   mode 0: p   1: p q   2: p^2   3: p q [q <= 0] (PReLU slope)   4: |p|
//   mode 5: (p - q[b][a])^2 with q an fp32 per-(b, a) centre (the mean): the variance of
//   BatchNorm / MVN as E[(x - EX)^2] (batch_norm_layer.cu:50-59, mvn_layer.cu:31-36) —
//   E[x^2] - EX^2 cancels when |mean| >> std
// Pass 1 writes partials part[split][b][a]; pass 2 combines the splits in order.
// ---------------------------------------------------------------------------------------
template <int MODE>
SN_DEV float rf(float a, float b) {
  if (MODE == 0) return a;
  if (MODE == 1) return a * b;
  if (MODE == 2) return a * a;
  if (MODE == 3) return b <= 0.f ? a * b : 0.f;
  if (MODE == 5) return (a - b) * (a - b);
  return fabsf(a);
}

// inner == 1: a [rows = outer] x [A] column reduction.  Block = 4 row lanes x 64 columns.
template <int MODE>
__global__ void __launch_bounds__(256) colred_k(const void* __restrict__ p, const void* __restrict__ q, int dtp,
                                                int dtq, long long outer, int A, int splits, float* __restrict__ part,
                                                int B) {
  const int col = blockIdx.x * 64 + (threadIdx.x & 63), rl = threadIdx.x >> 6;
  const int b = blockIdx.z, s = blockIdx.y;
  const long long per = (outer + splits - 1) / splits;
  const long long r0 = s * per, r1 = min(outer, r0 + per);
  float acc = 0.f;
  if (col < A) {
    const long long base = (long long)b * outer * A;
    const float cen = MODE == 5 ? reinterpret_cast<const float*>(q)[(long long)b * A + col] : 0.f;
    for (long long r = r0 + rl; r < r1; r += 4) {
      const long long e = base + r * A + col;
      acc += rf<MODE>(ldv(p, e, dtp), MODE == 5 ? cen : (q ? ldv(q, e, dtq) : 0.f));
    }
  }
  __shared__ float red[4][64];
  red[rl][threadIdx.x & 63] = acc;
  __syncthreads();
  if (rl == 0 && col < A)
    part[((long long)s * B + b) * A + col] =
        red[0][threadIdx.x] + red[1][threadIdx.x] + red[2][threadIdx.x] + red[3][threadIdx.x];
}

// inner > 1: one block per (a, split, b) strides over the outer x inner elements of a.
template <int MODE>
__global__ void __launch_bounds__(256) segred_k(const void* __restrict__ p, const void* __restrict__ q, int dtp,
                                                int dtq, long long outer, int A, long long inner, int splits,
                                                float* __restrict__ part, int B) {
  const int a = blockIdx.x, s = blockIdx.y, b = blockIdx.z;
  const long long tot = outer * inner, per = (tot + splits - 1) / splits;
  const long long e0 = s * per, e1 = min(tot, e0 + per);
  float acc = 0.f;
  const float cen = MODE == 5 ? reinterpret_cast<const float*>(q)[(long long)b * A + a] : 0.f;
  for (long long e = e0 + threadIdx.x; e < e1; e += blockDim.x) {
    const long long o = e / inner, i = e - o * inner;
    const long long idx = (((long long)b * outer + o) * A + a) * inner + i;
    acc += rf<MODE>(ldv(p, idx, dtp), MODE == 5 ? cen : (q ? ldv(q, idx, dtq) : 0.f));
  }
  acc = wave_sum(acc);
  __shared__ float red[4];
  if ((threadIdx.x & 63) == 0) red[threadIdx.x >> 6] = acc;
  __syncthreads();
  if (threadIdx.x == 0) part[((long long)s * B + b) * A + a] = red[0] + red[1] + red[2] + red[3];
}

__global__ void combine_k(const float* __restrict__ part, int splits, long long BA, float* __restrict__ out,
                          float scale, int acc) {
  for (long long j = blockIdx.x * (long long)blockDim.x + threadIdx.x; j < BA; j += (long long)gridDim.x * blockDim.x) {
    float s = 0.f;
    for (int k = 0; k < splits; ++k) s += part[k * BA + j];
    out[j] = acc ? out[j] + scale * s : scale * s;
  }
}

// ---------------------------------------------------------------------------------------
// Normalisation (BatchNorm / MVN): per-(b, a) affine and its backward
// ---------------------------------------------------------------------------------------
// y = (x - mean[ba]) * inv[ba]   (mean may be null)
__global__ void __launch_bounds__(256) chan_affine_k(const void* __restrict__ x, void* __restrict__ y, long long n,
                                                     long long outer, int A, long long inner,
                                                     const float* __restrict__ mean, const float* __restrict__ inv,
                                                     int dtx, int dty) {
  const long long stride = (long long)gridDim.x * blockDim.x, per_b = outer * A * inner;
  for (long long e = blockIdx.x * (long long)blockDim.x + threadIdx.x; e < n; e += stride) {
    const long long b = e / per_b;
    const int a = (int)((e / inner) % A);
    const long long k = b * A + a;
    float v = ldv(x, e, dtx);
    if (mean) v -= mean[k];
    stv(y, e, dty, inv ? v * inv[k] : v);
  }
}

// dx = (dy - m1[ba] - xhat * m2[ba]) * inv[ba]   (m1 / m2 / inv / xhat may be null)
__global__ void __launch_bounds__(256) norm_bwd_k(const void* __restrict__ dy, const void* __restrict__ xhat,
                                                  void* __restrict__ dx, long long n, long long outer, int A,
                                                  long long inner, const float* __restrict__ m1,
                                                  const float* __restrict__ m2, const float* __restrict__ inv,
                                                  int dtd, int dtx) {
  const long long stride = (long long)gridDim.x * blockDim.x, per_b = outer * A * inner;
  for (long long e = blockIdx.x * (long long)blockDim.x + threadIdx.x; e < n; e += stride) {
    const long long b = e / per_b;
    const int a = (int)((e / inner) % A);
    const long long k = b * A + a;
    float g = ldv(dy, e, dtd);
    if (m1) g -= m1[k];
    if (m2) g -= ldv(xhat, e, dtx) * m2[k];
    stv(dx, e, dtd, inv ? g * inv[k] : g);
  }
}

// From sums s1 = sum x and s2 over `count` elements per (b, a): mean = s1 / count and
//   var = s2 / count (mode & 4: s2 = sum (x - mean)^2, centred — the default now), or
//   var = s2 / count - mean^2 clamped at 0 (s2 = sum x^2)
//   mode 0 (BatchNorm): inv = 1 / sqrt(var + eps)     mode 1 (MVN): inv = 1 / (sqrt(var) + eps)
//   mode 2 (MVN without variance): inv = 1
__global__ void stats_finalize_k(const float* __restrict__ s1, const float* __restrict__ s2, int n, float inv_count,
                                 float eps, int mode, float* __restrict__ mean, float* __restrict__ var,
                                 float* __restrict__ inv) {
  const int j = blockIdx.x * blockDim.x + threadIdx.x;
  if (j >= n) return;
  const float m = s1[j] * inv_count;
  const bool centred = (mode & 4) != 0;
  mode &= 3;
  const float v = s2 ? (centred ? s2[j] * inv_count : fmaxf(s2[j] * inv_count - m * m, 0.f)) : 0.f;
  mean[j] = m;
  if (var) var[j] = v;
  if (inv) inv[j] = mode == 0 ? rsqrtf(v + eps) : (mode == 1 ? 1.f / (sqrtf(v) + eps) : 1.f);
}

// BatchNorm running statistics (batch_norm_layer.cpp Forward_gpu):
//   factor = frac * factor + 1; mean = frac * mean + bmean; var = frac * var + unbias * bvar
__global__ void bn_running_k(float* __restrict__ mean, float* __restrict__ var, float* __restrict__ factor,
                             const float* __restrict__ bmean, const float* __restrict__ bvar, int C, float frac,
                             float unbias) {
  const int j = blockIdx.x * blockDim.x + threadIdx.x;
  if (j == 0) factor[0] = frac * factor[0] + 1.f;
  if (j < C) {
    mean[j] = frac * mean[j] + bmean[j];
    var[j] = frac * var[j] + unbias * bvar[j];
  }
}

// Global-stats BatchNorm: mean = rm * s, inv = 1 / sqrt(rv * s + eps), s = 1 / factor (0 if factor == 0)
__global__ void bn_global_k(const float* __restrict__ rm, const float* __restrict__ rv, const float* __restrict__ factor,
                            int C, float eps, float* __restrict__ mean, float* __restrict__ inv) {
  const int j = blockIdx.x * blockDim.x + threadIdx.x;
  if (j >= C) return;
  const float f = factor[0], s = f == 0.f ? 0.f : 1.f / f;
  mean[j] = rm[j] * s;
  inv[j] = rsqrtf(rv[j] * s + eps);
}

// ---------------------------------------------------------------------------------------
// Eltwise
// ---------------------------------------------------------------------------------------
struct EPtrs {
  const void* p[16];
  float coeff[16];
};

// op: 0 PROD, 1 SUM, 2 MAX (mask = index of the first maximum, eltwise_layer.cu)
__global__ void __launch_bounds__(256) eltwise_fwd_k(EPtrs in, int K, int op, void* __restrict__ y,
                                                     int* __restrict__ mask, long long n, int dt) {
  const long long stride = (long long)gridDim.x * blockDim.x;
  for (long long i = blockIdx.x * (long long)blockDim.x + threadIdx.x; i < n; i += stride) {
    float acc = ldv(in.p[0], i, dt);
    int arg = 0;
    if (op == 1) acc *= in.coeff[0];
    for (int k = 1; k < K; ++k) {
      const float v = ldv(in.p[k], i, dt);
      if (op == 0)
        acc *= v;
      else if (op == 1)
        acc = fmaf(in.coeff[k], v, acc);
      else if (v > acc) {
        acc = v;
        arg = k;
      }
    }
    stv(y, i, dt, acc);
    if (op == 2) mask[i] = arg;
  }
}

// gradient of bottom `which`: PROD (stable: product of the other bottoms, else y / x),
// SUM (coeff * dy), MAX (dy where the mask selects this bottom)
__global__ void __launch_bounds__(256) eltwise_bwd_k(EPtrs in, int K, int op, int which, int stable,
                                                     const void* __restrict__ y, const void* __restrict__ dy,
                                                     const int* __restrict__ mask, void* __restrict__ dx, long long n,
                                                     int dt) {
  const long long stride = (long long)gridDim.x * blockDim.x;
  for (long long i = blockIdx.x * (long long)blockDim.x + threadIdx.x; i < n; i += stride) {
    const float d = ldv(dy, i, dt);
    float g;
    if (op == 0) {
      if (stable) {
        g = 1.f;
        for (int k = 0; k < K; ++k)
          if (k != which) g *= ldv(in.p[k], i, dt);
      } else {
        g = ldv(y, i, dt) / ldv(in.p[which], i, dt);
      }
      g *= d;
    } else if (op == 1) {
      g = in.coeff[which] * d;
    } else {
      g = mask[i] == which ? d : 0.f;
    }
    stv(dx, i, dt, g);
  }
}

// ---------------------------------------------------------------------------------------
// Layout / copies
// ---------------------------------------------------------------------------------------
// dst[o][dst_off + a][i] (+)= src[o][src_off + a][i] for a < cnt  (Slice / Concat / Tile)
__global__ void __launch_bounds__(256) axis_copy_k(const void* __restrict__ src, void* __restrict__ dst, long long outer,
                                                   long long srcA, long long dstA, long long inner, long long src_off,
                                                   long long dst_off, long long cnt, int dts, int dtd, int acc) {
  const long long n = outer * cnt * inner, stride = (long long)gridDim.x * blockDim.x;
  for (long long e = blockIdx.x * (long long)blockDim.x + threadIdx.x; e < n; e += stride) {
    const long long i = e % inner, t = e / inner, a = t % cnt, o = t / cnt;
    const long long si = (o * srcA + src_off + a) * inner + i, di = (o * dstA + dst_off + a) * inner + i;
    const float v = ldv(src, si, dts);
    stv(dst, di, dtd, acc ? ldv(dst, di, dtd) + v : v);
  }
}

// Tile backward: dst[o][a][i] = sum_t src[o][t A + a][i]
__global__ void __launch_bounds__(256) tile_bwd_k(const void* __restrict__ src, void* __restrict__ dst, long long outer,
                                                  long long A, long long inner, int tiles, int dt) {
  const long long n = outer * A * inner, stride = (long long)gridDim.x * blockDim.x;
  for (long long e = blockIdx.x * (long long)blockDim.x + threadIdx.x; e < n; e += stride) {
    const long long i = e % inner, t = e / inner, a = t % A, o = t / A;
    float s = 0.f;
    for (int k = 0; k < tiles; ++k) s += ldv(src, (o * tiles * A + k * A + a) * inner + i, dt);
    stv(dst, e, dt, s);
  }
}

// [N][HW][C] <-> [N][C][HW] through a 64 x 64 LDS tile (both sides coalesced)
__global__ void __launch_bounds__(256) transpose_k(const void* __restrict__ src, void* __restrict__ dst, long long R,
                                                  long long Ccols, int dts, int dtd) {
  // src: [N][R][Ccols] -> dst: [N][Ccols][R]
  __shared__ float tile[64][65];
  const long long n = blockIdx.z;
  const long long r0 = (long long)blockIdx.y * 64, c0 = (long long)blockIdx.x * 64;
  const int tx = threadIdx.x & 63, ty = threadIdx.x >> 6;
  const long long base = n * R * Ccols;
  for (int k = ty; k < 64; k += 4) {
    const long long r = r0 + k, c = c0 + tx;
    tile[k][tx] = (r < R && c < Ccols) ? ldv(src, base + r * Ccols + c, dts) : 0.f;
  }
  __syncthreads();
  for (int k = ty; k < 64; k += 4) {
    const long long c = c0 + k, r = r0 + tx;
    if (r < R && c < Ccols) stv(dst, base + c * R + r, dtd, tile[tx][k]);
  }
}

// ---------------------------------------------------------------------------------------
// Row gathers / deterministic scatter-add (BatchReindex, Filter, Embed)
// ---------------------------------------------------------------------------------------
// dst[j][:] = src[idx[j]][:] (+ bias)   idx as float (Caffe blobs) or int32
__global__ void __launch_bounds__(256) gather_rows_k(const void* __restrict__ src, const void* __restrict__ idx,
                                                     int idx_int, void* __restrict__ dst, long long rows,
                                                     long long row_len, const float* __restrict__ bias, int dts,
                                                     int dtd) {
  const long long n = rows * row_len, stride = (long long)gridDim.x * blockDim.x;
  for (long long e = blockIdx.x * (long long)blockDim.x + threadIdx.x; e < n; e += stride) {
    const long long j = e / row_len, c = e - j * row_len;
    const long long r = idx_int ? (long long)reinterpret_cast<const int*>(idx)[j]
                                : (long long)reinterpret_cast<const float*>(idx)[j];
    float v = ldv(src, r * row_len + c, dts);
    if (bias) v += bias[c];
    stv(dst, e, dtd, v);
  }
}

// dst[r][:] (+)= sum over j with idx[j] == r (ascending j) of src[j][:]   — one block per
// (destination row, 256-column chunk); rows nobody selects are zeroed unless acc.
__global__ void __launch_bounds__(256) index_add_rows_k(const void* __restrict__ src, const void* __restrict__ idx,
                                                        int idx_int, long long n_idx, void* __restrict__ dst,
                                                        long long r0, long long row_len, int dts, int dtd, int acc) {
  const long long r = r0 + blockIdx.y;
  const long long c = (long long)blockIdx.x * blockDim.x + threadIdx.x;
  if (c >= row_len) return;
  float s = acc ? ldv(dst, r * row_len + c, dtd) : 0.f;
  for (long long j = 0; j < n_idx; ++j) {
    const long long rj = idx_int ? (long long)reinterpret_cast<const int*>(idx)[j]
                                 : (long long)reinterpret_cast<const float*>(idx)[j];
    if (rj == r) s += ldv(src, j * row_len + c, dts);
  }
  stv(dst, r * row_len + c, dtd, s);
}

// ---------------------------------------------------------------------------------------
// Reduction layer backward and ArgMax
// ---------------------------------------------------------------------------------------
// Reduction (reduction_layer.cu): segment s of length L: op 1 SUM, 2 ASUM, 3 SUMSQ, 4 MEAN
__global__ void __launch_bounds__(256) reduction_bwd_k(const void* __restrict__ x, const float* __restrict__ dy,
                                                       void* __restrict__ dx, long long segs, long long L, int op,
                                                       float coeff, int dt) {
  const long long n = segs * L, stride = (long long)gridDim.x * blockDim.x;
  for (long long e = blockIdx.x * (long long)blockDim.x + threadIdx.x; e < n; e += stride) {
    const float d = dy[e / L] * coeff;
    float g;
    if (op == 2) {
      const float v = ldv(x, e, dt);
      g = d * (float)((v > 0.f) - (v < 0.f));
    } else if (op == 3) {
      g = d * 2.f * ldv(x, e, dt);
    } else if (op == 4) {
      g = d / (float)L;
    } else {
      g = d;
    }
    stv(dx, e, dt, g);
  }
}

// ArgMax / top-k over segments [outer][A][inner] along A (k <= 64): one thread per
// (o, i) segment, k selection passes (ties -> lowest index, as std::partial_sort on
// (value, index) pairs with greater<> picks the higher index... Caffe sorts pairs
// descending, so among equal values the HIGHER index wins; replicate that).
__global__ void __launch_bounds__(256) topk_k(const void* __restrict__ x, long long outer, long long A, long long inner,
                                              int k, int out_max_val, int axis_mode, float* __restrict__ out, int dt) {
  const long long segs = outer * inner;
  const long long sgi = blockIdx.x * (long long)blockDim.x + threadIdx.x;
  if (sgi >= segs) return;
  const long long o = sgi / inner, i = sgi - o * inner;
  float last_v = INFINITY;
  long long last_i = A;  // previous pick: (value, index) strictly greater than what remains
  for (int t = 0; t < k; ++t) {
    float bv = -INFINITY;
    long long bi = -1;
    for (long long a = 0; a < A; ++a) {
      const float v = ldv(x, (o * A + a) * inner + i, dt);
      // candidates strictly after the previous pick in (value desc, index desc) order
      const bool after = v < last_v || (v == last_v && a < last_i);
      if (!after) continue;
      if (bi < 0 || v > bv || (v == bv && a > bi)) {
        bv = v;
        bi = a;
      }
    }
    last_v = bv;
    last_i = bi;
    if (axis_mode) {  // out [outer][k][inner]: value or index
      out[(o * k + t) * inner + i] = out_max_val ? bv : (float)bi;
    } else {          // out [outer][1 or 2][k]
      if (out_max_val) {
        out[o * 2 * k + t] = (float)bi;
        out[o * 2 * k + k + t] = bv;
      } else {
        out[o * k + t] = (float)bi;
      }
    }
  }
}

// ---------------------------------------------------------------------------------------
// Im2col layer with Caffe's channel order (c, kh, kw) on NHWC input -> NHWC output
// [N][P][Q][C R S]; and its col2im backward (gather form, deterministic)
// ---------------------------------------------------------------------------------------
struct I2C {
  int N, H, W, C, P, Q, R, S, sh, sw, ph, pw, dh, dw;
};

__global__ void __launch_bounds__(256) im2col_caffe_k(const void* __restrict__ x, void* __restrict__ col, I2C g, int dt) {
  const long long CRS = (long long)g.C * g.R * g.S, n = (long long)g.N * g.P * g.Q * CRS;
  const long long stride = (long long)gridDim.x * blockDim.x;
  for (long long e = blockIdx.x * (long long)blockDim.x + threadIdx.x; e < n; e += stride) {
    const long long k = e % CRS, pix = e / CRS;
    const int s = (int)(k % g.S), r = (int)((k / g.S) % g.R), c = (int)(k / ((long long)g.R * g.S));
    const int q = (int)(pix % g.Q), p = (int)((pix / g.Q) % g.P), nn = (int)(pix / ((long long)g.P * g.Q));
    const int h = p * g.sh - g.ph + r * g.dh, w = q * g.sw - g.pw + s * g.dw;
    float v = 0.f;
    if ((unsigned)h < (unsigned)g.H && (unsigned)w < (unsigned)g.W)
      v = ldv(x, (((long long)nn * g.H + h) * g.W + w) * g.C + c, dt);
    stv(col, e, dt, v);
  }
}

__global__ void __launch_bounds__(256) col2im_caffe_k(const void* __restrict__ dcol, void* __restrict__ dx, I2C g,
                                                      int dt) {
  const long long CRS = (long long)g.C * g.R * g.S, n = (long long)g.N * g.H * g.W * g.C;
  const long long stride = (long long)gridDim.x * blockDim.x;
  for (long long e = blockIdx.x * (long long)blockDim.x + threadIdx.x; e < n; e += stride) {
    const int c = (int)(e % g.C), w = (int)((e / g.C) % g.W), h = (int)((e / ((long long)g.C * g.W)) % g.H);
    const int nn = (int)(e / ((long long)g.C * g.W * g.H));
    float s = 0.f;
    for (int r = 0; r < g.R; ++r) {
      const int hp = h + g.ph - r * g.dh;
      if (hp < 0 || hp % g.sh) continue;
      const int p = hp / g.sh;
      if (p >= g.P) continue;
      for (int ss = 0; ss < g.S; ++ss) {
        const int wq = w + g.pw - ss * g.dw;
        if (wq < 0 || wq % g.sw) continue;
        const int q = wq / g.sw;
        if (q >= g.Q) continue;
        const long long k = ((long long)c * g.R + r) * g.S + ss;
        s += ldv(dcol, (((long long)nn * g.P + p) * g.Q + q) * CRS + k, dt);
      }
    }
    stv(dx, e, dt, s);
  }
}

// ---------------------------------------------------------------------------------------
// Loss family: per-row loss terms (fwd) and gradients (bwd).  Rows are [M][C] views.
//   kind 0 EUCLIDEAN   row m: sum_c (x - t)^2 / 2              dx = +-(x - t) s
//   kind 1 HINGE_L1    sum_c max(0, 1 - sgn x)                  dx = -sgn [margin > 0] s
//   kind 2 HINGE_L2    sum_c max(0, 1 - sgn x)^2                dx = -2 sgn margin s
//   kind 3 MULTINOMIAL -log max(p[label], 1e-20)                dx[label] = -s / max(p, 1e-20)
//   kind 4 INFOGAIN    -sum_c H[label][c] log max(p_c, 1e-20)   dx = -H[label][c] s / max(p_c, 1e-20)
//   kind 5 SIGMOID_XE  sum_c x (t - [x >= 0]) - log(1 + exp(x - 2 x [x >= 0]))  (negated)
//                                                               dx = (sigmoid(x) - t) s
//   kind 6 CONTRASTIVE (a = x, b = t, y = label): d2 = |a - b|^2
//          similar: d2 / 2, dissimilar: max(margin - d2, 0) / 2 (legacy) or
//          max(margin - d, 0)^2 / 2; dx = +-s coef (a - b)
// Labels are float; s = (*loss_weight) * scale (loss_weight: the loss top's diff).
// ---------------------------------------------------------------------------------------
struct LossP {
  int kind, M, C, dtx, dtt;
  const void* x;
  const void* t;        // targets (kinds 0, 5, 6: same layout as x)
  const float* label;   // kinds 1-4, 6 (similarity)
  const float* H;       // kind 4: [C][C] row-major
  float margin;
  int legacy;
};

__global__ void __launch_bounds__(64) loss_rows_fwd_k(LossP P, float* __restrict__ row_loss) {
  const int m = blockIdx.x, lane = threadIdx.x;
  const long long base = (long long)m * P.C;
  float acc = 0.f;
  const int lab = (P.kind >= 1 && P.kind <= 4) ? (int)P.label[m] : 0;
  if (P.kind == 3) {
    acc = lane == 0 ? -logf(fmaxf(ldv(P.x, base + lab, P.dtx), 1e-20f)) : 0.f;
  } else {
    for (int c = lane; c < P.C; c += 64) {
      const float x = ldv(P.x, base + c, P.dtx);
      if (P.kind == 0 || P.kind == 6) {
        const float d = x - ldv(P.t, base + c, P.dtt);
        acc += d * d;
      } else if (P.kind == 1 || P.kind == 2) {
        const float mg = fmaxf(0.f, 1.f - (c == lab ? x : -x));
        acc += P.kind == 1 ? mg : mg * mg;
      } else if (P.kind == 4) {
        acc -= P.H[(long long)lab * P.C + c] * logf(fmaxf(x, 1e-20f));
      } else {  // 5
        const float t = ldv(P.t, base + c, P.dtt), pos = x >= 0.f ? 1.f : 0.f;
        acc -= x * (t - pos) - log1pf(expf(x - 2.f * x * pos));
      }
    }
  }
  acc = wave_sum(acc);
  if (lane == 0) {
    if (P.kind == 0) acc *= 0.5f;
    if (P.kind == 6) {
      row_loss[P.M + m] = acc;  // d2, kept for the backward
      const bool similar = P.label[m] > 0.f;
      float v;
      if (similar)
        v = acc;
      else if (P.legacy)
        v = fmaxf(P.margin - acc, 0.f);
      else {
        const float d = fmaxf(P.margin - sqrtf(acc), 0.f);
        v = d * d;
      }
      acc = 0.5f * v;
    }
    row_loss[m] = acc;
  }
}

// sign: +1 for bottom 0, -1 for bottom 1 (Euclidean / Contrastive); d2 (kind 6) from fwd
__global__ void __launch_bounds__(256) loss_rows_bwd_k(LossP P, const float* __restrict__ loss_weight, float scale,
                                                       float sign, const float* __restrict__ d2,
                                                       void* __restrict__ dx) {
  const long long n = (long long)P.M * P.C, stride = (long long)gridDim.x * blockDim.x;
  const float s = loss_weight[0] * scale * sign;
  for (long long e = blockIdx.x * (long long)blockDim.x + threadIdx.x; e < n; e += stride) {
    const int m = (int)(e / P.C), c = (int)(e - (long long)m * P.C);
    const float x = ldv(P.x, e, P.dtx);
    float g = 0.f;
    if (P.kind == 0) {
      g = (x - ldv(P.t, e, P.dtt)) * s;
    } else if (P.kind == 1 || P.kind == 2) {
      const int lab = (int)P.label[m];
      const float sg = c == lab ? 1.f : -1.f, mg = fmaxf(0.f, 1.f - sg * x);
      g = -sg * (P.kind == 1 ? (mg > 0.f ? 1.f : 0.f) : 2.f * mg) * s;
    } else if (P.kind == 3) {
      const int lab = (int)P.label[m];
      g = c == lab ? -s / fmaxf(x, 1e-20f) : 0.f;
    } else if (P.kind == 4) {
      const int lab = (int)P.label[m];
      g = -P.H[(long long)lab * P.C + c] * s / fmaxf(x, 1e-20f);
    } else if (P.kind == 5) {
      g = (0.5f * tanhf(0.5f * x) + 0.5f - ldv(P.t, e, P.dtt)) * s;
    } else {
      const float dd = d2[m];
      float coef;
      if (P.label[m] > 0.f)
        coef = 1.f;
      else if (P.legacy)
        coef = P.margin - dd > 0.f ? -1.f : 0.f;
      else {
        const float dist = sqrtf(dd), md = P.margin - dist;
        coef = md > 0.f ? -md / (dist + 1e-4f) : 0.f;
      }
      g = coef * (x - ldv(P.t, e, P.dtt)) * s;
    }
    stv(dx, e, P.dtx, g);
  }
}

// ---------------------------------------------------------------------------------------
// Stochastic pooling (pooling_layer.cu StoPoolForwardTrain / StoPoolForwardTest) on NHWC
// bf16, windows without padding.  Train: u ~ U[0,1) from Philox(seed, counter, layer
// stream, element), take the first window element whose running sum reaches u * sum, and
// record its window offset in the uint8 mask that the max-pool backward gathers with.
// Test: sum(x^2) / sum(x) (running sum starts at FLT_MIN, as in Caffe).
// ---------------------------------------------------------------------------------------
__global__ void __launch_bounds__(256) stopool_k(const bf16_t* __restrict__ x, bf16_t* __restrict__ y,
                                                 uint8_t* __restrict__ mask, int N, int H, int W, int C, int P, int Q,
                                                 int kh, int kw, int sh, int sw, const long long* __restrict__ rng,
                                                 int stream, int train) {
  const long long n = (long long)N * P * Q * C, stride = (long long)gridDim.x * blockDim.x;
  const unsigned long long seed = rng ? (unsigned long long)rng[0] : 0ull;
  const unsigned long long counter = rng ? (unsigned long long)rng[1] : 0ull;
  const uint2 key = make_uint2((uint32_t)seed, (uint32_t)(seed >> 32));
  for (long long e = blockIdx.x * (long long)blockDim.x + threadIdx.x; e < n; e += stride) {
    const int c = (int)(e % C);
    const long long pix = e / C;
    const int q = (int)(pix % Q), p = (int)((pix / Q) % P), nn = (int)(pix / ((long long)P * Q));
    const int hs = p * sh, ws = q * sw, he = min(hs + kh, H), we = min(ws + kw, W);
    const bf16_t* base = x + ((long long)nn * H * W) * C + c;
    if (train) {
      float sum = 0.f;
      for (int h = hs; h < he; ++h)
        for (int w = ws; w < we; ++w) sum += bf2f(base[((long long)h * W + w) * C]);
      const uint4 ctr = make_uint4((uint32_t)e, (uint32_t)(e >> 32) | ((uint32_t)(stream & 0xffff) << 16),
                                   (uint32_t)counter, (uint32_t)(counter >> 32) ^ 0x5170u);
      const float u = (float)(philox4x32(key, ctr).x >> 8) * (1.f / 16777216.f);
      const float thr = u * sum;
      float cum = 0.f, pick = 0.f;
      int widx = 0;
      bool found = false;
      for (int h = hs; h < he && !found; ++h)
        for (int w = ws; w < we; ++w) {
          const float v = bf2f(base[((long long)h * W + w) * C]);
          cum += v;
          if (cum >= thr) {
            pick = v;
            widx = (h - hs) * kw + (w - ws);
            found = true;
            break;
          }
        }
      y[e] = f2bf(pick);
      mask[e] = (uint8_t)widx;
    } else {
      float cs = 1.17549435e-38f, cv = 0.f;
      for (int h = hs; h < he; ++h)
        for (int w = ws; w < we; ++w) {
          const float v = bf2f(base[((long long)h * W + w) * C]);
          cs += v;
          cv += v * v;
        }
      y[e] = f2bf(cv / cs);
    }
  }
}

}  // namespace

// =========================================================================================
// C ABI
// =========================================================================================
extern "C" {

int sn_neuron_fwd(long long kind, const void* x, void* y, long long n, long long dtx, long long dty, float a, float b,
                  float c, hipStream_t st) {
  const NP p{a, b, c};
  const int g = grid_for((n & 7) ? n : n / 8);
  switch (kind) {
#define SN_NF(K) \
  case K: hipLaunchKernelGGL(neuron_fwd_k<K>, dim3(g), dim3(256), 0, st, x, y, n, (int)dtx, (int)dty, p); break;
    SN_NF(NK_SIGMOID) SN_NF(NK_TANH) SN_NF(NK_ABSVAL) SN_NF(NK_BNLL) SN_NF(NK_EXP) SN_NF(NK_LOG) SN_NF(NK_POWER)
    SN_NF(NK_THRESHOLD)
#undef SN_NF
    default: return 2;
  }
  return SN_CHECK_LAUNCH();
}

int sn_neuron_bwd(long long kind, const void* x, const void* y, const void* dy, void* dx, long long n, long long dtx,
                  long long dty, long long dtd, float a, float b, float c, hipStream_t st) {
  const NP p{a, b, c};
  const int g = grid_for((n & 7) ? n : n / 8);
  switch (kind) {
#define SN_NB(K)                                                                                              \
  case K:                                                                                                     \
    hipLaunchKernelGGL(neuron_bwd_k<K>, dim3(g), dim3(256), 0, st, x, y, dy, dx, n, (int)dtx, (int)dty, (int)dtd, \
                       p);                                                                                    \
    break;
    SN_NB(NK_SIGMOID) SN_NB(NK_TANH) SN_NB(NK_ABSVAL) SN_NB(NK_BNLL) SN_NB(NK_EXP) SN_NB(NK_LOG) SN_NB(NK_POWER)
#undef SN_NB
    default: return 2;
  }
  return SN_CHECK_LAUNCH();
}

int sn_prelu_fwd(const void* x, const float* slope, void* y, long long n, long long C, long long inner, long long dtx,
                 long long dt, hipStream_t st) {
  hipLaunchKernelGGL(prelu_fwd_k, dim3(grid_for(n)), dim3(256), 0, st, x, slope, y, n, (int)C, inner, (int)dtx, (int)dt);
  return SN_CHECK_LAUNCH();
}

int sn_prelu_bwd(const void* x, const void* dy, const float* slope, void* dx, long long n, long long C,
                 long long inner, long long dtx, long long dt, hipStream_t st) {
  hipLaunchKernelGGL(prelu_bwd_k, dim3(grid_for(n)), dim3(256), 0, st, x, dy, slope, dx, n, (int)C, inner, (int)dtx,
                     (int)dt);
  return SN_CHECK_LAUNCH();
}

// workspace `part` must hold splits * B * A floats; sn_axis_reduce_splits tells how many
long long sn_axis_reduce_splits(long long B, long long outer, long long A, long long inner) {
  const long long blocks = inner == 1 ? B * ((A + 63) / 64) : B * A;
  const long long work = inner == 1 ? outer / 256 : outer * inner / 2048;
  long long s = 512 / (blocks > 0 ? blocks : 1);
  if (s > work) s = work;
  if (s < 1) s = 1;
  if (s > 256) s = 256;
  return s;
}

int sn_axis_reduce(long long mode, const void* p, const void* q, long long dtp, long long dtq, long long B,
                   long long outer, long long A, long long inner, float* part, float* out, float scale, long long acc,
                   hipStream_t st) {
  const int splits = (int)sn_axis_reduce_splits(B, outer, A, inner);
  if (B > 65535 || splits > 65535) return 3;
  if (inner == 1) {
    const dim3 grid((unsigned)((A + 63) / 64), splits, (unsigned)B);
    switch (mode) {
#define SN_CR(M) \
  case M: hipLaunchKernelGGL(colred_k<M>, grid, dim3(256), 0, st, p, q, (int)dtp, (int)dtq, outer, (int)A, splits, part, (int)B); break;
      SN_CR(0) SN_CR(1) SN_CR(2) SN_CR(3) SN_CR(4) SN_CR(5)
#undef SN_CR
      default: return 2;
    }
  } else {
    if (A > 2147483647LL) return 3;
    const dim3 grid((unsigned)A, splits, (unsigned)B);
    switch (mode) {
#define SN_SR(M)                                                                                                 \
  case M:                                                                                                        \
    hipLaunchKernelGGL(segred_k<M>, grid, dim3(256), 0, st, p, q, (int)dtp, (int)dtq, outer, (int)A, inner, splits, \
                       part, (int)B);                                                                            \
    break;
      SN_SR(0) SN_SR(1) SN_SR(2) SN_SR(3) SN_SR(4) SN_SR(5)
#undef SN_SR
      default: return 2;
    }
  }
  if (hipGetLastError() != hipSuccess) return 1;
  hipLaunchKernelGGL(combine_k, dim3(grid_for(B * A)), dim3(256), 0, st, part, splits, B * A, out, scale, (int)acc);
  return SN_CHECK_LAUNCH();
}

int sn_chan_affine(const void* x, void* y, long long n, long long outer, long long A, long long inner,
                   const float* mean, const float* inv, long long dtx, long long dty, hipStream_t st) {
  hipLaunchKernelGGL(chan_affine_k, dim3(grid_for(n)), dim3(256), 0, st, x, y, n, outer, (int)A, inner, mean, inv,
                     (int)dtx, (int)dty);
  return SN_CHECK_LAUNCH();
}

int sn_norm_bwd(const void* dy, const void* xhat, void* dx, long long n, long long outer, long long A, long long inner,
                const float* m1, const float* m2, const float* inv, long long dtd, long long dtx, hipStream_t st) {
  hipLaunchKernelGGL(norm_bwd_k, dim3(grid_for(n)), dim3(256), 0, st, dy, xhat, dx, n, outer, (int)A, inner, m1, m2,
                     inv, (int)dtd, (int)dtx);
  return SN_CHECK_LAUNCH();
}

int sn_stats_finalize(const float* s1, const float* s2, long long n, float inv_count, float eps, long long mode,
                      float* mean, float* var, float* inv, hipStream_t st) {
  hipLaunchKernelGGL(stats_finalize_k, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, st, s1, s2, (int)n, inv_count,
                     eps, (int)mode, mean, var, inv);
  return SN_CHECK_LAUNCH();
}

int sn_bn_running(float* mean, float* var, float* factor, const float* bmean, const float* bvar, long long C,
                  float frac, float unbias, hipStream_t st) {
  hipLaunchKernelGGL(bn_running_k, dim3((unsigned)((C + 255) / 256)), dim3(256), 0, st, mean, var, factor, bmean, bvar,
                     (int)C, frac, unbias);
  return SN_CHECK_LAUNCH();
}

int sn_bn_global(const float* rm, const float* rv, const float* factor, long long C, float eps, float* mean,
                 float* inv, hipStream_t st) {
  hipLaunchKernelGGL(bn_global_k, dim3((unsigned)((C + 255) / 256)), dim3(256), 0, st, rm, rv, factor, (int)C, eps,
                     mean, inv);
  return SN_CHECK_LAUNCH();
}

int sn_eltwise_fwd(const void* const* ptrs, const float* coeffs, long long K, long long op, void* y, int* mask,
                   long long n, long long dt, hipStream_t st) {
  if (K < 1 || K > 16) return 2;
  EPtrs e;
  for (int k = 0; k < 16; ++k) {
    e.p[k] = k < K ? ptrs[k] : nullptr;
    e.coeff[k] = (k < K && coeffs) ? coeffs[k] : 1.f;
  }
  hipLaunchKernelGGL(eltwise_fwd_k, dim3(grid_for(n)), dim3(256), 0, st, e, (int)K, (int)op, y, mask, n, (int)dt);
  return SN_CHECK_LAUNCH();
}

int sn_eltwise_bwd(const void* const* ptrs, const float* coeffs, long long K, long long op, long long which,
                   long long stable, const void* y, const void* dy, const int* mask, void* dx, long long n,
                   long long dt, hipStream_t st) {
  if (K < 1 || K > 16) return 2;
  EPtrs e;
  for (int k = 0; k < 16; ++k) {
    e.p[k] = k < K ? ptrs[k] : nullptr;
    e.coeff[k] = (k < K && coeffs) ? coeffs[k] : 1.f;
  }
  hipLaunchKernelGGL(eltwise_bwd_k, dim3(grid_for(n)), dim3(256), 0, st, e, (int)K, (int)op, (int)which, (int)stable,
                     y, dy, mask, dx, n, (int)dt);
  return SN_CHECK_LAUNCH();
}

int sn_axis_copy(const void* src, void* dst, long long outer, long long srcA, long long dstA, long long inner,
                 long long src_off, long long dst_off, long long cnt, long long dts, long long dtd, long long acc,
                 hipStream_t st) {
  hipLaunchKernelGGL(axis_copy_k, dim3(grid_for(outer * cnt * inner)), dim3(256), 0, st, src, dst, outer, srcA, dstA,
                     inner, src_off, dst_off, cnt, (int)dts, (int)dtd, (int)acc);
  return SN_CHECK_LAUNCH();
}

int sn_tile_bwd(const void* src, void* dst, long long outer, long long A, long long inner, long long tiles,
                long long dt, hipStream_t st) {
  hipLaunchKernelGGL(tile_bwd_k, dim3(grid_for(outer * A * inner)), dim3(256), 0, st, src, dst, outer, A, inner,
                     (int)tiles, (int)dt);
  return SN_CHECK_LAUNCH();
}

int sn_transpose(const void* src, void* dst, long long N, long long R, long long Ccols, long long dts, long long dtd,
                 hipStream_t st) {
  if (N > 65535 || (R + 63) / 64 > 65535) return 3;
  const dim3 grid((unsigned)((Ccols + 63) / 64), (unsigned)((R + 63) / 64), (unsigned)N);
  hipLaunchKernelGGL(transpose_k, grid, dim3(256), 0, st, src, dst, R, Ccols, (int)dts, (int)dtd);
  return SN_CHECK_LAUNCH();
}

int sn_gather_rows(const void* src, const void* idx, long long idx_int, void* dst, long long rows, long long row_len,
                   const float* bias, long long dts, long long dtd, hipStream_t st) {
  hipLaunchKernelGGL(gather_rows_k, dim3(grid_for(rows * row_len)), dim3(256), 0, st, src, idx, (int)idx_int, dst, rows,
                     row_len, bias, (int)dts, (int)dtd);
  return SN_CHECK_LAUNCH();
}

int sn_index_add_rows(const void* src, const void* idx, long long idx_int, long long n_idx, void* dst,
                      long long n_dst, long long row_len, long long dts, long long dtd, long long acc, hipStream_t st) {
  for (long long r0 = 0; r0 < n_dst; r0 += 65535) {
    const long long nr = n_dst - r0 < 65535 ? n_dst - r0 : 65535;
    const dim3 grid((unsigned)((row_len + 255) / 256), (unsigned)nr);
    hipLaunchKernelGGL(index_add_rows_k, grid, dim3(256), 0, st, src, idx, (int)idx_int, n_idx, dst, r0, row_len,
                       (int)dts, (int)dtd, (int)acc);
    if (hipGetLastError() != hipSuccess) return 1;
  }
  return 0;
}

int sn_reduction_bwd(const void* x, const float* dy, void* dx, long long segs, long long L, long long op, float coeff,
                     long long dt, hipStream_t st) {
  hipLaunchKernelGGL(reduction_bwd_k, dim3(grid_for(segs * L)), dim3(256), 0, st, x, dy, dx, segs, L, (int)op, coeff,
                     (int)dt);
  return SN_CHECK_LAUNCH();
}

int sn_topk(const void* x, long long outer, long long A, long long inner, long long k, long long out_max_val,
            long long axis_mode, float* out, long long dt, hipStream_t st) {
  if (k < 1 || k > A) return 2;
  const long long segs = outer * inner;
  hipLaunchKernelGGL(topk_k, dim3((unsigned)((segs + 255) / 256)), dim3(256), 0, st, x, outer, A, inner, (int)k,
                     (int)out_max_val, (int)axis_mode, out, (int)dt);
  return SN_CHECK_LAUNCH();
}

int sn_im2col_caffe(const void* x, void* col, long long N, long long H, long long W, long long C, long long P,
                    long long Q, long long R, long long S, long long sh, long long sw, long long ph, long long pw,
                    long long dh, long long dw, long long dt, hipStream_t st) {
  const I2C g{(int)N, (int)H, (int)W, (int)C, (int)P, (int)Q, (int)R, (int)S, (int)sh, (int)sw, (int)ph, (int)pw,
              (int)dh, (int)dw};
  hipLaunchKernelGGL(im2col_caffe_k, dim3(grid_for(N * P * Q * C * R * S)), dim3(256), 0, st, x, col, g, (int)dt);
  return SN_CHECK_LAUNCH();
}

int sn_col2im_caffe(const void* dcol, void* dx, long long N, long long H, long long W, long long C, long long P,
                    long long Q, long long R, long long S, long long sh, long long sw, long long ph, long long pw,
                    long long dh, long long dw, long long dt, hipStream_t st) {
  const I2C g{(int)N, (int)H, (int)W, (int)C, (int)P, (int)Q, (int)R, (int)S, (int)sh, (int)sw, (int)ph, (int)pw,
              (int)dh, (int)dw};
  hipLaunchKernelGGL(col2im_caffe_k, dim3(grid_for(N * H * W * C)), dim3(256), 0, st, dcol, dx, g, (int)dt);
  return SN_CHECK_LAUNCH();
}

// row_loss must hold 3 * M floats for kind 6 (loss, d2, spare), M otherwise
int sn_loss_rows_fwd(long long kind, const void* x, const void* t, const float* label, const float* H, long long M,
                     long long C, long long dtx, long long dtt, float margin, long long legacy, float* row_loss,
                     hipStream_t st) {
  if (M > 2147483647LL || M <= 0) return M == 0 ? 0 : 3;
  const LossP P{(int)kind, (int)M, (int)C, (int)dtx, (int)dtt, x, t, label, H, margin, (int)legacy};
  hipLaunchKernelGGL(loss_rows_fwd_k, dim3((unsigned)M), dim3(64), 0, st, P, row_loss);
  return SN_CHECK_LAUNCH();
}

int sn_loss_rows_bwd(long long kind, const void* x, const void* t, const float* label, const float* H, long long M,
                     long long C, long long dtx, long long dtt, float margin, long long legacy,
                     const float* loss_weight, float scale, float sign, const float* d2, void* dx, hipStream_t st) {
  const LossP P{(int)kind, (int)M, (int)C, (int)dtx, (int)dtt, x, t, label, H, margin, (int)legacy};
  hipLaunchKernelGGL(loss_rows_bwd_k, dim3(grid_for(M * C)), dim3(256), 0, st, P, loss_weight, scale, sign, d2, dx);
  return SN_CHECK_LAUNCH();
}

int sn_stopool(const bf16_t* x, bf16_t* y, uint8_t* mask, long long N, long long H, long long W, long long C,
               long long P, long long Q, long long kh, long long kw, long long sh, long long sw, const long long* rng,
               long long stream, long long train, hipStream_t st) {
  if (kh * kw > 255) return 2;
  hipLaunchKernelGGL(stopool_k, dim3(grid_for(N * P * Q * C)), dim3(256), 0, st, x, y, mask, (int)N, (int)H, (int)W,
                     (int)C, (int)P, (int)Q, (int)kh, (int)kw, (int)sh, (int)sw, rng, (int)stream, (int)train);
  return SN_CHECK_LAUNCH();
}

}  // extern "C"
