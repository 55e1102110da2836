// Local response normalisation on NHWC bf16 (fp32 math).
//
// ACROSS_CHANNELS — reference: LRNFillScale + LRNComputeOutput + LRNComputeDiff
// (caffe/src/caffe/layers/lrn_layer.cu:9-177), three launches with an fp32 scale buffer
// written and re-read in NCHW.  Here: channels are contiguous, so one thread owns 8
// channels of a pixel and reads its two neighbour chunks (the window never spans more
// than +-8 channels for local_size <= 9); forward is one pass (x -> y, no scale buffer),
// backward recomputes the scales from x and is one pass (x, dy -> dx).
//   scale_c = k + alpha/size * sum_{c' in [c-pre, c+post]} x_c'^2
//   y_c     = x_c * scale_c^-beta
//   dx_c    = dy_c * scale_c^-beta - 2 alpha beta / size * x_c *
//             sum_{c' : c in window(c')} dy_c' * y_c' / scale_c'
//
// WITHIN_CHANNEL — reference: a 5-layer composite (Split, Power, Pool AVE, Power,
// Eltwise PROD; lrn_layer.cpp:18-65).  Here two fused kernels:
//   s = 1 + alpha/size^2 * boxsum_{size x size}(x^2),  y = x * s^-beta
//   dx = dy * s^-beta - 2 alpha beta / size^2 * x * boxsum(dy * x * s^(-beta-1))
#include "common.h"

struct LrnP {
  int N, H, W, C, size, pre;
  float alpha, beta, k;
  FDiv fcv;  // C / 8
  int gate;  // backward: zero dx where x <= 0 (the in-place ReLU that produced x, fused)
};

SN_DEV float powneg(float s, float beta) { return sn_powneg(s, beta); }

// The across-channel kernels (here and in pool_lrn.hip) spell out every multiply-add that
// -ffp-contract=fast could otherwise fuse or not depending on how a loop is unrolled: the
// square sums and the scale are explicit fmas, and the products the backward sums are
// rounded on their own (an fma with a zero addend, which the adds cannot absorb).  A rolled
// square sum had compiled to v_fma_f32 and the unrolled one in the fused LRN -> pool
// backward to v_pk_mul_f32 + v_add_f32: the fused and unfused paths differed by one ulp.
// Load the 24 channels [c0-8, c0+16) of a pixel as fp32 (zeros outside [0, C)).  The
// three 16-B loads are unconditional (clamped chunk index) and masked afterwards, so
// they are all in flight together.
SN_DEV void load24(const bf16_t* row, int c0, int C, float* v) {
  uint4 raw[3];
#pragma unroll
  for (int j = 0; j < 3; ++j) {
    const int c = min(max(c0 - 8 + 8 * j, 0), C - 8);
    raw[j] = *reinterpret_cast<const uint4*>(row + c);
  }
#pragma unroll
  for (int j = 0; j < 3; ++j) {
    const int c = c0 - 8 + 8 * j;
    const bool ok = c >= 0 && c < C;
    unpack8(raw[j], v + 8 * j);
#pragma unroll
    for (int t = 0; t < 8; ++t) v[8 * j + t] = ok ? v[8 * j + t] : 0.f;
  }
}

template <int SIZE>
__global__ void lrn_across_fwd(const bf16_t* __restrict__ x, bf16_t* __restrict__ y, LrnP p) {
  constexpr int PRE = (SIZE - 1) / 2;
  const int cv = p.C / 8;
  const long long total = (long long)p.N * p.H * p.W * cv;
  const float a = p.alpha / p.size;
  for (long long i = blockIdx.x * (long long)blockDim.x + threadIdx.x; i < total;
       i += (long long)gridDim.x * blockDim.x) {
    const uint32_t pix = udiv((uint32_t)i, p.fcv);
    const int c0 = (int)((uint32_t)i - pix * cv) * 8;
    const bf16_t* row = x + (long long)pix * p.C;
    float v[24];
    load24(row, c0, p.C, v);
    float o[8];
#pragma unroll
    for (int t = 0; t < 8; ++t) {
      float s = 0.f;
#pragma unroll
      for (int d = 0; d < SIZE; ++d) {
        float e = v[8 + t - PRE + d];
        s = __builtin_fmaf(e, e, s);
      }
      float sc = __builtin_fmaf(a, s, p.k);
      o[t] = v[8 + t] * powneg(sc, p.beta);
    }
    *reinterpret_cast<uint4*>(y + (long long)pix * p.C + c0) = pack8(o);
  }
}

template <int SIZE>
__global__ void lrn_across_bwd(const bf16_t* __restrict__ x, const bf16_t* __restrict__ dy,
                               bf16_t* __restrict__ dx, LrnP p) {
  constexpr int PRE = (SIZE - 1) / 2, POST = SIZE - PRE - 1;
  const int cv = p.C / 8;
  const long long total = (long long)p.N * p.H * p.W * cv;
  const float a = p.alpha / p.size;
  const float cache_ratio = 2.f * p.alpha * p.beta / p.size;
  for (long long i = blockIdx.x * (long long)blockDim.x + threadIdx.x; i < total;
       i += (long long)gridDim.x * blockDim.x) {
    const uint32_t pix = udiv((uint32_t)i, p.fcv);
    const int c0 = (int)((uint32_t)i - pix * cv) * 8;
    const long long base = (long long)pix * p.C;
    float xv[24], gv[24];
    load24(x + base, c0, p.C, xv);
    load24(dy + base, c0, p.C, gv);
    // r_j = dy_j * y_j / scale_j = dy_j * x_j * scale_j^(-beta-1), for j in [c0-8+pre.., ...]
    float r[24];
#pragma unroll
    for (int j = 8 - POST; j < 16 + PRE; ++j) {
      float s = 0.f;
#pragma unroll
      for (int d = 0; d < SIZE; ++d) {
        float e = xv[j - PRE + d];
        s = __builtin_fmaf(e, e, s);
      }
      float sc = __builtin_fmaf(a, s, p.k);
      // channels outside [0, C) have x = dy = 0 (load24), so r is 0 there without a branch
      r[j] = __builtin_fmaf(gv[j] * xv[j], powneg(sc, p.beta + 1.f), 0.f);
      if (j >= 8 && j < 16) gv[j] = gv[j] * powneg(sc, p.beta);  // reuse: dy * scale^-beta
    }
    float o[8];
#pragma unroll
    for (int t = 0; t < 8; ++t) {
      float acc = 0.f;
      // windows that contain channel c = c0+t start at c' - pre <= c <= c' + post
#pragma unroll
      for (int d = -PRE; d <= POST; ++d) acc += r[8 + t - d];
      o[t] = __builtin_fmaf(-(cache_ratio * xv[8 + t]), acc, gv[8 + t]);
      if (p.gate && !(xv[8 + t] > 0.f)) o[t] = 0.f;
    }
    *reinterpret_cast<uint4*>(dx + base + c0) = pack8(o);
  }
}

// Generic scalar fallback (any C, any odd size): one thread per pixel, sliding window.
__global__ void lrn_across_fwd_scalar(const bf16_t* __restrict__ x, bf16_t* __restrict__ y, LrnP p) {
  const long long npix = (long long)p.N * p.H * p.W;
  const float a = p.alpha / p.size;
  for (long long i = blockIdx.x * (long long)blockDim.x + threadIdx.x; i < npix;
       i += (long long)gridDim.x * blockDim.x) {
    const bf16_t* row = x + i * p.C;
    for (int c = 0; c < p.C; ++c) {
      float s = 0.f;
      for (int d = 0; d < p.size; ++d) {
        int cc = c - p.pre + d;
        if (cc >= 0 && cc < p.C) { float e = bf2f(row[cc]); s = __builtin_fmaf(e, e, s); }
      }
      y[i * p.C + c] = f2bf(bf2f(row[c]) * powneg(__builtin_fmaf(a, s, p.k), p.beta));
    }
  }
}

__global__ void lrn_across_bwd_scalar(const bf16_t* __restrict__ x, const bf16_t* __restrict__ dy,
                                      bf16_t* __restrict__ dx, LrnP p) {
  const long long npix = (long long)p.N * p.H * p.W;
  const float a = p.alpha / p.size;
  const float cache_ratio = 2.f * p.alpha * p.beta / p.size;
  const int post = p.size - p.pre - 1;
  for (long long i = blockIdx.x * (long long)blockDim.x + threadIdx.x; i < npix;
       i += (long long)gridDim.x * blockDim.x) {
    const bf16_t* xr = x + i * p.C;
    const bf16_t* gr = dy + i * p.C;
    for (int c = 0; c < p.C; ++c) {
      float acc = 0.f, own = 0.f;
      for (int cp = c - post; cp <= c + p.pre; ++cp) {
        if (cp < 0 || cp >= p.C) continue;
        float s = 0.f;
        for (int d = 0; d < p.size; ++d) {
          int cc = cp - p.pre + d;
          if (cc >= 0 && cc < p.C) { float e = bf2f(xr[cc]); s = __builtin_fmaf(e, e, s); }
        }
        float sc = __builtin_fmaf(a, s, p.k);
        acc += __builtin_fmaf(bf2f(gr[cp]) * bf2f(xr[cp]), powneg(sc, p.beta + 1.f), 0.f);
        if (cp == c) own = bf2f(gr[c]) * powneg(sc, p.beta);
      }
      const float v = __builtin_fmaf(-(cache_ratio * bf2f(xr[c])), acc, own);
      dx[i * p.C + c] = f2bf(p.gate && !(bf2f(xr[c]) > 0.f) ? 0.f : v);
    }
  }
}

// ---- WITHIN_CHANNEL ----------------------------------------------------------------
// pass A (fwd): y = x * s^-beta, also writes t = s (fp32) for backward when t != null.
__global__ void lrn_within_fwd(const bf16_t* __restrict__ x, bf16_t* __restrict__ y, float* __restrict__ sbuf,
                               LrnP p) {
  const long long total = (long long)p.N * p.H * p.W * p.C;
  const float a = p.alpha / (float)(p.size * p.size);
  for (long long i = blockIdx.x * (long long)blockDim.x + threadIdx.x; i < total;
       i += (long long)gridDim.x * blockDim.x) {
    const int c = (int)(i % p.C);
    long long pix = i / p.C;
    const int w = (int)(pix % p.W), h = (int)((pix / p.W) % p.H), n = (int)(pix / ((long long)p.W * p.H));
    float s = 0.f;
    for (int dh = 0; dh < p.size; ++dh) {
      int hh = h - p.pre + dh;
      if (hh < 0 || hh >= p.H) continue;
      for (int dw = 0; dw < p.size; ++dw) {
        int ww = w - p.pre + dw;
        if (ww < 0 || ww >= p.W) continue;
        float e = bf2f(x[(((long long)n * p.H + hh) * p.W + ww) * p.C + c]);
        s += e * e;
      }
    }
    float sc = 1.f + a * s;
    if (sbuf) sbuf[i] = sc;
    y[i] = f2bf(bf2f(x[i]) * powneg(sc, p.beta));
  }
}

// pass B (bwd 1): u = dy * x * s^(-beta-1) (fp32)
__global__ void lrn_within_bwd_u(const bf16_t* __restrict__ x, const bf16_t* __restrict__ dy,
                                 const float* __restrict__ sbuf, float* __restrict__ u, LrnP p) {
  const long long total = (long long)p.N * p.H * p.W * p.C;
  for (long long i = blockIdx.x * (long long)blockDim.x + threadIdx.x; i < total;
       i += (long long)gridDim.x * blockDim.x)
    u[i] = bf2f(dy[i]) * bf2f(x[i]) * powneg(sbuf[i], p.beta + 1.f);
}

// pass C (bwd 2): dx = dy * s^-beta - 2 a beta x * boxsum(u)
__global__ void lrn_within_bwd_dx(const bf16_t* __restrict__ x, const bf16_t* __restrict__ dy,
                                  const float* __restrict__ sbuf, const float* __restrict__ u,
                                  bf16_t* __restrict__ dx, LrnP p) {
  const long long total = (long long)p.N * p.H * p.W * p.C;
  const float a = p.alpha / (float)(p.size * p.size);
  for (long long i = blockIdx.x * (long long)blockDim.x + threadIdx.x; i < total;
       i += (long long)gridDim.x * blockDim.x) {
    const int c = (int)(i % p.C);
    long long pix = i / p.C;
    const int w = (int)(pix % p.W), h = (int)((pix / p.W) % p.H), n = (int)(pix / ((long long)p.W * p.H));
    float acc = 0.f;
    // windows centred at (hh, ww) contain (h, w) iff |hh-h| <= pre (odd size, stride 1)
    for (int dh = 0; dh < p.size; ++dh) {
      int hh = h - p.pre + dh;
      if (hh < 0 || hh >= p.H) continue;
      for (int dw = 0; dw < p.size; ++dw) {
        int ww = w - p.pre + dw;
        if (ww < 0 || ww >= p.W) continue;
        acc += u[(((long long)n * p.H + hh) * p.W + ww) * p.C + c];
      }
    }
    dx[i] = f2bf(bf2f(dy[i]) * powneg(sbuf[i], p.beta) - 2.f * a * p.beta * bf2f(x[i]) * acc);
  }
}

static LrnP mk(long long N, long long H, long long W, long long C, long long size, float alpha, float beta,
               float k) {
  LrnP p;
  p.N = (int)N; p.H = (int)H; p.W = (int)W; p.C = (int)C; p.size = (int)size; p.pre = (int)((size - 1) / 2);
  p.alpha = alpha; p.beta = beta; p.k = k;
  p.fcv = make_fdiv((uint32_t)(C % 8 == 0 ? C / 8 : 1));
  p.gate = 0;
  return p;
}

extern "C" int sn_lrn_across_fwd(const bf16_t* x, bf16_t* y, long long N, long long H, long long W, long long C,
                                 long long size, float alpha, float beta, float k, hipStream_t st) {
  LrnP p = mk(N, H, W, C, size, alpha, beta, k);
  if (N * H * W * C >= (1ll << 32)) return 8;  // 32-bit index decode
  dim3 g8(sn_blocks(N * H * W * (C / 8), 256, 16384));
  if (C % 8 == 0 && size == 3) {
    hipLaunchKernelGGL(lrn_across_fwd<3>, g8, dim3(256), 0, st, x, y, p);
  } else if (C % 8 == 0 && size == 5) {
    hipLaunchKernelGGL(lrn_across_fwd<5>, g8, dim3(256), 0, st, x, y, p);
  } else if (C % 8 == 0 && size == 7) {
    hipLaunchKernelGGL(lrn_across_fwd<7>, g8, dim3(256), 0, st, x, y, p);
  } else if (C % 8 == 0 && size == 9) {
    hipLaunchKernelGGL(lrn_across_fwd<9>, g8, dim3(256), 0, st, x, y, p);
  } else {
    hipLaunchKernelGGL(lrn_across_fwd_scalar, dim3(sn_blocks(N * H * W, 256, 16384)), dim3(256), 0, st, x, y, p);
  }
  return SN_CHECK_LAUNCH();
}

extern "C" int sn_lrn_across_bwd(const bf16_t* x, const bf16_t* dy, bf16_t* dx, long long N, long long H,
                                 long long W, long long C, long long size, float alpha, float beta, float k,
                                 long long gate, hipStream_t st) {
  LrnP p = mk(N, H, W, C, size, alpha, beta, k);
  p.gate = (int)gate;
  if (N * H * W * C >= (1ll << 32)) return 8;  // 32-bit index decode
  dim3 g8(sn_blocks(N * H * W * (C / 8), 256, 16384));
  if (C % 8 == 0 && size == 3) {
    hipLaunchKernelGGL(lrn_across_bwd<3>, g8, dim3(256), 0, st, x, dy, dx, p);
  } else if (C % 8 == 0 && size == 5) {
    hipLaunchKernelGGL(lrn_across_bwd<5>, g8, dim3(256), 0, st, x, dy, dx, p);
  } else if (C % 8 == 0 && size == 7) {
    hipLaunchKernelGGL(lrn_across_bwd<7>, g8, dim3(256), 0, st, x, dy, dx, p);
  } else if (C % 8 == 0 && size == 9) {
    hipLaunchKernelGGL(lrn_across_bwd<9>, g8, dim3(256), 0, st, x, dy, dx, p);
  } else {
    hipLaunchKernelGGL(lrn_across_bwd_scalar, dim3(sn_blocks(N * H * W, 256, 16384)), dim3(256), 0, st, x, dy, dx,
                       p);
  }
  return SN_CHECK_LAUNCH();
}

extern "C" int sn_lrn_within_fwd(const bf16_t* x, bf16_t* y, float* sbuf, long long N, long long H, long long W,
                                 long long C, long long size, float alpha, float beta, hipStream_t st) {
  LrnP p = mk(N, H, W, C, size, alpha, beta, 1.f);
  hipLaunchKernelGGL(lrn_within_fwd, dim3(sn_blocks(N * H * W * C, 256, 16384)), dim3(256), 0, st, x, y, sbuf, p);
  return SN_CHECK_LAUNCH();
}

extern "C" int sn_lrn_within_bwd(const bf16_t* x, const bf16_t* dy, float* sbuf, float* u, bf16_t* dx, long long N,
                                 long long H, long long W, long long C, long long size, float alpha, float beta,
                                 hipStream_t st) {
  LrnP p = mk(N, H, W, C, size, alpha, beta, 1.f);
  dim3 grid(sn_blocks(N * H * W * C, 256, 16384));
  hipLaunchKernelGGL(lrn_within_fwd, grid, dim3(256), 0, st, x, dx, sbuf, p);  // recompute s (dx as scratch)
  hipLaunchKernelGGL(lrn_within_bwd_u, grid, dim3(256), 0, st, x, dy, sbuf, u, p);
  hipLaunchKernelGGL(lrn_within_bwd_dx, grid, dim3(256), 0, st, x, dy, sbuf, u, dx, p);
  return SN_CHECK_LAUNCH();
}
