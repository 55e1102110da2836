// Elementwise / data-movement kernels on bf16 tensors (16-B vectorised, grid-stride).
//
//  * ReLU fwd/bwd (caffe/src/caffe/layers/relu_layer.cu:9-41) — standalone form; the
//    common conv/IP + in-place ReLU pair is fused into the GEMM epilogue instead.
//  * Dropout fwd/bwd (dropout_layer.cu:10-45 + curandGenerate): the keep mask is
//    Philox4x32-10(seed, counter | element, layer stream) regenerated in backward,
//    so nothing is stored (reference: a uint32 per element).
//  * fp32 -> bf16 cast of the flat parameter buffer (compute shadow refresh).
//  * Philox counter advance (device side, so captured graphs get fresh masks per replay).
//  * Sum of bf16 tensors (Split backward / gradient accumulation).
//  * Channel concat fwd / bwd of NHWC blobs (+ fused ReLU-backward mask).
//  * im2col (explicit, for convs whose per-group channel count is not a multiple of 8 —
//    i.e. the 3-channel input layer), col2im (stride>1 dgrad), weight flip-transpose
//    (turns dgrad into a forward implicit-GEMM conv), batched over a net's layers.
#include "common.h"

#include <cstdint>
#include <cstdlib>
#include <cstring>

// ---------------- ReLU ----------------
// n % 8 != 0: the vector loop covers n / 8 chunks, block 0 finishes the tail scalar.
__global__ void relu_fwd(const bf16_t* __restrict__ x, bf16_t* __restrict__ y, long long n, float slope) {
  const long long n8 = n / 8;
  for (long long i = blockIdx.x * (long long)blockDim.x + threadIdx.x; i < n8; i += (long long)gridDim.x * blockDim.x) {
    float f[8];
    unpack8(reinterpret_cast<const uint4*>(x)[i], f);
#pragma unroll
    for (int k = 0; k < 8; ++k) f[k] = f[k] > 0.f ? f[k] : f[k] * slope;
    reinterpret_cast<uint4*>(y)[i] = pack8(f);
  }
  if (blockIdx.x == 0 && threadIdx.x < (n & 7)) {
    const long long e = n8 * 8 + threadIdx.x;
    const float f = bf2f(x[e]);
    y[e] = f2bf(f > 0.f ? f : f * slope);
  }
}

__global__ void relu_bwd(const bf16_t* __restrict__ dy, const bf16_t* __restrict__ x, bf16_t* __restrict__ dx,
                         long long n, float slope) {
  const long long n8 = n / 8;
  for (long long i = blockIdx.x * (long long)blockDim.x + threadIdx.x; i < n8; i += (long long)gridDim.x * blockDim.x) {
    float g[8], v[8];
    unpack8(reinterpret_cast<const uint4*>(dy)[i], g);
    unpack8(reinterpret_cast<const uint4*>(x)[i], v);
#pragma unroll
    for (int k = 0; k < 8; ++k) g[k] = v[k] > 0.f ? g[k] : g[k] * slope;
    reinterpret_cast<uint4*>(dx)[i] = pack8(g);
  }
  if (blockIdx.x == 0 && threadIdx.x < (n & 7)) {
    const long long e = n8 * 8 + threadIdx.x;
    const float g = bf2f(dy[e]);
    dx[e] = f2bf(bf2f(x[e]) > 0.f ? g : g * slope);
  }
}

extern "C" int sn_relu_fwd(const bf16_t* x, bf16_t* y, long long n, float slope, hipStream_t st) {
  hipLaunchKernelGGL(relu_fwd, dim3(sn_blocks(n / 8 > 0 ? n / 8 : 1, 256, 16384)), dim3(256), 0, st, x, y, n, slope);
  return SN_CHECK_LAUNCH();
}

extern "C" int sn_relu_bwd(const bf16_t* dy, const bf16_t* x, bf16_t* dx, long long n, float slope, hipStream_t st) {
  hipLaunchKernelGGL(relu_bwd, dim3(sn_blocks(n / 8 > 0 ? n / 8 : 1, 256, 16384)), dim3(256), 0, st, dy, x, dx, n,
                     slope);
  return SN_CHECK_LAUNCH();
}

// ---------------- Dropout ----------------
// keep(i) = word i%4 of philox(key=seed, ctr=(i/4 lo, i/4 hi | stream<<16, counter lo, hi)) > thr
// gate (optional, backward only): the in-place ReLU output feeding this dropout — its
// slope-0 backward mask (gate > 0) is applied here instead of in a separate pass.
__global__ void dropout_kernel(const bf16_t* __restrict__ x, bf16_t* __restrict__ y, long long n,
                               const long long* __restrict__ rng, int stream, uint32_t thr, float scale,
                               const bf16_t* __restrict__ gate) {
  auto keep = [&](unsigned long long e) { return dropout_keep(rng, stream, thr, e); };
  const long long n8 = n / 8;
  for (long long i = blockIdx.x * (long long)blockDim.x + threadIdx.x; i < n8; i += (long long)gridDim.x * blockDim.x) {
    float f[8];
    unpack8(reinterpret_cast<const uint4*>(x)[i], f);
    const uint4 u0 = dropout_bits4(rng, stream, (unsigned long long)i * 2), u1 = dropout_bits4(rng, stream, (unsigned long long)i * 2 + 1);
    const uint32_t b[8] = {u0.x, u0.y, u0.z, u0.w, u1.x, u1.y, u1.z, u1.w};
#pragma unroll
    for (int k = 0; k < 8; ++k) f[k] = b[k] > thr ? f[k] * scale : 0.f;
    if (gate) {
      float gv[8];
      unpack8(reinterpret_cast<const uint4*>(gate)[i], gv);
#pragma unroll
      for (int k = 0; k < 8; ++k) f[k] = gv[k] > 0.f ? f[k] : 0.f;
    }
    reinterpret_cast<uint4*>(y)[i] = pack8(f);
  }
  // element counts that are not a multiple of 8: the last n % 8 elements, scalar
  if (blockIdx.x == 0 && threadIdx.x < (n & 7)) {
    const long long e = n8 * 8 + threadIdx.x;
    float f = keep((unsigned long long)e) ? bf2f(x[e]) * scale : 0.f;
    if (gate && !(bf2f(gate[e]) > 0.f)) f = 0.f;
    y[e] = f2bf(f);
  }
}

extern "C" int sn_dropout(const bf16_t* x, bf16_t* y, long long n, const long long* rng, long long stream,
                          float ratio, const bf16_t* gate, hipStream_t st) {
  uint32_t thr = (uint32_t)((double)4294967295u * (double)ratio);
  float scale = 1.f / (1.f - ratio);
  hipLaunchKernelGGL(dropout_kernel, dim3(sn_blocks(n / 8 > 0 ? n / 8 : 1, 256, 16384)), dim3(256), 0, st, x, y, n,
                     rng, (int)stream, thr, scale, gate);
  return SN_CHECK_LAUNCH();
}

__global__ void advance_rng_kernel(long long* rng) {
  if (threadIdx.x == 0) rng[1] += 1;
}

extern "C" int sn_advance_rng(long long* rng, hipStream_t st) {
  hipLaunchKernelGGL(advance_rng_kernel, dim3(1), dim3(64), 0, st, rng);
  return SN_CHECK_LAUNCH();
}

// ---------------- casts / sums ----------------
__global__ void cast_f32_bf16(const float* __restrict__ src, bf16_t* __restrict__ dst, long long n) {
  long long n4 = n / 4;
  for (long long i = blockIdx.x * (long long)blockDim.x + threadIdx.x; i < n4; i += (long long)gridDim.x * blockDim.x) {
    float4 v = reinterpret_cast<const float4*>(src)[i];
    reinterpret_cast<uint2*>(dst)[i] = make_uint2(pack2(v.x, v.y), pack2(v.z, v.w));
  }
  for (long long i = n4 * 4 + blockIdx.x * (long long)blockDim.x + threadIdx.x; i < n; i += (long long)gridDim.x * blockDim.x)
    dst[i] = f2bf(src[i]);
}

extern "C" int sn_cast_f32_bf16(const float* src, bf16_t* dst, long long n, hipStream_t st) {
  hipLaunchKernelGGL(cast_f32_bf16, dim3(sn_blocks(n / 4 + 1, 256, 16384)), dim3(256), 0, st, src, dst, n);
  return SN_CHECK_LAUNCH();
}

// Host-fed input staging for the native step executor (csrc/core/sn_core.cpp): a logical
// NCHW fp32 minibatch (the JavaData callback contract, CaffeLibrary.java:12-14) converted
// to the blob's physical NHWC bf16 layout.  One thread per output element, so the bf16
// stores are coalesced; the fp32 reads stride by H*W (the minibatch sits in L2).
__global__ void stage_nchw_f32_bf16(const float* __restrict__ src, bf16_t* __restrict__ dst, int C, int HW,
                                    long long n) {
  for (long long i = blockIdx.x * (long long)blockDim.x + threadIdx.x; i < n; i += (long long)gridDim.x * blockDim.x) {
    const long long pix = i / C;
    const int c = (int)(i - pix * C);
    const long long img = pix / HW;
    const int hw = (int)(pix - img * HW);
    dst[i] = f2bf(src[(img * C + c) * HW + hw]);
  }
}

extern "C" int sn_stage_nchw_f32_bf16(const float* src, bf16_t* dst, long long N, long long C, long long H,
                                      long long W, hipStream_t st) {
  const long long n = N * C * H * W;
  if (n <= 0) return 0;
  hipLaunchKernelGGL(stage_nchw_f32_bf16, dim3(sn_blocks(n, 256, 16384)), dim3(256), 0, st, src, dst, (int)C,
                     (int)(H * W), n);
  return SN_CHECK_LAUNCH();
}

// out = sum_k in_k (k <= 8), bf16 with fp32 accumulation; K is a template parameter so
// the K loads of an iteration are issued together.
struct Ptrs8 { const bf16_t* p[8]; };
template <int K>
__global__ void sum_bf16(Ptrs8 in, bf16_t* __restrict__ out, long long n8) {
  for (long long i = blockIdx.x * (long long)blockDim.x + threadIdx.x; i < n8; i += (long long)gridDim.x * blockDim.x) {
    uint4 v[K];
#pragma unroll
    for (int j = 0; j < K; ++j) v[j] = reinterpret_cast<const uint4*>(in.p[j])[i];
    float acc[8] = {0, 0, 0, 0, 0, 0, 0, 0};
#pragma unroll
    for (int j = 0; j < K; ++j) {
      float f[8];
      unpack8(v[j], f);
#pragma unroll
      for (int t = 0; t < 8; ++t) acc[t] += f[t];
    }
    reinterpret_cast<uint4*>(out)[i] = pack8(acc);
  }
}

extern "C" int sn_sum_bf16(const bf16_t* const* ptrs, long long k, bf16_t* out, long long n, hipStream_t st) {
  if (n % 8 || k > 8 || k < 1) return 7;
  Ptrs8 in;
  for (int j = 0; j < 8; ++j) in.p[j] = j < k ? ptrs[j] : nullptr;
  const dim3 grid(sn_blocks(n / 8, 256, 16384));
  switch (k) {
#define SN_SUM_CASE(KK) \
  case KK: hipLaunchKernelGGL(sum_bf16<KK>, grid, dim3(256), 0, st, in, out, n / 8); break;
    SN_SUM_CASE(1) SN_SUM_CASE(2) SN_SUM_CASE(3) SN_SUM_CASE(4)
    SN_SUM_CASE(5) SN_SUM_CASE(6) SN_SUM_CASE(7) SN_SUM_CASE(8)
#undef SN_SUM_CASE
  }
  return SN_CHECK_LAUNCH();
}

// ---------------- Channel concat (NHWC) ----------------
// Concat on the channel axis of NHWC bf16 blobs (concat_layer.cu:6-71) as one launch per
// direction; blockIdx.y = part.  Forward copies part i into channels [off_i, off_i + c_i)
// of every pixel; backward slices the top gradient back out and, for parts produced by
// an in-place slope-0 ReLU, applies its mask (gate = the part's own ReLU output), which
// replaces that ReLU's separate backward pass.  Channel counts are multiples of 8.
struct ConcatDesc {
  const bf16_t* part[8];  // forward: part data; backward: part diff (written)
  const bf16_t* gate[8];  // backward only: ReLU output of the part, or null
  int c8[8], off8[8];     // channels / offset in 16-B chunks
  int ct8;                // top channels in chunks
  long long pix;          // N*H*W
};

template <bool BWD>
__global__ void concat_nhwc(ConcatDesc d, bf16_t* __restrict__ top) {
  const int part = blockIdx.y;
  if (!d.part[part]) return;  // backward: a part that needs no gradient
  const int ci8 = d.c8[part];
  const long long total = d.pix * ci8;
  const uint4* g = reinterpret_cast<const uint4*>(d.gate[part]);
  for (long long j = blockIdx.x * (long long)blockDim.x + threadIdx.x; j < total; j += (long long)gridDim.x * blockDim.x) {
    const long long p = j / ci8;
    const long long t = p * d.ct8 + d.off8[part] + (j - p * ci8);
    if (!BWD) {
      reinterpret_cast<uint4*>(top)[t] = reinterpret_cast<const uint4*>(d.part[part])[j];
    } else {
      uint4 v = reinterpret_cast<const uint4*>(top)[t];
      if (g) {
        const uint4 m = g[j];
        // bf16 > 0  <=>  sign clear and magnitude in (0, +inf]  (zero and NaN fail, as in relu_bwd)
        auto keep = [](unsigned int w, unsigned int x) {
          const unsigned int a = w & 0x7fffu, b = (w >> 16) & 0x7fffu;
          const unsigned int lo = ((w & 0x8000u) == 0 && a != 0 && a <= 0x7f80u) ? 0xffffu : 0u;
          const unsigned int hi = ((w & 0x80000000u) == 0 && b != 0 && b <= 0x7f80u) ? 0xffff0000u : 0u;
          return x & (lo | hi);
        };
        v.x = keep(m.x, v.x);
        v.y = keep(m.y, v.y);
        v.z = keep(m.z, v.z);
        v.w = keep(m.w, v.w);
      }
      reinterpret_cast<uint4*>(const_cast<bf16_t*>(d.part[part]))[j] = v;
    }
  }
}

extern "C" int sn_concat_nhwc(const bf16_t* const* parts, const bf16_t* const* gates, const long long* chans,
                              long long nparts, bf16_t* top, long long pix, long long bwd, hipStream_t st) {
  if (nparts < 1 || nparts > 8) return 7;
  ConcatDesc d;
  memset(&d, 0, sizeof(d));
  long long off = 0, maxc = 0;
  for (int i = 0; i < nparts; ++i) {
    if (chans[i] % 8 || chans[i] <= 0) return 7;
    d.part[i] = parts[i];
    d.gate[i] = gates ? gates[i] : nullptr;
    d.c8[i] = (int)(chans[i] / 8);
    d.off8[i] = (int)(off / 8);
    off += chans[i];
    if (chans[i] > maxc) maxc = chans[i];
  }
  d.ct8 = (int)(off / 8);
  d.pix = pix;
  const dim3 grid(sn_blocks(pix * (maxc / 8), 256, 8192), (unsigned)nparts);
  if (bwd)
    hipLaunchKernelGGL(concat_nhwc<true>, grid, dim3(256), 0, st, d, top);
  else
    hipLaunchKernelGGL(concat_nhwc<false>, grid, dim3(256), 0, st, d, top);
  return SN_CHECK_LAUNCH();
}

// ---------------- im2col / col2im / weight flip ----------------
struct ConvG {
  int N, H, W, C, P, Q, R, S, sh, sw, ph, pw, dh, dw, Cg, Kpad, coff;
};

// col[m][k] (row = pixel (n,p,q), k = (r, s, c) with c fastest, zero-padded to Kpad)
__global__ void im2col_nhwc(const bf16_t* __restrict__ x, bf16_t* __restrict__ col, ConvG g) {
  const int kc = g.Kpad / 8;
  const long long total = (long long)g.N * g.P * g.Q * kc;
  const int K = g.R * g.S * g.Cg;
  for (long long i = blockIdx.x * (long long)blockDim.x + threadIdx.x; i < total; i += (long long)gridDim.x * blockDim.x) {
    const int k0 = (int)(i % kc) * 8;
    const long long m = i / kc;
    const int q = (int)(m % g.Q), p = (int)((m / g.Q) % g.P), n = (int)(m / ((long long)g.Q * g.P));
    float f[8];
#pragma unroll
    for (int t = 0; t < 8; ++t) {
      int k = k0 + t;
      float v = 0.f;
      if (k < K) {
        int c = k % g.Cg, tap = k / g.Cg;
        int s = tap % g.S, r = tap / g.S;
        int h = p * g.sh - g.ph + r * g.dh, w = q * g.sw - g.pw + s * g.dw;
        if ((unsigned)h < (unsigned)g.H && (unsigned)w < (unsigned)g.W)
          v = bf2f(x[(((long long)n * g.H + h) * g.W + w) * g.C + g.coff + c]);
      }
      f[t] = v;
    }
    reinterpret_cast<uint4*>(col)[i] = pack8(f);
  }
}

// dx[n,h,w,coff+c] = sum over (p,q,r,s) mapping to (h,w) of dcol[(n,p,q)][(r,s,c)]  (gather)
__global__ void col2im_nhwc(const bf16_t* __restrict__ dcol, bf16_t* __restrict__ dx, ConvG g) {
  const long long total = (long long)g.N * g.H * g.W * g.Cg;
  for (long long i = blockIdx.x * (long long)blockDim.x + threadIdx.x; i < total; i += (long long)gridDim.x * blockDim.x) {
    const int c = (int)(i % g.Cg);
    const long long pix = i / g.Cg;
    const int w = (int)(pix % g.W), h = (int)((pix / g.W) % g.H), n = (int)(pix / ((long long)g.W * g.H));
    float acc = 0.f;
    for (int r = 0; r < g.R; ++r) {
      int hh = h + g.ph - r * g.dh;
      if (hh < 0 || hh % g.sh) continue;
      int p = hh / g.sh;
      if (p >= g.P) continue;
      for (int s = 0; s < g.S; ++s) {
        int ww = w + g.pw - s * g.dw;
        if (ww < 0 || ww % g.sw) continue;
        int q = ww / g.sw;
        if (q >= g.Q) continue;
        acc += bf2f(dcol[(((long long)n * g.P + p) * g.Q + q) * g.Kpad + (r * g.S + s) * g.Cg + c]);
      }
    }
    dx[pix * g.C + g.coff + c] = f2bf(acc);
  }
}

static ConvG mkconv(long long N, long long H, long long W, long long C, long long P, long long Q, long long R,
                    long long S, long long sh, long long sw, long long ph, long long pw, long long dh, long long dw,
                    long long Cg, long long Kpad, long long coff) {
  ConvG g;
  g.N = (int)N; g.H = (int)H; g.W = (int)W; g.C = (int)C; g.P = (int)P; g.Q = (int)Q; g.R = (int)R; g.S = (int)S;
  g.sh = (int)sh; g.sw = (int)sw; g.ph = (int)ph; g.pw = (int)pw; g.dh = (int)dh; g.dw = (int)dw;
  g.Cg = (int)Cg; g.Kpad = (int)Kpad; g.coff = (int)coff;
  return g;
}

extern "C" int sn_im2col(const bf16_t* x, bf16_t* col, long long N, long long H, long long W, long long C, long long P,
                         long long Q, long long R, long long S, long long sh, long long sw, long long ph, long long pw,
                         long long dh, long long dw, long long Cg, long long Kpad, long long coff, hipStream_t st) {
  if (Kpad % 8) return 7;
  ConvG g = mkconv(N, H, W, C, P, Q, R, S, sh, sw, ph, pw, dh, dw, Cg, Kpad, coff);
  long long total = N * P * Q * (Kpad / 8);
  hipLaunchKernelGGL(im2col_nhwc, dim3(sn_blocks(total, 256, 16384)), dim3(256), 0, st, x, col, g);
  return SN_CHECK_LAUNCH();
}

extern "C" int sn_col2im(const bf16_t* dcol, bf16_t* dx, long long N, long long H, long long W, long long C,
                         long long P, long long Q, long long R, long long S, long long sh, long long sw, long long ph,
                         long long pw, long long dh, long long dw, long long Cg, long long Kpad, long long coff,
                         hipStream_t st) {
  ConvG g = mkconv(N, H, W, C, P, Q, R, S, sh, sw, ph, pw, dh, dw, Cg, Kpad, coff);
  long long total = N * H * W * Cg;
  hipLaunchKernelGGL(col2im_nhwc, dim3(sn_blocks(total, 256, 16384)), dim3(256), 0, st, dcol, dx, g);
  return SN_CHECK_LAUNCH();
}

// w [G][Kg][R][S][Cg]  ->  wt [G][Cg][R][S][Kg] with (r, s) flipped: the dgrad of a
// stride-1 conv is a forward conv of dy with these weights and pad' = R-1-pad.
__global__ void flip_weights(const bf16_t* __restrict__ w, bf16_t* __restrict__ wt, int G, int Kg, int R, int S,
                             int Cg) {
  const long long total = (long long)G * Kg * R * S * Cg;
  for (long long i = blockIdx.x * (long long)blockDim.x + threadIdx.x; i < total; i += (long long)gridDim.x * blockDim.x) {
    int c = (int)(i % Cg);
    long long t = i / Cg;
    int s = (int)(t % S); t /= S;
    int r = (int)(t % R); t /= R;
    int k = (int)(t % Kg);
    int g = (int)(t / Kg);
    long long o = ((((long long)g * Cg + c) * R + (R - 1 - r)) * S + (S - 1 - s)) * Kg + k;
    wt[o] = w[i];
  }
}

extern "C" int sn_flip_weights(const bf16_t* w, bf16_t* wt, long long G, long long Kg, long long R, long long S,
                               long long Cg, hipStream_t st) {
  long long total = G * Kg * R * S * Cg;
  hipLaunchKernelGGL(flip_weights, dim3(sn_blocks(total, 256, 16384)), dim3(256), 0, st, w, wt, (int)G, (int)Kg,
                     (int)R, (int)S, (int)Cg);
  return SN_CHECK_LAUNCH();
}

// The same flip for every stride-1 convolution of a net in ONE launch (blockIdx.y =
// layer), run once at the start of backward: the weights are final for the iteration
// there, and one launch replaces a launch boundary per layer.
struct FlipDesc {
  const bf16_t* w;
  bf16_t* wt;
  int total, Kg, R, S;
  FDiv fKg, fS, fR, fCg;
  int vec;  // Kg, Cg multiples of 8 and both tensors 16-B aligned: 16-B loads and stores
};

// For a fixed group g and tap, W[g][k][tap][c] -> Wt[g][c][RS-1-tap][k] is a [Kg x Cg]
// transpose: one workgroup moves a 64 x 64 tile through LDS so both the reads (along c)
// and the writes (along k) are coalesced (a per-element gather read 2 B per cache line).
__global__ void __launch_bounds__(256) flip_weights_multi(const FlipDesc* __restrict__ descs) {
  __shared__ bf16_t tile[64][66];
  const FlipDesc d = descs[blockIdx.y];
  const int Cg = (int)d.fCg.d, RS = d.R * d.S;
  const int ntk = (d.Kg + 63) >> 6, ntc = (Cg + 63) >> 6;
  const int per_tap = ntk * ntc;
  const int G = d.total / (d.Kg * RS * Cg);
  int b = blockIdx.x;
  if (b >= G * RS * per_tap) return;  // this descriptor has fewer tiles than the grid
  const int gt = b / per_tap, tt = b - gt * per_tap;
  const int g = gt / RS, tap = gt - g * RS;
  const int k0 = (tt / ntc) * 64, c0 = (tt - (tt / ntc) * ntc) * 64;
  const int tapf = RS - 1 - tap;
  if (d.vec) {
    // 16-B chunks: 64 k-rows x 8 c-chunks read (2 per thread), 64 c-rows x 8 k-chunks written,
    // each gathered from 8 tile rows (row stride 66 elements: the 8 reads hit distinct banks);
    // 2 instead of 16 global accesses per thread each way (the 2-byte form ran at ~1.4 TB/s)
#pragma unroll
    for (int i = 0; i < 2; ++i) {
      const int q = threadIdx.x + 256 * i, k = q >> 3, ch = (q & 7) * 8;
      if (k0 + k < d.Kg && c0 + ch < Cg) {
        const uint4 v = *reinterpret_cast<const uint4*>(d.w + ((long long)(g * d.Kg + k0 + k) * RS + tap) * Cg + c0 + ch);
        const uint32_t u[4] = {v.x, v.y, v.z, v.w};
#pragma unroll
        for (int j = 0; j < 4; ++j) {
          tile[k][ch + 2 * j] = (bf16_t)(u[j] & 0xffffu);
          tile[k][ch + 2 * j + 1] = (bf16_t)(u[j] >> 16);
        }
      }
    }
    __syncthreads();
#pragma unroll
    for (int i = 0; i < 2; ++i) {
      const int q = threadIdx.x + 256 * i, c = q >> 3, kk = (q & 7) * 8;
      if (c0 + c < Cg && k0 + kk < d.Kg) {
        uint32_t u[4];
#pragma unroll
        for (int j = 0; j < 4; ++j) u[j] = (uint32_t)tile[kk + 2 * j][c] | ((uint32_t)tile[kk + 2 * j + 1][c] << 16);
        *reinterpret_cast<uint4*>(d.wt + ((long long)(g * Cg + c0 + c) * RS + tapf) * d.Kg + k0 + kk) =
            make_uint4(u[0], u[1], u[2], u[3]);
      }
    }
    return;
  }
  const int r = threadIdx.x >> 6, x = threadIdx.x & 63;
#pragma unroll
  for (int i = 0; i < 16; ++i) {
    const int k = k0 + r + 4 * i, c = c0 + x;
    if (k < d.Kg && c < Cg) tile[r + 4 * i][x] = d.w[((long long)(g * d.Kg + k) * RS + tap) * Cg + c];
  }
  __syncthreads();
#pragma unroll
  for (int i = 0; i < 16; ++i) {
    const int c = c0 + r + 4 * i, k = k0 + x;
    if (k < d.Kg && c < Cg) d.wt[((long long)(g * Cg + c) * RS + tapf) * d.Kg + k] = tile[x][r + 4 * i];
  }
}

// descs: device array of n FlipDesc built by sn_flip_desc (host) and uploaded once.
extern "C" int sn_flip_desc_size() { return (int)sizeof(FlipDesc); }

extern "C" int sn_flip_desc(void* out, const bf16_t* w, bf16_t* wt, long long G, long long Kg, long long R,
                            long long S, long long Cg) {
  FlipDesc d;
  d.w = w;
  d.wt = wt;
  d.total = (int)(G * Kg * R * S * Cg);
  d.Kg = (int)Kg;
  d.R = (int)R;
  d.S = (int)S;
  d.fKg = make_fdiv((uint32_t)Kg);
  d.fS = make_fdiv((uint32_t)S);
  d.fR = make_fdiv((uint32_t)R);
  d.fCg = make_fdiv((uint32_t)Cg);
  d.vec = Kg % 8 == 0 && Cg % 8 == 0 &&
          (reinterpret_cast<uintptr_t>(w) % 16) == 0 && (reinterpret_cast<uintptr_t>(wt) % 16) == 0;
  memcpy(out, &d, sizeof d);
  return 0;
}

extern "C" int sn_flip_weights_multi(const void* descs, long long n, long long max_tiles, hipStream_t st) {
  if (n <= 0 || max_tiles <= 0) return 0;
  dim3 grid((unsigned)max_tiles, (unsigned)n);  // the largest descriptor's 64 x 64 tile count
  hipLaunchKernelGGL(flip_weights_multi, grid, dim3(256), 0, st, reinterpret_cast<const FlipDesc*>(descs));
  return SN_CHECK_LAUNCH();
}

// ---------------- space-to-depth folding of strided low-channel convolutions -------------
// A stride-f conv with R x S taps on C channels (e.g. AlexNet conv1: f=4, 11x11x3) equals a
// stride-1 conv with ceil(R/f) x ceil(S/f) taps on f*f*Cp channels of the space-to-depth
// input, Cp >= C chosen so f*f*Cp % 8 == 0.  That turns the reference's per-image im2col
// + SGEMM (the single most expensive layer of the net) into the implicit-GEMM fast path.
//   x2[n][i][j][(dy*f + dx)*Cp + c] = x[n][i*f + dy - ph][j*f + dx - pw][c]   (0 outside)
__global__ void s2d_input(const bf16_t* __restrict__ x, bf16_t* __restrict__ x2, int N, int H, int W, int C,
                          int Hs, int Ws, int f, int Cp, int ph, int pw) {
  // one thread per 16-B output chunk (8 folded channels): coalesced stores, the scattered
  // 2-B gathers hit L1/L2 (neighbouring chunks read the same input rows).
  const int C2 = f * f * Cp;
  const int cv = C2 / 8;
  const long long total = (long long)N * Hs * Ws * cv;
  for (long long i = blockIdx.x * (long long)blockDim.x + threadIdx.x; i < total; i += (long long)gridDim.x * blockDim.x) {
    const int e0 = (int)(i % cv) * 8;
    const long long pix = i / cv;
    const int j = (int)(pix % Ws), r = (int)((pix / Ws) % Hs), n = (int)(pix / ((long long)Ws * Hs));
    uint32_t w32[4];
#pragma unroll
    for (int t = 0; t < 8; t += 2) {
      bf16_t v2[2];
#pragma unroll
      for (int u = 0; u < 2; ++u) {
        const int e = e0 + t + u;
        const int d = e / Cp, c = e - d * Cp;
        const int h = r * f + d / f - ph, w = j * f + d % f - pw;
        const bool v = c < C && (unsigned)h < (unsigned)H && (unsigned)w < (unsigned)W;
        const int hc = min(max(h, 0), H - 1), wc = min(max(w, 0), W - 1), cc = min(c, C - 1);
        const bf16_t ld = x[(((long long)n * H + hc) * W + wc) * C + cc];  // unconditional load
        v2[u] = v ? ld : (bf16_t)0;
      }
      w32[t / 2] = (uint32_t)v2[0] | ((uint32_t)v2[1] << 16);
    }
    reinterpret_cast<uint4*>(x2)[i] = make_uint4(w32[0], w32[1], w32[2], w32[3]);
  }
}

// W [K][R][S][C] (bf16) -> W2 [K][Rf][Sf][f*f*Cp] (bf16, zero padded)
__global__ void s2d_weight(const bf16_t* __restrict__ w, bf16_t* __restrict__ w2, int K, int R, int S, int C,
                           int f, int Cp, int Rf, int Sf) {
  const int C2 = f * f * Cp;
  const long long total = (long long)K * Rf * Sf * C2;
  for (long long i = blockIdx.x * (long long)blockDim.x + threadIdx.x; i < total; i += (long long)gridDim.x * blockDim.x) {
    int cc = (int)(i % C2);
    long long t = i / C2;
    const int sf = (int)(t % Sf); t /= Sf;
    const int rf = (int)(t % Rf);
    const int k = (int)(t / Rf);
    const int c = cc % Cp, d = cc / Cp, dx = d % f, dy = d / f;
    const int r = rf * f + dy, s = sf * f + dx;
    w2[i] = (r < R && s < S && c < C) ? w[(((long long)k * R + r) * S + s) * C + c] : (bf16_t)0;
  }
}

// dW [K][R][S][C] (f32) += fold(dW2 [K][Rf][Sf][f*f*Cp] (f32))
__global__ void s2d_weight_grad(const float* __restrict__ dw2, float* __restrict__ dw, int K, int R, int S, int C,
                                int f, int Cp, int Rf, int Sf, int accumulate) {
  const long long total = (long long)K * R * S * C;
  for (long long i = blockIdx.x * (long long)blockDim.x + threadIdx.x; i < total; i += (long long)gridDim.x * blockDim.x) {
    int c = (int)(i % C);
    long long t = i / C;
    const int s = (int)(t % S); t /= S;
    const int r = (int)(t % R);
    const int k = (int)(t / R);
    const int rf = r / f, dy = r % f, sf = s / f, dx = s % f;
    const float g = dw2[(((long long)k * Rf + rf) * Sf + sf) * (f * f * Cp) + (dy * f + dx) * Cp + c];
    dw[i] = accumulate ? dw[i] + g : g;
  }
}

extern "C" int sn_s2d_input(const bf16_t* x, bf16_t* x2, long long N, long long H, long long W, long long C,
                            long long Hs, long long Ws, long long f, long long Cp, long long ph, long long pw,
                            hipStream_t st) {
  if ((f * f * Cp) % 8) return 7;
  hipLaunchKernelGGL(s2d_input, dim3(sn_blocks(N * Hs * Ws * (f * f * Cp / 8), 256, 16384)), dim3(256), 0, st, x, x2,
                     (int)N, (int)H,
                     (int)W, (int)C, (int)Hs, (int)Ws, (int)f, (int)Cp, (int)ph, (int)pw);
  return SN_CHECK_LAUNCH();
}

extern "C" int sn_s2d_weight(const bf16_t* w, bf16_t* w2, long long K, long long R, long long S, long long C,
                             long long f, long long Cp, long long Rf, long long Sf, hipStream_t st) {
  hipLaunchKernelGGL(s2d_weight, dim3(sn_blocks(K * Rf * Sf * f * f * Cp, 256, 16384)), dim3(256), 0, st, w, w2,
                     (int)K, (int)R, (int)S, (int)C, (int)f, (int)Cp, (int)Rf, (int)Sf);
  return SN_CHECK_LAUNCH();
}

extern "C" int sn_s2d_weight_grad(const float* dw2, float* dw, long long K, long long R, long long S, long long C,
                                  long long f, long long Cp, long long Rf, long long Sf, long long accumulate,
                                  hipStream_t st) {
  hipLaunchKernelGGL(s2d_weight_grad, dim3(sn_blocks(K * R * S * C, 256, 16384)), dim3(256), 0, st, dw2, dw, (int)K,
                     (int)R, (int)S, (int)C, (int)f, (int)Cp, (int)Rf, (int)Sf, (int)accumulate);
  return SN_CHECK_LAUNCH();
}
