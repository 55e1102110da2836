// Fused solver updates over the flat fp32 parameter buffer.
//
// Reference: SGDSolver::ApplyUpdate -> ClipGradients / Normalize / Regularize /
// ComputeUpdateValue + Blob::Update (caffe/src/caffe/solvers/sgd_solver.cpp:81-239,
// caffe/src/caffe/blob.cpp:154-176) — per parameter blob, 4-6 cuBLAS/elementwise
// launches (scal, axpy, axpby, copy, axpy) — and the Nesterov / AdaGrad / RMSProp /
// AdaDelta / Adam variants (caffe/src/caffe/solvers/*.cpp).
//
// Here: ONE launch for the whole net.  Each workgroup owns one chunk of one parameter
// segment (chunk table built once on the host: start, count, lr_mult, decay_mult), reads
// w, g, history once with float4 loads and writes w, history and the bf16 compute
// shadow.  Hyper-parameters (rate, momentum, decay, clip, 1/iter_size, ...) are read from
// device memory so the launch can live in a captured hipGraph.  Gradient clipping uses
// a deterministic two-pass sum of squares written into hyper[15].
#include "common.h"

enum { H_LR = 0, H_MOM, H_WD, H_CLIP, H_NORM, H_DELTA, H_MOM2, H_RMS, H_CORR, H_T, H_SUMSQ = 15 };

// Gradient of 4 consecutive parameters of a chunk: from the flat gradient buffer, or —
// for a chunk whose gradient was left as split-K slabs by its weight-gradient GEMM
// (engine.fuse_splitk_updates) — the sum of the `splits` fp32 slabs in the order of the
// reduce kernel the product would otherwise have used (splitk_reduce_kernel: sequential;
// splitk_reduce_wide: 16 strided lane partials), so no flat gradient write + read and no
// reduce launch, at bitwise-identical values.
// src[4 * cid] = {slab byte address of the chunk's first element (0: flat), slab stride
// (elements), splits, element stride (1: a weight row; ldw: a strided bias column)}.
SN_DEV void chunk_grad(const float* __restrict__ g, long long o, const long long* __restrict__ src, int cid, int i,
                       float* G) {
  const long long sp = src ? src[4 * cid] : 0;
  if (sp == 0) {
    const float4 gv = *reinterpret_cast<const float4*>(g + o);
    G[0] = gv.x; G[1] = gv.y; G[2] = gv.z; G[3] = gv.w;
    return;
  }
  const float* sl = reinterpret_cast<const float*>(sp);
  const long long ss = src[4 * cid + 1], es = src[4 * cid + 3];
  const int splits = (int)src[4 * cid + 2];
  G[0] = G[1] = G[2] = G[3] = 0.f;
  if (splits >= 16) {
    // splitk_reduce_wide's order: 16 lane partials over s = l, l+16, ..., then the lanes in
    // order — the fused and unfused updates stay bitwise equal
    // (loads issued four at a time, summed in s order: a data-dependent loop around single
    // loads waits for each one — the update kernel must stay a streaming kernel)
    if (es == 1) {
      const float* p = sl + i;
      for (int l = 0; l < 16; ++l) {
        float P[4] = {0.f, 0.f, 0.f, 0.f};
        int s = l;
        for (; s + 48 < splits; s += 64) {
          float4 v[4];
#pragma unroll
          for (int u = 0; u < 4; ++u) v[u] = *reinterpret_cast<const float4*>(p + (s + 16 * u) * ss);
#pragma unroll
          for (int u = 0; u < 4; ++u) {
            P[0] += v[u].x; P[1] += v[u].y; P[2] += v[u].z; P[3] += v[u].w;
          }
        }
        for (; s < splits; s += 16) {
          const float4 v = *reinterpret_cast<const float4*>(p + s * ss);
          P[0] += v.x; P[1] += v.y; P[2] += v.z; P[3] += v.w;
        }
#pragma unroll
        for (int k = 0; k < 4; ++k) G[k] += P[k];
      }
    } else {
      for (int l = 0; l < 16; ++l) {
        float P[4] = {0.f, 0.f, 0.f, 0.f};
        for (int s = l; s < splits; s += 16) {
          float v[4];
#pragma unroll
          for (int k = 0; k < 4; ++k) v[k] = sl[(long long)(i + k) * es + s * ss];
#pragma unroll
          for (int k = 0; k < 4; ++k) P[k] += v[k];
        }
#pragma unroll
        for (int k = 0; k < 4; ++k) G[k] += P[k];
      }
    }
    return;
  }
  if (es == 1) {
    const float* p = sl + i;
    int s = 0;
    for (; s + 3 < splits; s += 4) {
      float4 v[4];
#pragma unroll
      for (int u = 0; u < 4; ++u) v[u] = *reinterpret_cast<const float4*>(p + (s + u) * ss);
#pragma unroll
      for (int u = 0; u < 4; ++u) {
        G[0] += v[u].x; G[1] += v[u].y; G[2] += v[u].z; G[3] += v[u].w;
      }
    }
    for (; s < splits; ++s) {
      const float4 v = *reinterpret_cast<const float4*>(p + s * ss);
      G[0] += v.x; G[1] += v.y; G[2] += v.z; G[3] += v.w;
    }
  } else {
    for (int s = 0; s < splits; ++s)
#pragma unroll
      for (int k = 0; k < 4; ++k) G[k] += sl[(long long)(i + k) * es + s * ss];
  }
}

template <int KIND, bool L1, bool CLIP, bool SHADOW>
__global__ void __launch_bounds__(256) solver_update_kernel(float* __restrict__ w, const float* __restrict__ g,
                                                            float* __restrict__ h0, float* __restrict__ h1,
                                                            bf16_t* __restrict__ shadow,
                                                            const long long* __restrict__ chunk_pos,
                                                            const float* __restrict__ chunk_mult,
                                                            const float* __restrict__ hyper, int nchunks,
                                                            const long long* __restrict__ chunk_src) {
  // a grid smaller than the chunk table loops over it (a background update running next to
  // the backward GEMMs on a side stream takes only a slice of the CUs)
  for (int cid = blockIdx.x; cid < nchunks; cid += gridDim.x) {
  const long long start = chunk_pos[2 * cid];
  const int count = (int)chunk_pos[2 * cid + 1];
  const float lr_mult = chunk_mult[2 * cid], decay_mult = chunk_mult[2 * cid + 1];
  const float rate = hyper[H_LR] * lr_mult;
  const float mom = hyper[H_MOM];
  const float decay = hyper[H_WD] * decay_mult;
  float gscale = hyper[H_NORM];
  if (CLIP) {
    const float clip = hyper[H_CLIP];
    const float l2 = sqrtf(hyper[H_SUMSQ]);
    if (clip > 0.f && l2 > clip) gscale *= clip / l2;
  }
  const float delta = hyper[H_DELTA], mom2 = hyper[H_MOM2], rms = hyper[H_RMS], corr = hyper[H_CORR];
  for (int i = threadIdx.x * 4; i < count; i += blockDim.x * 4) {
    const long long o = start + i;
    float4 wv = *reinterpret_cast<float4*>(w + o);
    float G[4];
    chunk_grad(g, o, chunk_src, cid, i, G);
    float4 a = *reinterpret_cast<float4*>(h0 + o);
    float4 b = make_float4(0.f, 0.f, 0.f, 0.f);
    if (KIND >= 4) b = *reinterpret_cast<float4*>(h1 + o);
    float W[4] = {wv.x, wv.y, wv.z, wv.w};
    float A[4] = {a.x, a.y, a.z, a.w}, B[4] = {b.x, b.y, b.z, b.w};
#pragma unroll
    for (int k = 0; k < 4; ++k) {
      float gg = G[k] * gscale;
      gg += decay * (L1 ? ((W[k] > 0.f) - (W[k] < 0.f)) : W[k]);
      float upd;
      if (KIND == 0) {            // SGD
        A[k] = mom * A[k] + rate * gg;
        upd = A[k];
      } else if (KIND == 1) {     // Nesterov
        float prev = A[k];
        A[k] = mom * A[k] + rate * gg;
        upd = (1.f + mom) * A[k] - mom * prev;
      } else if (KIND == 2) {     // AdaGrad
        A[k] += gg * gg;
        upd = rate * gg / (sqrtf(A[k]) + delta);
      } else if (KIND == 3) {     // RMSProp
        A[k] = rms * A[k] + (1.f - rms) * gg * gg;
        upd = rate * gg / (sqrtf(A[k]) + delta);
      } else if (KIND == 4) {     // AdaDelta
        A[k] = mom * A[k] + (1.f - mom) * gg * gg;
        float u = gg * sqrtf((B[k] + delta) / (A[k] + delta));
        B[k] = mom * B[k] + (1.f - mom) * u * u;
        upd = rate * u;
      } else {                    // Adam
        A[k] = mom * A[k] + (1.f - mom) * gg;
        B[k] = mom2 * B[k] + (1.f - mom2) * gg * gg;
        upd = rate * corr * A[k] / (sqrtf(B[k]) + delta);
      }
      W[k] -= upd;
    }
    *reinterpret_cast<float4*>(w + o) = make_float4(W[0], W[1], W[2], W[3]);
    *reinterpret_cast<float4*>(h0 + o) = make_float4(A[0], A[1], A[2], A[3]);
    if (KIND >= 4) *reinterpret_cast<float4*>(h1 + o) = make_float4(B[0], B[1], B[2], B[3]);
    if (SHADOW) *reinterpret_cast<uint2*>(shadow + o) = make_uint2(pack2(W[0], W[1]), pack2(W[2], W[3]));
  }
  }
}

// deterministic sum of squares of the flat gradient -> hyper[H_SUMSQ]
__global__ void sumsq_pass1(const float* __restrict__ g, long long n, float* __restrict__ part) {
  __shared__ float red[16];
  float s = 0.f;
  for (long long i = blockIdx.x * (long long)blockDim.x + threadIdx.x; i < n; i += (long long)gridDim.x * blockDim.x) {
    float v = g[i];
    s += v * v;
  }
  s = wave_sum(s);
  if ((threadIdx.x & 63) == 0) red[threadIdx.x >> 6] = s;
  __syncthreads();
  if (threadIdx.x == 0) {
    float t = 0.f;
    for (int w = 0; w < (int)(blockDim.x >> 6); ++w) t += red[w];
    part[blockIdx.x] = t;
  }
}

__global__ void sumsq_pass2(const float* __restrict__ part, int nparts, float* __restrict__ hyper) {
  __shared__ float red[16];
  float s = 0.f;
  for (int i = threadIdx.x; i < nparts; i += blockDim.x) s += part[i];
  s = wave_sum(s);
  if ((threadIdx.x & 63) == 0) red[threadIdx.x >> 6] = s;
  __syncthreads();
  if (threadIdx.x == 0) {
    float t = 0.f;
    for (int w = 0; w < (int)(blockDim.x >> 6); ++w) t += red[w];
    hyper[H_SUMSQ] = t;
  }
}

template <int KIND, bool L1, bool CLIP>
static void launch3(bool shadow, dim3 grid, hipStream_t st, float* w, const float* g, float* h0, float* h1,
                    bf16_t* sh, const long long* cp, const float* cm, const float* hyper, int n, const long long* src) {
  if (shadow)
    hipLaunchKernelGGL((solver_update_kernel<KIND, L1, CLIP, true>), grid, dim3(256), 0, st, w, g, h0, h1, sh, cp, cm,
                       hyper, n, src);
  else
    hipLaunchKernelGGL((solver_update_kernel<KIND, L1, CLIP, false>), grid, dim3(256), 0, st, w, g, h0, h1, sh, cp,
                       cm, hyper, n, src);
}

template <int KIND>
static void launch_kind(bool l1, bool clip, bool shadow, dim3 grid, hipStream_t st, float* w, const float* g,
                        float* h0, float* h1, bf16_t* sh, const long long* cp, const float* cm, const float* hyper,
                        int n, const long long* src) {
  if (l1) {
    if (clip) launch3<KIND, true, true>(shadow, grid, st, w, g, h0, h1, sh, cp, cm, hyper, n, src);
    else launch3<KIND, true, false>(shadow, grid, st, w, g, h0, h1, sh, cp, cm, hyper, n, src);
  } else {
    if (clip) launch3<KIND, false, true>(shadow, grid, st, w, g, h0, h1, sh, cp, cm, hyper, n, src);
    else launch3<KIND, false, false>(shadow, grid, st, w, g, h0, h1, sh, cp, cm, hyper, n, src);
  }
}

extern "C" int sn_solver_update(long long kind, float* w, const float* g, float* h0, float* h1, bf16_t* shadow,
                                const long long* chunk_pos, const float* chunk_mult, long long nchunks,
                                float* hyper, long long l1, long long clip, float* part, long long nparts,
                                long long total, long long grid_limit, const long long* chunk_src, hipStream_t st) {
  if (nchunks <= 0) return 0;
  if (clip && chunk_src) return 9;  // clipping needs every gradient in the flat buffer
  if (clip) {
    hipLaunchKernelGGL(sumsq_pass1, dim3((unsigned)nparts), dim3(256), 0, st, g, total, part);
    hipLaunchKernelGGL(sumsq_pass2, dim3(1), dim3(1024), 0, st, part, (int)nparts, hyper);
  }
  dim3 grid((unsigned)(grid_limit > 0 && grid_limit < nchunks ? grid_limit : nchunks));
  bool sh = shadow != nullptr;
  const int n = (int)nchunks;
  switch (kind) {
    case 0: launch_kind<0>(l1, clip, sh, grid, st, w, g, h0, h1, shadow, chunk_pos, chunk_mult, hyper, n, chunk_src); break;
    case 1: launch_kind<1>(l1, clip, sh, grid, st, w, g, h0, h1, shadow, chunk_pos, chunk_mult, hyper, n, chunk_src); break;
    case 2: launch_kind<2>(l1, clip, sh, grid, st, w, g, h0, h1, shadow, chunk_pos, chunk_mult, hyper, n, chunk_src); break;
    case 3: launch_kind<3>(l1, clip, sh, grid, st, w, g, h0, h1, shadow, chunk_pos, chunk_mult, hyper, n, chunk_src); break;
    case 4: launch_kind<4>(l1, clip, sh, grid, st, w, g, h0, h1, shadow, chunk_pos, chunk_mult, hyper, n, chunk_src); break;
    case 5: launch_kind<5>(l1, clip, sh, grid, st, w, g, h0, h1, shadow, chunk_pos, chunk_mult, hyper, n, chunk_src); break;
    default: return 8;
  }
  return SN_CHECK_LAUNCH();
}

// model averaging / gradient averaging helper: w = w * scale, shadow = bf16(w) (after an
// all-reduce SUM; shadow may be null).  16-B vectors over the aligned body, scalars for the
// (< 4-element) tail, so any bucket boundary works.
__global__ void scale_shadow(float* __restrict__ w, bf16_t* __restrict__ shadow, long long n, long long n4,
                             float scale) {
  const long long stride = (long long)gridDim.x * blockDim.x;
  for (long long i = blockIdx.x * (long long)blockDim.x + threadIdx.x; i < n4; i += stride) {
    float4 v = reinterpret_cast<float4*>(w)[i];
    v.x *= scale; v.y *= scale; v.z *= scale; v.w *= scale;
    reinterpret_cast<float4*>(w)[i] = v;
    if (shadow) reinterpret_cast<uint2*>(shadow)[i] = make_uint2(pack2(v.x, v.y), pack2(v.z, v.w));
  }
  for (long long i = 4 * n4 + blockIdx.x * (long long)blockDim.x + threadIdx.x; i < n; i += stride) {
    const float v = w[i] * scale;
    w[i] = v;
    if (shadow) shadow[i] = f2bf(v);
  }
}

extern "C" int sn_scale_shadow(float* w, bf16_t* shadow, long long n, float scale, hipStream_t st) {
  if (n <= 0) return 0;
  const bool vec = (reinterpret_cast<uintptr_t>(w) & 15) == 0 && (reinterpret_cast<uintptr_t>(shadow) & 7) == 0;
  const long long n4 = vec ? n / 4 : 0;
  hipLaunchKernelGGL(scale_shadow, dim3(sn_blocks(n4 > 0 ? n4 : n, 256, 16384)), dim3(256), 0, st, w, shadow, n, n4,
                     scale);
  return SN_CHECK_LAUNCH();
}
