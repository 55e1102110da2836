// Device-side data transform: uint8 planar (N, C, Hs, Ws) minibatch -> bf16 NHWC
// (N, crop, crop, C) with random crop, mirror, mean subtraction and scale in ONE pass.
//
// Reference: DataTransformer::Transform (caffe/src/caffe/data_transformer.cpp:17-130) on
// the host per image, and SparkNet's ImageNetApp crop/mean closures executed inside the
// JNA data callback (src/main/scala/apps/ImageNetApp.scala:160-176, whose mean
// subtraction is a no-op — SURVEY §7.5; here it is applied correctly).
// Crop offsets / mirror flags come from Philox(seed, counter) per image so the kernel can
// be replayed inside a graph without host involvement; TEST phase uses centre crops.
#include "common.h"

#include <cstdlib>

// OUT = bf16_t (the bf16 engine) or float (the fp32 device mode, ops.f32dev)
SN_DEV void store_px(bf16_t* o, float v) { *o = f2bf(v); }
SN_DEV void store_px(float* o, float v) { *o = v; }

template <typename OUT>
__global__ void augment_kernel(const uint8_t* __restrict__ src, OUT* __restrict__ dst, int N, int C, int Hs, int Ws,
                               int crop_h, int crop_w, const float* __restrict__ mean, int mean_mode, float scale,
                               const long long* __restrict__ rng, int train, int mirror, int* __restrict__ offs_out,
                               const int* __restrict__ labels, float* __restrict__ labels_out) {
  // the minibatch's labels -> the float label blob (ProtoLoader.scala:53), folded in here
  if (labels && blockIdx.x == 0)
    for (int i = threadIdx.x; i < N; i += blockDim.x) labels_out[i] = (float)labels[i];
  const long long total = (long long)N * crop_h * crop_w;
  const unsigned long long seed = rng ? (unsigned long long)rng[0] : 0ull;
  const unsigned long long counter = rng ? (unsigned long long)rng[1] : 0ull;
  for (long long i = blockIdx.x * (long long)blockDim.x + threadIdx.x; i < total; i += (long long)gridDim.x * blockDim.x) {
    const int w = (int)(i % crop_w);
    const int h = (int)((i / crop_w) % crop_h);
    const int n = (int)(i / ((long long)crop_w * crop_h));
    int ho, wo, mir;
    if (train) {
      uint4 u = philox4x32(make_uint2((uint32_t)seed, (uint32_t)(seed >> 32)),
                           make_uint4((uint32_t)n, 0xA5A50000u, (uint32_t)counter, (uint32_t)(counter >> 32)));
      ho = (int)(u.x % (uint32_t)(Hs - crop_h + 1));
      wo = (int)(u.y % (uint32_t)(Ws - crop_w + 1));
      mir = mirror ? (int)(u.z & 1u) : 0;
    } else {
      ho = (Hs - crop_h) / 2;
      wo = (Ws - crop_w) / 2;
      mir = 0;
    }
    if (offs_out && h == 0 && w == 0) {
      offs_out[3 * n] = ho;
      offs_out[3 * n + 1] = wo;
      offs_out[3 * n + 2] = mir;
    }
    const int sh = h + ho;
    const int sw = (mir ? (crop_w - 1 - w) : w) + wo;
    OUT* o = dst + i * C;
    for (int c = 0; c < C; ++c) {
      const long long si = (((long long)n * C + c) * Hs + sh) * Ws + sw;
      float v = (float)src[si];
      if (mean_mode == 1) v -= mean[c];
      else if (mean_mode == 2) v -= mean[((long long)c * Hs + sh) * Ws + sw];
      store_px(o + c, v * scale);
    }
  }
}

extern "C" int sn_augment(const uint8_t* src, bf16_t* dst, long long N, long long C, long long Hs, long long Ws,
                          long long crop_h, long long crop_w, const float* mean, long long mean_mode, float scale,
                          const long long* rng, long long train, long long mirror, int* offs_out,
                          const int* labels, float* labels_out, hipStream_t st) {
  if (crop_h > Hs || crop_w > Ws) return 9;
  long long total = N * crop_h * crop_w;
  hipLaunchKernelGGL(augment_kernel<bf16_t>, dim3(sn_blocks(total, 256, 16384)), dim3(256), 0, st, src, dst, (int)N,
                     (int)C, (int)Hs, (int)Ws, (int)crop_h, (int)crop_w, mean, (int)mean_mode, scale, rng, (int)train,
                     (int)mirror, offs_out, labels, labels_out);
  return SN_CHECK_LAUNCH();
}

extern "C" int sn_augment_f32(const uint8_t* src, float* dst, long long N, long long C, long long Hs, long long Ws,
                              long long crop_h, long long crop_w, const float* mean, long long mean_mode, float scale,
                              const long long* rng, long long train, long long mirror, int* offs_out,
                              const int* labels, float* labels_out, hipStream_t st) {
  if (crop_h > Hs || crop_w > Ws) return 9;
  long long total = N * crop_h * crop_w;
  hipLaunchKernelGGL(augment_kernel<float>, dim3(sn_blocks(total, 256, 16384)), dim3(256), 0, st, src, dst, (int)N,
                     (int)C, (int)Hs, (int)Ws, (int)crop_h, (int)crop_w, mean, (int)mean_mode, scale, rng, (int)train,
                     (int)mirror, offs_out, labels, labels_out);
  return SN_CHECK_LAUNCH();
}

// Fused augment + space-to-depth fold for an input layer whose only consumer is a
// stride-f convolution on the S2D path (see s2d_input in eltwise.hip): writes the folded
// bf16 tensor x2 [N][Hs2][Ws2][f*f*Cp] straight from the uint8 planar source, so the
// NHWC crop is never materialised (one pass instead of augment + s2d_input).  Same
// Philox crop / mirror draw as augment_kernel, so both produce identical samples.
// One thread per folded output pixel (the Philox draw is amortised over its f*f*Cp
// channels); F / CP are compile-time for the common RGB cases so the channel ->
// (dy, dx, c) decode is shifts, with a runtime fallback.
typedef uint32_t __attribute__((aligned(1))) u32_unaligned;  // gfx950 global loads allow any byte alignment

template <int F, int CP, int MM>
__global__ void __launch_bounds__(256) augment_s2d_kernel(const uint8_t* __restrict__ src, bf16_t* __restrict__ x2,
                                                          int N, int C, int Hs, int Ws, int crop_h, int crop_w,
                                                          const float* __restrict__ mean, int mean_mode, float scale,
                                                          const long long* __restrict__ rng, int train, int mirror,
                                                          int H2, int W2, int f_rt, int cp_rt, int ph, int pw,
                                                          int direct, const int* __restrict__ labels,
                                                          float* __restrict__ labels_out) {
  if (labels && blockIdx.x == 0)
    for (int i = threadIdx.x; i < N; i += blockDim.x) labels_out[i] = (float)labels[i];
  const int f = F ? F : f_rt, Cp = CP ? CP : cp_rt;
  const int cv = f * f * Cp / 8;
  const bool staged = F && !direct;
  // compile-time shapes: the block's 256 consecutive output pixels (contiguous in x2) are
  // assembled in LDS and stored by consecutive lanes — a per-thread store of its own
  // cv x 16 B pixel leaves each wave store instruction 64 scattered 16-B pieces
  constexpr int CVS = F ? F * F * CP / 8 : 1;
  __shared__ uint4 tile[F ? 256 * CVS : 1];
  const long long total = (long long)N * H2 * W2;
  const unsigned long long seed = rng ? (unsigned long long)rng[0] : 0ull;
  const unsigned long long counter = rng ? (unsigned long long)rng[1] : 0ull;
  for (long long base = (long long)blockIdx.x * blockDim.x; base < total; base += (long long)gridDim.x * blockDim.x) {
    const long long pix = base + threadIdx.x;
    if (pix < total) {
      const int j = (int)(pix % W2), r = (int)((pix / W2) % H2), n = (int)(pix / ((long long)W2 * H2));
      int ho, wo, mir;
      if (train) {
        uint4 u = philox4x32(make_uint2((uint32_t)seed, (uint32_t)(seed >> 32)),
                             make_uint4((uint32_t)n, 0xA5A50000u, (uint32_t)counter, (uint32_t)(counter >> 32)));
        ho = (int)(u.x % (uint32_t)(Hs - crop_h + 1));
        wo = (int)(u.y % (uint32_t)(Ws - crop_w + 1));
        mir = mirror ? (int)(u.z & 1u) : 0;
      } else {
        ho = (Hs - crop_h) / 2;
        wo = (Ws - crop_w) / 2;
        mir = 0;
      }
      uint4* out = reinterpret_cast<uint4*>(x2) + pix * cv;
      bool done = false;
      if constexpr (F == 4 && CP == 3) {
        // RGB into 4 x 4 folds (CaffeNet conv1): the 4 source columns of one (row, channel)
        // are 4 consecutive bytes (reversed under the mirror), so one unaligned 32-bit load
        // replaces four byte loads — 12 loads per folded pixel instead of 48.  Folded columns
        // that reach past the crop (the last one) keep the per-element path below.
        const int w0 = j * 4 - pw;
        if (C == 3 && w0 >= 0 && w0 + 3 < crop_w) {
          float v48[48];
#pragma unroll
          for (int dy = 0; dy < 4; ++dy) {
            const int h = r * 4 + dy - ph;
            const bool okh = (unsigned)h < (unsigned)crop_h;
            const int sh = min(max(h, 0), crop_h - 1) + ho;
            const int s0 = (mir ? crop_w - 4 - w0 : w0) + wo;  // leftmost of the 4 source bytes
#pragma unroll
            for (int c = 0; c < 3; ++c) {
              const uint8_t* row = src + (((long long)n * C + c) * Hs + sh) * Ws;
              const uint32_t word = *reinterpret_cast<const u32_unaligned*>(row + s0);
#pragma unroll
              for (int dx = 0; dx < 4; ++dx) {
                const int b = mir ? 3 - dx : dx;
                float x = (float)((word >> (8 * b)) & 0xffu);
                if (MM == 1) x -= mean[c];
                if (MM == 2) x -= mean[((long long)c * Hs + sh) * Ws + s0 + b];
                v48[(dy * 4 + dx) * 3 + c] = okh ? x * scale : 0.f;
              }
            }
          }
#pragma unroll
          for (int ch = 0; ch < 6; ++ch) {
            if (staged) tile[threadIdx.x * CVS + ch] = pack8(v48 + 8 * ch);
            else out[ch] = pack8(v48 + 8 * ch);
          }
          done = true;
        }
      }
      if (!done) {
#pragma unroll
        for (int ch = 0; ch < cv; ++ch) {
          float v[8];
#pragma unroll
          for (int t = 0; t < 8; ++t) {
            const int e = ch * 8 + t;
            const int d = e / Cp, c = e - d * Cp;
            const int h = r * f + d / f - ph, w = j * f + d % f - pw;  // crop coordinates
            // branch-free: load from a clamped in-image address, then select (a load under a
            // per-element condition makes hipcc wait vmcnt(0) per element)
            const bool ok = c < C && (unsigned)h < (unsigned)crop_h && (unsigned)w < (unsigned)crop_w;
            const int hc = min(max(h, 0), crop_h - 1), wc = min(max(w, 0), crop_w - 1), cc = min(c, C - 1);
            const int sh = hc + ho, sw = (mir ? (crop_w - 1 - wc) : wc) + wo;
            float x = (float)src[(((long long)n * C + cc) * Hs + sh) * Ws + sw];
            if (MM == 1) x -= mean[cc];  // mean mode is a template parameter: no per-element branch
            if (MM == 2) x -= mean[((long long)cc * Hs + sh) * Ws + sw];
            x = ok ? x * scale : 0.f;
            v[t] = x;
          }
          if (staged) tile[threadIdx.x * CVS + ch] = pack8(v);
          else out[ch] = pack8(v);
        }
      }
    }
    if (staged) {
      __syncthreads();
      const int n_out = (int)min((long long)blockDim.x, total - base) * CVS;
      uint4* dst = reinterpret_cast<uint4*>(x2) + base * CVS;
      for (int k = threadIdx.x; k < n_out; k += blockDim.x) dst[k] = tile[k];
      __syncthreads();
    }
  }
}

extern "C" int sn_augment_s2d(const uint8_t* src, bf16_t* x2, long long N, long long C, long long Hs, long long Ws,
                              long long crop_h, long long crop_w, const float* mean, long long mean_mode, float scale,
                              const long long* rng, long long train, long long mirror, long long H2, long long W2,
                              long long f, long long Cp, long long ph, long long pw, const int* labels,
                              float* labels_out, hipStream_t st) {
  if (crop_h > Hs || crop_w > Ws || (f * f * Cp) % 8 || Cp < C) return 9;
  long long total = N * H2 * W2;
  dim3 grid(sn_blocks(total, 256, 16384));
  const int direct = 0;  // per-thread pixel stores (slower than the block-staged stores, round 3)
#define SN_AUG_S2D_MM(FF, CC, MM)                                                                               \
  hipLaunchKernelGGL((augment_s2d_kernel<FF, CC, MM>), grid, dim3(256), 0, st, src, x2, (int)N, (int)C, (int)Hs, (int)Ws, \
                     (int)crop_h, (int)crop_w, mean, (int)mean_mode, scale, rng, (int)train, (int)mirror, (int)H2,     \
                     (int)W2, (int)f, (int)Cp, (int)ph, (int)pw, direct, labels, labels_out)
#define SN_AUG_S2D(FF, CC)              \
  do {                                  \
    if (mean_mode == 1)                 \
      SN_AUG_S2D_MM(FF, CC, 1);         \
    else if (mean_mode == 2)            \
      SN_AUG_S2D_MM(FF, CC, 2);         \
    else                                \
      SN_AUG_S2D_MM(FF, CC, 0);         \
  } while (0)
  if (f == 4 && Cp == 3)  // AlexNet / CaffeNet conv1: 11x11 stride 4 on RGB -> 3x3 on 48 channels
    SN_AUG_S2D(4, 3);
  else if (f == 2 && Cp == 4)  // GoogLeNet / ResNet conv1: 7x7 stride 2 on RGB -> 4x4 on 16 channels
    SN_AUG_S2D(2, 4);
  else if (f == 1 && Cp == 8)  // stride-1 input conv (VGG conv1_1, CIFAR conv1): channels padded to 8
    SN_AUG_S2D(1, 8);
  else
    SN_AUG_S2D(0, 0);
#undef SN_AUG_S2D
#undef SN_AUG_S2D_MM
  return SN_CHECK_LAUNCH();
}

// labels: uint8/int32 -> float (JavaData label blob is [B, 1] float, ProtoLoader.scala:53)
__global__ void labels_kernel(const int* __restrict__ src, float* __restrict__ dst, int n) {
  int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i < n) dst[i] = (float)src[i];
}

extern "C" int sn_labels_to_float(const int* src, float* dst, long long n, hipStream_t st) {
  hipLaunchKernelGGL(labels_kernel, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, st, src, dst, (int)n);
  return SN_CHECK_LAUNCH();
}
