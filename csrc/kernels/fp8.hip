// FP8 (OCP e4m3) quantisation with per-tensor delayed scaling for the fp8 forward GEMMs
// (VGG-16 fp8 configuration, SURVEY §7.6-3: fp32 masters, fp32 accumulation, per-tensor
// scales from an amax history).
//
// A scale slot is float[8]: [0] quantisation scale s (x_fp8 = sat(x * s)), [1] amax of the
// tensors quantised with this slot since the last update (float bits, atomicMax),
// [2] dequantisation factor 1/s (read by the GEMM epilogue), [3] 1 once a measured amax
// has been turned into a scale, [4] the format's largest normal (e4m3 448, e5m2 57344),
// [5] write position of the slot's amax-history ring (fp8_update_scales_kernel).
// fp8_update_scales (once per iteration, inside the captured graph) turns the running
// amax into the next iteration's scale: s = max / amax.  e4m3 (3 mantissa bits) carries
// activations and weights; e5m2 (2 mantissa bits, 2^32 of range) is the option for the
// output gradients of the fp8 data-gradient products.
// A slot that has never been updated (the first iteration; or the output gradients of the
// fp8 data-gradient products, which span orders of magnitude below the unit default
// scale) is scaled from the CURRENT tensor instead: fp8_init_amax measures its amax first
// (it returns at once, device-side, for an initialised slot, so a captured graph keeps the
// launch) and the quantiser derives the scale from it.
#include "common.h"

namespace {

constexpr float E4M3_MAX = 448.f, E5M2_MAX = 57344.f;
constexpr int SLOT = 8;  // floats per scale slot

template <int E5M2>
SN_DEV uint32_t pack4_fp8(float a, float b, float c, float d) {
  int w = 0;
  if (E5M2) {
    w = __builtin_amdgcn_cvt_pk_bf8_f32(a, b, w, false);
    w = __builtin_amdgcn_cvt_pk_bf8_f32(c, d, w, true);
  } else {
    w = __builtin_amdgcn_cvt_pk_fp8_f32(a, b, w, false);
    w = __builtin_amdgcn_cvt_pk_fp8_f32(c, d, w, true);
  }
  return (uint32_t)w;
}

SN_DEV void block_amax_to_slot(float amax, float* slot) {
  // one atomic per block (a per-wave atomic on one address serialises ~30k updates)
  __shared__ float red[4];
  amax = wave_max(amax);
  if ((threadIdx.x & 63) == 0) red[threadIdx.x >> 6] = amax;
  __syncthreads();
  if (threadIdx.x == 0) {
    amax = fmaxf(fmaxf(red[0], red[1]), fmaxf(red[2], red[3]));
    if (amax > 0.f)  // amax >= 0: uint order == float order
      atomicMax(reinterpret_cast<unsigned int*>(slot + 1), __float_as_uint(amax));
  }
}

__global__ void __launch_bounds__(256) fp8_init_amax_kernel(const bf16_t* __restrict__ x, long long n16,
                                                            float* __restrict__ slot) {
  if (slot[3] != 0.f) return;  // scale already derived from a measured amax
  float amax = 0.f;
  for (long long i = blockIdx.x * (long long)blockDim.x + threadIdx.x; i < n16; i += (long long)gridDim.x * blockDim.x) {
    float f[16];
    unpack8(reinterpret_cast<const uint4*>(x)[2 * i], f);
    unpack8(reinterpret_cast<const uint4*>(x)[2 * i + 1], f + 8);
#pragma unroll
    for (int k = 0; k < 16; ++k) amax = fmaxf(amax, fabsf(f[k]));
  }
  block_amax_to_slot(amax, slot);
}

template <int E5M2>
__global__ void __launch_bounds__(256) quant_fp8_kernel(const bf16_t* __restrict__ x, uint8_t* __restrict__ q,
                                                        long long n16, float* __restrict__ slot) {
  constexpr float FMAX = E5M2 ? E5M2_MAX : E4M3_MAX;
  float sc = slot[0];
  if (slot[3] == 0.f) {  // uninitialised slot: current scaling from fp8_init_amax's measurement
    const float am = slot[1];
    sc = am > 0.f ? FMAX / am : 1.f;
    if (blockIdx.x == 0 && threadIdx.x == 0) {  // no block reads [0] / [2] in this mode
      slot[0] = sc;
      slot[2] = 1.f / sc;
    }
  }
  float amax = 0.f;
  for (long long i = blockIdx.x * (long long)blockDim.x + threadIdx.x; i < n16; i += (long long)gridDim.x * blockDim.x) {
    const uint4 a = reinterpret_cast<const uint4*>(x)[2 * i];
    const uint4 b = reinterpret_cast<const uint4*>(x)[2 * i + 1];
    float f[16];
    unpack8(a, f);
    unpack8(b, f + 8);
#pragma unroll
    for (int k = 0; k < 16; ++k) {
      amax = fmaxf(amax, fabsf(f[k]));
      f[k] = fminf(fmaxf(f[k] * sc, -FMAX), FMAX);
    }
    uint4 o;
    o.x = pack4_fp8<E5M2>(f[0], f[1], f[2], f[3]);
    o.y = pack4_fp8<E5M2>(f[4], f[5], f[6], f[7]);
    o.z = pack4_fp8<E5M2>(f[8], f[9], f[10], f[11]);
    o.w = pack4_fp8<E5M2>(f[12], f[13], f[14], f[15]);
    reinterpret_cast<uint4*>(q)[i] = o;
  }
  block_amax_to_slot(amax, slot);
}

// Delayed scaling with an amax HISTORY: the iteration's measured amax goes into a ring of
// the last `hist_len` amaxes (hist[i][pos], pos = slot[5]) and the next scale is derived
// from the ring's maximum times `margin`, so one quiet iteration after a spike (or one
// spike) does not swing the scale and saturate / flush the next iteration's values.
// hist_len == 0: the one-iteration delayed scale (the ring is not used).
__global__ void fp8_update_scales_kernel(float* __restrict__ slots, float* __restrict__ hist, int hist_len, int n,
                                         float margin) {
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  float* s = slots + SLOT * i;
  float amax = s[1];
  if (hist_len > 0 && amax > 0.f) {
    float* h = hist + (long long)i * hist_len;
    int pos = (int)s[5];
    pos = pos >= 0 && pos < hist_len ? pos : 0;
    h[pos] = amax;
    s[5] = (float)(pos + 1 == hist_len ? 0 : pos + 1);
    for (int k = 0; k < hist_len; ++k) amax = fmaxf(amax, h[k]);
  }
  if (amax > 0.f) {
    const float sc = (s[4] > 0.f ? s[4] : E4M3_MAX) / (amax * margin);
    s[0] = sc;
    s[2] = 1.f / sc;
    s[3] = 1.f;
  }
  s[1] = 0.f;
}

// fold the GEMM side output's block |max| partials (SnGemmArgs.q_part: 256 floats 128 B
// apart) into the slot's running amax and clear them for the next iteration
__global__ void __launch_bounds__(256) fp8_fold_amax_kernel(float* __restrict__ part, float* __restrict__ slot) {
  float v = part[threadIdx.x * 32];
  part[threadIdx.x * 32] = 0.f;
  block_amax_to_slot(v, slot);
}

}  // namespace

extern "C" int sn_fp8_slot_floats() { return SLOT; }

extern "C" int sn_fp8_fold_amax(float* part, float* slot, hipStream_t st) {
  hipLaunchKernelGGL(fp8_fold_amax_kernel, dim3(1), dim3(256), 0, st, part, slot);
  return SN_CHECK_LAUNCH();
}

extern "C" int sn_quant_fp8(const bf16_t* x, uint8_t* q, long long n, float* slot, int e5m2, hipStream_t st) {
  if (n % 16) return 7;
  hipLaunchKernelGGL(fp8_init_amax_kernel, dim3(sn_blocks(n / 16, 256, 1024)), dim3(256), 0, st, x, n / 16, slot);
  if (e5m2)
    hipLaunchKernelGGL(quant_fp8_kernel<1>, dim3(sn_blocks(n / 16, 256, 1024)), dim3(256), 0, st, x, q, n / 16, slot);
  else
    hipLaunchKernelGGL(quant_fp8_kernel<0>, dim3(sn_blocks(n / 16, 256, 1024)), dim3(256), 0, st, x, q, n / 16, slot);
  return SN_CHECK_LAUNCH();
}

extern "C" int sn_fp8_update_scales(float* slots, float* hist, long long hist_len, long long n, float margin,
                                    hipStream_t st) {
  if (n <= 0) return 0;
  if (hist_len > 0 && !hist) return 7;
  hipLaunchKernelGGL(fp8_update_scales_kernel, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, st, slots, hist,
                     (int)hist_len, (int)n, margin);
  return SN_CHECK_LAUNCH();
}
