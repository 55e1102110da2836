// Shared helpers for the sparknet_amd HIP kernels (gfx950 / CDNA4 only).
//
// Conventions used by every kernel in this directory:
//  * activations are NHWC bf16 on device (channels innermost), params are fp32
//    masters with bf16 compute shadows;
//  * every entry point is `extern "C"` and takes an explicit hipStream_t so the
//    Python side (ctypes) can launch on torch's current stream and the whole
//    training step can be captured into a hipGraph;
//  * wave size is 64, blocks are multiples of 64 threads.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

typedef __attribute__((ext_vector_type(8))) __bf16 bf16x8_t;
typedef __attribute__((ext_vector_type(8))) short s16x8;
typedef __attribute__((ext_vector_type(4))) short s16x4;
typedef __attribute__((ext_vector_type(4))) float f32x4;
typedef __attribute__((ext_vector_type(16))) float f32x16;
typedef __attribute__((ext_vector_type(4))) unsigned u32x4;
typedef uint16_t bf16_t;  // raw storage type of a bf16 element

#define SN_DEV __device__ __forceinline__

SN_DEV float bf2f(bf16_t v) { return __uint_as_float(((uint32_t)v) << 16); }

// s^-beta for the LRN scales (s >= k > 0, never denormal): v_log_f32 (log2) and v_exp_f32 (2^x)
// directly.  __expf(-beta * __logf(s)) expanded to ~16 VALU ops (denormal range scaling, an
// extended-precision ln 2 product) and made the LRN kernels VALU-bound (profiles/r5_lrn_pow.txt).
SN_DEV float sn_powneg(float s, float beta) { return __builtin_amdgcn_exp2f(-beta * __builtin_amdgcn_logf(s)); }

// Round-to-nearest-even f32 -> bf16 (hipcc lowers the __bf16 cast to v_cvt_pk_bf16_f32,
// which keeps NaNs NaN — see MI355X_MICROARCH "Correctness boundaries").
SN_DEV bf16_t f2bf(float f) { return __builtin_bit_cast(bf16_t, (__bf16)f); }

SN_DEV void unpack8(const uint4& v, float* f) {
  const uint32_t w[4] = {v.x, v.y, v.z, v.w};
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    f[2 * i] = __uint_as_float(w[i] << 16);
    f[2 * i + 1] = __uint_as_float(w[i] & 0xffff0000u);
  }
}

SN_DEV uint32_t pack2(float a, float b) {
  return (uint32_t)f2bf(a) | ((uint32_t)f2bf(b) << 16);
}

SN_DEV uint4 pack8(const float* f) {
  uint4 r;
  r.x = pack2(f[0], f[1]);
  r.y = pack2(f[2], f[3]);
  r.z = pack2(f[4], f[5]);
  r.w = pack2(f[6], f[7]);
  return r;
}

// XCD-aware bijective block remap: the hardware deals consecutive block ids round-robin over
// the 8 XCDs (each with its own L2); after the remap the blocks that share an XCD hold a
// contiguous range of logical ids, so neighbouring tiles (stencil halos, shared input rows)
// meet in one L2 instead of being fetched by several.
SN_DEV int xcd_block(int bid, int nwg) {
  if (nwg < 16) return bid;
  const int xcd = bid & 7, q = nwg >> 3, r = nwg & 7;
  return (xcd < r ? xcd * (q + 1) : r * (q + 1) + (xcd - r) * q) + (bid >> 3);
}

// Fast division by a runtime-invariant divisor for 0 <= n < 2^24 (pixel / tap indices):
// fp32 reciprocal estimate + one correction step replaces the ~40-instruction integer
// division sequence in the implicit-GEMM address generators.
SN_DEV int fdiv(int n, int d, float inv) {
  int q = __float2int_rz((float)n * inv);
  int r = n - q * d;
  q += (r >= d) - (r < 0);
  return q;
}

// Exact unsigned 32-bit division by a runtime-invariant divisor (multiply-high + shift,
// Granlund-Montgomery): NHWC index decodes in the elementwise kernels otherwise compile
// to 64-bit division loops of ~100 instructions each.
struct FDiv {
  uint32_t d, m;
  int l;
};

static inline FDiv make_fdiv(uint32_t d) {
  int l = 0;
  while ((1ull << l) < d) ++l;
  FDiv f;
  f.d = d;
  f.m = (uint32_t)(((1ull << 32) * ((1ull << l) - d)) / d + 1);
  f.l = l;
  return f;
}

SN_DEV uint32_t udiv(uint32_t n, const FDiv& f) {
  const uint32_t t = __umulhi(n, f.m);
  return (uint32_t)(((uint64_t)t + n) >> f.l);
}

SN_DEV float wave_sum(float v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o, 64);
  return v;
}

SN_DEV float wave_max(float v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v = fmaxf(v, __shfl_xor(v, o, 64));
  return v;
}

// Philox4x32-10 counter-based RNG: dropout masks are regenerated in backward
// from (seed, offset, element index) instead of being stored.
SN_DEV uint4 philox4x32(uint2 key, uint4 ctr) {
  const uint32_t M0 = 0xD2511F53u, M1 = 0xCD9E8D57u;
  const uint32_t W0 = 0x9E3779B9u, W1 = 0xBB67AE85u;
#pragma unroll
  for (int i = 0; i < 10; ++i) {
    uint32_t hi0 = __umulhi(M0, ctr.x), lo0 = M0 * ctr.x;
    uint32_t hi1 = __umulhi(M1, ctr.z), lo1 = M1 * ctr.z;
    ctr = make_uint4(hi1 ^ ctr.y ^ key.x, lo1, hi0 ^ ctr.w ^ key.y, lo0);
    key.x += W0;
    key.y += W1;
  }
  return ctr;
}

// Dropout keep decisions (Philox4x32-10 keyed by the net's seed; counter = (e / 4, layer
// stream, per-iteration counter); element e uses output word e % 4, so one Philox call
// covers 4 consecutive elements.  dropout_layer.cu draws one curand uniform per element
// instead.)  Shared by dropout_kernel and the fused GEMM / split-K epilogues, which must
// draw identical masks.
SN_DEV uint4 dropout_bits4(const long long* rng, int stream, unsigned long long e4) {
  const unsigned long long seed = (unsigned long long)rng[0], counter = (unsigned long long)rng[1];
  const uint2 key = make_uint2((uint32_t)seed, (uint32_t)(seed >> 32));
  const uint4 ctr = make_uint4((uint32_t)e4, (uint32_t)(e4 >> 32) | ((uint32_t)(stream & 0xffff) << 16),
                               (uint32_t)counter, (uint32_t)(counter >> 32));
  return philox4x32(key, ctr);
}
SN_DEV uint32_t pick4(uint4 u, int k) { return k == 0 ? u.x : (k == 1 ? u.y : (k == 2 ? u.z : u.w)); }
SN_DEV bool dropout_keep(const long long* rng, int stream, unsigned thr, unsigned long long e) {
  return pick4(dropout_bits4(rng, stream, e >> 2), (int)(e & 3)) > thr;
}

#define SN_CHECK_LAUNCH() (hipGetLastError() == hipSuccess ? 0 : 1)

// CUs of the current device (persistent kernels launch one block per CU); cached per process
// (one process per GPU), 256 if the query fails.
static inline int sn_cu_count() {
  static int cus = 0;
  if (!cus) {
    int dev = 0;
    (void)hipGetDevice(&dev);
    if (hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess || cus <= 0) cus = 256;
  }
  return cus;
}

static inline int sn_blocks(long long n, int per_block, int cap = 65535 * 8) {
  long long b = (n + per_block - 1) / per_block;
  if (b < 1) b = 1;
  if (b > cap) b = cap;
  return (int)b;
}
