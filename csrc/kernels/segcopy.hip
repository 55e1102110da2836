// Multi-segment copy / accumulate in ONE launch: the gathers and scatters of merged-layer
// parameters (engine.fuse_siblings: the siblings' bf16 weights and fp32 biases into the
// merged operands every forward, the merged fp32 weight / bias gradients back into the
// per-layer gradient slices every backward).  A separate copy per segment cost ~4-9 us each
// (single-workgroup copy kernels; GoogLeNet: 72 of them, 379 us per step); here every
// segment is a range of one grid-stride loop.  Segments are kernel arguments (pointers are
// stable across hipGraph replays: persistent buffers and graph-pool temporaries).
#include "common.h"

namespace {

constexpr int SEG_MAX = 8;

struct SegTable {
  const void* src[SEG_MAX];
  void* dst[SEG_MAX];
  long long start[SEG_MAX + 1];  // element prefix sums (start[n] = total)
  int dts[SEG_MAX], dtd[SEG_MAX], acc[SEG_MAX];
  int n;
};

SN_DEV float seg_ld(const void* p, long long i, int dt) {
  return dt ? reinterpret_cast<const float*>(p)[i] : bf2f(reinterpret_cast<const bf16_t*>(p)[i]);
}

__global__ void __launch_bounds__(256) copy_segments_k(SegTable t) {
  const long long total = t.start[t.n];
  const long long stride = (long long)gridDim.x * blockDim.x;
  int s = 0;
  for (long long e = blockIdx.x * (long long)blockDim.x + threadIdx.x; e < total; e += stride) {
    while (e >= t.start[s + 1]) ++s;  // e only grows: the segment index only advances
    const long long i = e - t.start[s];
    float v = seg_ld(t.src[s], i, t.dts[s]);
    if (t.dtd[s]) {
      float* d = reinterpret_cast<float*>(t.dst[s]) + i;
      *d = t.acc[s] ? *d + v : v;
    } else {
      bf16_t* d = reinterpret_cast<bf16_t*>(t.dst[s]) + i;
      *d = f2bf(t.acc[s] ? bf2f(*d) + v : v);
    }
  }
}

}  // namespace

// segs: n rows of (src, dst, count, src dtype, dst dtype, accumulate) as int64 (pointers as
// integers); dtype 0 = bf16, 1 = fp32
extern "C" int sn_copy_segments(const long long* segs, long long n, hipStream_t st) {
  if (n <= 0) return 0;
  if (n > SEG_MAX) return 3;
  SegTable t;
  t.n = (int)n;
  t.start[0] = 0;
  for (int s = 0; s < n; ++s) {
    const long long* r = segs + 6 * s;
    t.src[s] = reinterpret_cast<const void*>(r[0]);
    t.dst[s] = reinterpret_cast<void*>(r[1]);
    t.start[s + 1] = t.start[s] + r[2];
    t.dts[s] = (int)r[3];
    t.dtd[s] = (int)r[4];
    t.acc[s] = (int)r[5];
  }
  const long long total = t.start[n];
  if (total == 0) return 0;
  long long blocks = (total + 255) / 256;
  if (blocks > 1024) blocks = 1024;
  hipLaunchKernelGGL(copy_segments_k, dim3((unsigned)blocks), dim3(256), 0, st, t);
  return SN_CHECK_LAUNCH();
}
