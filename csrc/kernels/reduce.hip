// Reductions: split-K combine for the MFMA GEMM, bias gradients (column sums of an
// [M x N] bf16 gradient), and small deterministic sums.
//
// Reference: bias gradients were cublasSgemv with a ones vector per image
// (caffe/src/caffe/layers/base_conv_layer.cpp:372-376, inner_product_layer.cu:45-47).
// Here one two-pass column reduction covers the whole batch; both passes are
// deterministic (no float atomics), so repeated runs are bitwise identical.
#include "common.h"

// out (op)= act(sum_s ws[s] + bias)
//   mode 0: out bf16 = act(sum + bias)     mode 1: out f32 = sum     mode 2: out f32 += sum
__global__ void splitk_reduce_kernel(const float* __restrict__ ws, int splits, long long sstride,
                                     int rows, int cols, long long ldw, void* out, long long ldo,
                                     int mode, const float* __restrict__ bias, int relu,
                                     int groups, long long ws_gstride, long long out_gstride) {
  const int cols4 = (cols + 3) >> 2;
  const long long total = (long long)rows * cols4;
  const int g = blockIdx.y;
  const float* wsg = ws + g * ws_gstride;
  for (long long i = blockIdx.x * (long long)blockDim.x + threadIdx.x; i < total;
       i += (long long)gridDim.x * blockDim.x) {
    const int r = (int)(i / cols4), c = (int)(i - (long long)r * cols4) * 4;
    float acc[4] = {0.f, 0.f, 0.f, 0.f};
    const bool vec = (c + 3 < cols) && ((ldw & 3) == 0);
    for (int s = 0; s < splits; ++s) {
      const float* p = wsg + s * sstride + (long long)r * ldw + c;
      if (vec) {
        float4 v = *reinterpret_cast<const float4*>(p);
        acc[0] += v.x; acc[1] += v.y; acc[2] += v.z; acc[3] += v.w;
      } else {
        for (int k = 0; k < 4; ++k)
          if (c + k < cols) acc[k] += p[k];
      }
    }
    if (mode == 0) {
      bf16_t* o = reinterpret_cast<bf16_t*>(out) + g * out_gstride + (long long)r * ldo + c;
      for (int k = 0; k < 4; ++k) {
        if (c + k >= cols) break;
        float v = acc[k] + (bias ? bias[(long long)g * cols + c + k] : 0.f);
        if (relu) v = fmaxf(v, 0.f);
        o[k] = f2bf(v);
      }
    } else {
      float* o = reinterpret_cast<float*>(out) + g * out_gstride + (long long)r * ldo + c;
      for (int k = 0; k < 4; ++k) {
        if (c + k >= cols) break;
        o[k] = (mode == 2 ? o[k] : 0.f) + acc[k];
      }
    }
  }
}

extern "C" int sn_splitk_reduce(const float* ws, long long splits, long long sstride, long long rows,
                                long long cols, long long ldw, void* out, long long ldo, long long mode,
                                const float* bias, long long relu, long long groups,
                                long long ws_gstride, long long out_gstride, hipStream_t st) {
  long long total = rows * ((cols + 3) / 4);
  dim3 grid(sn_blocks(total, 256, 4096), (unsigned)groups);
  hipLaunchKernelGGL(splitk_reduce_kernel, grid, dim3(256), 0, st, ws, (int)splits, sstride, (int)rows,
                     (int)cols, ldw, out, ldo, (int)mode, bias, (int)relu, (int)groups, ws_gstride,
                     out_gstride);
  return SN_CHECK_LAUNCH();
}

// ---- column sums of a bf16 [rows x cols] matrix (bias gradient) --------------------
// Pass 1: block b sums rows [b*rpb, (b+1)*rpb) for all columns -> part[b][cols] (f32).
// Each thread owns 8 consecutive columns (one 16-B load) and strides over rows.
__global__ void colsum_pass1(const bf16_t* __restrict__ x, long long rows, int cols, long long ld,
                             long long rpb, float* __restrict__ part) {
  extern __shared__ float red[];  // [threads][8]
  const int c8 = (cols + 7) >> 3;
  const int lanes_per_row = c8;  // threads covering one row
  const int rows_per_pass = blockDim.x / lanes_per_row;
  const int t = threadIdx.x;
  const int cc = t % lanes_per_row, rr = t / lanes_per_row;
  float acc[8] = {0, 0, 0, 0, 0, 0, 0, 0};
  const long long r0 = blockIdx.x * rpb, r1 = min(rows, r0 + rpb);
  const int c = cc * 8;
  if (rr < rows_per_pass) {
    const bool vec = (c + 7 < cols) && ((ld & 7) == 0);
    for (long long r = r0 + rr; r < r1; r += rows_per_pass) {
      const bf16_t* p = x + r * ld + c;
      if (vec) {
        float f[8];
        unpack8(*reinterpret_cast<const uint4*>(p), f);
#pragma unroll
        for (int k = 0; k < 8; ++k) acc[k] += f[k];
      } else {
        for (int k = 0; k < 8; ++k)
          if (c + k < cols) acc[k] += bf2f(p[k]);
      }
    }
  }
#pragma unroll
  for (int k = 0; k < 8; ++k) red[t * 8 + k] = (rr < rows_per_pass) ? acc[k] : 0.f;
  __syncthreads();
  // tree over rr for fixed cc (deterministic order)
  if (rr == 0) {
    for (int q = 1; q < rows_per_pass; ++q)
#pragma unroll
      for (int k = 0; k < 8; ++k) acc[k] += red[(q * lanes_per_row + cc) * 8 + k];
    for (int k = 0; k < 8; ++k)
      if (c + k < cols) part[blockIdx.x * (long long)cols + c + k] = acc[k];
  }
}

// Pass 2: one 256-thread block per group of 64 columns; the 4 waves split the partial
// rows, lanes own columns (coalesced), fixed-order combine in LDS (deterministic).
__global__ void __launch_bounds__(1024) colsum_pass2(const float* __restrict__ part, int nparts, int cols, float* out,
                                                     int accumulate) {
  __shared__ float red[16][64];
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;  // 16 waves split the partial rows
  const int c = blockIdx.x * 64 + lane;
  float s0 = 0.f, s1 = 0.f;
  if (c < cols) {
    int p = w;
    for (; p + 16 < nparts; p += 32) {
      s0 += part[(long long)p * cols + c];
      s1 += part[(long long)(p + 16) * cols + c];
    }
    if (p < nparts) s0 += part[(long long)p * cols + c];
  }
  red[w][lane] = s0 + s1;
  __syncthreads();
  if (w == 0 && c < cols) {
    float t = 0.f;
#pragma unroll
    for (int k = 0; k < 16; ++k) t += red[k][lane];
    out[c] = (accumulate ? out[c] : 0.f) + t;
  }
}

// part must hold nparts*cols floats; returns via out[cols] (+= if accumulate).
extern "C" int sn_colsum_bf16(const bf16_t* x, long long rows, long long cols, long long ld, float* part,
                              long long nparts, float* out, long long accumulate, hipStream_t st) {
  const int c8 = (int)((cols + 7) / 8);
  if (c8 > 1024) return 5;
  int threads = 256;
  while (threads < c8) threads *= 2;
  long long rpb = (rows + nparts - 1) / nparts;
  hipLaunchKernelGGL(colsum_pass1, dim3((unsigned)nparts), dim3(threads), threads * 8 * sizeof(float), st, x,
                     rows, (int)cols, ld, rpb, part);
  hipLaunchKernelGGL(colsum_pass2, dim3((unsigned)((cols + 63) / 64)), dim3(1024), 0, st, part, (int)nparts,
                     (int)cols, out, (int)accumulate);
  return SN_CHECK_LAUNCH();
}

// ---- deterministic block sum of an f32 vector into out[0] (+= if accumulate) --------
__global__ void vsum_kernel(const float* __restrict__ x, long long n, float* out, float scale, int accumulate) {
  __shared__ float red[16];
  float s = 0.f;
  for (long long i = threadIdx.x; i < n; i += blockDim.x) s += x[i];
  s = wave_sum(s);
  if ((threadIdx.x & 63) == 0) red[threadIdx.x >> 6] = s;
  __syncthreads();
  if (threadIdx.x == 0) {
    float t = 0.f;
    for (int w = 0; w < (int)(blockDim.x >> 6); ++w) t += red[w];
    out[0] = (accumulate ? out[0] : 0.f) + t * scale;
  }
}

extern "C" int sn_vsum(const float* x, long long n, float* out, float scale, long long accumulate, hipStream_t st) {
  hipLaunchKernelGGL(vsum_kernel, dim3(1), dim3(1024), 0, st, x, n, out, scale, (int)accumulate);
  return SN_CHECK_LAUNCH();
}
