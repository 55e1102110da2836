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
// (gate, mode 0: zero where gate <= 0 — a fused slope-0 ReLU backward)
// (modes 1/2, a GEMM with a bias-gradient ones column: column extra_col goes to
//  extra[g * extra_gstride + r], accumulated when extra_acc, instead of out)
struct ReduceOut {
  void* out;
  long long ldo, out_gstride;
  int cols, mode, relu;
  const float* bias;
  const bf16_t* gate;
  float* extra;
  long long extra_gstride;
  int extra_col, extra_acc;
  const long long* drop_rng;  // mode 0: fused dropout / gate scale, as the GEMM epilogue
  int drop_stream;
  unsigned drop_thr;
  float drop_scale, gate_scale;
};

// acc is taken by value and every index below is a compile-time constant (unrolled, guarded
// instead of `break`): a pointer to the caller's array with a runtime index put the four
// accumulators in scratch memory (32 B per lane, kernel-resource-usage report)
SN_DEV void reduce_store(const ReduceOut& o, int g, int r, int c, float4 a) {
  const float acc[4] = {a.x, a.y, a.z, a.w};
  if (o.extra && c <= o.extra_col && o.extra_col < c + 4) {
    float* e = o.extra + g * o.extra_gstride + r;
    const int q = o.extra_col - c;
    const float v = q == 0 ? a.x : (q == 1 ? a.y : (q == 2 ? a.z : a.w));
    *e = o.extra_acc ? *e + v : v;
  }
  if (o.mode == 0) {
    const long long base = g * o.out_gstride + (long long)r * o.ldo + c;
    bf16_t* p = reinterpret_cast<bf16_t*>(o.out) + base;
    float v[4];
#pragma unroll
    for (int k = 0; k < 4; ++k) {
      v[k] = acc[k] + ((o.bias && c + k < o.cols) ? o.bias[(long long)g * o.cols + c + k] : 0.f);
      if (o.relu) v[k] = fmaxf(v[k], 0.f);
      if (o.gate && c + k < o.cols) v[k] = bf2f(o.gate[base + k]) > 0.f ? v[k] * o.gate_scale : 0.f;
    }
    if (o.drop_rng) {
      if ((base & 3) == 0) {  // the 4 columns are one Philox draw (as the GEMM epilogue)
        const uint4 u = dropout_bits4(o.drop_rng, o.drop_stream, (unsigned long long)base >> 2);
        const uint32_t b[4] = {u.x, u.y, u.z, u.w};
#pragma unroll
        for (int k = 0; k < 4; ++k) v[k] = b[k] > o.drop_thr ? v[k] * o.drop_scale : 0.f;
      } else {
#pragma unroll
        for (int k = 0; k < 4; ++k)
          v[k] = dropout_keep(o.drop_rng, o.drop_stream, o.drop_thr, base + k) ? v[k] * o.drop_scale : 0.f;
      }
    }
    if (c + 3 < o.cols && (base & 3) == 0) {  // one 8-byte store for the 4 bf16 outputs
      *reinterpret_cast<uint2*>(p) = make_uint2(pack2(v[0], v[1]), pack2(v[2], v[3]));
    } else {
#pragma unroll
      for (int k = 0; k < 4; ++k)
        if (c + k < o.cols) p[k] = f2bf(v[k]);
    }
  } else {
    float* p = reinterpret_cast<float*>(o.out) + g * o.out_gstride + (long long)r * o.ldo + c;
    const int cols = o.extra ? o.extra_col : o.cols;
#pragma unroll
    for (int k = 0; k < 4; ++k)
      if (c + k < cols) p[k] = (o.mode == 2 ? p[k] : 0.f) + acc[k];
  }
}

// Few splits: one thread per 4 output columns, serial over the splits.
__global__ void splitk_reduce_kernel(const float* __restrict__ ws, int splits, long long sstride, int rows,
                                     long long ldw, long long ws_gstride, ReduceOut o) {
  const int cols = o.cols, cols4 = (cols + 3) >> 2;
  const long long total = (long long)rows * cols4;
  const int g = blockIdx.y;
  const float* wsg = ws + g * ws_gstride;
  for (long long i = blockIdx.x * (long long)blockDim.x + threadIdx.x; i < total;
       i += (long long)gridDim.x * blockDim.x) {
    const int r = (int)(i / cols4), c = (int)(i - (long long)r * cols4) * 4;
    float acc[4] = {0.f, 0.f, 0.f, 0.f};
    const bool vec = (c + 3 < cols) && ((ldw & 3) == 0);
    const float* p0 = wsg + (long long)r * ldw + c;
    if (vec) {
      // slab loads issued four at a time before they are summed (in split order): a load
      // inside a per-split branch made each split a dependent L2 round trip
      int s = 0;
      for (; s + 3 < splits; s += 4) {
        float4 v[4];
#pragma unroll
        for (int u = 0; u < 4; ++u) v[u] = *reinterpret_cast<const float4*>(p0 + (s + u) * sstride);
#pragma unroll
        for (int u = 0; u < 4; ++u) {
          acc[0] += v[u].x; acc[1] += v[u].y; acc[2] += v[u].z; acc[3] += v[u].w;
        }
      }
      for (; s < splits; ++s) {
        const float4 v = *reinterpret_cast<const float4*>(p0 + s * sstride);
        acc[0] += v.x; acc[1] += v.y; acc[2] += v.z; acc[3] += v.w;
      }
    } else {
      for (int s = 0; s < splits; ++s)
#pragma unroll
        for (int k = 0; k < 4; ++k)
          if (c + k < cols) acc[k] += p0[s * sstride + k];
    }
    reduce_store(o, g, r, c, make_float4(acc[0], acc[1], acc[2], acc[3]));
  }
}

// Many splits (e.g. 128-way split-K of a small weight gradient): 16 output float4s per
// block x 16 split lanes, four slab loads in flight per thread, fixed-order LDS combine.
// Needs cols % 4 == 0 and ldw % 4 == 0.
__global__ void __launch_bounds__(256) splitk_reduce_wide(const float* __restrict__ ws, int splits,
                                                          long long sstride, int rows, long long ldw,
                                                          long long ws_gstride, ReduceOut o) {
  __shared__ float4 red[16][16];
  const int it = threadIdx.x & 15, sl = threadIdx.x >> 4;
  const int cols4 = (o.cols + 3) >> 2;  // a ragged last float4 reads slab padding (ldw % 4 == 0)
  const long long total = (long long)rows * cols4;
  const long long i = blockIdx.x * 16LL + it;
  const int g = blockIdx.y;
  float4 acc = make_float4(0.f, 0.f, 0.f, 0.f);
  int r = 0, c = 0;
  if (i < total) {
    r = (int)(i / cols4);
    c = (int)(i - (long long)r * cols4) * 4;
    const float* p = ws + g * ws_gstride + (long long)r * ldw + c;
    int s = sl;
    for (; s + 48 < splits; s += 64) {
      float4 v[4];
#pragma unroll
      for (int u = 0; u < 4; ++u) v[u] = *reinterpret_cast<const float4*>(p + (s + 16 * u) * sstride);
#pragma unroll
      for (int u = 0; u < 4; ++u) {
        acc.x += v[u].x; acc.y += v[u].y; acc.z += v[u].z; acc.w += v[u].w;
      }
    }
    for (; s < splits; s += 16) {
      float4 v = *reinterpret_cast<const float4*>(p + s * sstride);
      acc.x += v.x; acc.y += v.y; acc.z += v.z; acc.w += v.w;
    }
  }
  red[sl][it] = acc;
  __syncthreads();
  if (sl == 0 && i < total) {
    float a[4] = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
    for (int q = 0; q < 16; ++q) {
      float4 v = red[q][it];
      a[0] += v.x; a[1] += v.y; a[2] += v.z; a[3] += v.w;
    }
    reduce_store(o, g, r, c, make_float4(a[0], a[1], a[2], a[3]));
  }
}

extern "C" int sn_splitk_reduce(const float* ws, long long splits, long long sstride, long long rows,
                                long long cols, long long ldw, void* out, long long ldo, long long mode,
                                const float* bias, long long relu, long long groups,
                                long long ws_gstride, long long out_gstride, const bf16_t* gate,
                                float* extra, long long extra_col, long long extra_acc, long long extra_gstride,
                                const long long* drop_rng, long long drop_stream, float drop_ratio,
                                float gate_scale, hipStream_t st) {
  ReduceOut o;
  o.drop_rng = drop_rng;
  o.drop_stream = (int)drop_stream;
  o.drop_thr = (uint32_t)((double)4294967295u * (double)drop_ratio);
  o.drop_scale = 1.f / (1.f - drop_ratio);
  o.gate_scale = gate_scale;
  o.out = out; o.ldo = ldo; o.out_gstride = out_gstride; o.cols = (int)cols; o.mode = (int)mode;
  o.relu = (int)relu; o.bias = bias; o.gate = gate;
  o.extra = extra; o.extra_col = (int)extra_col; o.extra_acc = (int)extra_acc; o.extra_gstride = extra_gstride;
  if (extra && (mode == 0 || extra_col != cols - 1)) return 5;
  long long total = rows * ((cols + 3) / 4);
  if (splits >= 16 && ((cols & 3) == 0 || ldw >= ((cols + 3) & ~3LL)) && (ldw & 3) == 0) {
    dim3 grid((unsigned)((total + 15) / 16), (unsigned)groups);
    hipLaunchKernelGGL(splitk_reduce_wide, grid, dim3(256), 0, st, ws, (int)splits, sstride, (int)rows, ldw,
                       ws_gstride, o);
  } else {
    dim3 grid(sn_blocks(total, 256, 4096), (unsigned)groups);
    hipLaunchKernelGGL(splitk_reduce_kernel, grid, dim3(256), 0, st, ws, (int)splits, sstride, (int)rows, ldw,
                       ws_gstride, o);
  }
  return SN_CHECK_LAUNCH();
}

// ---- column sums of a bf16 [rows x cols] matrix (bias gradient) --------------------
// Pass 1: block (b, cb) sums rows [b*rpb, (b+1)*rpb) of the column block cb (CL*8
// columns) -> part[b][cols] (f32).  256 threads = CL column lanes (8 columns = one 16-B
// load each) x RL row lanes; four rows in flight per thread.
__global__ void __launch_bounds__(256) colsum_pass1(const bf16_t* __restrict__ x, long long rows, int cols,
                                                    long long ld, long long rpb, int CL, float* __restrict__ part) {
  __shared__ float red[256 * 8];
  const int RL = 256 / CL;
  const int t = threadIdx.x;
  const int cc = t % CL, rr = t / CL;
  const int c = (blockIdx.y * CL + cc) * 8;
  float acc[8] = {0, 0, 0, 0, 0, 0, 0, 0};
  const long long r0 = blockIdx.x * rpb, r1 = min(rows, r0 + rpb);
  if (c < cols) {
    const bool vec = (c + 7 < cols) && ((ld & 7) == 0);
    long long r = r0 + rr;
    if (vec) {
      for (; r + 3 * RL < r1; r += 4 * RL) {
        uint4 v[4];
#pragma unroll
        for (int u = 0; u < 4; ++u) v[u] = *reinterpret_cast<const uint4*>(x + (r + u * RL) * ld + c);
#pragma unroll
        for (int u = 0; u < 4; ++u) {
          float f[8];
          unpack8(v[u], f);
#pragma unroll
          for (int k = 0; k < 8; ++k) acc[k] += f[k];
        }
      }
    }
    for (; r < r1; r += RL) {
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
  for (int k = 0; k < 8; ++k) red[t * 8 + k] = acc[k];
  __syncthreads();
  // fixed-order combine over the row lanes (deterministic)
  if (rr == 0 && c < cols) {
    for (int q = 1; q < RL; ++q)
#pragma unroll
      for (int k = 0; k < 8; ++k) acc[k] += red[(q * CL + cc) * 8 + k];
    for (int k = 0; k < 8; ++k)
      if (c + k < cols) part[blockIdx.x * (long long)cols + c + k] = acc[k];
  }
}

// Pass 2: one 1024-thread block per 64 columns; 16 waves split the partial rows (eight
// independent loads in flight per lane), lanes own columns (coalesced), fixed-order
// combine in LDS (deterministic).
__global__ void __launch_bounds__(1024) colsum_pass2(const float* __restrict__ part, int nparts, int cols, float* out,
                                                     int accumulate) {
  __shared__ float red[16][64];
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  const int c = blockIdx.x * 64 + lane;
  float s[8] = {0, 0, 0, 0, 0, 0, 0, 0};
  if (c < cols) {
    int p = w;
    for (; p + 7 * 16 < nparts; p += 8 * 16) {
#pragma unroll
      for (int u = 0; u < 8; ++u) s[u] += part[(long long)(p + u * 16) * cols + c];
    }
    for (; p < nparts; p += 16) s[0] += part[(long long)p * cols + c];
  }
  red[w][lane] = ((s[0] + s[1]) + (s[2] + s[3])) + ((s[4] + s[5]) + (s[6] + s[7]));
  __syncthreads();
  if (w == 0 && c < cols) {
    float tot = 0.f;
#pragma unroll
    for (int k = 0; k < 16; ++k) tot += red[k][lane];
    out[c] = (accumulate ? out[c] : 0.f) + tot;
  }
}

// part must hold nparts*cols floats; returns via out[cols] (+= if accumulate).
extern "C" int sn_colsum_bf16(const bf16_t* x, long long rows, long long cols, long long ld, float* part,
                              long long nparts, float* out, long long accumulate, hipStream_t st) {
  const int c8 = (int)((cols + 7) / 8);
  int CL = 1;
  while (CL < c8 && CL < 64) CL *= 2;
  const int cblocks = (c8 + CL - 1) / CL;
  long long rpb = (rows + nparts - 1) / nparts;
  hipLaunchKernelGGL(colsum_pass1, dim3((unsigned)nparts, (unsigned)cblocks), dim3(256), 0, st, x, rows,
                     (int)cols, ld, rpb, CL, part);
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

// ---------------------------------------------------------------------------------------
// Probe of the ds_read_b64_tr_b8 lane mapping (tests/test_gemm_fp8_mc_gpu.py): a 16 x 16
// byte image b[row][col] = row * 16 + col in LDS; lane l (group g = l >> 4, i = l & 15)
// addresses row 8 (g & 1) + (i >> 1), bytes 8 (i & 1) .. +7 and stores the 8 bytes it gets.
// Under the mapping read_frag8_mc assumes, lane i receives column i of the 8 rows.
namespace {
__global__ void probe_tr8_kernel(unsigned* out) {
  __shared__ __attribute__((aligned(16))) unsigned char img[256];
  const int l = threadIdx.x;
  for (int e = l; e < 256; e += 64) img[e] = (unsigned char)e;
  __syncthreads();
  typedef int v2i __attribute__((ext_vector_type(2)));
  const int g = l >> 4, i = l & 15;
  const int row = 8 * (g & 1) + (i >> 1);
  typedef __attribute__((address_space(3))) v2i lds_v2i;
  const v2i v = __builtin_amdgcn_ds_read_tr8_b64_v2i32(
      (lds_v2i*)((__attribute__((address_space(3))) unsigned char*)img + row * 16 + 8 * (i & 1)));
  out[2 * l] = (unsigned)v[0];
  out[2 * l + 1] = (unsigned)v[1];
}
}  // namespace

extern "C" int sn_probe_tr8(unsigned* out, hipStream_t st) {
  hipLaunchKernelGGL(probe_tr8_kernel, dim3(1), dim3(64), 0, st, out);
  return SN_CHECK_LAUNCH();
}
