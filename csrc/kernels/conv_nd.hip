// N-d convolution support (Caffe's num_spatial_axes != 2 / force_nd_im2col path:
// caffe/src/caffe/layers/base_conv_layer.cpp:16-40, caffe/src/caffe/util/im2col.cu:70-199,
// 295-430).  Rare in practice (3-D video / volumetric nets), so the design keeps the MFMA
// GEMM engine for the arithmetic and moves only the layout work here:
//
//   im2col_nd : x [num][Ctot][D_0..D_{n-1}] (Caffe's logical order, one channel group at
//               channel offset coff)  ->  col [num * P][Cg * T]  with P = prod(out dims),
//               T = prod(kernel dims); row = output pixel (pitch ldcol >= Cg * T, the pad
//               columns written as zeros so the row pitch can meet the GEMM's 16-B rule),
//               column = (c, tap) in Caffe's weight order, so col . W^T (a K-contiguous NT
//               product) is the forward.
//   col2im_nd : the adjoint, in gather form (every input element sums the col entries
//               that read it: no atomics, deterministic), written into the group's
//               channel slice of dx (overwrite) or added to it.
//
// Element-parallel over the OUTPUT of each kernel so consecutive threads write consecutive
// addresses; the index decode runs on exact 32/64-bit integer division (a handful of
// divisions per element is noise next to the product these feed).
#include "common.h"

namespace {

constexpr int ND_MAX = 6;

struct NdGeom {
  int nd;
  int num, Ctot, Cg, coff;
  int in[ND_MAX], out[ND_MAX], k[ND_MAX], st[ND_MAX], pad[ND_MAX];
  long long Sin, P, T;  // prod(in), prod(out), prod(k)
  long long ldcol;      // col row pitch (elements), >= Cg * T
};

SN_DEV float nd_ld(const void* p, long long i, int dt) {
  return dt ? reinterpret_cast<const float*>(p)[i] : bf2f(reinterpret_cast<const bf16_t*>(p)[i]);
}

__global__ void __launch_bounds__(256) im2col_nd_k(const void* __restrict__ x, void* __restrict__ col, NdGeom g,
                                                   int dtx, int dtc) {
  const long long CT = (long long)g.Cg * g.T, n_el = (long long)g.num * g.P * g.ldcol;
  const long long stride = (long long)gridDim.x * blockDim.x;
  for (long long e = blockIdx.x * (long long)blockDim.x + threadIdx.x; e < n_el; e += stride) {
    const long long j = e % g.ldcol;
    if (j >= CT) {  // row padding
      if (dtc)
        reinterpret_cast<float*>(col)[e] = 0.f;
      else
        reinterpret_cast<bf16_t*>(col)[e] = f2bf(0.f);
      continue;
    }
    long long t = j % g.T;
    const long long r = (e / g.ldcol) * g.Cg + j / g.T;
    const int c = (int)(r % g.Cg);
    const long long pix = r / g.Cg;
    long long p = pix % g.P;
    const long long n = pix / g.P;
    // decode the output pixel and the tap from the innermost (last) spatial axis outwards
    long long lin = 0, mul = 1;
    bool ok = true;
#pragma unroll
    for (int d = ND_MAX - 1; d >= 0; --d) {
      if (d >= g.nd) continue;
      const int o = (int)(p % g.out[d]), kk = (int)(t % g.k[d]);
      p /= g.out[d];
      t /= g.k[d];
      const int i = o * g.st[d] - g.pad[d] + kk;
      ok = ok && (unsigned)i < (unsigned)g.in[d];
      lin += (long long)i * mul;
      mul *= g.in[d];
    }
    float v = 0.f;
    if (ok) v = nd_ld(x, ((long long)n * g.Ctot + g.coff + c) * g.Sin + lin, dtx);
    if (dtc)
      reinterpret_cast<float*>(col)[e] = v;
    else
      reinterpret_cast<bf16_t*>(col)[e] = f2bf(v);
  }
}

__global__ void __launch_bounds__(256) col2im_nd_k(const void* __restrict__ col, void* __restrict__ dx, NdGeom g,
                                                   int dtc, int dtx, int acc) {
  const long long n_el = (long long)g.num * g.Cg * g.Sin;
  const long long stride = (long long)gridDim.x * blockDim.x;
  for (long long e = blockIdx.x * (long long)blockDim.x + threadIdx.x; e < n_el; e += stride) {
    const long long lin = e % g.Sin;
    const long long r = e / g.Sin;
    const int c = (int)(r % g.Cg);
    const long long n = r / g.Cg;
    int idx[ND_MAX];
    long long rem = lin;
#pragma unroll
    for (int d = ND_MAX - 1; d >= 0; --d) {
      if (d >= g.nd) continue;
      idx[d] = (int)(rem % g.in[d]);
      rem /= g.in[d];
    }
    float s = 0.f;
    // every tap t: the output pixel o_d = (i_d + pad_d - k_d) / st_d, when divisible and inside
    for (long long t = 0; t < g.T; ++t) {
      long long tt = t, p = 0, pm = 1;
      bool ok = true;
#pragma unroll
      for (int d = ND_MAX - 1; d >= 0; --d) {
        if (d >= g.nd) continue;
        const int kk = (int)(tt % g.k[d]);
        tt /= g.k[d];
        const int num = idx[d] + g.pad[d] - kk;
        const int o = num / g.st[d];
        ok = ok && num >= 0 && num == o * g.st[d] && o < g.out[d];
        p += (long long)o * pm;
        pm *= g.out[d];
      }
      if (ok) s += nd_ld(col, (n * g.P + p) * g.ldcol + (long long)c * g.T + t, dtc);
    }
    const long long o = (n * g.Ctot + g.coff + c) * g.Sin + lin;
    if (dtx) {
      float* q = reinterpret_cast<float*>(dx) + o;
      *q = acc ? *q + s : s;
    } else {
      bf16_t* q = reinterpret_cast<bf16_t*>(dx) + o;
      *q = f2bf(acc ? bf2f(*q) + s : s);
    }
  }
}

inline int nd_grid(long long n) {
  long long b = (n + 255) / 256;
  return (int)(b < 1 ? 1 : (b > 8192 ? 8192 : b));
}

int nd_geom(NdGeom& g, long long nd, long long num, long long Ctot, long long Cg, long long coff, long long ldcol,
            const int* dims) {
  // dims: in[nd], out[nd], k[nd], st[nd], pad[nd]
  if (nd < 1 || nd > ND_MAX) return 3;
  g.nd = (int)nd;
  g.num = (int)num;
  g.Ctot = (int)Ctot;
  g.Cg = (int)Cg;
  g.coff = (int)coff;
  g.Sin = g.P = g.T = 1;
  for (int d = 0; d < ND_MAX; ++d) {
    const bool on = d < nd;
    g.in[d] = on ? dims[d] : 1;
    g.out[d] = on ? dims[nd + d] : 1;
    g.k[d] = on ? dims[2 * nd + d] : 1;
    g.st[d] = on ? dims[3 * nd + d] : 1;
    g.pad[d] = on ? dims[4 * nd + d] : 0;
    if (on && (g.in[d] <= 0 || g.out[d] <= 0 || g.k[d] <= 0 || g.st[d] <= 0)) return 3;
    g.Sin *= g.in[d];
    g.P *= g.out[d];
    g.T *= g.k[d];
  }
  g.ldcol = ldcol;
  if (ldcol < (long long)g.Cg * g.T) return 3;
  return 0;
}

}  // namespace

extern "C" {

int sn_im2col_nd(const void* x, void* col, long long nd, long long num, long long Ctot, long long Cg, long long coff,
                 long long ldcol, const int* dims, long long dtx, long long dtc, hipStream_t st) {
  NdGeom g;
  if (int rc = nd_geom(g, nd, num, Ctot, Cg, coff, ldcol, dims)) return rc;
  hipLaunchKernelGGL(im2col_nd_k, dim3(nd_grid((long long)g.num * g.P * g.ldcol)), dim3(256), 0, st, x, col, g,
                     (int)dtx, (int)dtc);
  return SN_CHECK_LAUNCH();
}

int sn_col2im_nd(const void* col, void* dx, long long nd, long long num, long long Ctot, long long Cg, long long coff,
                 long long ldcol, const int* dims, long long dtc, long long dtx, long long acc, hipStream_t st) {
  NdGeom g;
  if (int rc = nd_geom(g, nd, num, Ctot, Cg, coff, ldcol, dims)) return rc;
  hipLaunchKernelGGL(col2im_nd_k, dim3(nd_grid((long long)g.num * g.Cg * g.Sin)), dim3(256), 0, st, col, dx, g,
                     (int)dtc, (int)dtx, (int)acc);
  return SN_CHECK_LAUNCH();
}

}  // extern "C"
