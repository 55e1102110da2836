// Max / average pooling on NHWC bf16 tensors (Caffe ceil-mode geometry).
//
// Reference: MaxPoolForward / AvePoolForward / MaxPoolBackward / AvePoolBackward
// (caffe/src/caffe/layers/pooling_layer.cu:11-80, 217-296): one thread per NCHW output
// element with a float/int mask.  Here one thread owns 8 consecutive channels of one
// output pixel (16-B loads/stores), the argmax mask is a uint8 window offset (4x less
// traffic than Caffe's int mask) and the backward pass is a gather (no atomics).
#include "common.h"

#include <cstdlib>

struct PoolGeom {
  int N, H, W, C, P, Q, kh, kw, sh, sw, ph, pw;
  FDiv fcv, fW, fH, fQ, fP, fsh, fsw;  // cv = channel chunks per pixel (C/8 or C)
};

template <bool VEC>
__global__ void maxpool_fwd(const bf16_t* __restrict__ x, bf16_t* __restrict__ y, uint8_t* __restrict__ mask,
                            PoolGeom g, int gate) {
  const int cv = VEC ? g.C / 8 : g.C;
  const long long total = (long long)g.N * g.P * g.Q * cv;
  for (long long i = xcd_block(blockIdx.x, gridDim.x) * (long long)blockDim.x + threadIdx.x; i < total;
       i += (long long)gridDim.x * blockDim.x) {
    const uint32_t pix = udiv((uint32_t)i, g.fcv), pq = udiv(pix, g.fQ), n = udiv(pq, g.fP);
    const int c0 = (int)((uint32_t)i - pix * cv) * (VEC ? 8 : 1);
    const int q = (int)(pix - pq * g.Q), p = (int)(pq - n * g.P);
    const int hs = p * g.sh - g.ph, ws = q * g.sw - g.pw;
    const int he = min(hs + g.kh, g.H), we = min(ws + g.kw, g.W);
    const int h0 = max(hs, 0), w0 = max(ws, 0);
    float best[8];
    int arg[8];
#pragma unroll
    for (int k = 0; k < 8; ++k) { best[k] = -INFINITY; arg[k] = 0; }
    for (int h = h0; h < he; ++h)
      for (int w = w0; w < we; ++w) {
        const bf16_t* src = x + (((long long)n * g.H + h) * g.W + w) * g.C + c0;
        const int widx = (h - hs) * g.kw + (w - ws);
        if (VEC) {
          float f[8];
          unpack8(*reinterpret_cast<const uint4*>(src), f);
#pragma unroll
          for (int k = 0; k < 8; ++k)
            if (f[k] > best[k]) { best[k] = f[k]; arg[k] = widx; }
        } else {
          float f = bf2f(src[0]);
          if (f > best[0]) { best[0] = f; arg[0] = widx; }
        }
      }
    // ReLU gate (the pooled input is the output of an in-place slope-0 ReLU whose
    // backward is folded in here): a window whose max is <= 0 passes no gradient, which
    // the mask encodes as the impossible window index 255.
    if (gate) {
#pragma unroll
      for (int k = 0; k < 8; ++k)
        if (!(best[k] > 0.f)) arg[k] = 255;
    }
    const long long o = (long long)pix * g.C + c0;
    if (VEC) {
      *reinterpret_cast<uint4*>(y + o) = pack8(best);
      if (mask) {
        uint2 m;
        m.x = arg[0] | (arg[1] << 8) | (arg[2] << 16) | (arg[3] << 24);
        m.y = arg[4] | (arg[5] << 8) | (arg[6] << 16) | (arg[7] << 24);
        *reinterpret_cast<uint2*>(mask + o) = m;
      }
    } else {
      y[o] = f2bf(best[0]);
      if (mask) mask[o] = (uint8_t)arg[0];
    }
  }
}

template <bool VEC>
__global__ void avepool_fwd(const bf16_t* __restrict__ x, bf16_t* __restrict__ y, PoolGeom g) {
  const int cv = VEC ? g.C / 8 : g.C;
  const long long total = (long long)g.N * g.P * g.Q * cv;
  for (long long i = xcd_block(blockIdx.x, gridDim.x) * (long long)blockDim.x + threadIdx.x; i < total;
       i += (long long)gridDim.x * blockDim.x) {
    const uint32_t pix = udiv((uint32_t)i, g.fcv), pq = udiv(pix, g.fQ), n = udiv(pq, g.fP);
    const int c0 = (int)((uint32_t)i - pix * cv) * (VEC ? 8 : 1);
    const int q = (int)(pix - pq * g.Q), p = (int)(pq - n * g.P);
    int hs = p * g.sh - g.ph, ws = q * g.sw - g.pw;
    int he = min(hs + g.kh, g.H + g.ph), we = min(ws + g.kw, g.W + g.pw);
    const float inv = 1.f / (float)((he - hs) * (we - ws));
    hs = max(hs, 0); ws = max(ws, 0); he = min(he, g.H); we = min(we, g.W);
    float acc[8] = {0, 0, 0, 0, 0, 0, 0, 0};
    if (VEC) {
      // the window in row-major order, 8 loads issued before any is summed (a load inside the
      // data-dependent window loop waited for each one: GoogLeNet's 7 x 7 global average pool
      // took 49 dependent L2 / HBM round trips per thread); same summation order as before
      const int ww = we - ws, win = (he - hs) * ww;
      int hh = hs, wq = ws;  // window position of the next load
      for (int base = 0; base < win; base += 8) {
        uint4 v[8];
#pragma unroll
        for (int u = 0; u < 8; ++u) {
          const bool ok = base + u < win;
          v[u] = *reinterpret_cast<const uint4*>(x + (((long long)n * g.H + (ok ? hh : hs)) * g.W + (ok ? wq : ws)) * g.C + c0);
          if (ok && ++wq == we) {
            wq = ws;
            ++hh;
          }
        }
#pragma unroll
        for (int u = 0; u < 8; ++u) {
          if (base + u < win) {
            float f[8];
            unpack8(v[u], f);
#pragma unroll
            for (int k = 0; k < 8; ++k) acc[k] += f[k];
          }
        }
      }
    } else {
      for (int h = hs; h < he; ++h)
        for (int w = ws; w < we; ++w) acc[0] += bf2f(x[(((long long)n * g.H + h) * g.W + w) * g.C + c0]);
    }
    const long long o = (long long)pix * g.C + c0;
    if (VEC) {
#pragma unroll
      for (int k = 0; k < 8; ++k) acc[k] *= inv;
      *reinterpret_cast<uint4*>(y + o) = pack8(acc);
    } else {
      y[o] = f2bf(acc[0] * inv);
    }
  }
}

// Backward: one thread per 8 channels of one INPUT pixel; gathers every output window
// that contains the pixel.
template <bool VEC, bool MAX>
__global__ void pool_bwd(const bf16_t* __restrict__ dy, const uint8_t* __restrict__ mask, bf16_t* __restrict__ dx,
                         PoolGeom g) {
  const int cv = VEC ? g.C / 8 : g.C;
  const long long total = (long long)g.N * g.H * g.W * cv;
  for (long long i = xcd_block(blockIdx.x, gridDim.x) * (long long)blockDim.x + threadIdx.x; i < total;
       i += (long long)gridDim.x * blockDim.x) {
    const uint32_t pix = udiv((uint32_t)i, g.fcv), ph_ = udiv(pix, g.fW), n = udiv(ph_, g.fH);
    const int c0 = (int)((uint32_t)i - pix * cv) * (VEC ? 8 : 1);
    const int w = (int)(pix - ph_ * g.W), h = (int)(ph_ - n * g.H);
    const int hp = h + g.ph, wp = w + g.pw;
    const int p0 = hp < g.kh ? 0 : (int)udiv((uint32_t)(hp - g.kh), g.fsh) + 1;
    const int p1 = min((int)udiv((uint32_t)hp, g.fsh) + 1, g.P);
    const int q0 = wp < g.kw ? 0 : (int)udiv((uint32_t)(wp - g.kw), g.fsw) + 1;
    const int q1 = min((int)udiv((uint32_t)wp, g.fsw) + 1, g.Q);
    float acc[8] = {0, 0, 0, 0, 0, 0, 0, 0};
    for (int p = p0; p < p1; ++p)
      for (int q = q0; q < q1; ++q) {
        const long long o = (((long long)n * g.P + p) * g.Q + q) * g.C + c0;
        const int hs = p * g.sh - g.ph, ws = q * g.sw - g.pw;
        float scale = 1.f;
        if (!MAX) {
          int he = min(hs + g.kh, g.H + g.ph), we = min(ws + g.kw, g.W + g.pw);
          scale = 1.f / (float)((he - hs) * (we - ws));
        }
        const int widx = (h - hs) * g.kw + (w - ws);
        if (VEC) {
          float f[8];
          unpack8(*reinterpret_cast<const uint4*>(dy + o), f);
          if (MAX) {
            uint2 m = *reinterpret_cast<const uint2*>(mask + o);
            const uint32_t mw[2] = {m.x, m.y};
#pragma unroll
            for (int k = 0; k < 8; ++k)
              if ((int)((mw[k >> 2] >> ((k & 3) * 8)) & 0xff) == widx) acc[k] += f[k];
          } else {
#pragma unroll
            for (int k = 0; k < 8; ++k) acc[k] += f[k] * scale;
          }
        } else {
          float f = bf2f(dy[o]);
          if (MAX) {
            if ((int)mask[o] == widx) acc[0] += f;
          } else {
            acc[0] += f * scale;
          }
        }
      }
    const long long o = (long long)pix * g.C + c0;
    if (VEC)
      *reinterpret_cast<uint4*>(dx + o) = pack8(acc);
    else
      dx[o] = f2bf(acc[0]);
  }
}

// ---- fp8 side output (engine.fuse_fp8_quant): the pooled output / the input gradient also
// stored as the fp8 bytes the consuming fp8 product reads (a conv's e4m3 input after a pool,
// the fp8 output gradient of the conv before a pool), scaled by an initialised delayed-scaling
// slot; block |max| into one of 256 partials 128 B apart (folded by sn_fp8_fold_amax).
struct QSide {
  uint8_t* q;
  const float* slot;
  float* part;
  int e5m2;
};

SN_DEV uint2 q_pack8(const QSide& qs, float sc, const float* v, float& qmax) {
  const float fmax = qs.e5m2 ? 57344.f : 448.f;
  float f[8];
#pragma unroll
  for (int r = 0; r < 8; ++r) {
    const float b = bf2f(f2bf(v[r]));  // the stored bf16 value
    qmax = fmaxf(qmax, fabsf(b));
    f[r] = fminf(fmaxf(b * sc, -fmax), fmax);
  }
  int w0 = 0, w1 = 0;
  if (qs.e5m2) {
    w0 = __builtin_amdgcn_cvt_pk_bf8_f32(f[0], f[1], w0, false);
    w0 = __builtin_amdgcn_cvt_pk_bf8_f32(f[2], f[3], w0, true);
    w1 = __builtin_amdgcn_cvt_pk_bf8_f32(f[4], f[5], w1, false);
    w1 = __builtin_amdgcn_cvt_pk_bf8_f32(f[6], f[7], w1, true);
  } else {
    w0 = __builtin_amdgcn_cvt_pk_fp8_f32(f[0], f[1], w0, false);
    w0 = __builtin_amdgcn_cvt_pk_fp8_f32(f[2], f[3], w0, true);
    w1 = __builtin_amdgcn_cvt_pk_fp8_f32(f[4], f[5], w1, false);
    w1 = __builtin_amdgcn_cvt_pk_fp8_f32(f[6], f[7], w1, true);
  }
  return make_uint2((uint32_t)w0, (uint32_t)w1);
}

SN_DEV void q_flush(const QSide& qs, float qmax) {  // every thread of the block calls it
  __shared__ float red[4];
  qmax = wave_max(qmax);
  if ((threadIdx.x & 63) == 0) red[threadIdx.x >> 6] = qmax;
  __syncthreads();
  if (threadIdx.x == 0) {
    const float m = fmaxf(fmaxf(red[0], red[1]), fmaxf(red[2], red[3]));
    if (m > 0.f) atomicMax(reinterpret_cast<unsigned int*>(qs.part + (blockIdx.x & 255) * 32), __float_as_uint(m));
  }
}

// ---- fixed-window fast paths (VEC, compile-time window) --------------------------------
// Same semantics as the generic kernels above, but every window load is issued up front
// from a clamped in-bounds address and masked afterwards: a load inside a data-dependent
// loop / branch makes hipcc wait vmcnt(0) per element (one L2 round trip each).

template <int KH, int KW>
__global__ void maxpool_fwd_k(const bf16_t* __restrict__ x, bf16_t* __restrict__ y, uint8_t* __restrict__ mask,
                              PoolGeom g, int gate, QSide qs) {
  const int cv = g.C / 8;
  float qmax = 0.f;
  const float qsc = qs.q ? qs.slot[0] : 0.f;
  const long long total = (long long)g.N * g.P * g.Q * cv;
  for (long long i = xcd_block(blockIdx.x, gridDim.x) * (long long)blockDim.x + threadIdx.x; i < total;
       i += (long long)gridDim.x * blockDim.x) {
    const uint32_t pix = udiv((uint32_t)i, g.fcv), pq = udiv(pix, g.fQ), n = udiv(pq, g.fP);
    const int c0 = (int)((uint32_t)i - pix * cv) * 8;
    const int q = (int)(pix - pq * g.Q), p = (int)(pq - n * g.P);
    const int hs = p * g.sh - g.ph, ws = q * g.sw - g.pw;
    uint4 v[KH * KW];
    bool ok[KH * KW];
#pragma unroll
    for (int a = 0; a < KH; ++a)
#pragma unroll
      for (int b = 0; b < KW; ++b) {
        const int h = hs + a, w = ws + b;
        ok[a * KW + b] = (unsigned)h < (unsigned)g.H && (unsigned)w < (unsigned)g.W;
        const int hc = min(max(h, 0), g.H - 1), wc = min(max(w, 0), g.W - 1);
        v[a * KW + b] = *reinterpret_cast<const uint4*>(x + (((long long)n * g.H + hc) * g.W + wc) * g.C + c0);
      }
    float best[8];
    int arg[8];
#pragma unroll
    for (int k = 0; k < 8; ++k) { best[k] = -INFINITY; arg[k] = 0; }
#pragma unroll
    for (int widx = 0; widx < KH * KW; ++widx) {
      float f[8];
      unpack8(v[widx], f);
#pragma unroll
      for (int k = 0; k < 8; ++k)
        if (ok[widx] && f[k] > best[k]) { best[k] = f[k]; arg[k] = widx; }
    }
    if (gate) {
#pragma unroll
      for (int k = 0; k < 8; ++k)
        if (!(best[k] > 0.f)) arg[k] = 255;
    }
    const long long o = (long long)pix * g.C + c0;
    *reinterpret_cast<uint4*>(y + o) = pack8(best);
    if (qs.q) *reinterpret_cast<uint2*>(qs.q + o) = q_pack8(qs, qsc, best, qmax);
    if (mask) {
      uint2 m;
      m.x = arg[0] | (arg[1] << 8) | (arg[2] << 16) | (arg[3] << 24);
      m.y = arg[4] | (arg[5] << 8) | (arg[6] << 16) | (arg[7] << 24);
      *reinterpret_cast<uint2*>(mask + o) = m;
    }
  }
  if (qs.q) q_flush(qs, qmax);
}

// NH x NW = max number of windows covering one input pixel (ceil(k / stride) per axis).
template <int NH, int NW, bool MAX>
__global__ void pool_bwd_k(const bf16_t* __restrict__ dy, const uint8_t* __restrict__ mask, bf16_t* __restrict__ dx,
                           PoolGeom g, QSide qs) {
  const int cv = g.C / 8;
  float qmax = 0.f;
  const float qsc = qs.q ? qs.slot[0] : 0.f;
  const long long total = (long long)g.N * g.H * g.W * cv;
  for (long long i = xcd_block(blockIdx.x, gridDim.x) * (long long)blockDim.x + threadIdx.x; i < total;
       i += (long long)gridDim.x * blockDim.x) {
    const uint32_t pix = udiv((uint32_t)i, g.fcv), ph_ = udiv(pix, g.fW), n = udiv(ph_, g.fH);
    const int c0 = (int)((uint32_t)i - pix * cv) * 8;
    const int w = (int)(pix - ph_ * g.W), h = (int)(ph_ - n * g.H);
    const int hp = h + g.ph, wp = w + g.pw;
    const int p0 = hp < g.kh ? 0 : (int)udiv((uint32_t)(hp - g.kh), g.fsh) + 1;
    const int p1 = min((int)udiv((uint32_t)hp, g.fsh) + 1, g.P);
    const int q0 = wp < g.kw ? 0 : (int)udiv((uint32_t)(wp - g.kw), g.fsw) + 1;
    const int q1 = min((int)udiv((uint32_t)wp, g.fsw) + 1, g.Q);
    uint4 dv[NH * NW];
    uint2 mv[NH * NW];
    bool ok[NH * NW];
#pragma unroll
    for (int a = 0; a < NH; ++a)
#pragma unroll
      for (int b = 0; b < NW; ++b) {
        const int p = p0 + a, q = q0 + b;
        ok[a * NW + b] = p < p1 && q < q1;
        const int pc = min(p, g.P - 1), qc = min(q, g.Q - 1);
        const long long o = (((long long)n * g.P + pc) * g.Q + qc) * g.C + c0;
        dv[a * NW + b] = *reinterpret_cast<const uint4*>(dy + o);
        if (MAX) mv[a * NW + b] = *reinterpret_cast<const uint2*>(mask + o);
      }
    float acc[8] = {0, 0, 0, 0, 0, 0, 0, 0};
#pragma unroll
    for (int a = 0; a < NH; ++a)
#pragma unroll
      for (int b = 0; b < NW; ++b) {
        const int t = a * NW + b;
        const int p = p0 + a, q = q0 + b;
        const int hs = p * g.sh - g.ph, ws = q * g.sw - g.pw;
        float f[8];
        unpack8(dv[t], f);
        if (MAX) {
          const int widx = (h - hs) * g.kw + (w - ws);
          const uint32_t mw[2] = {mv[t].x, mv[t].y};
#pragma unroll
          for (int k = 0; k < 8; ++k)
            if (ok[t] && (int)((mw[k >> 2] >> ((k & 3) * 8)) & 0xff) == widx) acc[k] += f[k];
        } else {
          const int he = min(hs + g.kh, g.H + g.ph), we = min(ws + g.kw, g.W + g.pw);
          const float scale = ok[t] ? 1.f / (float)((he - hs) * (we - ws)) : 0.f;
#pragma unroll
          for (int k = 0; k < 8; ++k) acc[k] += f[k] * scale;
        }
      }
    if (dx) *reinterpret_cast<uint4*>(dx + (long long)pix * g.C + c0) = pack8(acc);
    if (qs.q) *reinterpret_cast<uint2*>(qs.q + (long long)pix * g.C + c0) = q_pack8(qs, qsc, acc, qmax);
  }
  if (qs.q) q_flush(qs, qmax);
}

// 3x3 / stride-2 windows (AlexNet / CaffeNet / GoogLeNet pools): in padded coordinates
// (hp = h + ph) input rows 2b and 2b+1 are covered by windows {b-1, b} and {b}, so ONE
// thread handles a 2x2 block of input pixels from the same 4 windows — a quarter of the
// window loads of the per-pixel gather above (which is L2-bandwidth bound: every window
// is re-read by the ~4 pixels it covers).
template <bool MAX>
__global__ void pool_bwd_k3s2(const bf16_t* __restrict__ dy, const uint8_t* __restrict__ mask,
                              bf16_t* __restrict__ dx, PoolGeom g, FDiv fBW, FDiv fBH, int BW, int BH) {
  const int cv = g.C / 8;
  const long long total = (long long)g.N * BH * BW * cv;
  for (long long i = xcd_block(blockIdx.x, gridDim.x) * (long long)blockDim.x + threadIdx.x; i < total;
       i += (long long)gridDim.x * blockDim.x) {
    const uint32_t blk = udiv((uint32_t)i, g.fcv), bh_ = udiv(blk, fBW), n = udiv(bh_, fBH);
    const int c0 = (int)((uint32_t)i - blk * cv) * 8;
    const int bw = (int)(blk - bh_ * BW), bh = (int)(bh_ - n * BH);
    uint4 dv[4];
    uint2 mv[4];
    bool ok[4];
#pragma unroll
    for (int a = 0; a < 2; ++a)
#pragma unroll
      for (int b = 0; b < 2; ++b) {
        const int p = bh - 1 + a, q = bw - 1 + b, t = a * 2 + b;
        ok[t] = p >= 0 && p < g.P && q >= 0 && q < g.Q;
        const int pc = min(max(p, 0), g.P - 1), qc = min(max(q, 0), g.Q - 1);
        const long long o = (((long long)n * g.P + pc) * g.Q + qc) * g.C + c0;
        dv[t] = *reinterpret_cast<const uint4*>(dy + o);
        if (MAX) mv[t] = *reinterpret_cast<const uint2*>(mask + o);
      }
    float f[4][8];
#pragma unroll
    for (int t = 0; t < 4; ++t) unpack8(dv[t], f[t]);
    float scale[4] = {1.f, 1.f, 1.f, 1.f};
    if (!MAX) {
#pragma unroll
      for (int t = 0; t < 4; ++t) {
        const int p = bh - 1 + (t >> 1), q = bw - 1 + (t & 1);
        const int hs = 2 * p - g.ph, ws = 2 * q - g.pw;
        const int he = min(hs + 3, g.H + g.ph), we = min(ws + 3, g.W + g.pw);
        scale[t] = ok[t] ? 1.f / (float)((he - hs) * (we - ws)) : 0.f;
      }
    }
#pragma unroll
    for (int a = 0; a < 2; ++a)
#pragma unroll
      for (int b = 0; b < 2; ++b) {
        const int h = 2 * bh + a - g.ph, w = 2 * bw + b - g.pw;
        if ((unsigned)h >= (unsigned)g.H || (unsigned)w >= (unsigned)g.W) continue;
        float acc[8] = {0, 0, 0, 0, 0, 0, 0, 0};
#pragma unroll
        for (int t = 0; t < 4; ++t) {
          const int wa = t >> 1, wb = t & 1;  // window p = bh-1+wa covers row a iff wa == 1 or a == 0
          if ((wa == 0 && a == 1) || (wb == 0 && b == 1)) continue;
          if (MAX) {
            // window-relative offset of this pixel: row (2bh+a) - 2p = a + 2(1-wa)
            const int widx = (a + 2 * (1 - wa)) * 3 + (b + 2 * (1 - wb));
            const uint32_t mw[2] = {mv[t].x, mv[t].y};
#pragma unroll
            for (int k = 0; k < 8; ++k)
              if (ok[t] && (int)((mw[k >> 2] >> ((k & 3) * 8)) & 0xff) == widx) acc[k] += f[t][k];
          } else {
#pragma unroll
            for (int k = 0; k < 8; ++k) acc[k] += f[t][k] * scale[t];
          }
        }
        *reinterpret_cast<uint4*>(dx + (((long long)n * g.H + h) * g.W + w) * g.C + c0) = pack8(acc);
      }
  }
}

static PoolGeom mkgeom(long long N, long long H, long long W, long long C, long long P, long long Q, long long kh,
                       long long kw, long long sh, long long sw, long long ph, long long pw) {
  PoolGeom g;
  g.N = (int)N; g.H = (int)H; g.W = (int)W; g.C = (int)C; g.P = (int)P; g.Q = (int)Q;
  g.kh = (int)kh; g.kw = (int)kw; g.sh = (int)sh; g.sw = (int)sw; g.ph = (int)ph; g.pw = (int)pw;
  g.fcv = make_fdiv((uint32_t)((C % 8) == 0 ? C / 8 : C));
  g.fW = make_fdiv((uint32_t)W); g.fH = make_fdiv((uint32_t)H);
  g.fQ = make_fdiv((uint32_t)Q); g.fP = make_fdiv((uint32_t)P);
  g.fsh = make_fdiv((uint32_t)sh); g.fsw = make_fdiv((uint32_t)sw);
  return g;
}

// (Round 6 removed the measured-and-rejected opt-in variants: LDS row-band 3x3 / stride-1 pooling,
// block-per-thread 2x2 / stride-2 backward and 3x3 / stride-1 forward / backward —
// docs/PERF_NOTES.md rounds 4-5.)
extern "C" int sn_pool_fwd(const bf16_t* x, bf16_t* y, uint8_t* mask, long long N, long long H, long long W,
                           long long C, long long P, long long Q, long long kh, long long kw, long long sh,
                           long long sw, long long ph, long long pw, long long method, long long gate,
                           uint8_t* q, const float* qslot, float* qpart, long long qe5m2, hipStream_t st) {
  PoolGeom g = mkgeom(N, H, W, C, P, Q, kh, kw, sh, sw, ph, pw);
  const QSide qs{q, qslot, qpart, (int)qe5m2};
  // fp8 side output: the vectorised fixed-window max-pool only
  if (q && !(method == 0 && (C % 8) == 0 && kh == kw && (kh == 2 || kh == 3) && qslot && qpart)) return 9;
  if (method == 0 && kh * kw > 254) return 6;
  if (N * H * W * C >= (1ll << 32)) return 8;  // 32-bit index decode
  const bool vec = (C % 8) == 0;
  long long total = N * P * Q * (vec ? C / 8 : C);
  dim3 grid(sn_blocks(total, 256, 16384));
  if (method == 0 && vec && kh == kw && (kh == 2 || kh == 3)) {
    if (kh == 3)
      hipLaunchKernelGGL((maxpool_fwd_k<3, 3>), grid, dim3(256), 0, st, x, y, mask, g, (int)gate, qs);
    else hipLaunchKernelGGL((maxpool_fwd_k<2, 2>), grid, dim3(256), 0, st, x, y, mask, g, (int)gate, qs);
  } else if (method == 0) {
    if (vec) hipLaunchKernelGGL(maxpool_fwd<true>, grid, dim3(256), 0, st, x, y, mask, g, (int)gate);
    else hipLaunchKernelGGL(maxpool_fwd<false>, grid, dim3(256), 0, st, x, y, mask, g, (int)gate);
  } else {
    // one-wave blocks when the output is small: GoogLeNet's global 7 x 7 pool has 16384 threads
    // (64 blocks of 256 left 3/4 of the CUs idle)
    const int bs = total < 256 * 1024 ? 64 : 256;
    const dim3 ag(sn_blocks(total, bs, 16384));
    if (vec) hipLaunchKernelGGL(avepool_fwd<true>, ag, dim3(bs), 0, st, x, y, g);
    else hipLaunchKernelGGL(avepool_fwd<false>, ag, dim3(bs), 0, st, x, y, g);
  }
  return SN_CHECK_LAUNCH();
}

extern "C" int sn_pool_bwd(const bf16_t* dy, const uint8_t* mask, bf16_t* dx, long long N, long long H, long long W,
                           long long C, long long P, long long Q, long long kh, long long kw, long long sh,
                           long long sw, long long ph, long long pw, long long method,
                           uint8_t* q, const float* qslot, float* qpart, long long qe5m2, hipStream_t st) {
  PoolGeom g = mkgeom(N, H, W, C, P, Q, kh, kw, sh, sw, ph, pw);
  const QSide qs{q, qslot, qpart, (int)qe5m2};
  if (N * H * W * C >= (1ll << 32)) return 8;  // 32-bit index decode
  const bool vec = (C % 8) == 0;
  long long total = N * H * W * (vec ? C / 8 : C);
  dim3 grid(sn_blocks(total, 256, 16384));
  const long long nh = (kh + sh - 1) / sh, nw = (kw + sw - 1) / sw;
  // fp8 side output: the pool_bwd_k paths only.  dx null: the side output alone (the consuming
  // conv reads nothing but the fp8 bytes, engine.fuse_fp8_quant fp8_dx_only)
  if (q && (!vec || (kh == 3 && kw == 3 && sh == 2 && sw == 2) || nh != nw || nh < 1 || nh > 3)) return 9;
  if (!dx && !q) return 9;
  if (vec && kh == 3 && kw == 3 && sh == 2 && sw == 2) {
    // 2x2 input pixels per thread over the padded extent [0, H + ph) x [0, W + pw)
    const int BH = (int)((H + ph + 1) / 2), BW = (int)((W + pw + 1) / 2);
    const long long nt = N * BH * BW * (C / 8);
    dim3 g2(sn_blocks(nt, 256, 16384));
    if (method == 0)
      hipLaunchKernelGGL((pool_bwd_k3s2<true>), g2, dim3(256), 0, st, dy, mask, dx, g, make_fdiv((uint32_t)BW),
                         make_fdiv((uint32_t)BH), BW, BH);
    else
      hipLaunchKernelGGL((pool_bwd_k3s2<false>), g2, dim3(256), 0, st, dy, mask, dx, g, make_fdiv((uint32_t)BW),
                         make_fdiv((uint32_t)BH), BW, BH);
  } else if (vec && nh == nw && nh >= 1 && nh <= 3) {
    if (q && !(qslot && qpart)) return 9;
#define SN_POOL_BWD_K(NN)                                                                                  \
  do {                                                                                                     \
    if (method == 0) hipLaunchKernelGGL((pool_bwd_k<NN, NN, true>), grid, dim3(256), 0, st, dy, mask, dx, g, qs); \
    else hipLaunchKernelGGL((pool_bwd_k<NN, NN, false>), grid, dim3(256), 0, st, dy, mask, dx, g, qs);            \
  } while (0)
    if (nh == 1) SN_POOL_BWD_K(1);
    else if (nh == 2) SN_POOL_BWD_K(2);
    else SN_POOL_BWD_K(3);
#undef SN_POOL_BWD_K
  } else if (method == 0) {
    if (vec) hipLaunchKernelGGL((pool_bwd<true, true>), grid, dim3(256), 0, st, dy, mask, dx, g);
    else hipLaunchKernelGGL((pool_bwd<false, true>), grid, dim3(256), 0, st, dy, mask, dx, g);
  } else {
    if (vec) hipLaunchKernelGGL((pool_bwd<true, false>), grid, dim3(256), 0, st, dy, mask, dx, g);
    else hipLaunchKernelGGL((pool_bwd<false, false>), grid, dim3(256), 0, st, dy, mask, dx, g);
  }
  return SN_CHECK_LAUNCH();
}
