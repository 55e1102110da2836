// Fused 3x3 / stride-2 max pooling + cross-channel LRN on NHWC bf16 — the pool1 -> norm1
// and pool2 -> norm2 pairs of CaffeNet (and GoogLeNet's pool1 -> norm1).
//
// Reference: two layers, each a full pass over HBM (pooling_layer.cu:11-47 MaxPoolForward,
// 217-260 MaxPoolBackward; lrn_layer.cu:9-177 fill-scale / compute-output / compute-diff).
// Unfused here they are maxpool_fwd_k + lrn_across_fwd and lrn_across_bwd + pool_bwd_k3s2:
// the pooled tensor is written, read back by the LRN, and in backward the LRN's input
// gradient (the pooling layer's top diff) is written and read back by the pooling
// backward.  Fused:
//   forward : one workgroup pools a run of output pixels (all channels) into LDS, stores
//             the pooled tensor (the LRN backward needs it) and the argmax mask, then
//             normalises across channels out of LDS — the LRN never re-reads HBM;
//   backward: one workgroup owns RB rows of 2x2 input blocks of one image and a group of
//             channel chunks: it computes the LRN input gradient of the RB+1 pooled rows
//             those blocks read (one halo row) into LDS, then gathers the pooling gradient
//             out of LDS — the pooled gradient never exists in HBM.
// The arithmetic is the unfused kernels' own, in the same order, on the same bf16-rounded
// intermediates, so the fused pair is bitwise equal to the two separate launches.
#include "common.h"

#include <cmath>

#include <cstdlib>

struct PLGeom {
  int N, H, W, C, P, Q, ph, pw;
  int gate;         // forward: the pooled input is an in-place ReLU output (mask 255 = no gradient)
  int pix;          // forward: pooled pixels per workgroup
  int BH, BW;       // backward: 2x2 input blocks over the padded extent
  int rows, nb;     // backward: block rows per workgroup, row runs per image
  int cg, ngrp;     // backward: channel chunks per workgroup, channel groups
  int size;
  float alpha, beta, k;
  FDiv fcv, fQ, fP, fcg, fQcg, fBWcg, fBW, fBH;
};

SN_DEV float plrn_pow(float s, float beta) { return sn_powneg(s, beta); }

template <int SIZE>
__global__ void __launch_bounds__(256) pool_lrn_fwd(const bf16_t* __restrict__ x, bf16_t* __restrict__ pooled,
                                                    uint8_t* __restrict__ mask, bf16_t* __restrict__ y, PLGeom g) {
  extern __shared__ uint4 tile[];  // g.pix x cv pooled chunks
  constexpr int PRE = (SIZE - 1) / 2;
  const int cv = g.C >> 3;
  const long long npix = (long long)g.N * g.P * g.Q;
  const long long pix0 = (long long)xcd_block(blockIdx.x, gridDim.x) * g.pix;
  const int npx = (int)min((long long)g.pix, npix - pix0);
  const int items = npx * cv;
  for (int it = threadIdx.x; it < items; it += blockDim.x) {
    const uint32_t lp = udiv((uint32_t)it, g.fcv);
    const int c0 = (it - (int)lp * cv) * 8;
    const uint32_t pix = (uint32_t)(pix0 + lp);
    const uint32_t pq = udiv(pix, g.fQ), n = udiv(pq, g.fP);
    const int q = (int)(pix - pq * g.Q), p = (int)(pq - n * g.P);
    const int hs = 2 * p - g.ph, ws = 2 * q - g.pw;
    uint4 v[9];
    bool ok[9];
#pragma unroll
    for (int a = 0; a < 3; ++a)
#pragma unroll
      for (int b = 0; b < 3; ++b) {
        const int h = hs + a, w = ws + b;
        ok[a * 3 + b] = (unsigned)h < (unsigned)g.H && (unsigned)w < (unsigned)g.W;
        const int hc = min(max(h, 0), g.H - 1), wc = min(max(w, 0), g.W - 1);
        v[a * 3 + b] = *reinterpret_cast<const uint4*>(x + (((long long)n * g.H + hc) * g.W + wc) * g.C + c0);
      }
    float best[8];
    int arg[8];
#pragma unroll
    for (int t = 0; t < 8; ++t) { best[t] = -INFINITY; arg[t] = 0; }
#pragma unroll
    for (int widx = 0; widx < 9; ++widx) {
      float f[8];
      unpack8(v[widx], f);
#pragma unroll
      for (int t = 0; t < 8; ++t)
        if (ok[widx] && f[t] > best[t]) { best[t] = f[t]; arg[t] = widx; }
    }
    if (g.gate) {
#pragma unroll
      for (int t = 0; t < 8; ++t)
        if (!(best[t] > 0.f)) arg[t] = 255;
    }
    const uint4 packed = pack8(best);
    const long long o = (long long)pix * g.C + c0;
    *reinterpret_cast<uint4*>(pooled + o) = packed;
    uint2 m;
    m.x = arg[0] | (arg[1] << 8) | (arg[2] << 16) | (arg[3] << 24);
    m.y = arg[4] | (arg[5] << 8) | (arg[6] << 16) | (arg[7] << 24);
    *reinterpret_cast<uint2*>(mask + o) = m;
    tile[it] = packed;
  }
  __syncthreads();
  const float a = g.alpha / g.size;
  for (int it = threadIdx.x; it < items; it += blockDim.x) {
    const uint32_t lp = udiv((uint32_t)it, g.fcv);
    const int ch = it - (int)lp * cv;
    float v[24];
#pragma unroll
    for (int j = 0; j < 3; ++j) {
      const int c = ch - 1 + j;
      const bool ok = c >= 0 && c < cv;
      unpack8(tile[(int)lp * cv + min(max(c, 0), cv - 1)], v + 8 * j);
#pragma unroll
      for (int t = 0; t < 8; ++t) v[8 * j + t] = ok ? v[8 * j + t] : 0.f;
    }
    float o[8];
#pragma unroll
    for (int t = 0; t < 8; ++t) {
      float s = 0.f;
#pragma unroll
      for (int d = 0; d < SIZE; ++d) {
        float e = v[8 + t - PRE + d];
        s = __builtin_fmaf(e, e, s);
      }
      float sc = __builtin_fmaf(a, s, g.k);
      o[t] = v[8 + t] * plrn_pow(sc, g.beta);
    }
    *reinterpret_cast<uint4*>(y + (pix0 + lp) * g.C + ch * 8) = pack8(o);
  }
}

// The 24 channels [c0-8, c0+16) of one pixel row as fp32, zero outside [0, C).
SN_DEV void plrn_load24(const bf16_t* row, int c0, int C, float* v) {
  uint4 raw[3];
#pragma unroll
  for (int j = 0; j < 3; ++j) raw[j] = *reinterpret_cast<const uint4*>(row + min(max(c0 - 8 + 8 * j, 0), C - 8));
#pragma unroll
  for (int j = 0; j < 3; ++j) {
    const int c = c0 - 8 + 8 * j;
    const bool ok = c >= 0 && c < C;
    unpack8(raw[j], v + 8 * j);
#pragma unroll
    for (int t = 0; t < 8; ++t) v[8 * j + t] = ok ? v[8 * j + t] : 0.f;
  }
}

// Phase 1 of the fused backward: the LRN input gradient of pooled rows bh0-1 .. bh0+rows-1,
// channel chunks [ch0, ch0 + cg), of image n into the LDS tile (lrn_across_bwd, gate off);
// MLDS also stages the argmax mask of those rows after the gradient tile.
template <int SIZE, bool MLDS>
SN_DEV void plrn_bwd_phase1(const bf16_t* __restrict__ xp, const bf16_t* __restrict__ dyn,
                            const uint8_t* __restrict__ mask, const PLGeom& g, uint4* tile, int n, int bh0, int ch0,
                            int cg, int items1) {
  constexpr int PRE = (SIZE - 1) / 2, POST = SIZE - PRE - 1;
  const int qcg = g.Q * cg;
  const float a = g.alpha / g.size;
  const float cache_ratio = 2.f * g.alpha * g.beta / g.size;
  for (int it = threadIdx.x; it < items1; it += blockDim.x) {
    const uint32_t r = udiv((uint32_t)it, g.fQcg);
    const int rem = it - (int)r * qcg;
    const uint32_t q = udiv((uint32_t)rem, g.fcg);
    const int c0 = (ch0 + rem - (int)q * cg) * 8;
    const int p = bh0 - 1 + (int)r;
    if (p < 0 || p >= g.P) {
      tile[it] = make_uint4(0u, 0u, 0u, 0u);
      if (MLDS) reinterpret_cast<uint2*>(tile + items1)[it] = make_uint2(0u, 0u);
      continue;
    }
    const long long base = (((long long)n * g.P + p) * g.Q + q) * g.C;
    if (MLDS) reinterpret_cast<uint2*>(tile + items1)[it] = *reinterpret_cast<const uint2*>(mask + base + c0);
    float xv[24], gv[24];
    plrn_load24(xp + base, c0, g.C, xv);
    plrn_load24(dyn + base, c0, g.C, gv);
    float rr[24];
#pragma unroll
    for (int j = 8 - POST; j < 16 + PRE; ++j) {
      float s = 0.f;
#pragma unroll
      for (int d = 0; d < SIZE; ++d) {
        float e = xv[j - PRE + d];
        s = __builtin_fmaf(e, e, s);
      }
      float sc = __builtin_fmaf(a, s, g.k);
      // channels outside [0, C) have x = dy = 0 (plrn_load24): rr is 0 there without a branch
      rr[j] = __builtin_fmaf(gv[j] * xv[j], plrn_pow(sc, g.beta + 1.f), 0.f);
      if (j >= 8 && j < 16) gv[j] = gv[j] * plrn_pow(sc, g.beta);
    }
    float o[8];
#pragma unroll
    for (int t = 0; t < 8; ++t) {
      float acc = 0.f;
#pragma unroll
      for (int d = -PRE; d <= POST; ++d) acc += rr[8 + t - d];
      o[t] = __builtin_fmaf(-(cache_ratio * xv[8 + t]), acc, gv[8 + t]);
    }
    tile[it] = pack8(o);
  }
}

// MLDS: phase 1 also stages the argmax mask of the pooled rows in LDS (after the gradient
// tile), so phase 2's window reads are LDS reads instead of dependent global loads.
template <int SIZE, bool MLDS>
__global__ void __launch_bounds__(256) lrn_pool_bwd(const bf16_t* __restrict__ xp, const bf16_t* __restrict__ dyn,
                                                    const uint8_t* __restrict__ mask, bf16_t* __restrict__ dx,
                                                    PLGeom g) {
  // workgroup = (image, run of `rows` block rows, group of `cg` channel chunks): the LRN's
  // channel window only widens the global loads of phase 1, so channel groups cost no
  // recomputation; only the one halo pooled row above the run is computed twice
  extern __shared__ uint4 tile[];  // (rows + 1) x Q x cg chunks of the pooled gradient
  const int cg = g.cg;
  const int bid = xcd_block(blockIdx.x, gridDim.x);
  const int wg = bid / g.ngrp;
  const int ch0 = (bid - wg * g.ngrp) * cg;
  const int n = wg / g.nb;
  const int bh0 = (wg - n * g.nb) * g.rows;
  const int qcg = g.Q * cg;
  const int items1 = (g.rows + 1) * qcg;
  plrn_bwd_phase1<SIZE, MLDS>(xp, dyn, mask, g, tile, n, bh0, ch0, cg, items1);
  __syncthreads();
  // phase 2: the 2x2 input blocks of rows bh0 .. bh0+rows-1 (pool_bwd_k3s2<true>)
  const int bwcg = g.BW * cg;
  const int items2 = min(g.rows, g.BH - bh0) * bwcg;
  for (int it = threadIdx.x; it < items2; it += blockDim.x) {
    const uint32_t r = udiv((uint32_t)it, g.fBWcg);
    const int rem = it - (int)r * bwcg;
    const uint32_t bwu = udiv((uint32_t)rem, g.fcg);
    const int lc = rem - (int)bwu * cg, c0 = (ch0 + lc) * 8;
    const int bw = (int)bwu, bh = bh0 + (int)r;
    uint4 dv[4];
    uint2 mv[4];
    bool ok[4];
#pragma unroll
    for (int wa = 0; wa < 2; ++wa)
#pragma unroll
      for (int wb = 0; wb < 2; ++wb) {
        const int p = bh - 1 + wa, q = bw - 1 + wb, t = wa * 2 + wb;
        ok[t] = p >= 0 && p < g.P && q >= 0 && q < g.Q;
        const int pc = min(max(p, 0), g.P - 1), qc = min(max(q, 0), g.Q - 1);
        dv[t] = tile[((int)r + wa) * qcg + qc * cg + lc];
        if (MLDS)
          mv[t] = reinterpret_cast<const uint2*>(tile + items1)[((int)r + wa) * qcg + qc * cg + lc];
        else
          mv[t] = *reinterpret_cast<const uint2*>(mask + (((long long)n * g.P + pc) * g.Q + qc) * g.C + c0);
      }
    float f[4][8];
#pragma unroll
    for (int t = 0; t < 4; ++t) unpack8(dv[t], f[t]);
#pragma unroll
    for (int ia = 0; ia < 2; ++ia)
#pragma unroll
      for (int ib = 0; ib < 2; ++ib) {
        const int h = 2 * bh + ia - g.ph, w = 2 * bw + ib - g.pw;
        if ((unsigned)h >= (unsigned)g.H || (unsigned)w >= (unsigned)g.W) continue;
        float acc[8] = {0, 0, 0, 0, 0, 0, 0, 0};
#pragma unroll
        for (int t = 0; t < 4; ++t) {
          const int wa = t >> 1, wb = t & 1;
          if ((wa == 0 && ia == 1) || (wb == 0 && ib == 1)) continue;
          const int widx = (ia + 2 * (1 - wa)) * 3 + (ib + 2 * (1 - wb));
          const uint32_t mw[2] = {mv[t].x, mv[t].y};
#pragma unroll
          for (int kk = 0; kk < 8; ++kk)
            if (ok[t] && (int)((mw[kk >> 2] >> ((kk & 3) * 8)) & 0xff) == widx) acc[kk] += f[t][kk];
        }
        *reinterpret_cast<uint4*>(dx + (((long long)n * g.H + h) * g.W + w) * g.C + c0) = pack8(acc);
      }
  }
}

// The other order — a cross-channel LRN whose output feeds a 3x3 / stride-2 max pooling
// (AlexNet's norm1 -> pool1 and norm2 -> pool2, GoogLeNet's conv2/norm2 -> pool2) — fused in
// BACKWARD only.  A workgroup owns a run of g.pix 2x2 input blocks (linear over image, block
// row, block column) with ALL their channels:
//   phase 1: one item per (block, 8-channel chunk) gathers the pooling gradient of the block's
//            4 pixels from the 4 windows covering it (pool_bwd_k3s2's order), rounded to bf16
//            as that kernel stores it, into LDS;
//   phase 2: one item per (pixel, chunk) runs the LRN backward (lrn_across_bwd's arithmetic,
//            with the fused ReLU gate), its neighbour channels read from the LDS tile.
// The LRN-output gradient (the full-resolution tensor the unfused pair writes and re-reads)
// never reaches HBM; the result is bitwise equal to the two launches.  (The forward stays two
// launches: the LRN of a 3x3 window's 9 pixels would be recomputed by up to 4 windows.)
template <int SIZE>
__global__ void __launch_bounds__(256) pool_lrn_bwd_rev(const bf16_t* __restrict__ dy, const uint8_t* __restrict__ mask,
                                                        const bf16_t* __restrict__ x, bf16_t* __restrict__ dx,
                                                        PLGeom g) {
  extern __shared__ uint4 tile[];  // g.pix blocks x 4 pixels x cv chunks of the pooling gradient
  constexpr int PRE = (SIZE - 1) / 2, POST = SIZE - PRE - 1;
  const int cv = g.C >> 3;
  const long long nblk = (long long)g.N * g.BH * g.BW;
  const long long blk0 = (long long)xcd_block(blockIdx.x, gridDim.x) * g.pix;
  const int nb = (int)min((long long)g.pix, nblk - blk0);
  // phase 1: pooling backward of the run's blocks into LDS
  const int items1 = nb * cv;
  for (int it = threadIdx.x; it < items1; it += blockDim.x) {
    const uint32_t lb = udiv((uint32_t)it, g.fcv);
    const int ch = it - (int)lb * cv, c0 = ch * 8;
    const uint32_t blk = (uint32_t)(blk0 + lb), bh_ = udiv(blk, g.fBW), n = udiv(bh_, g.fBH);
    const int bw = (int)(blk - bh_ * g.BW), bh = (int)(bh_ - n * g.BH);
    uint4 dv[4];
    uint2 mv[4];
    bool ok[4];
#pragma unroll
    for (int wa = 0; wa < 2; ++wa)
#pragma unroll
      for (int wb = 0; wb < 2; ++wb) {
        const int p = bh - 1 + wa, q = bw - 1 + wb, t = wa * 2 + wb;
        ok[t] = p >= 0 && p < g.P && q >= 0 && q < g.Q;
        const int pc = min(max(p, 0), g.P - 1), qc = min(max(q, 0), g.Q - 1);
        const long long o = (((long long)n * g.P + pc) * g.Q + qc) * g.C + c0;
        dv[t] = *reinterpret_cast<const uint4*>(dy + o);
        mv[t] = *reinterpret_cast<const uint2*>(mask + o);
      }
    float f[4][8];
#pragma unroll
    for (int t = 0; t < 4; ++t) unpack8(dv[t], f[t]);
#pragma unroll
    for (int ia = 0; ia < 2; ++ia)
#pragma unroll
      for (int ib = 0; ib < 2; ++ib) {
        float acc[8] = {0, 0, 0, 0, 0, 0, 0, 0};
#pragma unroll
        for (int t = 0; t < 4; ++t) {
          const int wa = t >> 1, wb = t & 1;
          if ((wa == 0 && ia == 1) || (wb == 0 && ib == 1)) continue;
          const int widx = (ia + 2 * (1 - wa)) * 3 + (ib + 2 * (1 - wb));
          const uint32_t mw[2] = {mv[t].x, mv[t].y};
#pragma unroll
          for (int kk = 0; kk < 8; ++kk)
            if (ok[t] && (int)((mw[kk >> 2] >> ((kk & 3) * 8)) & 0xff) == widx) acc[kk] += f[t][kk];
        }
        tile[((int)lb * 4 + ia * 2 + ib) * cv + ch] = pack8(acc);
      }
  }
  __syncthreads();
  // phase 2: LRN backward of the run's pixels
  const float a = g.alpha / g.size;
  const float cache_ratio = 2.f * g.alpha * g.beta / g.size;
  const int items2 = 4 * nb * cv;
  for (int it = threadIdx.x; it < items2; it += blockDim.x) {
    const uint32_t lp = udiv((uint32_t)it, g.fcv);
    const int ch = it - (int)lp * cv, c0 = ch * 8;
    const uint32_t lb = lp >> 2, sub = lp & 3;
    const uint32_t blk = (uint32_t)(blk0 + lb), bh_ = udiv(blk, g.fBW), n = udiv(bh_, g.fBH);
    const int bw = (int)(blk - bh_ * g.BW), bh = (int)(bh_ - n * g.BH);
    const int h = 2 * bh + (int)(sub >> 1) - g.ph, w = 2 * bw + (int)(sub & 1) - g.pw;
    if ((unsigned)h >= (unsigned)g.H || (unsigned)w >= (unsigned)g.W) continue;
    const long long base = (((long long)n * g.H + h) * g.W + w) * g.C;
    float xv[24], gv[24];
    plrn_load24(x + base, c0, g.C, xv);
#pragma unroll
    for (int j = 0; j < 3; ++j) {
      const int c = ch - 1 + j;
      const bool cok = c >= 0 && c < cv;
      unpack8(tile[(int)lp * cv + min(max(c, 0), cv - 1)], gv + 8 * j);
#pragma unroll
      for (int t = 0; t < 8; ++t) gv[8 * j + t] = cok ? gv[8 * j + t] : 0.f;
    }
    float rr[24];
#pragma unroll
    for (int j = 8 - POST; j < 16 + PRE; ++j) {
      float s2 = 0.f;
#pragma unroll
      for (int d = 0; d < SIZE; ++d) {
        float ev = xv[j - PRE + d];
        s2 = __builtin_fmaf(ev, ev, s2);
      }
      float sc = __builtin_fmaf(a, s2, g.k);
      rr[j] = __builtin_fmaf(gv[j] * xv[j], plrn_pow(sc, g.beta + 1.f), 0.f);
      if (j >= 8 && j < 16) gv[j] = gv[j] * plrn_pow(sc, g.beta);
    }
    float o[8];
#pragma unroll
    for (int t = 0; t < 8; ++t) {
      float acc = 0.f;
#pragma unroll
      for (int d = -PRE; d <= POST; ++d) acc += rr[8 + t - d];
      o[t] = __builtin_fmaf(-(cache_ratio * xv[8 + t]), acc, gv[8 + t]);
      if (g.gate && !(xv[8 + t] > 0.f)) o[t] = 0.f;
    }
    *reinterpret_cast<uint4*>(dx + base + c0) = pack8(o);
  }
}

static PLGeom plgeom(long long N, long long H, long long W, long long C, long long P, long long Q, long long ph,
                     long long pw, long long size, float alpha, float beta, float k) {
  PLGeom g{};
  g.N = (int)N; g.H = (int)H; g.W = (int)W; g.C = (int)C; g.P = (int)P; g.Q = (int)Q;
  g.ph = (int)ph; g.pw = (int)pw;
  g.size = (int)size; g.alpha = alpha; g.beta = beta; g.k = k;
  g.fcv = make_fdiv((uint32_t)(C / 8));
  g.fQ = make_fdiv((uint32_t)Q); g.fP = make_fdiv((uint32_t)P);
  return g;
}

static bool plrn_ok(long long N, long long H, long long W, long long C, long long P, long long Q, long long ph,
                    long long pw, long long size) {
  // 3x3 / stride-2 ceil-mode windows, every window starting inside the padded input
  return C % 8 == 0 && C >= 8 && (size == 3 || size == 5 || size == 7 || size == 9) && ph < 3 && pw < 3 &&
         2 * (P - 1) - ph < H && 2 * (Q - 1) - pw < W && N * H * W * C < (1ll << 32);
}

// Workgroup shapes (host side, shared with the Python eligibility check).
static int plrn_fwd_pix(long long C) {
  // (pixel, chunk) items per workgroup: 256 (one per thread) beat 512 / 1024 / 2048 at both
  // CaffeNet shapes (pool1/norm1 51.5 -> 47.8 us, pool2/norm2 31.1 -> 28.3 us,
  // profiles/r4_plrn_tiles.txt)
  const long long items = 256;
  return (int)(items / (C / 8) > 0 ? items / (C / 8) : 1);
}
// backward tile: for each channel group cg (a divisor of the C / 8 chunks, at least 4 chunks =
// 64 B of a pixel, or the whole pixel) the most block rows (<= 7, least halo recomputation)
// whose (rows + 1) x Q x cg tile fits the LDS budget (32 KB); of
// those, the shape whose grid is closest to 2560 workgroups (10 per CU: enough to fill every
// CU with short blocks, few enough that the halo rows stay a small share).  Measured on CaffeNet
// (profiles/r4_plrn_tiles.txt): pool1/norm1 74.4 -> 63.3 us (cg 12 -> 4), pool2/norm2 45.4 ->
// 42.4 us (cg 16 -> 8).
static bool plrn_bwd_tile(long long N, long long Q, long long C, long long BH, int item_bytes, int* rows, int* cg) {
  const int cv = (int)(C / 8);
  const long long budget = 32 * 1024;
  double best = 1e30;
  bool found = false;
  for (int c = cv; c >= 1; --c) {
    if (cv % c) continue;
    if (c != cv && c < 4) continue;
    int r = 7;
    while (r >= 1 && (long long)(r + 1) * Q * c * item_bytes > budget) --r;
    if (r < 1) continue;
    const double grid = (double)N * (double)((BH + r - 1) / r) * (double)(cv / c);
    const double d = std::fabs(std::log(grid / 2560.0));
    if (d < best - 1e-9) {
      best = d;
      *rows = r;
      *cg = c;
      found = true;
    }
  }
  return found;
}

extern "C" int sn_pool_lrn_fwd(const bf16_t* x, bf16_t* pooled, uint8_t* mask, bf16_t* y, long long N, long long H,
                               long long W, long long C, long long P, long long Q, long long ph, long long pw,
                               long long gate, long long size, float alpha, float beta, float k, hipStream_t st) {
  if (!plrn_ok(N, H, W, C, P, Q, ph, pw, size)) return 4;
  PLGeom g = plgeom(N, H, W, C, P, Q, ph, pw, size, alpha, beta, k);
  g.gate = (int)gate;
  g.pix = plrn_fwd_pix(C);
  const long long npix = N * P * Q;
  dim3 grid((unsigned)((npix + g.pix - 1) / g.pix));
  const size_t lds = (size_t)g.pix * (C / 8) * sizeof(uint4);
  switch (size) {
    case 3: hipLaunchKernelGGL(pool_lrn_fwd<3>, grid, dim3(256), lds, st, x, pooled, mask, y, g); break;
    case 5: hipLaunchKernelGGL(pool_lrn_fwd<5>, grid, dim3(256), lds, st, x, pooled, mask, y, g); break;
    case 7: hipLaunchKernelGGL(pool_lrn_fwd<7>, grid, dim3(256), lds, st, x, pooled, mask, y, g); break;
    default: hipLaunchKernelGGL(pool_lrn_fwd<9>, grid, dim3(256), lds, st, x, pooled, mask, y, g); break;
  }
  return SN_CHECK_LAUNCH();
}

// Host probe for the Python eligibility check (ops.hip.pool_lrn_eligible): 1 when both
// sn_pool_lrn_fwd and sn_lrn_pool_bwd accept the shape with the current environment's
// backward tile (the same plrn_ok / plrn_bwd_tile / row-coverage tests they apply).
extern "C" int sn_pool_lrn_supported(long long N, long long H, long long W, long long C, long long P, long long Q,
                                     long long ph, long long pw, long long size) {
  if (!plrn_ok(N, H, W, C, P, Q, ph, pw, size)) return 0;
  const int item_bytes = 24;  // argmax mask staged in LDS (sn_lrn_pool_bwd)
  const long long BH = (H + ph + 1) / 2, BW = (W + pw + 1) / 2;
  int rows = 0, cg = 0;
  if (!plrn_bwd_tile(N, Q, C, BH, item_bytes, &rows, &cg)) return 0;
  return BH <= P + 1 && BW <= Q + 1 ? 1 : 0;
}

extern "C" int sn_lrn_pool_bwd(const bf16_t* xp, const bf16_t* dyn, const uint8_t* mask, bf16_t* dx, long long N,
                               long long H, long long W, long long C, long long P, long long Q, long long ph,
                               long long pw, long long size, float alpha, float beta, float k, hipStream_t st) {
  if (!plrn_ok(N, H, W, C, P, Q, ph, pw, size)) return 4;
  PLGeom g = plgeom(N, H, W, C, P, Q, ph, pw, size, alpha, beta, k);
  g.BH = (int)((H + ph + 1) / 2);
  g.BW = (int)((W + pw + 1) / 2);
  // every pooled row the blocks read exists in the tile: blocks bh read rows bh-1, bh
  if (g.BH > P + 1 || g.BW > Q + 1) return 4;
  // argmax mask staged in LDS by phase 1 (instead of phase 2 reading it from global memory):
  // pool1/norm1 63.5 -> 62.2 us, pool2/norm2 42.5 -> 41.3 us (profiles/r4_plrn_tiles.txt)
  const int mlds = 1;
  const int item_bytes = mlds ? 24 : 16;
  if (!plrn_bwd_tile(N, Q, C, g.BH, item_bytes, &g.rows, &g.cg)) return 4;
  g.ngrp = (int)(C / 8) / g.cg;
  g.nb = (g.BH + g.rows - 1) / g.rows;
  g.fcg = make_fdiv((uint32_t)g.cg);
  g.fQcg = make_fdiv((uint32_t)(Q * g.cg));
  g.fBWcg = make_fdiv((uint32_t)(g.BW * g.cg));
  dim3 grid((unsigned)(N * g.nb * g.ngrp));
  const size_t lds = (size_t)(g.rows + 1) * Q * g.cg * item_bytes;
#define SN_PLRN_BWD(S)                                                                                          \
  do {                                                                                                          \
    if (mlds) hipLaunchKernelGGL((lrn_pool_bwd<S, true>), grid, dim3(256), lds, st, xp, dyn, mask, dx, g);   \
    else hipLaunchKernelGGL((lrn_pool_bwd<S, false>), grid, dim3(256), lds, st, xp, dyn, mask, dx, g);       \
  } while (0)
  switch (size) {
    case 3: SN_PLRN_BWD(3); break;
    case 5: SN_PLRN_BWD(5); break;
    case 7: SN_PLRN_BWD(7); break;
    default: SN_PLRN_BWD(9); break;
  }
#undef SN_PLRN_BWD
  return SN_CHECK_LAUNCH();
}

// LRN -> 3x3 / stride-2 max pooling, backward (pool_lrn_bwd_rev): dx at the LRN input from
// the pooled gradient dy and the argmax mask (pool_forward_mask's format), with the gate of
// the in-place ReLU that produced x when `gate` is set
extern "C" int sn_pool_lrn_bwd_rev(const bf16_t* dy, const uint8_t* mask, const bf16_t* x, bf16_t* dx, long long N,
                                   long long H, long long W, long long C, long long P, long long Q, long long ph,
                                   long long pw, long long size, float alpha, float beta, float k, long long gate,
                                   hipStream_t st) {
  if (!plrn_ok(N, H, W, C, P, Q, ph, pw, size)) return 4;
  PLGeom g = plgeom(N, H, W, C, P, Q, ph, pw, size, alpha, beta, k);
  g.gate = (int)gate;
  g.BH = (int)((H + ph + 1) / 2);
  g.BW = (int)((W + pw + 1) / 2);
  if (g.BH > P + 1 || g.BW > Q + 1) return 4;
  g.fBW = make_fdiv((uint32_t)g.BW);
  g.fBH = make_fdiv((uint32_t)g.BH);
  // blocks per workgroup: about 256 phase-1 items (one per thread) and 1024 phase-2 items.
  // Isolated at AlexNet b256 / GoogLeNet b128 (scripts/plrn_rev_probe.py, profiles/r6_lrn_pool_rev.txt):
  // 128 / 256 / 512 / 1024 items -> norm1 152.5 / 141.4 / 139.0 / 181.2 us, norm2 84.4 / 77.0 /
  // 83.5 / 106.9, GoogLeNet conv2/norm2 139.8 / 119.2 / 129.5 / 177.8 (unfused 150.1 / 89.3 / 141.1)
  g.pix = (int)max(1LL, 256 / (C / 8));
  const long long nblk = N * g.BH * g.BW;
  if (nblk >= (1ll << 31) || 4 * nblk * (C / 8) >= (1ll << 32)) return 4;
  const dim3 grid((unsigned)((nblk + g.pix - 1) / g.pix));
  const size_t lds = (size_t)g.pix * 4 * (C / 8) * sizeof(uint4);
  if (lds > 64 * 1024) return 4;
  switch (size) {
    case 3: hipLaunchKernelGGL(pool_lrn_bwd_rev<3>, grid, dim3(256), lds, st, dy, mask, x, dx, g); break;
    case 5: hipLaunchKernelGGL(pool_lrn_bwd_rev<5>, grid, dim3(256), lds, st, dy, mask, x, dx, g); break;
    case 7: hipLaunchKernelGGL(pool_lrn_bwd_rev<7>, grid, dim3(256), lds, st, dy, mask, x, dx, g); break;
    default: hipLaunchKernelGGL(pool_lrn_bwd_rev<9>, grid, dim3(256), lds, st, dy, mask, x, dx, g); break;
  }
  return SN_CHECK_LAUNCH();
}
