// Direct 3x3 / stride-1 / pad-1 convolution, 64 -> 64 channels, on e4m3 operands (VGG-16
// conv1_2 forward and data gradient under --dtype fp8).
//
// The bf16 kernel (conv3x3.hip) keeps the weights resident in LDS and stages one input patch
// per 16 x 16 output tile; on the implicit-GEMM path these 64-channel products would run an
// fp8 tile with half its columns idle (the cost model keeps them bf16, engine.enable_fp8).
// Here the same persistent structure runs v_mfma_scale_f32_16x16x128_f8f6f4: one MFMA
// reduces TWO taps x 64 channels (k = 32 g + j: taps 2p / 2p+1 for lane groups g < 2 / >= 2,
// channels 32 (g & 1) + j), so the 9 taps are five tap pairs (the last pair's second tap is
// zero: an all-zero tenth weight tap, read with tap 8's patch rows).  LDS: weights 10 taps x
// 64 x 64 B = 40 KB, double-buffered 18 x 18-pixel patches
// 2 x 25.3 KB; rows padded to 80 B, so 16 consecutive rows fall in distinct banks and every
// fragment read is one per-lane base + an immediate offset.  fp32 accumulation, epilogue: dequantise
// (the two per-tensor factors), + bias, ReLU, ReLU-backward gate, bf16 NHWC store.
// Reference: caffe/src/caffe/layers/conv_layer.cu:8-56 (im2col + SGEMM per image).
#include "common.h"

namespace {

constexpr int TILE = 16, PATCH = TILE + 2, PROWS = PATCH * PATCH;  // 324 patch pixels
constexpr int ROWB = 80;  // 64 e4m3 channels + 16 B pad: 16 consecutive rows -> 16 distinct banks
constexpr int W_BYTES = 10 * 64 * ROWB, P_BYTES = PROWS * ROWB;    // 51200 (9 taps + a zero tap), 25920
constexpr int CHUNKS = PROWS * 4;                                  // 16-B patch chunks

typedef __attribute__((ext_vector_type(8))) int i32x8_t;

SN_DEV int off64(int row, int c) { return row * ROWB + (c << 4); }

// 32 bytes at lds + o (two ds_read_b128; o = the lane's row and half + an immediate offset)
SN_DEV i32x8_t read32(const char* lds, int o) {
  const uint4 a = *reinterpret_cast<const uint4*>(lds + o);
  const uint4 b = *reinterpret_cast<const uint4*>(lds + o + 16);
  return i32x8_t{(int)a.x, (int)a.y, (int)a.z, (int)a.w, (int)b.x, (int)b.y, (int)b.z, (int)b.w};
}

struct Geo8 {
  int N, H, W;  // input (= output: stride 1, pad 1)
  int th, tw;   // output tiles per image
  long long tiles;
};

SN_DEV void tile_coords8(const Geo8& g, long long t, int& n, int& ty, int& tx) {
  const int per_img = g.th * g.tw;
  n = (int)(t / per_img);
  const int r = (int)(t - (long long)n * per_img);
  ty = r / g.tw;
  tx = r - ty * g.tw;
}

SN_DEV uint4 patch_load8(const uint8_t* __restrict__ x, const Geo8& g, long long t, int q) {
  const int pix = q >> 2, c = q & 3;
  int n, ty, tx;
  tile_coords8(g, t, n, ty, tx);
  const int py = pix / PATCH, px = pix - py * PATCH;
  const int h = ty * TILE - 1 + py, w = tx * TILE - 1 + px;
  if ((unsigned)h >= (unsigned)g.H || (unsigned)w >= (unsigned)g.W) return make_uint4(0, 0, 0, 0);
  return *reinterpret_cast<const uint4*>(x + (((long long)n * g.H + h) * g.W + w) * 64 + c * 16);
}

// 8 waves: wave (mi = w & 3, ni = w >> 2) owns output rows 4 mi .. 4 mi + 3 (four 16-pixel M
// fragments) x output channels 32 ni .. 32 ni + 31 (two N fragments).
template <bool GATE>
__global__ void __launch_bounds__(512, 1)
conv3x3_fp8_kernel(const uint8_t* __restrict__ x, const uint8_t* __restrict__ w, const float* __restrict__ deq_x,
                   const float* __restrict__ deq_w, const float* __restrict__ bias, const bf16_t* __restrict__ gate,
                   bf16_t* __restrict__ y, Geo8 g, int relu) {
  constexpr int NT = 512, PER_T = (CHUNKS + NT - 1) / NT;
  __shared__ __attribute__((aligned(16))) char smem[W_BYTES + 2 * P_BYTES];
  char* wl = smem;
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int mi = wave & 3, n0w = (wave >> 2) * 32;
  const int gq = lane >> 4, li = lane & 15, hsel = gq & 1, tsel = gq >> 1;

  // resident weights w[64][3][3][64] (e4m3): row = tap * 64 + output channel; tap 9 = zeros
  for (int q = tid; q < 10 * 64 * 4; q += NT) {
    const int t = q >> 8, rem = q & 255, n = rem >> 2, c = rem & 3;
    const uint4 v = t < 9 ? *reinterpret_cast<const uint4*>(w + ((long long)n * 9 + t) * 64 + c * 16)
                          : make_uint4(0, 0, 0, 0);
    *reinterpret_cast<uint4*>(wl + off64(t * 64 + n, c)) = v;
  }
  long long tile = blockIdx.x;
  if (tile < g.tiles) {
    for (int i = 0; i < PER_T; ++i) {
      const int q = tid + i * NT;
      if (q < CHUNKS) *reinterpret_cast<uint4*>(smem + W_BYTES + off64(q >> 2, q & 3)) = patch_load8(x, g, tile, q);
    }
  }
  __syncthreads();
  const float dq = deq_x[0] * deq_w[0];

  int cur = 0;
  const int mrow = lane & 15, ncol = (lane >> 4) * 4;
  // this lane's output channels are the same in every tile: bias values stay in registers (a
  // per-tile global load of them stalled each epilogue on an L2 round trip)
  float bv[2][4];
#pragma unroll
  for (int i = 0; i < 2; ++i)
#pragma unroll
    for (int k = 0; k < 4; ++k) bv[i][k] = bias ? bias[n0w + 16 * i + ncol + k] : 0.f;
  for (; tile < g.tiles; tile += gridDim.x) {
    const long long next = tile + gridDim.x;
    uint4 pre[PER_T];
    if (next < g.tiles) {
#pragma unroll
      for (int i = 0; i < PER_T; ++i) {
        const int q = tid + i * NT;
        pre[i] = q < CHUNKS ? patch_load8(x, g, next, q) : make_uint4(0, 0, 0, 0);
      }
    }
    int n_img, ty, tx;
    tile_coords8(g, tile, n_img, ty, tx);
    // data gradient: this tile's ReLU-backward gate, loaded before the MFMAs so the epilogue
    // does not wait on it
    uint2 gpf[4][GATE ? 2 : 1];
#pragma unroll
    for (int j = 0; j < 4; ++j)
#pragma unroll
      for (int i = 0; i < (GATE ? 2 : 1); ++i) {
        const int h = ty * TILE + 4 * mi + j, wc = tx * TILE + mrow;
        gpf[j][i] = make_uint2(0u, 0u);
        if (GATE && h < g.H && wc < g.W)
          gpf[j][i] = *reinterpret_cast<const uint2*>(
              gate + (((long long)n_img * g.H + h) * g.W + wc) * 64 + n0w + 16 * i + ncol);
      }
    f32x4 acc[2][4];
#pragma unroll
    for (int i = 0; i < 2; ++i)
#pragma unroll
      for (int j = 0; j < 4; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};
    const char* p = smem + W_BYTES + cur * P_BYTES;
    // tap pair pp + 1's fragments load while pair pp's eight MFMAs run
    i32x8_t fb[2][2], fa[2][4];
    auto load = [&](int pp, i32x8_t* b, i32x8_t* a) {
      const int t = 2 * pp + tsel, ta = t < 9 ? t : 8;  // tap 9: zero weights x tap 8's rows
      const int r = ta / 3, s = ta - r * 3;
      const int ob = (t * 64 + n0w + li) * ROWB + hsel * 32, oa = ((4 * mi + r) * PATCH + s + li) * ROWB + hsel * 32;
#pragma unroll
      for (int i = 0; i < 2; ++i) b[i] = read32(wl, ob + 16 * i * ROWB);
#pragma unroll
      for (int j = 0; j < 4; ++j) a[j] = read32(p, oa + j * PATCH * ROWB);
    };
    load(0, fb[0], fa[0]);
#pragma unroll
    for (int pp = 0; pp < 5; ++pp) {
      if (pp < 4) load(pp + 1, fb[(pp + 1) & 1], fa[(pp + 1) & 1]);
      __builtin_amdgcn_s_setprio(1);
#pragma unroll
      for (int i = 0; i < 2; ++i)
#pragma unroll
        for (int j = 0; j < 4; ++j)
          acc[i][j] = __builtin_amdgcn_mfma_scale_f32_16x16x128_f8f6f4(fb[pp & 1][i], fa[pp & 1][j], acc[i][j], 0, 0,
                                                                        0, 127, 0, 127);
      __builtin_amdgcn_s_setprio(0);
      // pin pair pp's MFMAs before pair pp + 2's loads: one pair of fragments in flight, not five
#pragma unroll
      for (int i = 0; i < 2; ++i)
#pragma unroll
        for (int j = 0; j < 4; ++j) asm volatile("" : "+v"(acc[i][j])::"memory");
    }
    // hand the next tile's patch to LDS before this tile's stores (its loads have landed; a
    // wait after the stores would also wait for them); the other buffer's last reader was tile
    // t - 1, behind the barrier
    if (next < g.tiles) {
      char* pn = smem + W_BYTES + (cur ^ 1) * P_BYTES;
#pragma unroll
      for (int i = 0; i < PER_T; ++i) {
        const int q = tid + i * NT;
        if (q < CHUNKS) *reinterpret_cast<uint4*>(pn + off64(q >> 2, q & 3)) = pre[i];
      }
    }
    // epilogue: lane holds output channels n .. n+3 of pixel (4 mi + j, mrow)
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      const int h = ty * TILE + 4 * mi + j, wc = tx * TILE + mrow;
      if (h >= g.H || wc >= g.W) continue;
      const long long o = (((long long)n_img * g.H + h) * g.W + wc) * 64;
#pragma unroll
      for (int i = 0; i < 2; ++i) {
        const int n = n0w + 16 * i + ncol;
        float v[4] = {acc[i][j][0] * dq, acc[i][j][1] * dq, acc[i][j][2] * dq, acc[i][j][3] * dq};
        if (bias) {
#pragma unroll
          for (int k = 0; k < 4; ++k) v[k] += bv[i][k];
        }
        if (relu) {
#pragma unroll
          for (int k = 0; k < 4; ++k) v[k] = fmaxf(v[k], 0.f);
        }
        if (GATE) {
          const uint2 gv = gpf[j][GATE ? i : 0];
          const uint32_t gw[2] = {gv.x, gv.y};
#pragma unroll
          for (int k = 0; k < 4; ++k) {
            const float gf = __uint_as_float((k & 1) ? (gw[k >> 1] & 0xffff0000u) : (gw[k >> 1] << 16));
            if (!(gf > 0.f)) v[k] = 0.f;
          }
        }
        *reinterpret_cast<uint2*>(y + o + n) = make_uint2(pack2(v[0], v[1]), pack2(v[2], v[3]));
      }
    }
    __syncthreads();  // next patch in LDS, and every wave is done reading this one
    cur ^= 1;
  }
}

}  // namespace

// y[N][H][W][64] (bf16) = deq_x * deq_w * conv3x3(x[N][H][W][64] e4m3, w[64][3][3][64] e4m3)
// (+ bias, ReLU, gate), stride 1, pad 1 — a forward conv, or a data gradient with the flip-
// transposed weights.
extern "C" int sn_conv3x3_fp8(const uint8_t* x, const uint8_t* w, const float* deq_x, const float* deq_w,
                              const float* bias, const bf16_t* gate, bf16_t* y, long long N, long long H, long long W,
                              long long relu, hipStream_t st) {
  if (N <= 0 || H <= 0 || W <= 0) return 0;
  if (!deq_x || !deq_w) return 3;
  if ((reinterpret_cast<uintptr_t>(x) | reinterpret_cast<uintptr_t>(w)) & 15) return 3;
  Geo8 g;
  g.N = (int)N; g.H = (int)H; g.W = (int)W;
  g.th = (g.H + TILE - 1) / TILE;
  g.tw = (g.W + TILE - 1) / TILE;
  g.tiles = N * g.th * g.tw;
  const int cus = sn_cu_count();
  const long long grid = g.tiles < cus ? g.tiles : cus;  // persistent: one block per CU
  if (gate)
    hipLaunchKernelGGL(conv3x3_fp8_kernel<true>, dim3((unsigned)grid), dim3(512), 0, st, x, w, deq_x, deq_w, bias, gate, y, g,
                     (int)relu);
  else
    hipLaunchKernelGGL(conv3x3_fp8_kernel<false>, dim3((unsigned)grid), dim3(512), 0, st, x, w, deq_x, deq_w, bias, gate, y, g,
                     (int)relu);
  return SN_CHECK_LAUNCH();
}
