// Direct 3x3 / stride-1 / pad-1 convolution for 64 input and 64 output channels (VGG-16's
// conv1_2 forward and data gradient: 64 % of VGG's bf16 conv time outside the fp8 products
// went to these two thin products on the implicit-GEMM path).
//
// Why a separate kernel: the implicit GEMM stages every tap of its A operand from L2 (a
// 256 x 64 tile reads 256 x 576 x 2 B = 295 KB of im2col rows for 9.4 M MACs, the input
// pixels 9x over), and with only 64 output columns per A byte that L2 -> LDS stream, not the
// MFMA pipe, sets the speed.  Here a block keeps the whole weight tensor (9 taps x 64 x 64
// bf16 = 72 KB) resident in LDS, stages one 18 x 18-pixel input patch (41 KB, 1/7 of the
// implicit-GEMM bytes) per 16 x 16-pixel output tile and reads the 9 tap-shifted A fragments
// straight out of the patch.  Blocks are persistent (one per CU, 153 KB of LDS) and
// double-buffer the patch: the next tile's global loads are in flight in registers while the
// current tile's 288 MFMAs per wave run.
//
// Same XOR-swizzled 128-B-row LDS images as the GEMM engine (a row = one pixel's 64 channels
// or one output channel's 64 weights), v_mfma_f32_16x16x32_bf16 with fp32 accumulation,
// epilogue: + bias, ReLU, ReLU-backward gate (dgrad), bf16 NHWC store.
#include "common.h"

#include <cstdlib>

namespace {

constexpr int TILE = 16, PATCH = TILE + 2, PROWS = PATCH * PATCH;  // 324 patch pixels
constexpr int ROWB = 128;                                           // 64 bf16 channels
constexpr int W_BYTES = 9 * 64 * ROWB, P_BYTES = PROWS * ROWB;      // 73728, 41472
constexpr int CHUNKS = PROWS * 8;                                   // 16-B patch chunks

SN_DEV int kc_off(int row, int kc) { return row * ROWB + ((kc ^ ((row >> 1) & 7)) << 4); }

SN_DEV bf16x8_t frag(const char* lds, int row0, int ks, int lane) {
  const uint4 v = *reinterpret_cast<const uint4*>(lds + kc_off(row0 + (lane & 15), ks * 4 + (lane >> 4)));
  return __builtin_bit_cast(bf16x8_t, v);
}

struct Geo {
  int N, H, W;   // input
  int P, Q;      // output (P = H + 2 pad - 2)
  int C, pad;    // input channels (<= 64, multiple of 8: stored as 128-B rows, zero-filled), padding
  int th, tw;    // output tiles per image
  int ldy;       // output pixel stride in elements (K, or wider: a channel slice of a K-wide output)
  long long tiles;
};

SN_DEV void tile_coords(const Geo& g, long long t, int& n, int& ty, int& tx) {
  const int per_img = g.th * g.tw;
  n = (int)(t / per_img);
  const int r = (int)(t - (long long)n * per_img);
  ty = r / g.tw;
  tx = r - ty * g.tw;
}

// 16-B chunk q (pixel q / 8, channel chunk q % 8) of tile t's input patch; zeros outside the
// image and beyond the C input channels
SN_DEV uint4 patch_load(const bf16_t* __restrict__ x, const Geo& g, long long t, int q) {
  const int pix = q >> 3, kc = q & 7;
  int n, ty, tx;
  tile_coords(g, t, n, ty, tx);
  const int py = pix / PATCH, px = pix - py * PATCH;
  const int h = ty * TILE - g.pad + py, w = tx * TILE - g.pad + px;
  if ((unsigned)h >= (unsigned)g.H || (unsigned)w >= (unsigned)g.W || kc * 8 >= g.C) return make_uint4(0, 0, 0, 0);
  return *reinterpret_cast<const uint4*>(x + (((long long)n * g.H + h) * g.W + w) * g.C + kc * 8);
}

// NW = 4: wave w owns output rows 4w..4w+3 x all KOUT channels; NW = 8: wave (mi, ni) owns rows
// 4mi..4mi+3 x channels ni*KOUT/2 .. (two waves per SIMD to hide the LDS read latency).
// DBUF: double-buffered patch (KOUT = 64); KOUT = 96 weights (108 KB) leave room for one
// patch, written after a barrier while the next tile's loads wait in registers.
template <int NW, int KOUT, bool DBUF, bool GATE>
__global__ void __launch_bounds__(NW * 64, 1)
conv3x3_kernel(const bf16_t* __restrict__ x, const bf16_t* __restrict__ w, const float* __restrict__ bias,
               const bf16_t* __restrict__ gate, bf16_t* __restrict__ y, Geo g, int relu) {
  constexpr int NT = NW * 64, PER_T = (CHUNKS + NT - 1) / NT;
  constexpr int NF = (NW == 4 ? KOUT : KOUT / 2) / 16;  // N fragments per wave
  constexpr int WB = 9 * KOUT * ROWB;
  __shared__ __attribute__((aligned(16))) char smem[WB + (DBUF ? 2 : 1) * P_BYTES];
  char* wl = smem;
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int mi = NW == 4 ? wave : (wave & 3), n0w = NW == 4 ? 0 : (wave >> 2) * (KOUT / 2);

  // resident weights w[KOUT][3][3][C]: tap t image, row = output channel n, chunk = 8 inputs
  for (int q = tid; q < 9 * KOUT * 8; q += NT) {
    const int t = q / (KOUT * 8), rem = q - t * (KOUT * 8), n = rem >> 3, kc = rem & 7;
    const uint4 v = kc * 8 < g.C ? *reinterpret_cast<const uint4*>(w + ((long long)n * 9 + t) * g.C + kc * 8)
                                 : make_uint4(0, 0, 0, 0);
    *reinterpret_cast<uint4*>(wl + t * KOUT * ROWB + kc_off(n, kc)) = v;
  }
  long long tile = blockIdx.x;
  if (tile < g.tiles) {
    for (int i = 0; i < PER_T; ++i) {
      const int q = tid + i * NT;
      if (q < CHUNKS) *reinterpret_cast<uint4*>(smem + WB + kc_off(q >> 3, q & 7)) = patch_load(x, g, tile, q);
    }
  }
  __syncthreads();

  int cur = 0;
  const int mrow = lane & 15, ncol = (lane >> 4) * 4;
  // this lane's output channels are the same in every tile: bias values stay in registers (a
  // per-tile global load of them stalled each epilogue on an L2 round trip)
  float bv[NF][4];
#pragma unroll
  for (int i = 0; i < NF; ++i)
#pragma unroll
    for (int k = 0; k < 4; ++k) bv[i][k] = bias ? bias[n0w + 16 * i + ncol + k] : 0.f;
  for (; tile < g.tiles; tile += gridDim.x) {
    const long long next = tile + gridDim.x;
    uint4 pre[PER_T];
    if (next < g.tiles) {
#pragma unroll
      for (int i = 0; i < PER_T; ++i) {
        const int q = tid + i * NT;
        pre[i] = q < CHUNKS ? patch_load(x, g, next, q) : make_uint4(0, 0, 0, 0);
      }
    }
    int n_img, ty, tx;
    tile_coords(g, tile, n_img, ty, tx);
    // data gradient: this tile's ReLU-backward gate, loaded before the MFMAs so the epilogue
    // does not wait on it
    uint2 gpf[4][GATE ? NF : 1];
#pragma unroll
    for (int j = 0; j < 4; ++j)
#pragma unroll
      for (int i = 0; i < (GATE ? NF : 1); ++i) {
        const int h = ty * TILE + 4 * mi + j, wc = tx * TILE + mrow;
        gpf[j][i] = make_uint2(0u, 0u);
        if (GATE && h < g.P && wc < g.Q)
          gpf[j][i] = *reinterpret_cast<const uint2*>(
              gate + (((long long)n_img * g.P + h) * g.Q + wc) * KOUT + n0w + 16 * i + ncol);
      }
    f32x4 acc[NF][4];
#pragma unroll
    for (int i = 0; i < NF; ++i)
#pragma unroll
      for (int j = 0; j < 4; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};
    const char* p = smem + WB + cur * P_BYTES;
#pragma unroll
    for (int t = 0; t < 9; ++t) {
      const int r = t / 3, s = t - r * 3;
      const char* wt = wl + t * KOUT * ROWB;
#pragma unroll
      for (int ks = 0; ks < 2; ++ks) {
        bf16x8_t fb[NF], fa[4];
#pragma unroll
        for (int i = 0; i < NF; ++i) fb[i] = frag(wt, n0w + 16 * i, ks, lane);
#pragma unroll
        for (int j = 0; j < 4; ++j) fa[j] = frag(p, (4 * mi + j + r) * PATCH + s, ks, lane);
        __builtin_amdgcn_s_setprio(1);
#pragma unroll
        for (int i = 0; i < NF; ++i)
#pragma unroll
          for (int j = 0; j < 4; ++j) acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(fb[i], fa[j], acc[i][j], 0, 0, 0);
        __builtin_amdgcn_s_setprio(0);
      }
    }
    // DBUF: hand the next tile's patch to LDS before this tile's stores (its loads have landed;
    // a wait after the stores would also wait for them); the other buffer's last reader was
    // tile t - 1, behind the barrier
    if (DBUF && next < g.tiles) {
      char* pn = smem + WB + (cur ^ 1) * P_BYTES;
#pragma unroll
      for (int i = 0; i < PER_T; ++i) {
        const int q = tid + i * NT;
        if (q < CHUNKS) *reinterpret_cast<uint4*>(pn + kc_off(q >> 3, q & 7)) = pre[i];
      }
    }
    // epilogue: lane holds output channels n .. n+3 of pixel (4 mi + j, mrow)
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      const int h = ty * TILE + 4 * mi + j, wc = tx * TILE + mrow;
      if (h >= g.P || wc >= g.Q) continue;
      const long long o = (((long long)n_img * g.P + h) * g.Q + wc) * g.ldy;
#pragma unroll
      for (int i = 0; i < NF; ++i) {
        const int n = n0w + 16 * i + ncol;
        float v[4] = {acc[i][j][0], acc[i][j][1], acc[i][j][2], acc[i][j][3]};
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
    if (!DBUF) {
      __syncthreads();  // single patch buffer: every wave is done reading it
      if (next < g.tiles) {
        char* pn = smem + WB;
#pragma unroll
        for (int i = 0; i < PER_T; ++i) {
          const int q = tid + i * NT;
          if (q < CHUNKS) *reinterpret_cast<uint4*>(pn + kc_off(q >> 3, q & 7)) = pre[i];
        }
      }
    }
    __syncthreads();  // next patch in LDS (DBUF: and every wave is done reading this one)
    if (DBUF) cur ^= 1;
  }
}

}  // namespace

// y[N][P][Q][K] = conv3x3(x[N][H][W][C], w[K][3][3][C]) (+ bias, ReLU, gate), stride 1, pad
// 0 or 1 (P = H + 2 pad - 2) — a forward conv, or a data gradient with flip-transposed
// weights.  K = 64 (VGG-16 conv1_2: C = 64, pad 1) or 96 (CaffeNet / AlexNet conv1 after the
// space-to-depth fold: C = 48, pad 0); C <= 64, multiple of 8.
// ldy: pixel stride of y in elements (0 = K): GoogLeNet's conv2/3x3 (64 -> 192) runs as two
// 96-output launches into the channel halves of one 192-wide output (64.6 us each vs 155 us for
// the implicit GEMM, scripts/direct96_probe.py).  A gated launch (data gradient) keeps ldy = K.
extern "C" int sn_conv3x3_direct(const bf16_t* x, const bf16_t* w, const float* bias, const bf16_t* gate, bf16_t* y,
                                 long long N, long long H, long long W, long long C, long long K, long long pad,
                                 long long relu, long long ldy, hipStream_t st) {
  if (N <= 0 || H <= 0 || W <= 0) return 0;
  if (C <= 0 || C > 64 || C % 8 || (K != 64 && K != 96) || (pad != 0 && pad != 1)) return 3;
  if (ldy == 0) ldy = K;
  if (ldy < K || ldy % 4 || (gate && ldy != K)) return 3;
  Geo g;
  g.N = (int)N; g.H = (int)H; g.W = (int)W; g.C = (int)C; g.pad = (int)pad;
  g.ldy = (int)ldy;
  g.P = (int)(H + 2 * pad - 2);
  g.Q = (int)(W + 2 * pad - 2);
  if (g.P <= 0 || g.Q <= 0) return 3;
  g.th = (g.P + TILE - 1) / TILE;
  g.tw = (g.Q + TILE - 1) / TILE;
  g.tiles = N * g.th * g.tw;
  const int cus = sn_cu_count();
  const long long grid = g.tiles < cus ? g.tiles : cus;  // persistent: one block per CU
  const int nw = 8;  // 8 waves (2 per SIMD) beat 4 (docs/PERF_NOTES.md round 3)
#define SN_C3(NWV, KV, DB, NTH)                                                                             \
  do {                                                                                                     \
    if (gate)                                                                                              \
      hipLaunchKernelGGL((conv3x3_kernel<NWV, KV, DB, true>), dim3((unsigned)grid), dim3(NTH), 0, st, x, w, bias, \
                         gate, y, g, (int)relu);                                                           \
    else                                                                                                   \
      hipLaunchKernelGGL((conv3x3_kernel<NWV, KV, DB, false>), dim3((unsigned)grid), dim3(NTH), 0, st, x, w, bias, \
                         gate, y, g, (int)relu);                                                           \
  } while (0)
  if (K == 96)
    SN_C3(8, 96, false, 512);
  else if (nw == 4)
    SN_C3(4, 64, true, 256);
  else
    SN_C3(8, 64, true, 512);
#undef SN_C3
  return SN_CHECK_LAUNCH();
}
