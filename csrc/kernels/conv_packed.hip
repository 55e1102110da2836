// Direct stride-1 / pad-0 convolution with the reduction packed across taps: CaffeNet /
// AlexNet conv1 after the space-to-depth fold (227 x 227 x 3, 11 x 11 / 4 -> 57 x 57 x 48,
// 3 x 3 / 1, 96 outputs, 55 x 55), and GoogLeNet conv1 after its fold (224 x 224 x 3, 7 x 7 / 2,
// pad 3 -> 115 x 115 x 16, 4 x 4 / 1, 64 outputs, 112 x 112) on a <4, 64> instance.
//
// The 64-channel direct kernel (conv3x3.hip, K = 96 instance) ran this product at 837 TF/s
// of issued MFMA work but only 389 TF/s of useful work (profiles/r4_step_kernels_caffenet.txt:
// 139 us per step), because three paddings multiply: 48 channels zero-filled to the 64 of a
// 128-B LDS row (x 1.33), 16 x 16 output tiles over a 55 x 55 image (x 1.35), and the fold's
// 12 x 12 kernel for an 11 x 11 one (x 1.19, inherent to the fold).  Here
//   * the reduction index is k = tap * C + c (9 x 48 = 432 = 13.5 x 32): a 32-wide MFMA K step
//     may span two taps, each lane group (lane >> 4) reading its own tap's 16-B channel chunk,
//     so 14 K steps replace 18 (a per-lane k-offset table, built once);
//   * a tile is 192 consecutive output pixels of one image in row-major order (16 tiles per
//     55 x 55 image, 1.5 % over), so the output offset is (n P Q + m) K and the input patch is the
//     7 contiguous input rows r0 .. r0 + 6 — one linear copy, stored linearly in LDS;
//   * weights sit in LDS in MFMA-fragment order (K step, N fragment, lane), 1 KB per read, and
//     the 96-B pixel rows make the 16-row A reads conflict-free under ds_read_b128's lane
//     groups because consecutive k chunks alternate in parity (MI355X_MICROARCH.md §LDS).
// LDS: 84 KB weights + 2 x 37.5 KB patches; persistent blocks (one per CU, 8 waves: wave
// (mi, ni) owns 48 pixels x 48 channels, 3 x 3 MFMA fragments), the next tile's patch in
// registers while the current tile's 126 MFMAs per wave run.  Epilogue: + bias, ReLU, bf16.
// Reference: caffe/src/caffe/layers/conv_layer.cu:8-33 (im2col + GEMM per image).
#include "common.h"

namespace {

constexpr int TP = 192;  // output pixels per tile (12 M fragments)
constexpr int NT = 512;

struct GeoP {
  int N, H, W, C;  // folded input (pad 0)
  int P, Q;        // output = H - TAPS + 1, W - TAPS + 1
  int PR;          // input rows staged per tile
  int tpi;         // tiles per image
  long long tiles;
};

// TAPS x TAPS taps, KOUT output channels, KS 32-wide K steps (covering TAPS^2 x the largest C),
// PCAP patch bytes per buffer.  Instances:
//   <3, 96, 14, 38400>: CaffeNet / AlexNet conv1 after the 4x4 fold (57 x 57 x 48 -> 55 x 55 x 96;
//                       up to 56 16-B chunks = 9 taps x 48 channels; 7 rows x 57 px x 96 B)
//   <4, 64,  8, 22528>: GoogLeNet conv1 after the 2x2 fold (115 x 115 x 16 -> 112 x 112 x 64;
//                       32 chunks = 16 taps x 16 channels; 6 rows x 115 px x 32 B)
//   <3, 64,  3, 16384>: VGG-16 conv1_1 after its fold (226 x 226 x 8 -> 224 x 224 x 64;
//                       9 chunks = 9 taps x 8 channels; 4 rows x 226 px x 16 B)
// 8 waves: wave (mi, ni) owns 48 pixels x KOUT / 2 channels (3 x KOUT / 32 MFMA fragments).
// q (optional, engine.fuse_fp8_quant): the output also stored as e4m3 with the scale of the
// (initialised) delayed-scaling slot qslot — the bytes quant_fp8 would produce from the bf16
// output — and the block's |max| into one of 256 partials 128 B apart (sn_fp8_fold_amax).
template <int TAPS, int KOUT, int KS, int PCAP>
__global__ void __launch_bounds__(NT, 1)
conv_packed_kernel(const bf16_t* __restrict__ x, const bf16_t* __restrict__ w, const float* __restrict__ bias,
                   bf16_t* __restrict__ y, GeoP g, int relu, uint8_t* __restrict__ q, const float* __restrict__ qslot,
                   float* __restrict__ qpart) {
  constexpr int NF = KOUT / 16, NFW = NF / 2;     // N fragments: all, per wave
  constexpr int W_BYTES = KS * NF * 1024;         // fragment-ordered weights
  constexpr int PER_T = (PCAP / 16 + NT - 1) / NT;
  static_assert(NF % 2 == 0 && PCAP % 16 == 0, "two N halves, whole 16-B chunks");
  __shared__ __attribute__((aligned(16))) char smem[W_BYTES + 2 * PCAP];
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int mi = wave & 3, ni = wave >> 2;
  const int CB = g.C * 2, CH = g.C >> 3, KC = TAPS * TAPS * CH;  // pixel bytes, chunks per pixel, real chunks

  // weights w[KOUT][TAPS][TAPS][C]: row n is the packed reduction k = tap * C + c; LDS chunk q =
  // ((ks * NF + nf) * 64 + lane) holds row nf * 16 + (lane & 15), chunk 4 ks + (lane >> 4)
  for (int q = tid; q < KS * NF * 64; q += NT) {
    const int ks = q / (NF * 64), rem = q - ks * (NF * 64), nf = rem >> 6, l = rem & 63;
    const int n = nf * 16 + (l & 15), kc = ks * 4 + (l >> 4);
    const uint4 v = kc < KC ? *reinterpret_cast<const uint4*>(w + (long long)n * TAPS * TAPS * g.C + kc * 8)
                            : make_uint4(0, 0, 0, 0);
    *reinterpret_cast<uint4*>(smem + q * 16) = v;
  }
  // this lane's patch offset of K step ks: tap t = kc / CH at row t / TAPS, column t % TAPS,
  // chunk kc % CH; the zero-weight tail chunks read tap 0's (finite) data
  int koff[KS];
#pragma unroll
  for (int ks = 0; ks < KS; ++ks) {
    const int kc = ks * 4 + (lane >> 4);
    const int t = kc / CH, cc = kc - t * CH, r = t / TAPS, s = t - r * TAPS;
    koff[ks] = kc < KC ? (r * g.W + s) * CB + cc * 16 : 0;
  }
  const int PQ = g.P * g.Q;

  // 16-B chunk q of tile t's patch: input rows r0 .. r0 + PR - 1 (clipped to the image)
  auto patch_src = [&](long long t, int& nch) -> const char* {
    const int n = (int)(t / g.tpi), p0 = (int)(t - (long long)n * g.tpi) * TP, r0 = p0 / g.Q;
    const int rows = min(g.PR, g.H - r0);
    nch = rows * g.W * CB / 16;
    return reinterpret_cast<const char*>(x) + (((long long)n * g.H + r0) * g.W) * CB;
  };

long long tile = blockIdx.x;
  if (tile < g.tiles) {
    int nch;
    const char* src = patch_src(tile, nch);
    for (int q = tid; q < nch; q += NT)
      *reinterpret_cast<uint4*>(smem + W_BYTES + q * 16) = *reinterpret_cast<const uint4*>(src + q * 16);
  }
  __syncthreads();

  const char* wb = smem + lane * 16 + ni * NFW * 1024;
  // this lane's 4 x NFW output channels are the same in every tile: their bias values stay in
  // registers (a per-tile global load of them stalled each epilogue on an L2 round trip)
  float bv[NFW][4];
#pragma unroll
  for (int i = 0; i < NFW; ++i)
#pragma unroll
    for (int k = 0; k < 4; ++k) bv[i][k] = bias ? bias[ni * (KOUT / 2) + i * 16 + (lane >> 4) * 4 + k] : 0.f;
  const float qsc = q ? qslot[0] : 0.f;
  float qmax = 0.f;
  int cur = 0;
  for (; tile < g.tiles; tile += gridDim.x) {
    const long long next = tile + gridDim.x;
    uint4 pre[PER_T];
    if (next < g.tiles) {
      int nch;
      const char* src = patch_src(next, nch);
#pragma unroll
      for (int i = 0; i < PER_T; ++i) {
        const int q = tid + i * NT;
        pre[i] = q < nch ? *reinterpret_cast<const uint4*>(src + q * 16) : make_uint4(0, 0, 0, 0);
      }
    }
    const int n_img = (int)(tile / g.tpi), p0 = (int)(tile - (long long)n_img * g.tpi) * TP, r0 = p0 / g.Q;
    int pixb[3];
#pragma unroll
    for (int j = 0; j < 3; ++j) {
      const int m = min(p0 + mi * 48 + j * 16 + (lane & 15), PQ - 1);  // past the image: a valid pixel, not stored
      const int oh = m / g.Q, ow = m - oh * g.Q;
      pixb[j] = ((oh - r0) * g.W + ow) * CB;
    }
    const char* p = smem + W_BYTES + cur * PCAP;
    f32x4 acc[NFW][3];
#pragma unroll
    for (int i = 0; i < NFW; ++i)
#pragma unroll
      for (int j = 0; j < 3; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};
    bf16x8_t fb[2][NFW], fa[2][3];
    auto load = [&](int ks, bf16x8_t* b, bf16x8_t* a) {
#pragma unroll
      for (int i = 0; i < NFW; ++i) b[i] = *reinterpret_cast<const bf16x8_t*>(wb + (ks * NF + i) * 1024);
#pragma unroll
      for (int j = 0; j < 3; ++j) a[j] = *reinterpret_cast<const bf16x8_t*>(p + pixb[j] + koff[ks]);
    };
    load(0, fb[0], fa[0]);
#pragma unroll
    for (int ks = 0; ks < KS; ++ks) {
      if (ks + 1 < KS) load(ks + 1, fb[(ks + 1) & 1], fa[(ks + 1) & 1]);
      __builtin_amdgcn_s_setprio(1);
#pragma unroll
      for (int i = 0; i < NFW; ++i)
#pragma unroll
        for (int j = 0; j < 3; ++j)
          acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(fb[ks & 1][i], fa[ks & 1][j], acc[i][j], 0, 0, 0);
      __builtin_amdgcn_s_setprio(0);
      // pin step ks's MFMAs before step ks + 2's reads: one step of fragments in flight
#pragma unroll
      for (int i = 0; i < NFW; ++i)
#pragma unroll
        for (int j = 0; j < 3; ++j) asm volatile("" : "+v"(acc[i][j])::"memory");
    }
    // hand the next tile's patch to LDS before this tile's stores: its loads were issued before
    // the MFMAs and have landed, while a wait placed after the stores would also wait for them
    // (vmcnt counts stores); the other buffer's last reader was tile t - 1, behind the barrier
    if (next < g.tiles) {
      char* pn = smem + W_BYTES + (cur ^ 1) * PCAP;
#pragma unroll
      for (int i = 0; i < PER_T; ++i) {
        const int q = tid + i * NT;
        if (q < PCAP / 16) *reinterpret_cast<uint4*>(pn + q * 16) = pre[i];
      }
    }
    // epilogue: lane holds output channels ch .. ch + 3 of pixel m
#pragma unroll
    for (int j = 0; j < 3; ++j) {
      const int m = p0 + mi * 48 + j * 16 + (lane & 15);
      if (m >= PQ) continue;
      bf16_t* yo = y + ((long long)n_img * PQ + m) * KOUT;
#pragma unroll
      for (int i = 0; i < NFW; ++i) {
        const int ch = ni * (KOUT / 2) + i * 16 + (lane >> 4) * 4;
        float v[4] = {acc[i][j][0], acc[i][j][1], acc[i][j][2], acc[i][j][3]};
        if (bias) {
#pragma unroll
          for (int k = 0; k < 4; ++k) v[k] += bv[i][k];
        }
        if (relu) {
#pragma unroll
          for (int k = 0; k < 4; ++k) v[k] = fmaxf(v[k], 0.f);
        }
        *reinterpret_cast<uint2*>(yo + ch) = make_uint2(pack2(v[0], v[1]), pack2(v[2], v[3]));
        if (q) {
          float f[4];
#pragma unroll
          for (int k = 0; k < 4; ++k) {
            const float b = bf2f(f2bf(v[k]));  // the stored bf16 value
            qmax = fmaxf(qmax, fabsf(b));
            f[k] = fminf(fmaxf(b * qsc, -448.f), 448.f);
          }
          int wq = 0;
          wq = __builtin_amdgcn_cvt_pk_fp8_f32(f[0], f[1], wq, false);
          wq = __builtin_amdgcn_cvt_pk_fp8_f32(f[2], f[3], wq, true);
          *reinterpret_cast<uint32_t*>(q + ((long long)n_img * PQ + m) * KOUT + ch) = (uint32_t)wq;
        }
      }
    }
    __syncthreads();  // next patch in LDS, and every wave is done reading this one
    cur ^= 1;
  }
  if (q) {  // block |max| -> partial (every thread reaches this: the tile loop has no early exit)
    __shared__ float red[NT / 64];
    qmax = wave_max(qmax);
    if (lane == 0) red[wave] = qmax;
    __syncthreads();
    if (tid == 0) {
      float m = 0.f;
#pragma unroll
      for (int i = 0; i < NT / 64; ++i) m = fmaxf(m, red[i]);
      if (m > 0.f) atomicMax(reinterpret_cast<unsigned int*>(qpart + (blockIdx.x & 255) * 32), __float_as_uint(m));
    }
  }
}

template <int TAPS, int KOUT, int KS, int PCAP>
int launch_packed(const bf16_t* x, const bf16_t* w, const float* bias, bf16_t* y, long long N, long long H,
                  long long W, long long C, long long K, long long relu, hipStream_t st, uint8_t* q = nullptr,
                  const float* qslot = nullptr, float* qpart = nullptr) {
  if (q && !(qslot && qpart)) return 9;
  if (N <= 0 || H <= 0 || W <= 0) return 0;
  if (K != KOUT || C <= 0 || C % 8 || (long long)TAPS * TAPS * (C / 8) > 4LL * KS || H < TAPS || W < TAPS ||
      W > 4096)
    return 3;
  GeoP g;
  g.N = (int)N; g.H = (int)H; g.W = (int)W; g.C = (int)C;
  g.P = g.H - TAPS + 1; g.Q = g.W - TAPS + 1;
  // output rows a run of TP pixels can touch, + the TAPS - 1 extra input rows of the window
  g.PR = (TP - 1 + g.Q - 1) / g.Q + 1 + (TAPS - 1);
  if (g.PR > g.H) g.PR = g.H;
  if ((long long)g.PR * g.W * g.C * 2 > PCAP) return 3;
  if ((long long)g.P * g.Q >= (1LL << 31) / KOUT) return 3;
  g.tpi = (g.P * g.Q + TP - 1) / TP;
  g.tiles = N * g.tpi;
  const int cus = sn_cu_count();
  const long long grid = g.tiles < cus ? g.tiles : cus;  // persistent: one block per CU
  hipLaunchKernelGGL((conv_packed_kernel<TAPS, KOUT, KS, PCAP>), dim3((unsigned)grid), dim3(NT), 0, st, x, w, bias, y,
                     g, (int)relu, q, qslot, qpart);
  return SN_CHECK_LAUNCH();
}

}  // namespace

// y[N][H-2][W-2][96] = conv3x3(x[N][H][W][C], w[96][3][3][C]) (+ bias, ReLU), stride 1, pad 0;
// C a multiple of 8, at most 48.  Returns 3 for shapes outside the kernel.
extern "C" int sn_conv_packed3x3(const bf16_t* x, const bf16_t* w, const float* bias, bf16_t* y, long long N,
                                 long long H, long long W, long long C, long long K, long long relu, hipStream_t st) {
  return launch_packed<3, 96, 14, 38400>(x, w, bias, y, N, H, W, C, K, relu, st);
}

// y[N][H-3][W-3][64] = conv4x4(x[N][H][W][C], w[64][4][4][C]) (+ bias, ReLU), stride 1, pad 0;
// C a multiple of 8, at most 16 (GoogLeNet conv1 after the 2x2 space-to-depth fold).
// <1, 64, 2, 36864>: a 1x1 convolution with <= 64 input and 64 output channels (GoogLeNet's
// conv2/3x3_reduce, 56 x 56 x 64 -> 64: 5 input rows x 56 px x 128 B per 192-pixel tile) —
// the implicit GEMM runs it as one K step per 128-row tile
extern "C" int sn_conv_packed1x1(const bf16_t* x, const bf16_t* w, const float* bias, bf16_t* y, long long N,
                                 long long H, long long W, long long C, long long K, long long relu, hipStream_t st) {
  return launch_packed<1, 64, 2, 36864>(x, w, bias, y, N, H, W, C, K, relu, st);
}

// <3, 64, 3, 16384>: y[N][H-2][W-2][64] = conv3x3(x[N][H][W][8], w[64][3][3][8]), stride 1, pad 0 —
// VGG-16 conv1_1 (224 x 224 x 3, 3x3 pad 1) after its fold (the pad baked in, channels padded to
// 8: 226 x 226 x 8): 9 taps x one 16-B chunk = 3 K steps (the implicit GEMM ran its 72-deep
// reduction as two 64-deep steps of 128-row tiles, one output write per 16 KB tile, 84 TF/s)
// q / qslot / qpart: the e4m3 side output of conv1_2's input under --dtype fp8 (null: none)
extern "C" int sn_conv_packed3x3k64(const bf16_t* x, const bf16_t* w, const float* bias, bf16_t* y, long long N,
                                    long long H, long long W, long long C, long long K, long long relu,
                                    uint8_t* q, const float* qslot, float* qpart, hipStream_t st) {
  return launch_packed<3, 64, 3, 16384>(x, w, bias, y, N, H, W, C, K, relu, st, q, qslot, qpart);
}

extern "C" int sn_conv_packed4x4(const bf16_t* x, const bf16_t* w, const float* bias, bf16_t* y, long long N,
                                 long long H, long long W, long long C, long long K, long long relu, hipStream_t st) {
  return launch_packed<4, 64, 8, 22528>(x, w, bias, y, N, H, W, C, K, relu, st);
}
