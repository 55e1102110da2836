// MFMA GEMM for gfx950 — the single matrix engine behind Convolution (fwd / dgrad /
// wgrad, implicit-GEMM over NHWC activations), InnerProduct and Deconvolution.
//
// Replaces the reference's per-image im2col + cublasSgemm loop
// (caffe/src/caffe/layers/conv_layer.cu:14-21, base_conv_layer.cpp:312-376,
//  inner_product_layer.cu:22-54, math_functions.cu:14-28) with ONE launch per layer
// over the whole batch.
//
//   C_g[m][n] (op)= sum_k A_g(m, k) * B_g(n, k)          g = group, split-K over k
//
// Operands are bf16, accumulation is fp32 on v_mfma_f32_16x16x32_bf16.  Each operand
// is a "virtual row-major matrix" that is either
//   KC : [rows = M (or N)] x [cols = K]   (reduction dim contiguous)  -> ds_read_b128
//   MC : [rows = K] x [cols = M (or N)]   (reduction dim strided)     -> ds_read_b64_tr_b16
// so NT / NN / TN products all stage their tiles straight from global memory without a
// transpose pass: the transposition happens in the LDS read (CDNA4 tr_b16).
// A virtual matrix is DENSE (ptr + row*ld + col), IM2COL (the implicit [N*P*Q pixels] x
// [R*S*Cg] patch matrix of an NHWC tensor, gathered on the fly with zero-fill for
// padding — no column buffer in HBM) or FLIPW (conv weights read flipped / transposed
// for the data gradient).
//
// Block tile BM x BN x 64 with 256 threads = 4 waves, each wave owning a 64x64 output
// sub-tile (4x4 MFMA tiles): (BM, BN) = (128, 128) or (256, 64) for skinny N (e.g.
// 48-channel grouped dgrad).  Tiles are staged by LDS-DMA (global_load_lds_dwordx4) into
// two LDS stages held in two distinct __shared__ objects, XOR-swizzled on the source
// side so both the b128 row reads and the tr_b16 transposed reads are bank-conflict
// free; the DMA of tile k+1 runs under the MFMAs of tile k; XCD-aware bijective block
// remap; fused bias / ReLU / ReLU-backward-gate epilogue; deterministic split-K.
#include "gemm_impl.h"

namespace {

// 128x96 tile (waves own 64x48): output widths that are multiples of 96 (AlexNet conv1's
// 96 filters, conv4's 192 per group) without the 25 % dead columns of a 128-wide tile.
// The 96-row B image has 12-chunk MC rows, so only K-contiguous (KC) B operands.
int launch_tile96(const SnGemmArgs& a, hipStream_t stream) {
  const int tiles = ((a.M + 127) / 128) * ((a.N + 95) / 96);
  dim3 grid(tiles * a.splits * a.groups);
  if (a.b_mc || a.b_mode != OP_DENSE) return 4;
  if (a.a_mc == 0 && a.a_mode == OP_IM2COL) return launch_epi<0, OP_IM2COL, 0, OP_DENSE, 128, 96, 4, 2, 3>(a, grid, stream);
  if (a.a_mc == 0 && a.a_mode == OP_DENSE) return launch_epi<0, OP_DENSE, 0, OP_DENSE, 128, 96, 4, 2, 3>(a, grid, stream);
  if (a.a_mc == 1 && a.a_mode == OP_DENSE) return launch_epi<1, OP_DENSE, 0, OP_DENSE, 128, 96, 4, 2, 3>(a, grid, stream);
  return 4;
}

// 256x48 tile (4 waves of 64x48; B staged as 64 rows): 48-wide outputs such as AlexNet
// conv2's dgrad (48 input channels per group) without a quarter of dead MFMA columns.
template <int NS_ = 2>
int launch_tile48(const SnGemmArgs& a, hipStream_t stream) {
  const int tiles = ((a.M + 255) / 256) * ((a.N + 47) / 48);
  dim3 grid(tiles * a.splits * a.groups);
  const int key = (a.a_mc << 3) | (a.a_mode << 2) | (a.b_mc << 1) | a.b_mode;
  switch (key) {
    case 0b0000: return launch_epi<0, OP_DENSE, 0, OP_DENSE, 256, 48, 4, NS_, 3>(a, grid, stream);
    case 0b0100: return launch_epi<0, OP_IM2COL, 0, OP_DENSE, 256, 48, 4, NS_, 3>(a, grid, stream);
    case 0b0010: return launch_epi<0, OP_DENSE, 1, OP_DENSE, 256, 48, 4, NS_, 3>(a, grid, stream);
    case 0b1010: return launch_epi<1, OP_DENSE, 1, OP_DENSE, 256, 48, 4, NS_, 3>(a, grid, stream);
    case 0b1011: return launch_epi<1, OP_DENSE, 1, OP_IM2COL, 256, 48, 4, NS_, 3>(a, grid, stream);
    case 0b1000: return launch_epi<1, OP_DENSE, 0, OP_DENSE, 256, 48, 4, NS_, 3>(a, grid, stream);
    default: break;
  }
  if (a.a_mc == 0 && a.a_mode == OP_IM2COL && a.b_mc == 1 && a.b_mode == OP_FLIPW)
    return launch_epi<0, OP_IM2COL, 1, OP_FLIPW, 256, 48, 4, NS_, 3>(a, grid, stream);
  return 4;
}

template <int AMODE, int FMT>
int launch_fp8(const SnGemmArgs& a, dim3 grid, hipStream_t st) {
  switch (a.epi) {
    case EPI_BF16:
      hipLaunchKernelGGL((gemm_kernel<0, AMODE, 0, OP_DENSE, EPI_BF16, 128, 128, 4, 2, FMT>), grid, dim3(256), 0, st, a);
      break;
    case EPI_BF16_DROP:
      if (AMODE != OP_DENSE || FMT != 1) return 4;
      hipLaunchKernelGGL((gemm_kernel<0, OP_DENSE, 0, OP_DENSE, EPI_BF16_DROP, 128, 128, 4, 2, 1>), grid, dim3(256), 0,
                         st, a);
      break;
    case EPI_F32:
      hipLaunchKernelGGL((gemm_kernel<0, AMODE, 0, OP_DENSE, EPI_F32, 128, 128, 4, 2, FMT>), grid, dim3(256), 0, st, a);
      break;
    default:
      return 2;
  }
  return SN_CHECK_LAUNCH();
}

// fp8 weight gradients: dy^T (MC dense, e4m3 / e5m2) x x (MC: implicit im2col of the
// layer input, or a dense activation matrix), reduction over the pixel / batch rows, fp32
// (split-K slab / accumulate) epilogues only; 128x128 tile (read_frag8_mc)
template <int BMODE, int FMT>
int launch_fp8_mc(const SnGemmArgs& a, dim3 grid, hipStream_t st) {
  switch (a.epi) {
    case EPI_F32:
      hipLaunchKernelGGL((gemm_kernel<1, OP_DENSE, 1, BMODE, EPI_F32, 128, 128, 4, 2, FMT>), grid, dim3(256), 0, st, a);
      break;
    case EPI_F32_ACC:
      hipLaunchKernelGGL((gemm_kernel<1, OP_DENSE, 1, BMODE, EPI_F32_ACC, 128, 128, 4, 2, FMT>), grid, dim3(256), 0, st,
                         a);
      break;
    default:
      return 2;
  }
  return SN_CHECK_LAUNCH();
}

}  // namespace


extern "C" int sn_gemm(const SnGemmArgs* args, hipStream_t stream) {
  const SnGemmArgs& a = *args;
  if (a.M <= 0 || a.N <= 0) return 0;
  // the ones column is a whole 16-B chunk of an MC B operand, inside the product's N
  // (fp8: MC weight-gradient products only, the column on a 16-byte chunk boundary)
  if (a.ones_col >= 0 && (!a.b_mc || a.b_mode == OP_FLIPW || (a.ones_col & (a.fp8 ? 15 : 7)) || a.ones_col >= a.N ||
                          (a.fp8 && !a.a_mc)))
    return 5;
  if (a.bias_out && (a.ones_col < 0 || a.epi == EPI_BF16 || a.epi == EPI_BF16_DROP)) return 5;
  // fused fp8 side output: unsplit bf16 epilogues of gemm_kernel (not gemm256_kernel, tiles
  // 6-9), whole 8-byte chunks
  if (a.q_out && (a.splits != 1 || (a.epi != EPI_BF16 && a.epi != EPI_BF16_DROP) || (a.tile >= 6 && a.tile <= 7) ||
                  (a.N % 8) || (a.q_ld % 8) || (a.q_gstride % 8) || !a.q_slot || !a.q_part ||
                  (reinterpret_cast<unsigned long long>(a.q_out) & 7)))
    return 6;
  if (a.fp8) {
    if (a.kchunk <= 0 || (a.kchunk % 128) != 0 || !a.deq_a || !a.deq_b) return 3;
    if (a.a_mc || a.b_mc) {
      if (!a.a_mc || a.a_mode != OP_DENSE || !a.b_mc || (a.b_mode != OP_IM2COL && a.b_mode != OP_DENSE) ||
          (a.fp8 != 1 && a.fp8 != 2))
        return 3;
      const int tiles = ((a.M + 127) / 128) * ((a.N + 127) / 128);
      dim3 grid(tiles * a.splits * a.groups);
      if (a.b_mode == OP_IM2COL)
        return a.fp8 == 1 ? launch_fp8_mc<OP_IM2COL, 1>(a, grid, stream) : launch_fp8_mc<OP_IM2COL, 2>(a, grid, stream);
      return a.fp8 == 1 ? launch_fp8_mc<OP_DENSE, 1>(a, grid, stream) : launch_fp8_mc<OP_DENSE, 2>(a, grid, stream);
    }
    // e4m3 forward products: A (dense or implicit im2col) and B dense, both K-contiguous
    if (a.b_mode != OP_DENSE) return 3;
    if (a.tile == 11 || a.tile == 16) return sn_gemm_fp8_big(a, stream);  // gemm_fp8big.hip
    const int tiles = ((a.M + 127) / 128) * ((a.N + 127) / 128);
    dim3 grid(tiles * a.splits * a.groups);
    if (a.fp8 == 2)  // e5m2 output gradients: the fp8 data-gradient products (implicit im2col A)
      return a.a_mode == OP_IM2COL ? launch_fp8<OP_IM2COL, 2>(a, grid, stream) : 4;
    if (a.fp8 != 1) return 4;
    return a.a_mode == OP_IM2COL ? launch_fp8<OP_IM2COL, 1>(a, grid, stream) : launch_fp8<OP_DENSE, 1>(a, grid, stream);
  }
  if (a.kchunk <= 0 || (a.kchunk % BK) != 0) return 3;
  switch (a.tile) {
    case 1:
    case 2:
    case 3:
    case 10:
    case 19:
    case 20: return sn_gemm_tiles_b(a, stream);  // gemm_tiles_b.hip
    case 4: return launch_tile96(a, stream);
    case 5: return launch_tile48(a, stream);
    case 6:
    case 7: return a.epi == EPI_SGD ? 4 : sn_gemm_t256(a, stream);  // gemm_t256.hip
    case 11:
    case 12:
    case 13:
    case 14: return a.epi == EPI_SGD ? 4 : sn_gemm_big8(a, stream);  // gemm_big8.hip
    case 21:
    case 22: return sn_gemm_tiles_c(a, stream);  // gemm_tiles_c.hip (64-row tiles)
    case 15:
    case 16:
    case 17:
    case 18: return a.epi == EPI_SGD ? 4 : sn_gemm_big4(a, stream);  // gemm_big4.hip
    default: return launch_tile<128, 128, 4, 2>(a, stream);
  }
}
