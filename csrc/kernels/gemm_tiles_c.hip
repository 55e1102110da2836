// Tile-family translation unit of the MFMA GEMM engine (see gemm.hip, gemm_impl.h):
// 64-row tiles for products whose M is 64 or less — the weight gradients of 64-channel
// convolutions (VGG-16 conv1_2 / conv2_1, M = K_out = 64) and GoogLeNet's thin reduce
// layers (M = 16-64), which on a 128-row tile leave half or more of every MFMA idle.
#include "gemm_impl.h"

namespace {

template <int BM, int BN, int NW, int NS, int NFR, int MFR>
int launch_tile_nf(const SnGemmArgs& a, hipStream_t stream) {
  const int tiles = ((a.M + BM - 1) / BM) * ((a.N + BN - 1) / BN);
  dim3 grid(tiles * a.splits * a.groups);
  const int key = (a.a_mc << 3) | (a.a_mode << 2) | (a.b_mc << 1) | a.b_mode;
  if (a.epi == EPI_SGD) {
    if (key != 0b1010 || a.splits != 1 || !a.sgd_w || !a.sgd_h || !a.sgd_shadow || !a.sgd_hyper) return 6;
    hipLaunchKernelGGL((gemm_kernel<1, OP_DENSE, 1, OP_DENSE, EPI_SGD, BM, BN, NW, NS, 0, NFR, MFR>), grid,
                       dim3(NW * 64), 0, stream, a);
    return SN_CHECK_LAUNCH();
  }
  switch (key) {
    case 0b0000: return launch_epi<0, OP_DENSE, 0, OP_DENSE, BM, BN, NW, NS, NFR, MFR>(a, grid, stream);
    case 0b0100: return launch_epi<0, OP_IM2COL, 0, OP_DENSE, BM, BN, NW, NS, NFR, MFR>(a, grid, stream);
    case 0b0010: return launch_epi<0, OP_DENSE, 1, OP_DENSE, BM, BN, NW, NS, NFR, MFR>(a, grid, stream);
    case 0b1010: return launch_epi<1, OP_DENSE, 1, OP_DENSE, BM, BN, NW, NS, NFR, MFR>(a, grid, stream);
    case 0b1011: return launch_epi<1, OP_DENSE, 1, OP_IM2COL, BM, BN, NW, NS, NFR, MFR>(a, grid, stream);
    default: break;
  }
  return 4;
}

}  // namespace

int sn_gemm_tiles_c(const SnGemmArgs& a, hipStream_t stream) {
  switch (a.tile) {
    case 21: return launch_tile_nf<64, 256, 4, 2, 4, 4>(a, stream);  // waves 1x4 of 64x64, 2 blocks / CU
    case 22: return launch_tile_nf<64, 128, 4, 2, 2, 4>(a, stream);  // waves 1x4 of 64x32, 3 blocks / CU
    default: return 4;
  }
}
