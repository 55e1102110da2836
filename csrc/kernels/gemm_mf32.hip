// Tile-family translation unit of the MFMA GEMM engine (see gemm.hip, gemm_impl.h): the
// v_mfma_f32_32x32x16_bf16 twins of the production tiles (gemm_kernel MF32 = 1).  Each
// wave-tile is (MFR/2) x (NFR/2) blocks of 32x32; per K-step the LDS fragment bytes are those
// of the 16x16x32 tile, with half the MFMA instructions and three times the VALU issue slack
// per MFMA cycle (24 of 32 cycles instead of 8 of 16), which is what the implicit-im2col
// address paths (the weight gradients' pixel-row walk above all) spend.
#include "gemm_impl.h"

namespace {

template <int BM, int BN, int NW, int NS, int NFR, int MFR>
int launch_mf32(const SnGemmArgs& a, hipStream_t stream) {
  const int tiles = ((a.M + BM - 1) / BM) * ((a.N + BN - 1) / BN);
  dim3 grid(tiles * a.splits * a.groups);
  const int key = (a.a_mc << 3) | (a.a_mode << 2) | (a.b_mc << 1) | a.b_mode;
  constexpr bool mc_b_ok = (BN / 8) == 8 || (BN / 8) == 16 || (BN / 8) == 32;  // MC images: whole rows per DMA
  constexpr bool mc_a_ok = (BM / 8) == 8 || (BM / 8) == 16 || (BM / 8) == 32;
  switch (key) {
    case 0b0000: return launch_epi<0, OP_DENSE, 0, OP_DENSE, BM, BN, NW, NS, NFR, MFR, 1>(a, grid, stream);   // NT dense
    case 0b0100: return launch_epi<0, OP_IM2COL, 0, OP_DENSE, BM, BN, NW, NS, NFR, MFR, 1>(a, grid, stream);  // conv fwd/dgrad
    default: break;
  }
  if constexpr (mc_b_ok) {
    if (key == 0b0010) return launch_epi<0, OP_DENSE, 1, OP_DENSE, BM, BN, NW, NS, NFR, MFR, 1>(a, grid, stream);  // NN
    if constexpr (mc_a_ok) {
      if (key == 0b1010) return launch_epi<1, OP_DENSE, 1, OP_DENSE, BM, BN, NW, NS, NFR, MFR, 1>(a, grid, stream);  // TN
      if (key == 0b1011)  // conv weight gradient
        return launch_epi<1, OP_DENSE, 1, OP_IM2COL, BM, BN, NW, NS, NFR, MFR, 1>(a, grid, stream);
    }
  }
  return 4;
}

}  // namespace

int sn_gemm_mf32(const SnGemmArgs& a, hipStream_t stream) {
  if (a.epi == EPI_SGD) return 4;
  switch (a.tile) {
    case 23: return launch_mf32<128, 128, 4, 2, 4, 4>(a, stream);  // tile 0's twin: waves 2x2 of 64x64
    case 24: return launch_mf32<128, 64, 4, 2, 2, 4>(a, stream);   // tile 10's twin: waves 2x2 of 64x32
    case 25: return launch_mf32<192, 128, 4, 2, 4, 6>(a, stream);  // tile 16's twin: waves 2x2 of 96x64
    case 26: return launch_mf32<256, 128, 8, 2, 4, 4>(a, stream);  // tile 13's twin: waves 4x2 of 64x64
    case 27: return launch_mf32<256, 64, 4, 2, 4, 4>(a, stream);   // tile 1's twin: waves 4x1 of 64x64
    case 28: return launch_mf32<256, 256, 8, 2, 4, 8>(a, stream);  // tile 11's twin: waves 2x4 of 128x64
    default: return 4;
  }
}
