// Tile-family translation unit of the MFMA GEMM engine (see gemm.hip, gemm_impl.h):
// compiled separately so the instantiations build in parallel.
#include "gemm_impl.h"

// 8-wave, 2-stage gemm_kernel tiles with 256 rows (one block per CU)
int sn_gemm_big8(const SnGemmArgs& a, hipStream_t stream) {
  switch (a.tile) {
    case 11: return launch_big<256, 256, 8, 4>(a, stream);  // waves 2x4 of 128x64
    case 12: return launch_big<256, 128, 8, 2>(a, stream);  // waves 2x4 of 128x32
    case 13: return launch_big<256, 128, 4, 4>(a, stream);  // waves 4x2 of 64x64
    case 14: return launch_big<256, 192, 8, 3>(a, stream);  // waves 2x4 of 128x48
    default: return 4;
  }
}
