// Tile-family translation unit of the MFMA GEMM engine (see gemm.hip, gemm_impl.h):
// compiled separately so the instantiations build in parallel.
#include "gemm_impl.h"

// 4-wave tiles of 320 rows + columns (40 KB LDS stages: two blocks per CU, like 128x128)
// with 17 % fewer operand bytes per MFMA than 128x128
int sn_gemm_big4(const SnGemmArgs& a, hipStream_t stream) {
  switch (a.tile) {
    case 15: return launch_big<128, 192, 4, 6, 4>(a, stream);  // waves 2x2 of 64x96
    case 16: return launch_big<192, 128, 6, 4, 4>(a, stream);  // waves 2x2 of 96x64
    case 17: return launch_big<192, 96, 6, 3, 4>(a, stream);   // waves 2x2 of 96x48
    case 18: return launch_big<192, 64, 6, 2, 4>(a, stream);   // waves 2x2 of 96x32
    default: return 4;
  }
}
