// Tile-family translation unit of the MFMA GEMM engine (see gemm.hip, gemm_impl.h):
// gemm256_kernel with the 8-phase schedule (PH 8: four phases per K-tile, one C-quadrant per
// phase, one half-tile LDS-DMA per phase, counted vmcnt once per K-tile), compiled apart so
// the instantiations build in parallel.
#include "gemm_impl.h"

int sn_gemm_t256p8(const SnGemmArgs& a, hipStream_t stream) {
  switch (a.tile) {
    case 40: return launch256<256, 8>(a, stream);
    case 41: return launch256<128, 8>(a, stream);
    default: return 4;
  }
}
