// Tile-family translation unit of the MFMA GEMM engine (see gemm.hip, gemm_impl.h):
// compiled separately so the instantiations build in parallel.
#include "gemm_impl.h"

// gemm256_kernel: 256x256 / 256x128 8-wave tiles, half-tile phased DMA pipeline
int sn_gemm_t256(const SnGemmArgs& a, hipStream_t stream) {
  switch (a.tile) {
    case 6: return launch256<256>(a, stream);
    case 7: return launch256<128>(a, stream);
    default: return 4;
  }
}
