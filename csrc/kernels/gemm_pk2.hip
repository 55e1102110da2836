// Persistent ring-pipelined GEMM tiles 33-36 (see gemm_pk.h); own TU for parallel builds.
#include "gemm_pk.h"

int sn_gemm_pk_b(const SnGemmArgs& a, hipStream_t stream) {
  switch (a.tile) {
    case 33: return pk_launch<128, 128, 4, 2, 4, 5>(a, stream);  // waves 4x2 of 32x64, 5 x 32 KB ring
    case 34: return pk_launch<256, 192, 2, 8, 3, 2>(a, stream);  // waves 2x4 of 128x48, 2 x 56 KB ring
    case 36: return pk_launch<128, 256, 2, 4, 4, 3>(a, stream);  // waves 2x4 of 64x64, 3 x 48 KB ring
    case 37: return pk_launch<192, 384, 2, 6, 6, 2>(a, stream);  // waves 2x4 of 96x96, 2 x 72 KB ring
    case 38: return pk_launch<256, 256, 2, 8, 4, 2>(a, stream);  // waves 2x4 of 128x64, 2 x 64 KB ring
    default: return 4;
  }
}
