// Persistent ring-pipelined GEMM tiles 30-32 (see gemm_pk.h); own TU for parallel builds.
#include "gemm_pk.h"

int sn_gemm_pk_a(const SnGemmArgs& a, hipStream_t stream) {
  switch (a.tile) {
    case 30: return pk_launch<256, 128, 4, 4, 4, 3>(a, stream);  // waves 4x2 of 64x64, 3 x 48 KB ring
    case 31: return pk_launch<256, 64, 4, 4, 2, 4>(a, stream);   // waves 4x2 of 64x32, 4 x 40 KB ring
    case 32: return pk_launch<256, 96, 4, 4, 3, 3>(a, stream);   // waves 4x2 of 64x48, 3 x 48 KB ring
    case 39: return pk_launch_probe<256, 128, 4, 4, 4, 3>(a, stream);  // tile 30 with the unstaggered loop
    default: return 4;
  }
}
