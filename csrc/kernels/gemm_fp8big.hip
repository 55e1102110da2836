// Large e4m3 tiles for the fp8 forward products (VGG-16 --dtype fp8): 256x256 (8 waves of
// 128x64, one block per CU, tile 11) and 192x128 (4 waves of 96x64, two blocks per CU,
// tile 16).  At twice the bf16 MFMA rate an fp8 K-step is half as long, so the 128x128
// tile (gemm.hip launch_fp8) is even more bound by its operand traffic and LDS-DMA latency
// than in bf16: these tiles cut the L2 -> LDS bytes per MFMA by 1/2 and 1/6.
#include "gemm_impl.h"

namespace {

template <int AMODE, int BM, int BN, int NW, int NFR, int MFR, int FMT>
int launch_fp8_big(const SnGemmArgs& a, hipStream_t st) {
  const int tiles = ((a.M + BM - 1) / BM) * ((a.N + BN - 1) / BN);
  dim3 grid(tiles * a.splits * a.groups);
  switch (a.epi) {
    case EPI_BF16:
      hipLaunchKernelGGL((gemm_kernel<0, AMODE, 0, OP_DENSE, EPI_BF16, BM, BN, NW, 2, FMT, NFR, MFR>), grid,
                         dim3(NW * 64), 0, st, a);
      break;
    case EPI_F32:
      hipLaunchKernelGGL((gemm_kernel<0, AMODE, 0, OP_DENSE, EPI_F32, BM, BN, NW, 2, FMT, NFR, MFR>), grid,
                         dim3(NW * 64), 0, st, a);
      break;
    default:
      return 4;
  }
  return SN_CHECK_LAUNCH();
}

}  // namespace

int sn_gemm_fp8_big(const SnGemmArgs& a, hipStream_t stream) {
  const bool im2col = a.a_mode == OP_IM2COL;
  if (a.fp8 == 2) {  // e5m2 A (output gradients of the fp8 data-gradient products): implicit im2col only
    if (!im2col) return 4;
    switch (a.tile) {
      case 11: return launch_fp8_big<OP_IM2COL, 256, 256, 8, 4, 8, 2>(a, stream);
      case 16: return launch_fp8_big<OP_IM2COL, 192, 128, 4, 4, 6, 2>(a, stream);
      default: return 4;
    }
  }
  if (a.fp8 != 1) return 4;
  switch (a.tile) {
    case 11:
      return im2col ? launch_fp8_big<OP_IM2COL, 256, 256, 8, 4, 8, 1>(a, stream)
                    : launch_fp8_big<OP_DENSE, 256, 256, 8, 4, 8, 1>(a, stream);
    case 16:
      return im2col ? launch_fp8_big<OP_IM2COL, 192, 128, 4, 4, 6, 1>(a, stream)
                    : launch_fp8_big<OP_DENSE, 192, 128, 4, 4, 6, 1>(a, stream);
    default:
      return 4;
  }
}
