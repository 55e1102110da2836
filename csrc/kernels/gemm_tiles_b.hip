// Tile-family translation unit of the MFMA GEMM engine (see gemm.hip, gemm_impl.h):
// compiled separately so the instantiations build in parallel.
#include "gemm_impl.h"

namespace {

// 128x64 tile (4 waves of 64x32, 48 KB of LDS): three co-resident blocks per CU (three
// waves per SIMD) to hide the LDS-DMA latency of latency-bound products (few K-steps,
// narrow outputs) at the price of 1.5x the operand bytes per MFMA of a 128x128 tile.
template <int NS = 2>
int launch_tile64(const SnGemmArgs& a, hipStream_t stream) {
  const int tiles = ((a.M + 127) / 128) * ((a.N + 63) / 64);
  dim3 grid(tiles * a.splits * a.groups);
  const int key = (a.a_mc << 3) | (a.a_mode << 2) | (a.b_mc << 1) | a.b_mode;
  switch (key) {
    case 0b0000: return launch_epi<0, OP_DENSE, 0, OP_DENSE, 128, 64, 4, NS, 2>(a, grid, stream);
    case 0b0100: return launch_epi<0, OP_IM2COL, 0, OP_DENSE, 128, 64, 4, NS, 2>(a, grid, stream);
    case 0b1010: return launch_epi<1, OP_DENSE, 1, OP_DENSE, 128, 64, 4, NS, 2>(a, grid, stream);
    case 0b1011: return launch_epi<1, OP_DENSE, 1, OP_IM2COL, 128, 64, 4, NS, 2>(a, grid, stream);
    case 0b0010: return NS == 3 ? launch_epi<0, OP_DENSE, 1, OP_DENSE, 128, 64, 4, NS, 2>(a, grid, stream) : 4;
    default: return 4;
  }
}

// Three-stage 4-wave tiles for latency-bound products (the batch-256 InnerProduct
// forward / data gradient: few K-steps per block, weights streamed from HBM): two
// K-steps of LDS-DMA in flight per block instead of one.  128x128 x 3 stages = 96 KB
// (one block per CU); 128x64 x 3 stages = 72 KB (two per CU).
int launch_tile_ns3(const SnGemmArgs& a, hipStream_t stream) {
  const int key = (a.a_mc << 3) | (a.a_mode << 2) | (a.b_mc << 1) | a.b_mode;
  // 128x64: also the weight-gradient forms (MC x MC dense / im2col), whose NS = 2 tile 10
  // waits for each K-step's DMA (one K-step in flight per block, three blocks per CU)
  if (a.tile == 20 && (key == 0b1010 || key == 0b1011)) return launch_tile64<3>(a, stream);
  if (key != 0b0000 && key != 0b0010) return 4;  // dense NT / NN
  if (a.tile == 20) return launch_tile64<3>(a, stream);
  const int tiles = ((a.M + 127) / 128) * ((a.N + 127) / 128);
  dim3 grid(tiles * a.splits * a.groups);
  if (key == 0b0000) return launch_epi<0, OP_DENSE, 0, OP_DENSE, 128, 128, 4, 3>(a, grid, stream);
  return launch_epi<0, OP_DENSE, 1, OP_DENSE, 128, 128, 4, 3>(a, grid, stream);
}

}  // namespace

// 256x64 (skinny N), 256x128 / 128x256 (8 waves, 3 stages), 128x64 (three blocks per CU),
// 128x128 / 128x64 with 3 stages (19: dense; 20: dense and the weight-gradient forms)
int sn_gemm_tiles_b(const SnGemmArgs& a, hipStream_t stream) {
  switch (a.tile) {
    case 1: return launch_tile<256, 64, 4, 2>(a, stream);
    case 2: return launch_tile<256, 128, 8, 3>(a, stream);
    case 3: return launch_tile<128, 256, 8, 3>(a, stream);
    case 10: return a.epi == EPI_SGD ? 4 : launch_tile64(a, stream);
    case 19:
    case 20: return a.epi == EPI_SGD ? 4 : launch_tile_ns3(a, stream);
    default: return 4;
  }
}
