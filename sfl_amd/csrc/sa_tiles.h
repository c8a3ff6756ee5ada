// sa_tiles.h -- workgroup -> tile mapping of the one-pass streaming kernels
// (device code: included by sa_api.hip and sa_dp.hip after hip_runtime.h)
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

namespace sa {

// Tile of a one-pass streaming kernel (one tile per workgroup, no grid
// stride: the server kernels, k_dp_perturb).  The dispatcher deals
// workgroup b to XCD b % 8, so tile b is workgroup b and the 8 XCDs stream
// interleaved tiles.  SA_XCD_TILES=1 gives each XCD one contiguous run of
// tiles instead (bijective for any grid: XCD x holds q + (x < r) tiles,
// q = G / 8, r = G % 8).  Nothing is re-read, so no per-XCD L2 locality is
// there to win: on MI355X the contiguous runs were 0.5-2 % SLOWER for
// k_sum_u64, k_sum_f64, k_decode<true> and k_dp_perturb and within noise
// for k_decode<false> (tools/r05_dpx.sh, profiles/r05/xcd_tiles_ab.txt);
// the interleaved order stays.
#ifndef SA_XCD_TILES
#define SA_XCD_TILES 0
#endif
__device__ __forceinline__ uint32_t stream_tile() {
#if SA_XCD_TILES
  const uint32_t G = gridDim.x, q = G / 8, r = G % 8, x = blockIdx.x % 8;
  return x * q + (x < r ? x : r) + blockIdx.x / 8;
#else
  return blockIdx.x;
#endif
}

}  // namespace sa
