// procx.hpp -- the seeded counter-based design generator as a device function.
//
// X[i, j] of the synthetic designs (sparkglm_amd/synth.py, bit-identical host copy) is a pure
// function of (seed, global row i, column j): integer hashing (splitmix64) and IEEE
// multiply/add only, no FMA contraction.  synth_kernel stores it in HBM; the procedural mode
// of the wide path (sglm_synth_procedural) regenerates it inside the kernels instead of
// reading it, for designs larger than HBM (BASELINE configs[4]: 2B x 512 = 8.19 TB).
#pragma once
#include <hip/hip_runtime.h>

#include <cstdint>

#include "common.hpp"

namespace sglm {

__device__ __forceinline__ uint64_t splitmix64(uint64_t x) {
  uint64_t z = x + 0x9E3779B97F4A7C15ull;
  z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
  z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
  return z ^ (z >> 31);
}
__device__ __forceinline__ double unif(uint64_t key) { return (double)(splitmix64(key) >> 11) * 0x1.0p-53; }

// X[gi, j] for j < p (column 0: the intercept); kind 3 is the positive gamma design.
__device__ __forceinline__ double gen_x(int kind, uint64_t kx, uint64_t gi, int p, int j, double scale) {
#pragma clang fp contract(off)
  if (j == 0) return 1.0;
  const double u = unif(kx + gi * (uint64_t)p + (uint64_t)j);
  return kind == 3 ? (0.5 + u) * scale : (2.0 * u - 1.0) * scale;
}

// gen_x for one row, the design kind fixed at compile time (POS: kind 3): kb = kx + gi * p, the
// row's key base (unsigned wrap-around, so kb + j is gen_x's key bit for bit).
template <bool POS>
__device__ __forceinline__ double gen_x_row(uint64_t kb, int j, double scale) {
#pragma clang fp contract(off)
  if (j == 0) return 1.0;
  const double u = unif(kb + (uint64_t)j);
  return POS ? (0.5 + u) * scale : (2.0 * u - 1.0) * scale;
}

// X[row, col] of a procedural shard: zero past p and on the padding rows (>= n), exactly as
// the resident, zero-padded image.
__device__ __forceinline__ double proc_x(const ProcX& g, int64_t row, int col) {
  if (col >= g.p || row >= g.n) return 0.0;
  return gen_x(g.kind, g.kx, (uint64_t)(g.row0 + row), g.p, col, g.scale);
}

}  // namespace sglm
