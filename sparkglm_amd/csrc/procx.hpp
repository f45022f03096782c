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

// The design's two affine maps of u = (h >> 11) * 2^-53 (h = splitmix64(key)), (2u - 1) and (0.5 + u),
// built from the bits of h with integer ops and ONE fp64 add -- bit for bit the fp64 expressions
// (synth.py), without the u64 -> f64 conversion (two cvt, two ldexp, one add) and the two affine fp64
// ops: on gfx950 the fp64 VALU shares its pipe with the fp64 MFMA of the Gram launch this runs beside,
// integer VALU does not.  With h >> 11 = b 2^52 + r (b = bit 63 of h, r = its bits
// 11..62) and d(E) the double of biased exponent E and mantissa r, i.e. (1 + r 2^-52) 2^(E - 1023):
//   2u - 1  = r 2^-52 + b - 1    = d(0x3FF) - (b ? 1 : 2)   exact on both sides (Sterbenz), signed zero included;
//   0.5 + u = 0.5 + r 2^-53 + b/2 = d(0x3FE) + (b ? 0.5 : 0) the one rounding of 0.5 + u when b = 1
//                                                          (u = d(0x3FE) then), exact when b = 0.
template <bool POS>
__device__ __forceinline__ double affine_u(uint64_t h) {
#pragma clang fp contract(off)
  const uint64_t e = POS ? 0x3FEull : 0x3FFull;
  const double d = __builtin_bit_cast(double, (e << 52) | ((h >> 11) & 0xFFFFFFFFFFFFFull));
  const bool b = (h >> 63) != 0;
  const uint64_t cbits = POS ? (b ? 0x3FE0000000000000ull : 0ull) : (b ? 0xBFF0000000000000ull : 0xC000000000000000ull);
  return d + __builtin_bit_cast(double, cbits);
}

// X[gi, j] for j < p (column 0: the intercept); kind 3 is the positive gamma design.
__device__ __forceinline__ double gen_x(int kind, uint64_t kx, uint64_t gi, int p, int j, double scale) {
#pragma clang fp contract(off)
  if (j == 0) return 1.0;
  const uint64_t h = splitmix64(kx + gi * (uint64_t)p + (uint64_t)j);
  return (kind == 3 ? affine_u<true>(h) : affine_u<false>(h)) * scale;
}

// gen_x for one row, the design kind fixed at compile time (POS: kind 3): kb = kx + gi * p, the
// row's key base (unsigned wrap-around, so kb + j is gen_x's key bit for bit).
template <bool POS>
__device__ __forceinline__ double gen_x_row(uint64_t kb, int j, double scale) {
#pragma clang fp contract(off)
  if (j == 0) return 1.0;
  return affine_u<POS>(splitmix64(kb + (uint64_t)j)) * scale;
}

// X[row, col] of a procedural shard: zero past p and on the padding rows (>= n), exactly as
// the resident, zero-padded image.
__device__ __forceinline__ double proc_x(const ProcX& g, int64_t row, int col) {
  if (col >= g.p || row >= g.n) return 0.0;
  return gen_x(g.kind, g.kx, (uint64_t)(g.row0 + row), g.p, col, g.scale);
}

}  // namespace sglm
