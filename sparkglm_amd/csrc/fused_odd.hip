// fused_odd.hip -- the fused passes at odd column-block counts (fused.hpp): K1r
// (irls_pass_r_kernel) for P16 = 5, 7, ..., 15 -- by default 129..144, 161..176, ..., 225..240
// columns (P16 >= 9) -- and K1 (irls_pass_kernel) for P16 = 5, 7 (65..80, 97..112 columns): ceil(p / 16)
// blocks of 16 instead of the next even count (P16 (P16 + 1) / 2 tiles per k-step instead of
// (P16 + 1) (P16 + 2) / 2).  A separate object so the kernel sets compile in parallel.
#include "fused.hpp"

namespace sglm {

hipError_t launch_pass_odd(int P16, const PassArgs& a, int grid, hipStream_t st, hipEvent_t e0, hipEvent_t e1) {
  if (!pass_uses_split(P16, a.fused_split, a.ld)) {  // K1 (5, 7; pass_variant rounds larger odd counts up)
    if (P16 == 5) return launch_pass_k1<5>(a, grid, st, e0, e1);
    if (P16 == 7) return launch_pass_k1<7>(a, grid, st, e0, e1);
    return hipErrorInvalidValue;
  }
  switch (P16) {
    case 5: return launch_pass_r_fl<5>(a, grid, st, e0, e1);
    case 7: return launch_pass_r_fl<7>(a, grid, st, e0, e1);
    case 9: return launch_pass_r_fl<9>(a, grid, st, e0, e1);
    case 11: return launch_pass_r_fl<11>(a, grid, st, e0, e1);
    case 13: return launch_pass_r_fl<13>(a, grid, st, e0, e1);
    case 15: return launch_pass_r_fl<15>(a, grid, st, e0, e1);
    default: return hipErrorInvalidValue;
  }
}

}  // namespace sglm
