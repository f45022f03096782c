// fused_odd.hip -- K1r (irls_pass_r_kernel, fused.hpp) for the odd column-block counts
// P16 = 5, 7, ..., 15: 65..80, 97..112, ..., 225..240 columns run ceil(p / 16) blocks of 16
// instead of K1's next even count (P16 (P16 + 1) / 2 tiles per k-step instead of (P16 + 1)
// (P16 + 2) / 2).  A separate object so the two kernel sets compile in parallel.
#include "fused.hpp"

namespace sglm {

hipError_t launch_pass_odd(int P16, const PassArgs& a, int grid, hipStream_t st) {
  switch (P16) {
    case 5: return launch_pass_r_fl<5>(a, grid, st);
    case 7: return launch_pass_r_fl<7>(a, grid, st);
    case 9: return launch_pass_r_fl<9>(a, grid, st);
    case 11: return launch_pass_r_fl<11>(a, grid, st);
    case 13: return launch_pass_r_fl<13>(a, grid, st);
    case 15: return launch_pass_r_fl<15>(a, grid, st);
    default: return hipErrorInvalidValue;
  }
}

}  // namespace sglm
