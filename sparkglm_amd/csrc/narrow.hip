// narrow.hip -- the narrow-design (p <= 64) fused IRLS pass for gfx950.
//
// At p <= 64 one row of X is <= 536 bytes and the pass sits at the HBM / fp64-MFMA balance
// point (~8 flop/B), so the workgroup-lockstep pipeline of irls_pass_kernel
// (two barriers per row block, row stage on one wave while its partners wait) leaves both
// the MFMA pipe and HBM idle.  Here every wave is an independent streaming pipeline with
// no barriers in its main loop:
//
//   * wave gw owns a contiguous range of row blocks (NRB = 32 rows for p <= 32, 16 above)
//     and the WHOLE lower-triangular Gram
//     (T = P16(P16+1)/2 <= 10 16x16 fp64 tiles, <= 80 accumulator VGPRs);
//   * its blocks land in a wave-private, double-buffered LDS image by LDS-DMA
//     (global_load_lds_dwordx4; block i+2 is issued as soon as block i is consumed), one
//     wave-instruction per column octet plus one for the y/m/offset/prior values;
//   * row stage (etaCreate GLM.scala:321-332, zwCreateBinomial GLM.scala:359-395, deviance
//     GLM.scala:162-170): 64/NRB lanes per row form eta over interleaved columns (xor-16 /
//     xor-32 lane swaps), then the family arithmetic (rowmath.hpp) on NRB lanes, w and w*z
//     to LDS;
//   * Gramian on v_mfma_f64_16x16x4_f64, A operand scaled by w, X'Wz on the VALU
//     (partitionComponents, utils.scala:84-92);
//   * two waves per SIMD (8 per workgroup, one workgroup per CU) interleave MFMA and VALU
//     work; the 8 wave partials are summed in LDS in a fixed tree order after the loop and
//     one partial per workgroup goes to reduce_partials_kernel (deterministic).
//
// LDS image of one block (per wave, per buffer): column c at c*NRB doubles, row r in slot
// r ^ f(c) (swz below), applied on the DMA source address.  MFMA fragment reads (lane
// (rq, cl) reads row 4s+rq of column 16b+cl) and row-stage reads (lane (g, rl) reads row rl
// of column (64/NRB)u+g) are both bank-conflict free for ds_read_b64.
#include <hip/hip_runtime.h>

#include <cstdint>
#include <type_traits>

#include "common.hpp"
#include "kernels.hpp"
#include "rowmath.hpp"

namespace sglm {

namespace {

typedef double d4 __attribute__((ext_vector_type(4)));
typedef __attribute__((address_space(3))) void lds_void;

// Issue priority by phase: a wave runs its row stage (eta, the family arithmetic: a dependent fp64
// chain) at high priority and its Grams at low, so the partner wave's MFMA stream fills the row
// stage's latencies instead of delaying its instructions (round 5: p = 32 -2 %, p = 48 -1 %, p = 64
// +-0 against priorities alternating between the two waves every 4 blocks; 12 waves a CU on 8-row
// blocks at p > 32: +18-20 %, DESIGN.md 4 K1').  Measured and not kept: the diagonal tiles on three
// v_mfma_f64_4x4x4f64 (rotated B operands from LDS or by DPP: slower at p = 32 and 64); a
// batched Gram phase (all operands, then all VALU, then all MFMAs per block: p = 64 +25 %).
constexpr int PRIO_ROWS = 2, PRIO_GRAM = 0;

// Rows per block NRB: 32 for p <= 32 (the family arithmetic then runs on 32 lanes), 16 above
// (LDS: 8 waves x 2 buffers).  Row swizzle f(c): 2((c >> 1) & 7) at NRB = 16 (the column
// parity separates the bank halves), 2(c & 15) at NRB = 32.
template <int P16>
struct NGeo {
  static_assert(P16 >= 1 && P16 <= 4, "narrow variants: p <= 64");
  // 8 waves per workgroup (two per SIMD), one workgroup per CU.  (Measured at p <= 32: 12 or
  // 16 waves on 16-row blocks run 1.2-1.7x slower -- the family arithmetic's lane efficiency,
  // not latency, bounds these variants -- and 4 waves on 64-row blocks (all 64 lanes in the
  // family arithmetic, no partner wave) 1.07-1.17x slower.)
  static constexpr int NW = 8;
  static constexpr int NRB = P16 <= 2 ? 32 : 16;     // rows per block
  static constexpr int LPR = 64 / NRB;               // row-stage lanes per row
  static constexpr int NC = 16 * P16;                // padded columns
  // Lower-triangular 16x16 tiles.  (Measured and not kept: at P16 = 2 the two diagonal tiles
  // as 4x4 blocks on v_mfma_f64_4x4x4f64 -- full rate on gfx950, tools/mfma44_*.hip -- with
  // the off-diagonal tile on 16x16x4: 5 x 16 instead of 2 x 64 MFMA cycles per k-step, but the
  // rotated operands' LDS reads and scaling made the compute-only pass 2-3 % slower.)
  static constexpr int T = P16 * (P16 + 1) / 2;
  static constexpr int CPI = 128 / NRB;              // columns per DMA wave-instruction (1 KiB)
  static constexpr int NOCT = NC / CPI;              // DMA wave-instructions for X per block
  static constexpr int SPER = NRB == 16 ? 2 : 16 / CPI;  // period of the swizzle over column groups
  static constexpr int LPER = NOCT < SPER ? NOCT : SPER;
  // 16-column blocks BSTR = 16 NRB + 2 doubles apart: the pad keeps the per-block MFMA operand
  // reads plain ds_read_b64 (no ds_read2st64_b64 pairing: 32-bank rule, 2-way conflicts)
  static constexpr int BSTR = 16 * NRB + 2;         // (+2: keeps LDS-DMA destinations 16-B aligned)
  static constexpr int XB = P16 * BSTR;              // doubles of X per buffer
  static constexpr int BUF = XB + 4 * NRB;           // + y, m, offset, prior
  static constexpr int OFF_W = 2 * BUF;              // w[NRB], w*z[NRB] (PAIR: w[2 NRB], w*z[2 NRB])
  // Row pairs (NRB = 32, p <= 32): the family arithmetic runs on 32 of the wave's 64 lanes, so
  // blocks are taken in pairs -- the first block's eta, row values and Gram operands are stashed
  // in registers and its buffer released at once; with the second block, the family arithmetic
  // covers both blocks' rows on all 64 lanes (upper half: the stashed block), then both blocks'
  // MFMAs run from registers.  Half the family-arithmetic instructions per row.
  static constexpr bool PAIR = NRB == 32;
  static constexpr int WAVE_LDS = OFF_W + 4 * NRB;  // doubles per wave (w / w*z of a block pair)
  // one wave partial (tiles | X'Wz | dev, sum w, pearson, ll, bad | LMX: X'1)
  static constexpr int PSZ = T * 256 + NC + 5 + NC;
  static constexpr int LDS = (NW * WAVE_LDS > (NW / 2) * PSZ) ? NW * WAVE_LDS : (NW / 2) * PSZ;
  static_assert(NW % 4 == 0, "whole waves per SIMD");
  // global partial (reduce_partials_kernel layout): tiles | X'Wz | NS scalars | LMX: X'1 [NC]
  static constexpr int STRIDE = T * 256 + NC + NS + NC;
  static_assert(LDS * 8 <= 160 * 1024, "LDS budget");
};

// vmcnt accounting.  A wave waits for one block's DMA with s_waitcnt vmcnt(N), N = the vector-memory
// instructions issued AFTER that DMA (vmcnt counts down in issue order).  Every wait names what it lets
// fly -- whole block DMAs and eta stores younger than the block it needs -- and N follows from the
// instruction counts here, which nstage / stage_next issue by construction (their loops run DMA_X
// column-octet loads plus DMA_V row-vector load).  A loop change then changes a named operand of
// younger(), not a literal.
template <int P16>
struct VmCount {
  static constexpr int DMA_X = NGeo<P16>::NOCT;  // column-octet wave-instructions per block
  static constexpr int DMA_V = 1;                // the y / m / offset / prior slice
  static constexpr int DMA_BLOCK = DMA_X + DMA_V;
  static constexpr int ETA_STORE = 1;            // one global_store_dwordx2 per block (pair)
  static constexpr int younger(int blocks, int eta_stores) { return blocks * DMA_BLOCK + eta_stores * ETA_STORE; }
};
static_assert(VmCount<4>::younger(1, 1) == 4 * 16 / 8 + 2 && VmCount<1>::younger(1, 0) == 16 / 4 + 1,
              "NOCT + 1 per block DMA (p = 64: 8 + 1; p = 16: 4 + 1), one per eta store");

template <int NRB>
__device__ __forceinline__ constexpr int swz(int c) { return NRB == 16 ? 2 * ((c >> 1) & 7) : 2 * (c & 15); }

template <int N>
__device__ __forceinline__ void wait_vm() {
  static_assert(N >= 0 && N < 64, "vmcnt range");
  __builtin_amdgcn_s_waitcnt((N & 15) | ((N >> 4) << 14) | (7 << 4) | (15 << 8));
}

__device__ __forceinline__ double xor16_sum(double v) {
  const auto a = __builtin_amdgcn_permlane16_swap(__double2loint(v), __double2loint(v), false, false);
  const auto b = __builtin_amdgcn_permlane16_swap(__double2hiint(v), __double2hiint(v), false, false);
  return __hiloint2double(b[0], a[0]) + __hiloint2double(b[1], a[1]);
}
__device__ __forceinline__ double xor32_sum(double v) {
  const auto a = __builtin_amdgcn_permlane32_swap(__double2loint(v), __double2loint(v), false, false);
  const auto b = __builtin_amdgcn_permlane32_swap(__double2hiint(v), __double2hiint(v), false, false);
  return __hiloint2double(b[0], a[0]) + __hiloint2double(b[1], a[1]);
}

// DMA of block blk into buffer buf of this wave's image: NOCT wave-instructions of CPI
// columns x NRB rows (1 KiB each) + one for the block's slices of y, m, offset, prior
// (4 x NRB doubles on 2 NRB lanes).  Column groups past the stored columns re-load the last
// stored group (finite data; beta is 0 and the tiles are discarded past p), so every block
// issues exactly NOCT + 1 vector-memory operations.
template <int P16, int AUX>
__device__ __forceinline__ void nstage(double* wl, int buf, const PassArgs& a, int64_t blk, int ngrp_stored,
                                       const int64_t (&loff)[NGeo<P16>::LPER], const double* vsrc, int lane) {
  using G = NGeo<P16>;
  const double* xb = a.X + blk * G::NRB;
  double* dst = wl + buf * G::BUF;
#pragma unroll
  for (int o = 0; o < VmCount<P16>::DMA_X; ++o) {
    const int os = o < ngrp_stored ? o : ngrp_stored - 1;  // uniform
    __builtin_amdgcn_global_load_lds((const void*)(xb + (int64_t)(G::CPI * os) * a.ld + loff[o % G::LPER]),
                                     (lds_void*)(dst + (o * G::CPI / 16) * G::BSTR + (o * G::CPI % 16) * G::NRB), 16, 0, AUX);
  }
  if (G::NRB == 32 || lane < 2 * G::NRB)
    __builtin_amdgcn_global_load_lds((const void*)(vsrc + blk * G::NRB), (lds_void*)(dst + G::XB), 16, 0, AUX);
}

// Lane l of a 16-lane row takes the value of lane l & ~12 (the first 4-lane group's lane of the same
// position): ds_swizzle in bit mode, and_mask 0b10011 on the lane id within 32.
__device__ __forceinline__ double bcast_quad0(double v) {
  const int lo = __builtin_amdgcn_ds_swizzle(__double2loint(v), 0x13);
  const int hi = __builtin_amdgcn_ds_swizzle(__double2hiint(v), 0x13);
  return __hiloint2double(hi, lo);
}

// One k-step (4 rows) of the lower-triangular Gram on v_mfma_f64_16x16x4_f64.
// T4 (P16 = 2, p <= 20: the second column block holds at most 4 real columns, 16..19): the two
// tiles of that block's row run on v_mfma_f64_4x4x4f64, which takes its operands in the 16x16x4
// lane layout with 4x4 block j on columns 4j..4j+3 (tools/mfma_layout.hip) and writes block j's
// D(m, n) to lane 16 m + 4 j + n -- exactly where the 16x16x4 tile keeps rows 0..3 of its D in
// acc[t][0].  Tile (1, 1): block 0 is columns 16..19 x 16..19; tile (1, 0): the A operand's first
// 4-lane group (columns 16..19) broadcast to all four groups gives columns 16..19 x 4j..4j+3 in
// block j.  16 MFMA cycles each instead of 64 (the LM Gram of configs[0], p = 20: 96 per k-step
// instead of 192); rows 4..15 of those tiles (columns 20..31: padding) are never formed.
template <int P16, bool T4 = false>
__device__ __forceinline__ void gram_kstep(d4 (&acc)[NGeo<P16>::T], const double (&av)[P16], const double (&xv)[P16]) {
  if constexpr (T4) {
    static_assert(P16 == 2, "T4: two column blocks");
    acc[0] = __builtin_amdgcn_mfma_f64_16x16x4f64(av[0], xv[0], acc[0], 0, 0, 0);
    acc[1][0] = __builtin_amdgcn_mfma_f64_4x4x4f64(bcast_quad0(av[1]), xv[0], acc[1][0], 0, 0, 0);
    acc[2][0] = __builtin_amdgcn_mfma_f64_4x4x4f64(av[1], xv[1], acc[2][0], 0, 0, 0);
  } else {
    int t = 0;
#pragma unroll
    for (int bi = 0; bi < P16; ++bi)
#pragma unroll
      for (int bj = 0; bj <= bi; ++bj, ++t) acc[t] = __builtin_amdgcn_mfma_f64_16x16x4f64(av[bi], xv[bj], acc[t], 0, 0, 0);
  }
}

// IRLS: compile-time a.mode == MODE_IRLS (the iterations); the init and LM Gram passes run the
// IRLS = false instantiation, so the iterations' main loop carries none of their branches.
// STATS (PassArgs::stats_in_pass: binomial / logit IRLS without m, Poisson / log, Gamma /
// inverse): the pass also accumulates the final statistics -- pearsonCalc / llBinomial, the R
// families' loglik ingredients -- at this pass's mu and stores no eta; the last pass of a fit then
// carries them (no stats_kernel pass; the eta store was ~6 % of a p = 32 pass, ~1 % at p = 64).
// The Poisson / Gamma statistics' per-fit constants (rowmath.hpp init_stats_const) are summed by
// the initial pass (IRLS = false) into S_AUX2.
// LMX (the LM Gram pass of LM.fit's one device round trip, PassArgs::lm_extras): the pass also sums
// X'1 (column sums) and y'y, from which lm_chol_kernel forms the residual statistics without a second
// pass over X (SSE = y'y - 2 b'X'y + b'X'X b, LM.scala:160-188's three sums; engine.cpp lm_device).
template <int P16, int FAM, int LNK, bool IRLS, bool STATS = false, bool T4 = false, bool LMX = false>
__global__ void __launch_bounds__(64 * NGeo<P16>::NW, 1) irls_narrow_kernel(PassArgs a) {
  using G = NGeo<P16>;
  using VM = VmCount<P16>;
  constexpr int NRB = G::NRB, LPR = G::LPR, CPL = G::NC / LPR;  // row stage: columns per lane
  // Poisson: per-row functions of the count y tabulated in LDS after the waves' images -- the
  // initial pass's unit deviance at mu0 and lgamma(y + 1) (rowmath.hpp poisson_init_table), the
  // IRLS passes' y log y (poisson_ylogy_table, pass_row ylogy)
  constexpr bool PTAB = !IRLS && FAM == FAM_POISSON && (G::LDS + 2 * POIS_TAB + 8) * 8 <= 160 * 1024;
  constexpr bool YTAB = IRLS && FAM == FAM_POISSON && (G::LDS + POIS_TAB) * 8 <= 160 * 1024;
  static_assert(FAM != FAM_POISSON || PTAB || YTAB, "the Poisson tables fit every narrow variant's LDS");
  __shared__ double lds[G::LDS + (PTAB ? 2 * POIS_TAB + 8 : (YTAB ? POIS_TAB : 0))];
  const int lane = threadIdx.x & 63;
  const int wv = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  double* wl = lds + wv * G::WAVE_LDS;
  double* ptab = lds + G::LDS;     // PTAB: [2][POIS_TAB]; YTAB: [POIS_TAB]
  double* pconst = ptab + 2 * POIS_TAB;  // init_const (PTAB)
  const double* ylogy = YTAB ? ptab : nullptr;
  if constexpr (YTAB) {
    for (int k = threadIdx.x; k < POIS_TAB; k += 64 * G::NW) poisson_ylogy_table(ptab, k);
    __syncthreads();
  }
  if constexpr (PTAB) {
    for (int k = threadIdx.x; k < POIS_TAB; k += 64 * G::NW) poisson_init_table(ptab, a.mu0, k);
    if (threadIdx.x == 0) {
      const InitConst ic = init_const(FAM, LNK, a.mode, a.mu0);
      for (int k = 0; k < 6; ++k) pconst[k] = ic.v[k];
    }
    __syncthreads();
  }

  const int64_t nb = a.nblocks * (RB / NRB);  // NRB-row blocks (n_pad = nblocks * RB)
  const int64_t gw = (int64_t)blockIdx.x * G::NW + wv, nwt = (int64_t)gridDim.x * G::NW;
  const int64_t b0 = nb * gw / nwt, b1 = nb * (gw + 1) / nwt;
  const int ngrp_stored = ((a.p + 7) / 8 * 8) / G::CPI;  // X stores whole column octets
  constexpr bool irls = IRLS;
  const int mode = IRLS ? (int)MODE_IRLS : a.mode;
  const bool has_eta = irls && !STATS && a.eta_out != nullptr;
  // the initial pass of a Poisson / Gamma fit sums the in-pass statistics' constants (S_AUX2)
  constexpr bool INIT_CONST = !IRLS && (FAM == FAM_POISSON || FAM == FAM_GAMMA);
  static_assert(!LMX || (!IRLS && !STATS && FAM == FAM_GAUSSIAN), "LMX: the LM Gram pass");
  constexpr bool XS = STATS || INIT_CONST || LMX;  // the extra scalar accumulators are live
  using SL = StatsSlots<FAM>;

  // per-lane parts of the DMA source addresses: lane -> (column cc of the group, row pair j);
  // the swizzle repeats every LPER column groups
  int64_t loff[G::LPER];
  {
    const int cc = lane / (NRB / 2), j = lane % (NRB / 2);
#pragma unroll
    for (int o = 0; o < G::LPER; ++o) loff[o] = (int64_t)cc * a.ld + ((2 * j) ^ swz<NRB>(G::CPI * o + cc));
  }
  const double* vsrc;
  {
    const int v = (lane / (NRB / 2)) & 3;  // 0 y, 1 m, 2 offset, 3 prior (absent: y again)
    const double* p = a.y;
    if (v == 1 && a.m) p = a.m;
    if (v == 2 && a.off) p = a.off;
    if (v == 3 && a.prior) p = a.prior;
    vsrc = p + 2 * (lane % (NRB / 2));
  }
  // row stage: lane (g, rl), g < LPR, covers columns LPR*u + g of row rl
  const int g = lane / NRB, rl = lane % NRB;
  double bcol[CPL];
#pragma unroll
  for (int u = 0; u < CPL; ++u) {
    const int c = LPR * u + g;
    bcol[u] = (a.beta && c < a.p) ? a.beta[c] : 0.0;
  }

  d4 acc[G::T];
#pragma unroll
  for (int t = 0; t < G::T; ++t) acc[t] = d4{0.0, 0.0, 0.0, 0.0};
  double xz[P16], x1[P16];
#pragma unroll
  for (int b = 0; b < P16; ++b) xz[b] = 0.0;
  if constexpr (LMX)
#pragma unroll
    for (int b = 0; b < P16; ++b) x1[b] = 0.0;
  double s_dev = 0.0, s_aux = 0.0, s_pear = 0.0, s_ll = 0.0, s_bad = 0.0;

  const int cl = lane & 15, rq = lane >> 4;
  const int fcl = swz<NRB>(cl);  // f(16b + cl) does not depend on b
  const bool do_gram = !a.no_gram;
  // Cache policy of the design stream: non-temporal in the IRLS passes (a large shard streamed once
  // per pass), the default in the LM Gram pass and the initial pass, whose X the next pass re-reads --
  // at configs[0]'s 1M x 20 (160 MB) the LM residual pass finds it in the Infinity Cache (31.3 us
  // against 36.7 us after a non-temporal Gram pass)
  constexpr int DAUX = IRLS ? DMA_NT : 0;  // (spelled out in stage_next)

  if (b0 < b1) nstage<P16, DAUX>(wl, 0, a, b0, ngrp_stored, loff, vsrc, lane);
  if (b0 + 1 < b1) nstage<P16, DAUX>(wl, 1, a, b0 + 1, ngrp_stored, loff, vsrc, lane);

  // The blocks alternate the two buffers, so the loops take them in pairs with the buffer a
  // compile-time constant: every LDS address is a per-lane base fixed for the kernel plus an immediate
  // offset (the compiler had formed the eta reads' swizzled addresses with one v_add3 per read and
  // block), and the DMA keeps one 64-bit source pointer per swizzle class, advanced once per block (it
  // had carried two 64-bit adds per column group and block).
  // eta reads: lane (g, rl), column c = LPR u + g at (c >> 4) BSTR + (c & 15) NRB + (rl ^ swz(c)); for
  // u = EC j + k the lane part depends on k only, j moves by BSTR (immediate)
  constexpr int EC = 16 / LPR;
  int eoff[EC];
#pragma unroll
  for (int k = 0; k < EC; ++k) {
    const int c = LPR * k + g;
    eoff[k] = (c & 15) * NRB + (rl ^ swz<NRB>(c));
  }
  // Gram operand reads: lane (rq, cl) reads row 4 s + rq of column 16 b + cl
  int goff[NRB / 4];
#pragma unroll
  for (int s = 0; s < NRB / 4; ++s) goff[s] = cl * NRB + ((4 * s + rq) ^ fcl);
  // DMA sources of the next block to stage (blocks are staged in order, b0 + 2 onwards): one 64-bit
  // pointer per swizzle class, the column group's offset added per instruction from SGPRs
  const double* dsrc[G::LPER];
#pragma unroll
  for (int o = 0; o < G::LPER; ++o) dsrc[o] = a.X + (b0 + 2) * NRB + loff[o];
  const double* vnext = vsrc + (b0 + 2) * NRB;
  auto stage_next = [&](auto bufc) {
    constexpr int BUFI = decltype(bufc)::value;
    double* dst = wl + BUFI * G::BUF;
    // the column groups' offsets are formed here on the scalar unit (an opaque copy of the stride keeps
    // the compiler from hoisting all of them out of the loop into SGPRs, which then spilled)
    int64_t cs = (int64_t)G::CPI * a.ld;
    asm volatile("" : "+s"(cs));
    int64_t co = 0;
#pragma unroll
    for (int o = 0; o < VM::DMA_X; ++o) {
      if (o > 0 && o < ngrp_stored) co += cs;  // uniform: groups past the stored columns repeat the last
      __builtin_amdgcn_global_load_lds((const void*)(dsrc[o % G::LPER] + co),
                                       (lds_void*)(dst + (o * G::CPI / 16) * G::BSTR + (o * G::CPI % 16) * NRB), 16, 0, IRLS ? DMA_NT : 0);
    }
#pragma unroll
    for (int o = 0; o < G::LPER; ++o) dsrc[o] += NRB;
    if (G::NRB == 32 || lane < 2 * NRB) __builtin_amdgcn_global_load_lds((const void*)vnext, (lds_void*)(dst + G::XB), 16, 0, IRLS ? DMA_NT : 0);
    vnext += NRB;
  };
  // eta: every LDS read of the row's columns issued before the first FMA (the scheduler had
  // interleaved them one read, one wait, one FMA -- CPL dependent LDS round trips per block)
  auto eta_of = [&](const double* xs) {
    double e4[4] = {0.0, 0.0, 0.0, 0.0};
    double xv[CPL];
#pragma unroll
    for (int u = 0; u < CPL; ++u) xv[u] = xs[eoff[u % EC] + (u / EC) * G::BSTR];
    __builtin_amdgcn_sched_barrier(0);
#pragma unroll
    for (int u = 0; u < CPL; ++u) e4[u & 3] += xv[u] * bcol[u];
    double e = (e4[0] + e4[1]) + (e4[2] + e4[3]);
    if constexpr (LPR == 4) e = xor16_sum(e);
    if constexpr (LPR >= 2) e = xor32_sum(e);
    return e;
  };
  // a block's m / offset / prior slots always hold data (absent vectors: y again, nstage), so they are
  // read unconditionally and selected: no scalar branch per value between the row stage's LDS reads
  const bool hm = a.m != nullptr, ho = a.off != nullptr, hp = a.prior != nullptr;
  auto rowv = [&](const double* vv, int k, bool present, double dflt) {
    const double v = vv[k * NRB + rl];
    return present ? v : dflt;
  };

  if constexpr (G::PAIR) {
    constexpr int KS = NRB / 4;
    // Row pairs (NRB = 32, p <= 32): the family arithmetic would run on 32 of the wave's 64 lanes.
    // The first block of a pair leaves its eta, row values and Gram operands in registers and
    // releases its buffer at once; with the second block the family arithmetic covers both blocks'
    // rows on all 64 lanes (lanes 32..63: the first block), then both blocks' MFMAs run from
    // registers, the first block's first.
    auto pair_blocks = [&](int64_t blk) {
      double xp[KS][P16];  // the first block's Gram operands (lane (rq, cl): row 4s + rq, column 16b + cl)
      double eta_p = 0.0, y_p, m_p, off_p, pw_p;
      __builtin_amdgcn_s_setprio(PRIO_ROWS);
      // the first block landed; younger than its DMA (issued in the last pair's first half): the
      // last pair's eta store and the second block's DMA (the first pair: that DMA only)
      if (has_eta && blk > b0) wait_vm<VM::younger(1, 1)>();
      else wait_vm<VM::younger(1, 0)>();
      {
        const double* xs = wl;
        const double* vv = xs + G::XB;
        if (irls) eta_p = eta_of(xs);
        y_p = vv[rl];
        m_p = rowv(vv, 1, hm, 1.0);
        off_p = rowv(vv, 2, ho, 0.0);
        pw_p = rowv(vv, 3, hp, 1.0);
        if (irls) eta_p = eta_p + off_p;
#pragma unroll
        for (int k = 0; k < KS; ++k)
#pragma unroll
          for (int b = 0; b < P16; ++b) xp[k][b] = xs[goff[k] + G::BSTR * b];
        asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
        if (blk + 2 < b1) stage_next(std::integral_constant<int, 0>{});
      }
      // the second block landed; younger than its DMA: block blk + 2's (issued above)
      if (blk + 2 < b1) wait_vm<VM::younger(1, 0)>();
      else wait_vm<0>();
      const double* xs = wl + G::BUF;
      const double* vv = xs + G::XB;
      double eta = irls ? eta_of(xs) : 0.0;
      const double yv = vv[rl];
      const double mv = rowv(vv, 1, hm, 1.0);
      const double ov = rowv(vv, 2, ho, 0.0);
      const double pv = rowv(vv, 3, hp, 1.0);
      if (irls) eta = eta + ov;
      // family arithmetic: lanes [0, 32) this block's row rl, lanes [32, 64) the first block's
      const bool hi = lane >= NRB;
      const int64_t row = hi ? blk * NRB + rl : (blk + 1) * NRB + rl;
      double w = 0.0, wz = 0.0;
      {
        const double et = hi ? eta_p : eta;
        if (irls && has_eta) a.eta_out[row] = et;
        if (row < a.n) {
          const double y = hi ? y_p : yv, m = hi ? m_p : mv, off = hi ? off_p : ov, pw = hi ? pw_p : pv;
          if constexpr (STATS)
            pass_row_stats<FAM>(et, y, off, pw, w, wz, s_dev, s_aux, s_pear, s_ll, s_bad, true, ylogy);
          else if (!(PTAB && poisson_init_row(pconst, ptab, y, off, pw, w, wz, s_dev, s_aux, s_ll))) {
            pass_row(FAM, LNK, mode, et, y, m, off, pw, a.mu0, a.ybar, a.m != nullptr, w, wz, s_dev, s_aux, true,
                     !IRLS, ylogy);
            if constexpr (LMX) s_pear += y * y;
            if constexpr (INIT_CONST)
              if (mode != MODE_LM_GRAM) s_ll += init_stats_const<FAM>(y, pw);
          }
        }
      }
      // w / w*z at [half * NRB + rl]: the first block in the upper half
      wl[G::OFF_W + lane] = w;
      wl[G::OFF_W + 2 * NRB + lane] = wz;
      // this block's Gram operands into registers, then release the buffer
      double xc[KS][P16];
#pragma unroll
      for (int k = 0; k < KS; ++k)
#pragma unroll
        for (int b = 0; b < P16; ++b) xc[k][b] = xs[goff[k] + G::BSTR * b];
      asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
      if (blk + 3 < b1) stage_next(std::integral_constant<int, 1>{});
      __builtin_amdgcn_s_setprio(PRIO_GRAM);
      if (do_gram) {
        // rows in order: the first block (upper-half w), then this one
#pragma unroll
        for (int h = 0; h < 2; ++h) {
#pragma unroll
          for (int k = 0; k < KS; ++k) {
            const int r = 4 * k + rq + (h == 0 ? NRB : 0);
            const double wr = wl[G::OFF_W + r], wzr = wl[G::OFF_W + 2 * NRB + r];
            double av[P16], xk[P16];
#pragma unroll
            for (int b = 0; b < P16; ++b) {
              xk[b] = h == 0 ? xp[k][b] : xc[k][b];
              av[b] = xk[b] * wr;
              xz[b] += xk[b] * wzr;
              if constexpr (LMX) x1[b] += xk[b];
            }
            gram_kstep<P16, T4>(acc, av, xk);
          }
        }
      }
    };
    // the range's last block when it has no partner: the family arithmetic on lanes [0, 32)
    auto single_block = [&](int64_t blk) {
      __builtin_amdgcn_s_setprio(PRIO_ROWS);
      wait_vm<0>();
      const double* xs = wl;
      const double* vv = xs + G::XB;
      double eta = irls ? eta_of(xs) : 0.0;
      const double yv = vv[rl];
      const double mv = rowv(vv, 1, hm, 1.0);
      const double ov = rowv(vv, 2, ho, 0.0);
      const double pv = rowv(vv, 3, hp, 1.0);
      if (irls) eta = eta + ov;
      double w = 0.0, wz = 0.0;
      if (lane < NRB) {
        const int64_t row = blk * NRB + rl;
        if (irls && has_eta) a.eta_out[row] = eta;
        if (row < a.n) {
          if constexpr (STATS)
            pass_row_stats<FAM>(eta, yv, ov, pv, w, wz, s_dev, s_aux, s_pear, s_ll, s_bad, true, ylogy);
          else if (!(PTAB && poisson_init_row(pconst, ptab, yv, ov, pv, w, wz, s_dev, s_aux, s_ll))) {
            pass_row(FAM, LNK, mode, eta, yv, mv, ov, pv, a.mu0, a.ybar, a.m != nullptr, w, wz, s_dev, s_aux, true,
                     !IRLS, ylogy);
            if constexpr (LMX) s_pear += yv * yv;
            if constexpr (INIT_CONST)
              if (mode != MODE_LM_GRAM) s_ll += init_stats_const<FAM>(yv, pv);
          }
        }
      }
      wl[G::OFF_W + lane] = w;
      wl[G::OFF_W + 2 * NRB + lane] = wz;
      __builtin_amdgcn_s_setprio(PRIO_GRAM);
      if (do_gram) {
#pragma unroll
        for (int k = 0; k < KS; ++k) {
          const int r = 4 * k + rq;
          const double wr = wl[G::OFF_W + r], wzr = wl[G::OFF_W + 2 * NRB + r];
          double av[P16], xk[P16];
#pragma unroll
          for (int b = 0; b < P16; ++b) {
            xk[b] = xs[goff[k] + G::BSTR * b];
            av[b] = xk[b] * wr;
            xz[b] += xk[b] * wzr;
            if constexpr (LMX) x1[b] += xk[b];
          }
          gram_kstep<P16, T4>(acc, av, xk);
        }
      }
    };
    int64_t blk = b0;
#pragma unroll 1
    for (; blk + 1 < b1; blk += 2) pair_blocks(blk);
    if (blk < b1) single_block(blk);
  } else {
  auto block = [&](auto bufc, int64_t blk) {
    constexpr int BUFI = decltype(bufc)::value;
    __builtin_amdgcn_s_setprio(PRIO_ROWS);
    // block blk landed; younger than its DMA: block blk + 1's and the previous block's eta store
    if (blk + 1 >= b1) wait_vm<0>();
    else if (has_eta && blk > b0) wait_vm<VM::younger(1, 1)>();
    else wait_vm<VM::younger(1, 0)>();
    const double* xs = wl + BUFI * G::BUF;

    // ---- row stage ----
    double eta = irls ? eta_of(xs) : 0.0;
    if (lane < NRB) {
      const double* vv = xs + G::XB;
      const int64_t row = blk * NRB + rl;
      double w = 0.0, wz = 0.0;
      if (irls) {
        eta = eta + rowv(vv, 2, ho, 0.0);
        if (has_eta) a.eta_out[row] = eta;  // always issued (row < n_pad): keeps vmcnt exact
      }
      if (row < a.n) {
        const double y = vv[rl];
        const double m = rowv(vv, 1, hm, 1.0);
        const double off = rowv(vv, 2, ho, 0.0);
        const double pw = rowv(vv, 3, hp, 1.0);
        if constexpr (STATS)
          pass_row_stats<FAM>(eta, y, off, pw, w, wz, s_dev, s_aux, s_pear, s_ll, s_bad, true, ylogy);
        else if (!(PTAB && poisson_init_row(pconst, ptab, y, off, pw, w, wz, s_dev, s_aux, s_ll))) {
          pass_row(FAM, LNK, mode, eta, y, m, off, pw, a.mu0, a.ybar, a.m != nullptr, w, wz, s_dev, s_aux, true,
                   !IRLS, ylogy);
          if constexpr (LMX) s_pear += y * y;
          if constexpr (INIT_CONST)
            if (mode != MODE_LM_GRAM) s_ll += init_stats_const<FAM>(y, pw);
        }
      }
      wl[G::OFF_W + rl] = w;
      wl[G::OFF_W + NRB + rl] = wz;
    }

    // ---- Gramian: NRB/4 k-steps of 4 rows ----
    __builtin_amdgcn_s_setprio(PRIO_GRAM);
    if (do_gram) {
#pragma unroll
      for (int s = 0; s < NRB / 4; ++s) {
        const int r = 4 * s + rq;
        const double wr = wl[G::OFF_W + r], wzr = wl[G::OFF_W + NRB + r];
        double xv[P16], av[P16];
#pragma unroll
        for (int b = 0; b < P16; ++b) {
          xv[b] = xs[goff[s] + G::BSTR * b];
          av[b] = xv[b] * wr;
          xz[b] += xv[b] * wzr;
          if constexpr (LMX) x1[b] += xv[b];
        }
        gram_kstep<P16, T4>(acc, av, xv);
      }
    }
    // every LDS read of this buffer has returned before the DMA may overwrite it
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    if (blk + 2 < b1) stage_next(bufc);
  };
  // Block pairs: the family arithmetic ran on 16 of the wave's 64 lanes (ablation: ~3 ms of a 15 ms
  // p = 64 pass).  Both blocks of a pair are formed first -- eta of the first block, its row values
  // kept in registers, eta of the second -- then the family arithmetic covers both blocks' rows on 32
  // lanes (lanes 16..31: the first block), then the two Grams, the first block's first (the rows in
  // the same order as block by block).  Unlike the p <= 32 loop the first block's Gram operands are
  // not stashed in registers (at P16 = 4 they do not fit beside the accumulators): its buffer is
  // released after its Gram, so block blk + 2's DMA flies under the second block's Gram only.
  auto pair_blocks = [&](int64_t blk) {
    __builtin_amdgcn_s_setprio(PRIO_ROWS);
    // the first block landed, the second may fly.  The last pair's eta store was issued before both
    // blocks' DMAs (in its row stage, ahead of the Grams), so it is older than the first block's and
    // must not be counted as in flight: with younger(1, 1) the first block's row-vector DMA (y, offset,
    // prior) could still be landing while the row stage read it (a run-to-run difference of ~1e-6
    // in the Poisson / Gaussian passes at p > 32, tests/test_gpu_determinism.py)
    wait_vm<VM::younger(1, 0)>();
    double eta_p = 0.0, y_p, m_p, off_p, pw_p;
    {
      const double* xs = wl;
      if (irls) eta_p = eta_of(xs);
      const double* vv = xs + G::XB;
      y_p = vv[rl];
      m_p = rowv(vv, 1, hm, 1.0);
      off_p = rowv(vv, 2, ho, 0.0);
      pw_p = rowv(vv, 3, hp, 1.0);
      if (irls) eta_p = eta_p + off_p;
    }
    wait_vm<0>();  // the second block landed
    const double* xs1 = wl + G::BUF;
    double eta = irls ? eta_of(xs1) : 0.0;
    if (lane < 2 * NRB) {
      // lanes [0, 16): the second block's row rl; lanes [16, 32): the first block's row rl
      const bool hi = lane >= NRB;
      const double* vv = xs1 + G::XB;
      const int64_t row = hi ? blk * NRB + rl : (blk + 1) * NRB + rl;
      double et = eta_p, y = y_p, m = m_p, off = off_p, pw = pw_p;
      if (!hi) {
        y = vv[rl];
        m = rowv(vv, 1, hm, 1.0);
        off = rowv(vv, 2, ho, 0.0);
        pw = rowv(vv, 3, hp, 1.0);
        et = irls ? eta + off : eta;
      }
      if (irls && has_eta) a.eta_out[row] = et;  // one store for the pair (row < n_pad)
      double w = 0.0, wz = 0.0;
      if (row < a.n) {
        if constexpr (STATS)
          pass_row_stats<FAM>(et, y, off, pw, w, wz, s_dev, s_aux, s_pear, s_ll, s_bad, true, ylogy);
        else if (!(PTAB && poisson_init_row(pconst, ptab, y, off, pw, w, wz, s_dev, s_aux, s_ll))) {
          pass_row(FAM, LNK, mode, et, y, m, off, pw, a.mu0, a.ybar, a.m != nullptr, w, wz, s_dev, s_aux, true,
                   !IRLS, ylogy);
          if constexpr (LMX) s_pear += y * y;
          if constexpr (INIT_CONST)
            if (mode != MODE_LM_GRAM) s_ll += init_stats_const<FAM>(y, pw);
        }
      }
      wl[G::OFF_W + lane] = w;
      wl[G::OFF_W + 2 * NRB + lane] = wz;
    }
    // the two Grams: the first block's rows (w at [16, 32)), then the second's
    auto gram = [&](auto bufc, int woff) {
      constexpr int BUFI = decltype(bufc)::value;
      const double* xs = wl + BUFI * G::BUF;
#pragma unroll
      for (int s2 = 0; s2 < NRB / 4; ++s2) {
        const int r = 4 * s2 + rq + woff;
        const double wr = wl[G::OFF_W + r], wzr = wl[G::OFF_W + 2 * NRB + r];
        double xv[P16], av[P16];
#pragma unroll
        for (int b = 0; b < P16; ++b) {
          xv[b] = xs[goff[s2] + G::BSTR * b];
          av[b] = xv[b] * wr;
          xz[b] += xv[b] * wzr;
          if constexpr (LMX) x1[b] += xv[b];
        }
        gram_kstep<P16, T4>(acc, av, xv);
      }
      asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");  // every read of the buffer returned
    };
    __builtin_amdgcn_s_setprio(PRIO_GRAM);
    if (do_gram) gram(std::integral_constant<int, 0>{}, NRB);
    else asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    if (blk + 2 < b1) stage_next(std::integral_constant<int, 0>{});
    if (do_gram) gram(std::integral_constant<int, 1>{}, 0);
    else asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    if (blk + 3 < b1) stage_next(std::integral_constant<int, 1>{});
  };
  int64_t blk = b0;
#pragma unroll 1
  for (; blk + 1 < b1; blk += 2) pair_blocks(blk);
  // the range's last block has no partner (outside the loop: inside it, the single-block path beside
  // the pair path made the compiler spill at P16 = 4)
  if (blk < b1) block(std::integral_constant<int, 0>{}, blk);
  }  // !PAIR

  // ---- wave partial: X'Wz over the 4 row lanes of each column, scalars over the wave ----
#pragma unroll
  for (int b = 0; b < P16; ++b) xz[b] = xor32_sum(xor16_sum(xz[b]));
  if constexpr (LMX)
#pragma unroll
    for (int b = 0; b < P16; ++b) x1[b] = xor32_sum(xor16_sum(x1[b]));
#pragma unroll
  for (int o = 1; o < 64; o <<= 1) {
    s_dev += __shfl_xor(s_dev, o);
    s_aux += __shfl_xor(s_aux, o);
    if constexpr (XS) {
      s_pear += __shfl_xor(s_pear, o);
      s_ll += __shfl_xor(s_ll, o);
      s_bad += __shfl_xor(s_bad, o);
    }
  }

  // ---- fixed-order fold over the NW waves in LDS: while n > 1, waves [h, n) (h = ceil(n/2))
  // hand their partials to waves [0, n - h) (NW = 8: ((w0+w4)+(w2+w6)) + ((w1+w5)+(w3+w7))) ----
  wait_vm<0>();
  __syncthreads();
#pragma unroll 1
  for (int n = G::NW; n > 1;) {
    const int h = (n + 1) / 2;
    if (wv >= h && wv < n) {
      double* reg = lds + (wv - h) * G::PSZ;
#pragma unroll
      for (int t = 0; t < G::T; ++t)
#pragma unroll
        for (int j = 0; j < 4; ++j) reg[t * 256 + 64 * j + lane] = acc[t][j];
      if (lane < 16) {
#pragma unroll
        for (int b = 0; b < P16; ++b) reg[G::T * 256 + 16 * b + lane] = xz[b];
        if constexpr (LMX)
#pragma unroll
          for (int b = 0; b < P16; ++b) reg[G::T * 256 + G::NC + 5 + 16 * b + lane] = x1[b];
      }
      if (lane == 0) {
        reg[G::T * 256 + G::NC] = s_dev;
        reg[G::T * 256 + G::NC + 1] = s_aux;
        reg[G::T * 256 + G::NC + 2] = s_pear;
        reg[G::T * 256 + G::NC + 3] = s_ll;
        reg[G::T * 256 + G::NC + 4] = s_bad;
      }
    }
    __syncthreads();
    if (wv < n - h) {
      const double* reg = lds + wv * G::PSZ;
#pragma unroll
      for (int t = 0; t < G::T; ++t)
#pragma unroll
        for (int j = 0; j < 4; ++j) acc[t][j] += reg[t * 256 + 64 * j + lane];
#pragma unroll
      for (int b = 0; b < P16; ++b) xz[b] += reg[G::T * 256 + 16 * b + (lane & 15)];
      if constexpr (LMX)
#pragma unroll
        for (int b = 0; b < P16; ++b) x1[b] += reg[G::T * 256 + G::NC + 5 + 16 * b + (lane & 15)];
      s_dev += reg[G::T * 256 + G::NC];
      s_aux += reg[G::T * 256 + G::NC + 1];
      if constexpr (XS) {
        s_pear += reg[G::T * 256 + G::NC + 2];
        s_ll += reg[G::T * 256 + G::NC + 3];
        s_bad += reg[G::T * 256 + G::NC + 4];
      }
    }
    __syncthreads();
    n = h;
  }
  if (wv == 0) {
    double* out = a.partials + (int64_t)blockIdx.x * a.stride;
    int t = 0;
#pragma unroll
    for (int bi = 0; bi < P16; ++bi)
#pragma unroll
      for (int bj = 0; bj <= bi; ++bj, ++t) {
#pragma unroll
        for (int j = 0; j < 4; ++j) out[t * 256 + 64 * j + lane] = acc[t][j];
      }
    if (lane < 16) {
#pragma unroll
      for (int b = 0; b < P16; ++b) out[G::T * 256 + 16 * b + lane] = xz[b];
      if constexpr (LMX)
#pragma unroll
        for (int b = 0; b < P16; ++b) out[G::T * 256 + G::NC + NS + 16 * b + lane] = x1[b];
    }
    if (lane < NS) {
      double v = lane == S_DEV ? s_dev : lane == S_SUMW ? s_aux : 0.0;
      if constexpr (STATS) {
        if (lane == SL::S2) v = s_pear;
        if (lane == SL::S3) v = s_ll;
        if (lane == SL::S4) v = s_bad;
      }
      if constexpr (INIT_CONST) {
        if (lane == S_AUX2) v = s_ll;
      }
      if constexpr (LMX) {
        if (lane == S_PEARSON) v = s_pear;  // y'y
      }
      out[G::T * 256 + G::NC + lane] = v;
    }
  }
}

template <int P16, int FAM, int LNK>
void launch_narrow_fl(const PassArgs& a, dim3 gr, dim3 bl, hipStream_t st, hipEvent_t e0, hipEvent_t e1) {
  constexpr bool SP = stats_in_pass_family(FAM, LNK);
  if constexpr (FAM == FAM_GAUSSIAN) {  // the LM Gram of the one-round-trip LM.fit: X'1 and y'y too
    if (a.mode == MODE_LM_GRAM && a.lm_extras) {
      if (P16 == 2 && a.p <= 20)
        hipExtLaunchKernelGGL((irls_narrow_kernel<P16, FAM, LNK, false, false, P16 == 2, true>), gr, bl, 0, st, e0, e1,
                              0, a);
      else
        hipExtLaunchKernelGGL((irls_narrow_kernel<P16, FAM, LNK, false, false, false, true>), gr, bl, 0, st, e0, e1, 0,
                              a);
      return;
    }
  }
  if constexpr (P16 == 2 && FAM == FAM_GAUSSIAN) {  // LM Gram / gaussian at p <= 20 (gram_kstep T4)
    if (a.p <= 20) {
      if (a.mode == MODE_IRLS)
        hipExtLaunchKernelGGL((irls_narrow_kernel<P16, FAM, LNK, true, false, true>), gr, bl, 0, st, e0, e1, 0, a);
      else
        hipExtLaunchKernelGGL((irls_narrow_kernel<P16, FAM, LNK, false, false, true>), gr, bl, 0, st, e0, e1, 0, a);
      return;
    }
  }
  if (a.mode == MODE_IRLS && SP && a.stats_in_pass && !(FAM == FAM_BINOMIAL && a.m))
    hipExtLaunchKernelGGL((irls_narrow_kernel<P16, FAM, LNK, true, SP>), gr, bl, 0, st, e0, e1, 0, a);
  else if (a.mode == MODE_IRLS)
    hipExtLaunchKernelGGL((irls_narrow_kernel<P16, FAM, LNK, true>), gr, bl, 0, st, e0, e1, 0, a);
  else
    hipExtLaunchKernelGGL((irls_narrow_kernel<P16, FAM, LNK, false>), gr, bl, 0, st, e0, e1, 0, a);
}

template <int P16>
hipError_t launch_narrow_p(const PassArgs& a, int grid, hipStream_t st, hipEvent_t e0, hipEvent_t e1) {
  const dim3 gr(grid), bl(64 * NGeo<P16>::NW);
  const int fam = (a.mode == MODE_LM_GRAM) ? FAM_GAUSSIAN : a.family;
  const int lnk = (a.mode == MODE_LM_GRAM) ? LNK_IDENTITY : a.link;
  if (fam == FAM_BINOMIAL && lnk == LNK_LOGIT)
    launch_narrow_fl<P16, FAM_BINOMIAL, LNK_LOGIT>(a, gr, bl, st, e0, e1);
  else if (fam == FAM_BINOMIAL && lnk == LNK_PROBIT)
    launch_narrow_fl<P16, FAM_BINOMIAL, LNK_PROBIT>(a, gr, bl, st, e0, e1);
  else if (fam == FAM_BINOMIAL)
    launch_narrow_fl<P16, FAM_BINOMIAL, LNK_CLOGLOG>(a, gr, bl, st, e0, e1);
  else if (fam == FAM_GAUSSIAN)
    launch_narrow_fl<P16, FAM_GAUSSIAN, LNK_IDENTITY>(a, gr, bl, st, e0, e1);
  else if (fam == FAM_POISSON)
    launch_narrow_fl<P16, FAM_POISSON, LNK_LOG>(a, gr, bl, st, e0, e1);
  else if (fam == FAM_GAMMA)
    launch_narrow_fl<P16, FAM_GAMMA, LNK_INVERSE>(a, gr, bl, st, e0, e1);
  else
    return hipErrorInvalidValue;
  return hipGetLastError();
}

}  // namespace

int narrow_variant(int p) { return (p + 15) / 16; }
int narrow_stride(int P16) { return (P16 * (P16 + 1) / 2) * 256 + 16 * P16 + NS + 16 * P16; }  // NGeo::STRIDE
int narrow_wg_per_cu() { return 1; }
int narrow_rows_per_wg(int P16) {
  switch (P16) {
    case 1: return NGeo<1>::NRB * NGeo<1>::NW;
    case 2: return NGeo<2>::NRB * NGeo<2>::NW;
    case 3: return NGeo<3>::NRB * NGeo<3>::NW;
    default: return NGeo<4>::NRB * NGeo<4>::NW;
  }
}

hipError_t launch_narrow(int P16, const PassArgs& a, int grid, hipStream_t st, hipEvent_t e0, hipEvent_t e1) {
  switch (P16) {
    case 1: return launch_narrow_p<1>(a, grid, st, e0, e1);
    case 2: return launch_narrow_p<2>(a, grid, st, e0, e1);
    case 3: return launch_narrow_p<3>(a, grid, st, e0, e1);
    case 4: return launch_narrow_p<4>(a, grid, st, e0, e1);
    default: return hipErrorInvalidValue;
  }
}

}  // namespace sglm
