// narrow_r.hip -- the split-role narrow IRLS pass for 17 <= p <= 64 (P16 = 2..4) on gfx950.
//
// irls_narrow_kernel (narrow.hip) runs every role on every wave: each wave streams its own 16-row
// blocks, forms eta on 4 lanes per row, runs the family arithmetic on 16 of its 64 lanes and the
// whole lower-triangular Gram on fp64 MFMA.  At p = 64 that kernel is bound by the SIMD's fp64
// pipe, which MFMAs and fp64 VALU share: per 16-row block 40 MFMAs (2560 cycles)
// beside ~200 VALU instructions -- the family arithmetic on a quarter of the lanes, the 64-bit
// address arithmetic of ten LDS-DMA pointers and the eta reads' swizzled addresses (PMC: 5.1 VALU
// instructions per MFMA, MFMA busy 64 %, 55 % of HBM).
//
// Here the roles have their own waves (twelve per workgroup, one workgroup per CU, three waves per
// SIMD), on 64-row blocks in a workgroup-shared LDS ring of NB slots:
//   * row waves 8..11 (one per SIMD): the LDS-DMA of the blocks -- each stages a quarter of every
//     block's column pairs plus one of the row vectors, wave-uniform base addresses on the scalar
//     unit and 32-bit lane offsets precomputed once (no per-block VALU address arithmetic) -- and
//     the row stage (etaCreate GLM.scala:321-332, zwCreateBinomial GLM.scala:359-395, the deviance
//     GLM.scala:162-170) of whole blocks, one row per lane: all 64 lanes run the family arithmetic.
//     The row stage of block j is row wave (j - b0) mod 4's, so each SIMD carries one in four;
//   * Gram waves 0..7 (two per SIMD): nothing but their two k-steps of every block -- the whole
//     lower-triangular tile set on v_mfma_f64_16x16x4_f64 with A scaled by w, and X'Wz on the VALU
//     from the same operand registers (partitionComponents, utils.scala:84-92).
// LDS counters order the ring (no block barrier): flag (+1 per row wave per block whose DMA part
// landed -- a barrier among the row waves), ready[s] (row stage of the block in slot s done),
// done[s] (+1 per Gram wave when it has read the block in slot s; the slot is restaged after 8).
// One partial per workgroup in narrow.hip's layout (reduce_partials_kernel): the eight Gram waves'
// tiles folded in LDS in a fixed tree, the row waves' scalars in wave order -- deterministic.
//
// LDS image of a block (slot s): column c of X at c * 64 doubles, row r in position r ^ 2 (c & 15)
// (an XOR of row pairs inside each 32-row half, applied on the DMA source address).  A DMA
// wave-instruction moves 1 KiB: two columns, lane l the row pair l & 31 of column 2q + (l >> 5).
// The eta reads (lane = row, one column) cover a 256-byte bank row per half-wave and the MFMA operand
// reads (lane (rq, cl): row 4k + rq of column 16b + cl) hit 32 distinct 8-byte positions of a bank
// row per half-wave: both conflict free.  Lane offsets of the DMA sources are 32-bit (column pair
// part h ld 8 bytes); a shard of n_pad >= 2^29 rows stages each column of a pair by its own half-wave
// instruction instead (the tall form).
#include <hip/hip_runtime.h>

#include <cstdint>

#include "common.hpp"
#include "kernels.hpp"
#include "rowmath.hpp"

namespace sglm {

namespace {

typedef double d4 __attribute__((ext_vector_type(4)));
typedef __attribute__((address_space(3))) void lds_void;
typedef __attribute__((address_space(3))) double lds_double;

constexpr int SB = 64;  // rows per block (one row per lane in the row stage)

template <int P16>
struct NR {
  static_assert(P16 >= 2 && P16 <= 4, "split-role narrow variants: 17 <= p <= 64");
  static constexpr int NW = 12, NGW = 8, NRW = 4;
  static constexpr int NC = 16 * P16;                    // padded columns
  static constexpr int T = P16 * (P16 + 1) / 2;          // lower-triangular 16x16 tiles
  static constexpr int XB = NC * SB;                     // X image doubles per slot
  static constexpr int NPAIR = NC / 2;                   // DMA wave-instructions of X per block
  static constexpr int PPW = NPAIR / NRW;                // ... per row wave
  static constexpr int VMEM = PPW + 1;                   // vector-memory operations per row wave and block
  static constexpr int VMEM_TALL = 2 * PPW + 1;          // ... on a tall shard (a column per half-wave instruction)
  static constexpr int OFF_V = XB;                       // y | m | offset | prior  [4][SB]
  static constexpr int OFF_W = XB + 4 * SB;              // w | w*z                 [2][SB]
  static constexpr int OFF_E = XB + 6 * SB;              // eta                     [SB]
  static constexpr int PER = XB + 7 * SB;                // doubles per slot
  static constexpr int TAB = 2 * POIS_TAB + 8;           // Poisson tables + init constants
  static constexpr int FIXED = NC + NW * 8 + 16 + TAB;   // beta | wave scalars | counters | tables
  static constexpr int LDS_MAX = 160 * 1024 / 8;
  static constexpr int NB = (LDS_MAX - FIXED) / PER > 8 ? 8 : (LDS_MAX - FIXED) / PER;  // ring slots
  static constexpr int OFF_BETA = NB * PER;
  static constexpr int OFF_RED = OFF_BETA + NC;
  static constexpr int OFF_CNT = OFF_RED + NW * 8;       // uint32: flag | ready[8] | done[8]
  static constexpr int OFF_TAB = OFF_CNT + 16;
  static constexpr int LDS = OFF_TAB + TAB;
  static constexpr int PSZ = T * 256 + NC + 8;           // one Gram wave's partial in the fold
  static_assert(NB >= 3, "ring depth");
  static_assert(LDS * 8 <= 160 * 1024, "LDS budget");
  static_assert((NGW / 2) * PSZ <= NB * PER, "the fold fits the ring");
  static_assert(VMEM_TALL * (NB - 1) < 64, "vmcnt range");
  static_assert(PER % 2 == 0 && XB % 2 == 0, "LDS-DMA destinations 16-byte aligned");
};

template <int N>
__device__ __forceinline__ void wait_vm() {
  static_assert(N >= 0 && N < 64, "vmcnt range");
  __builtin_amdgcn_s_waitcnt((N & 15) | ((N >> 4) << 14) | (7 << 4) | (15 << 8));
}

// wait until the DMA of a block has landed while `later` blocks staged after it may still fly
template <int VM, int NB, int L = NB - 1>
__device__ __forceinline__ void wait_landed(int later) {
  if constexpr (L == 0) {
    wait_vm<0>();
  } else {
    if (later >= L) return wait_vm<L * VM>();
    wait_landed<VM, NB, L - 1>(later);
  }
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

// LDS-DMA of row wave k's part of block blk into slot s: column pairs [k PPW, (k+1) PPW) and row
// vector k (0 y, 1 m, 2 offset, 3 prior; absent vectors re-load y so every block issues VMEM
// operations).  Pairs past the stored columns re-load the last stored pair (finite data; beta is 0
// there and their tiles are discarded).  The wave-uniform part of every source address is formed
// on the scalar unit; voff / vvoff are the lane parts (bytes).
// LDS-DMA through a buffer descriptor built from wave-uniform values: the SGPR base carries the
// column pair and the block (scalar arithmetic), the 32-bit lane offset is a VGPR computed once --
// the global_load_lds form kept one 64-bit VGPR pointer per instruction, advanced every block.
__device__ __forceinline__ void dma16(const void* base, uint32_t voff, lds_double* dst) {
  const __amdgpu_buffer_rsrc_t r = __builtin_amdgcn_make_buffer_rsrc(const_cast<void*>(base), 0, -1, 0x00020000);
  __builtin_amdgcn_raw_ptr_buffer_load_lds(r, (lds_void*)dst, 16, voff, 0, 0, 0);
}

// tall: a shard too tall for the second column's lane offset (n_pad 8 >= 2^32 - 1024) takes each
// column of a pair in its own half-wave instruction (lanes 0..31 / 32..63, the same LDS destination:
// the DMA writes lane-linearly), voff then holding only the row part.
template <int P16>
__device__ __forceinline__ void stage_r(lds_double* l3, int s, const PassArgs& a, const double* vsrc, int64_t blk,
                                        int k, int npair_stored, const uint32_t (&voff)[NR<P16>::PPW], uint32_t vvoff,
                                        int lane, bool tall) {
  using G = NR<P16>;
  lds_double* dst = l3 + s * G::PER;
  const int64_t r0 = blk * SB;
#pragma unroll
  for (int i = 0; i < G::PPW; ++i) {
    const int q = k * G::PPW + i;                                   // LDS column pair
    const int qs = __builtin_amdgcn_readfirstlane(q < npair_stored ? q : npair_stored - 1);
    if (!tall) {
      dma16(a.X + (int64_t)(2 * qs) * a.ld + r0, voff[i], dst + 2 * q * SB);
    } else {
      if (lane < 32) dma16(a.X + (int64_t)(2 * qs) * a.ld + r0, voff[i], dst + 2 * q * SB);
      if (lane >= 32) dma16(a.X + (int64_t)(2 * qs + 1) * a.ld + r0, voff[i], dst + 2 * q * SB);
    }
  }
  if (lane < 32) dma16(vsrc + r0, vvoff, dst + G::OFF_V + k * SB);
}

// One k-step (4 rows) of the lower-triangular Gram on v_mfma_f64_16x16x4_f64.
template <int P16>
__device__ __forceinline__ void gram_kstep(d4 (&acc)[NR<P16>::T], const double (&av)[P16], const double (&xv)[P16]) {
  int t = 0;
#pragma unroll
  for (int bi = 0; bi < P16; ++bi)
#pragma unroll
    for (int bj = 0; bj <= bi; ++bj, ++t) acc[t] = __builtin_amdgcn_mfma_f64_16x16x4f64(av[bi], xv[bj], acc[t], 0, 0, 0);
}

// IRLS / STATS as in irls_narrow_kernel: IRLS = compile-time MODE_IRLS (the init and LM Gram passes
// run the IRLS = false instantiation); STATS: the final statistics in the pass, no eta store.
template <int P16, int FAM, int LNK, bool IRLS, bool STATS = false>
__global__ void __launch_bounds__(64 * NR<P16>::NW, 3) irls_narrow_r_kernel(PassArgs a) {
  using G = NR<P16>;
  constexpr int NB = G::NB;
  __shared__ double lds[G::LDS];
  const int lane = threadIdx.x & 63;
  const int wv = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  lds_double* l3 = (lds_double*)__builtin_amdgcn_readfirstlane((int)(uintptr_t)(lds_void*)lds);

  // Poisson tables (as irls_narrow_kernel): the initial pass's unit deviance at mu0 and lgamma(y + 1),
  // the IRLS passes' y log y
  constexpr bool PTAB = !IRLS && FAM == FAM_POISSON;
  constexpr bool YTAB = IRLS && FAM == FAM_POISSON;
  double* ptab = lds + G::OFF_TAB;
  double* pconst = ptab + 2 * POIS_TAB;
  const double* ylogy = YTAB ? ptab : nullptr;
  unsigned* cnt = (unsigned*)(lds + G::OFF_CNT);
  for (int k = threadIdx.x; k < G::NC; k += 64 * G::NW) lds[G::OFF_BETA + k] = (IRLS && a.beta && k < a.p) ? a.beta[k] : 0.0;
  if (threadIdx.x < 32) cnt[threadIdx.x] = 0u;
  if constexpr (YTAB)
    for (int k = threadIdx.x; k < POIS_TAB; k += 64 * G::NW) poisson_ylogy_table(ptab, k);
  if constexpr (PTAB) {
    for (int k = threadIdx.x; k < POIS_TAB; k += 64 * G::NW) poisson_init_table(ptab, a.mu0, k);
    if (threadIdx.x == 0) {
      const InitConst ic = init_const(FAM, LNK, a.mode, a.mu0);
      for (int k = 0; k < 6; ++k) pconst[k] = ic.v[k];
    }
  }
  __syncthreads();

  const int64_t nb = (a.nblocks * RB + SB - 1) / SB;  // 64-row blocks (the last may hold 32 rows of the image)
  const int64_t b0 = nb * blockIdx.x / gridDim.x, b1 = nb * (blockIdx.x + 1) / gridDim.x;
  const int mode = IRLS ? (int)MODE_IRLS : a.mode;
  const bool do_gram = !a.no_gram;
  constexpr bool INIT_CONST = !IRLS && (FAM == FAM_POISSON || FAM == FAM_GAMMA);
  constexpr bool XS = STATS || INIT_CONST;
  using SL = StatsSlots<FAM>;
  unsigned* flag = cnt;
  unsigned* ready = cnt + 1;
  unsigned* done = cnt + 1 + 8;
  auto spin = [&](unsigned* c, unsigned target) {
    while (__hip_atomic_load(c, __ATOMIC_ACQUIRE, __HIP_MEMORY_SCOPE_WORKGROUP) < target) __builtin_amdgcn_s_sleep(1);
  };
  auto bump = [&](unsigned* c) {
    if (lane == 0) __hip_atomic_fetch_add(c, 1u, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_WORKGROUP);
  };

  // acc / xz: the Gram waves' (left undefined on the row waves, so the row stage does not keep
  // them in registers); the scalars: the row waves'
  d4 acc[G::T];
  double xz[P16];
  double s_dev = 0.0, s_aux = 0.0, s_pear = 0.0, s_ll = 0.0, s_bad = 0.0;

  if (wv >= G::NGW) {
    // ======================= row waves: LDS-DMA + row stage =======================
    const int k = wv - G::NGW;
    const int npair_stored = ((a.p + 7) / 8 * 8) / 2;  // X stores whole column octets
    // lane parts of the DMA source addresses of this wave's column pairs q = k PPW + i: column 2q + h
    // (h = lane >> 5), LDS row pair pp = lane & 31 holds source pair pp ^ ((2q + h) & 15)
    uint32_t voff[G::PPW];
    const int h = lane >> 5, pp = lane & 31;
    const bool tall = a.ld * 8 + 1024 >= ((int64_t)1 << 32);
#pragma unroll
    for (int i = 0; i < G::PPW; ++i)
      voff[i] = (uint32_t)((tall ? 0 : h * a.ld * 8) + 16 * (pp ^ ((2 * (k * G::PPW + i) + h) & 15)));
    uint32_t vvoff = (uint32_t)(16 * pp);
    const double* vsrc = a.y;
    if (k == 1 && a.m) vsrc = a.m;
    if (k == 2 && a.off) vsrc = a.off;
    if (k == 3 && a.prior) vsrc = a.prior;
    // the shard's last block may hold only 32 rows of the image (n_pad = 32 (2 nb - 1)): its upper
    // half re-reads the lower half's rows (finite data; those rows are past n, w = 0)
    const bool short_tail = (int64_t)nb * SB > a.nblocks * RB;
    auto stage = [&](int s, int64_t blk) {
      if (short_tail && blk == nb - 1) {
        uint32_t vt[G::PPW];
#pragma unroll
        for (int i = 0; i < G::PPW; ++i) vt[i] = voff[i] - (pp >= 16 ? 256u : 0u);
        stage_r<P16>(l3, s, a, vsrc, blk, k, npair_stored, vt, vvoff - (pp >= 16 ? 256u : 0u), lane, tall);
      } else {
        stage_r<P16>(l3, s, a, vsrc, blk, k, npair_stored, voff, vvoff, lane, tall);
      }
    };
    const int64_t nblk = b1 - b0;
#pragma unroll 1
    for (int c = 0; c < NB; ++c)
      if (c < nblk) stage(c, b0 + c);
    __builtin_amdgcn_s_setprio(2);

    // row stage of block j (slot s) on this wave, one row per lane
    auto row_stage = [&](int s, int64_t blk) {
      const double* xs = lds + s * G::PER;
      const double* vv = xs + G::OFF_V;
      const int r = lane;
      const int64_t row = blk * SB + r;
      double eta = 0.0;
      if (IRLS) {
        // eta over 16-column chunks (every read of a chunk issued before its FMAs; the scheduling
        // barrier keeps the next chunk's reads from being hoisted, which would need 4 NC registers)
        double e4[4] = {0.0, 0.0, 0.0, 0.0};
        const double* bt = lds + G::OFF_BETA;
#pragma unroll
        for (int c0 = 0; c0 < G::NC; c0 += 16) {
          double xv[16], bv[16];
#pragma unroll
          for (int u = 0; u < 16; ++u) {
            xv[u] = xs[(c0 + u) * SB + (r ^ (2 * u))];
            bv[u] = bt[c0 + u];
          }
#pragma unroll
          for (int u = 0; u < 16; ++u) e4[u & 3] += xv[u] * bv[u];
          // the chunk's sums formed before the next chunk's reads (without this the IR hoists every
          // read of the row stage and the 2 NC values spill)
          asm volatile("" : "+v"(e4[0]), "+v"(e4[1]), "+v"(e4[2]), "+v"(e4[3])::"memory");
        }
        eta = (e4[0] + e4[1]) + (e4[2] + e4[3]);
      }
      const double y = vv[r];
      const double m = a.m ? vv[SB + r] : 1.0;
      const double off = a.off ? vv[2 * SB + r] : 0.0;
      const double pw = a.prior ? vv[3 * SB + r] : 1.0;
      if (IRLS) eta = eta + off;
      double w = 0.0, wz = 0.0;
      if (row < a.n) {
        if constexpr (STATS)
          pass_row_stats<FAM>(eta, y, off, pw, w, wz, s_dev, s_aux, s_pear, s_ll, s_bad, true, ylogy);
        else if (!(PTAB && poisson_init_row(pconst, ptab, y, off, pw, w, wz, s_dev, s_aux, s_ll))) {
          pass_row(FAM, LNK, mode, eta, y, m, off, pw, a.mu0, a.ybar, a.m != nullptr, w, wz, s_dev, s_aux, true, !IRLS,
                   ylogy);
          if constexpr (INIT_CONST)
            if (mode != MODE_LM_GRAM) s_ll += init_stats_const<FAM>(y, pw);
        }
      }
      double* wd = lds + s * G::PER + G::OFF_W;
      wd[r] = w;
      wd[SB + r] = wz;
      lds[s * G::PER + G::OFF_E + r] = eta;
    };

    // block i = blk - b0 sits in slot i mod NB; its row stage runs on row wave i mod 4, one block
    // ahead of the Gram.  Before iteration i's restage, blocks 0 .. i + NB - 1 have been issued.
    if (nblk > 0) {
      const int later = (int)((NB < nblk ? NB : nblk) - 1);  // this wave's part of block 0
      if (tall) wait_landed<G::VMEM_TALL, NB>(later);
      else wait_landed<G::VMEM, NB>(later);
      bump(flag);
      if (k == 0) {
        spin(flag, 4u);
        row_stage(0, b0);
        bump(ready + 0);
      }
    }
    int cur = 0;
    unsigned rnd = 0;
#pragma unroll 1
    for (int64_t i = 0; i < nblk; ++i) {
      if (i + 1 < nblk) {  // the row stage of block i + 1
        int s1 = cur + 1 == NB ? 0 : cur + 1;
        // blocks up to i + NB - 1 are issued here (block i + NB only after block i is consumed)
        const int later = (int)((i + NB - 1 < nblk ? i + NB - 1 : nblk - 1) - (i + 1));
        if (tall) wait_landed<G::VMEM_TALL, NB>(later);
        else wait_landed<G::VMEM, NB>(later);
        bump(flag);
        if (((i + 1) & 3) == k) {
          spin(flag, (unsigned)(4 * (i + 2)));
          row_stage(s1, b0 + i + 1);
          bump(ready + s1);
        }
      }
      if (i + NB < nblk) {  // restage slot cur once the Gram waves are done with block i
        spin(done + cur, 8u * (rnd + 1));
        stage(cur, b0 + i + NB);
      }
      if (++cur == NB) {
        cur = 0;
        ++rnd;
      }
    }
    __builtin_amdgcn_s_setprio(0);
    wait_vm<0>();
  } else {
    // ======================= Gram waves: k-steps 2 g, 2 g + 1 of every block =======================
    const int g = wv;
    const int cl = lane & 15, rq = lane >> 4;
    int koff[2];
#pragma unroll
    for (int t = 0; t < 2; ++t) {
      const int rr = 4 * (2 * g + t) + rq;
      koff[t] = cl * SB + (rr ^ (2 * cl));
    }
#pragma unroll
    for (int t = 0; t < G::T; ++t) acc[t] = d4{0.0, 0.0, 0.0, 0.0};
#pragma unroll
    for (int b = 0; b < P16; ++b) xz[b] = 0.0;
    const bool has_eta = IRLS && !STATS && a.eta_out != nullptr;
    int cur = 0;
    unsigned rnd = 0;
    const int64_t nblk = b1 - b0;
#pragma unroll 1
    for (int64_t i = 0; i < nblk; ++i) {
      spin(ready + cur, rnd + 1);
      const double* xs = lds + cur * G::PER;
      const double* wd = xs + G::OFF_W;
      if (do_gram) {
#pragma unroll
        for (int t = 0; t < 2; ++t) {
          // the two Gram waves of a SIMD (g, g + 4) take turns at the higher issue priority
          if (((g >> 2) ^ t) & 1) __builtin_amdgcn_s_setprio(1);
          else __builtin_amdgcn_s_setprio(0);
          const int rr = 4 * (2 * g + t) + rq;
          const double wr = wd[rr], wzr = wd[SB + rr];
          double xv[P16], av[P16];
#pragma unroll
          for (int b = 0; b < P16; ++b) {
            xv[b] = xs[koff[t] + b * 16 * SB];
            av[b] = xv[b] * wr;
            xz[b] += xv[b] * wzr;
          }
          gram_kstep<P16>(acc, av, xv);
        }
      }
      if (has_eta && g == 0) {
        const int64_t row = (b0 + i) * SB + lane;
        if (row < a.n) a.eta_out[row] = xs[G::OFF_E + lane];
      }
      asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");  // every read of the slot returned
      bump(done + cur);
      if (++cur == NB) {
        cur = 0;
        ++rnd;
      }
    }
    __builtin_amdgcn_s_setprio(0);
  }

  // ---- wave partials: X'Wz over the 4 row lanes of each column, scalars over the wave ----
  if (wv < G::NGW) {
#pragma unroll
    for (int b = 0; b < P16; ++b) xz[b] = xor32_sum(xor16_sum(xz[b]));
  }
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
  if (wv >= G::NGW && lane == 0) {
    double* red = lds + G::OFF_RED + wv * 8;
    red[0] = s_dev;
    red[1] = s_aux;
    red[2] = s_pear;
    red[3] = s_ll;
    red[4] = s_bad;
  }
  __syncthreads();  // every slot consumed and every DMA landed: the ring is free for the fold

  // ---- fixed-order fold of the 8 Gram waves' partials: ((g0+g4)+(g2+g6)) + ((g1+g5)+(g3+g7)) ----
#pragma unroll 1
  for (int n = G::NGW; n > 1;) {
    const int hh = (n + 1) / 2;
    if (wv >= hh && wv < n) {
      double* reg = lds + (wv - hh) * G::PSZ;
#pragma unroll
      for (int t = 0; t < G::T; ++t)
#pragma unroll
        for (int j = 0; j < 4; ++j) reg[t * 256 + 64 * j + lane] = acc[t][j];
      if (lane < 16) {
#pragma unroll
        for (int b = 0; b < P16; ++b) reg[G::T * 256 + 16 * b + lane] = xz[b];
      }
    }
    __syncthreads();
    if (wv < n - hh) {
      const double* reg = lds + wv * G::PSZ;
#pragma unroll
      for (int t = 0; t < G::T; ++t)
#pragma unroll
        for (int j = 0; j < 4; ++j) acc[t][j] += reg[t * 256 + 64 * j + lane];
#pragma unroll
      for (int b = 0; b < P16; ++b) xz[b] += reg[G::T * 256 + 16 * b + (lane & 15)];
    }
    __syncthreads();
    n = hh;
  }
  if (wv == 0) {
    double* out = a.partials + (int64_t)blockIdx.x * a.stride;
#pragma unroll
    for (int t = 0; t < G::T; ++t)
#pragma unroll
      for (int j = 0; j < 4; ++j) out[t * 256 + 64 * j + lane] = acc[t][j];
    if (lane < 16) {
#pragma unroll
      for (int b = 0; b < P16; ++b) out[G::T * 256 + 16 * b + lane] = xz[b];
    }
    if (lane < NS) {
      // the row waves' scalars in wave order
      double sv[5] = {0.0, 0.0, 0.0, 0.0, 0.0};
#pragma unroll
      for (int k = 0; k < G::NRW; ++k)
#pragma unroll
        for (int q = 0; q < 5; ++q) sv[q] += lds[G::OFF_RED + (G::NGW + k) * 8 + q];
      double v = lane == S_DEV ? sv[0] : lane == S_SUMW ? sv[1] : 0.0;
      if constexpr (STATS) {
        if (lane == SL::S2) v = sv[2];
        if (lane == SL::S3) v = sv[3];
        if (lane == SL::S4) v = sv[4];
      }
      if constexpr (INIT_CONST) {
        if (lane == S_AUX2) v = sv[3];
      }
      out[G::T * 256 + G::NC + lane] = v;
    }
  }
}

template <int P16, int FAM, int LNK>
void launch_r_fl(const PassArgs& a, dim3 gr, dim3 bl, hipStream_t st, hipEvent_t e0, hipEvent_t e1) {
  constexpr bool SP = stats_in_pass_family(FAM, LNK);
  if (a.mode == MODE_IRLS && SP && a.stats_in_pass && !(FAM == FAM_BINOMIAL && a.m))
    hipExtLaunchKernelGGL((irls_narrow_r_kernel<P16, FAM, LNK, true, SP>), gr, bl, 0, st, e0, e1, 0, a);
  else if (a.mode == MODE_IRLS)
    hipExtLaunchKernelGGL((irls_narrow_r_kernel<P16, FAM, LNK, true>), gr, bl, 0, st, e0, e1, 0, a);
  else
    hipExtLaunchKernelGGL((irls_narrow_r_kernel<P16, FAM, LNK, false>), gr, bl, 0, st, e0, e1, 0, a);
}

template <int P16>
hipError_t launch_r_p(const PassArgs& a, int grid, hipStream_t st, hipEvent_t e0, hipEvent_t e1) {
  const dim3 gr(grid), bl(64 * NR<P16>::NW);
  const int fam = (a.mode == MODE_LM_GRAM) ? FAM_GAUSSIAN : a.family;
  const int lnk = (a.mode == MODE_LM_GRAM) ? LNK_IDENTITY : a.link;
  if (fam == FAM_BINOMIAL && lnk == LNK_LOGIT)
    launch_r_fl<P16, FAM_BINOMIAL, LNK_LOGIT>(a, gr, bl, st, e0, e1);
  else if (fam == FAM_BINOMIAL && lnk == LNK_PROBIT)
    launch_r_fl<P16, FAM_BINOMIAL, LNK_PROBIT>(a, gr, bl, st, e0, e1);
  else if (fam == FAM_BINOMIAL)
    launch_r_fl<P16, FAM_BINOMIAL, LNK_CLOGLOG>(a, gr, bl, st, e0, e1);
  else if (fam == FAM_GAUSSIAN)
    launch_r_fl<P16, FAM_GAUSSIAN, LNK_IDENTITY>(a, gr, bl, st, e0, e1);
  else if (fam == FAM_POISSON)
    launch_r_fl<P16, FAM_POISSON, LNK_LOG>(a, gr, bl, st, e0, e1);
  else if (fam == FAM_GAMMA)
    launch_r_fl<P16, FAM_GAMMA, LNK_INVERSE>(a, gr, bl, st, e0, e1);
  else
    return hipErrorInvalidValue;
  return hipGetLastError();
}

}  // namespace

bool narrow_r_ok(int P16, int64_t n_pad) {
  // any shard: one past the 32-bit lane offsets of a column pair stages a column per half-wave
  // instruction (stage_r's tall form)
  return P16 >= 2 && P16 <= 4 && n_pad > 0;
}

hipError_t launch_narrow_r(int P16, const PassArgs& a, int grid, hipStream_t st, hipEvent_t e0, hipEvent_t e1) {
  switch (P16) {
    case 2: return launch_r_p<2>(a, grid, st, e0, e1);
    case 3: return launch_r_p<3>(a, grid, st, e0, e1);
    case 4: return launch_r_p<4>(a, grid, st, e0, e1);
    default: return hipErrorInvalidValue;
  }
}

}  // namespace sglm
