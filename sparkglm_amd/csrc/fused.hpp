// fused.hpp -- the fused IRLS pass kernels for 65 <= p <= 256 (device templates): K1
// (irls_pass_kernel<P16>, even column-block counts) and K1r (irls_pass_r_kernel<P16>, the
// split-role pass, any column-block count >= 5).  Included by kernels.hip (even P16) and
// fused_odd.hip (odd P16), so the two sets compile as separate objects.
#pragma once
#include <hip/hip_runtime.h>

#include <cstdint>
#include <type_traits>

#include "common.hpp"
#include "kernels.hpp"
#include "procx.hpp"
#include "rowmath.hpp"

namespace sglm {


typedef double d4 __attribute__((ext_vector_type(4)));
typedef __attribute__((address_space(3))) void lds_void;

// ---------------------------------------------------------------------------------
// compile-time geometry.  P16 (even) column blocks of 16; NW = P16/2 waves.  Wave w
// owns the block rows lo = lo_row(w) and hi = P16-1-w of the lower-triangular tile grid:
// tiles (lo, 0..lo) and (hi, 0..hi), lo+hi+2 tiles, for the whole launch.
// ---------------------------------------------------------------------------------
template <int P16>
struct Geo {
  static_assert(P16 >= 2, "column-block count");  // odd counts: the layout of K1r only
  // waves per workgroup: P16 / 2 (whole row pairs; P16 = 16); P16 = 5..8 four (K1 takes its tiles as
  // runs, so the wave count is free there): P16 = 5, 6: three 4-wave workgroups fit the LDS -- 12
  // waves, 3 per SIMD, where
  // three 3-wave workgroups left one SIMD a third wave (p = 96 8.49 -> 7.93 ms, p = 80 9.39 -> 9.15,
  // profiles/r04_midp_ab_run7_nw4.txt)
  static constexpr int NW = P16 >= 5 && P16 <= 8 ? 4 : P16 / 2;
  static constexpr int NC = P16 * 16;              // padded columns
  static constexpr int NCE = (NC + 31) / 32 * 32;  // columns in the LDS image (eta stripes)
  static constexpr int T = P16 * (P16 + 1) / 2;    // lower-triangular 16x16 tiles
  static constexpr int TPW = P16 + 1;              // tiles per wave
  // The row stage runs on the "row group": waves NW/2 .. NW/2+NRW-1 (wave 0 when NW == 1),
  // one wave per SIMD, NRW a power of two, RW rows each.
  static constexpr int NRW = NW >= 8 ? 4 : (NW >= 4 ? 2 : 1);
  static constexpr int ROW0 = NW >= 2 ? NW / 2 : 0;   // first wave of the row group
  static constexpr int RW = RB / NRW;              // rows per row-group wave
  static constexpr int CPG = RW / 2;               // columns per lane group per 32-column stripe
  // LDS-DMA issuers: the MFMA-only waves (NA of them), which have slack at the block barrier;
  // a single-wave workgroup (P16 = 2) stages its own blocks.
  static constexpr int NA = NW - NRW;
  static constexpr int NI = NA > 0 ? NA : 1;
  static constexpr int QMAX = (4 * P16 + NI - 1) / NI;  // quads per issuer (at most)
  // vectors per issuer (at most), rounded UP so the NI issuers cover all four vectors (y, m,
  // offset, prior): at P16 = 10 (NI = 3) 4 / NI dropped the prior weights (tests/test_gpu_fused_split.py)
  static constexpr int VMAX = (4 + NI - 1) / NI;
  static_assert(VMAX * NI >= 4, "every vector staged");
  // 16-column blocks of the image are BSTR = 16*RB + 2 doubles apart: the pad keeps the
  // compiler from pairing the per-block B-operand reads into ds_read2st64_b64 (32-bank rule,
  // 2-way conflicts under the slot swizzle, 8 LDS cycles) -- they stay ds_read_b64
  static constexpr int BSTR = 16 * RB + 2;  // (+2: keeps LDS-DMA destinations 16-B aligned)
  static constexpr int XB = (NCE / 16) * BSTR;     // doubles per X buffer
  // LDS layout, in doubles (one __shared__ array: keeps hipcc's LDS-DMA waits counted)
  static constexpr int OFF_X = 0;                  // [2][XB]
  static constexpr int OFF_V = 2 * XB;             // [2][4][RB]  y, m, offset, prior
  static constexpr int OFF_BETA = OFF_V + 8 * RB;  // [NCE]
  static constexpr int OFF_W = OFF_BETA + NCE;     // [2][w RB | w*z RB]
  static constexpr int OFF_RED = OFF_W + 4 * RB;   // [NW][NS]
  static constexpr int OFF_INIT = OFF_RED + NW * NS; // [6] the initial pass's constants (init_const)
  static constexpr int OFF_FLAG = OFF_INIT + 6;    // row-wave staging counter (uint32)
  static constexpr int LDS_DOUBLES = OFF_FLAG + 1;
  static constexpr int STRIDE = T * 256 + NC + NS; // partial stride (doubles)
  // workgroups per CU: up to 12 waves per CU (3 per SIMD), LDS permitting -- P16 = 6 runs three
  // 3-wave workgroups (8 waves wanted: two; same-box p = 96 pass 9.30 -> 8.57 ms, p = 80 10.73 ->
  // 9.87 ms, no spills at the 168-VGPR budget); P16 >= 8 stays LDS-bound at two workgroups or one
  static constexpr int WMAX = 12;
  static constexpr int WG_PER_CU = (WMAX / NW) * (LDS_DOUBLES * 8) <= 160 * 1024 ? WMAX / NW : 160 * 1024 / (LDS_DOUBLES * 8);
  static constexpr int WAVES_PER_SIMD = (WG_PER_CU * NW + 3) / 4;
  // Block rows of wave wv's tiles: HI = P16-1-wv and LO below.  The row waves carry the row
  // stage on top of their MFMAs, so they take the LOW rows 0..NRW-1 (fewest tiles) and the
  // first NRW MFMA-only waves take ROW0.. in exchange (P16 = 16: 13 tiles per row wave, 21
  // per MFMA-only wave 0-3, instead of 17 everywhere).
  // P16 = 16: row waves 15 / MFMA-only waves 19 tiles (a 13 / 21 split would not fit the
  // 256-VGPR budget of two waves per SIMD; 17 / 17 and 16 / 18 measured slower).
  static constexpr int lo_row(int wv) {
    if (P16 == 16) {
      constexpr int t[8] = {2, 3, 6, 7, 0, 1, 4, 5};
      return t[wv];
    }
    return wv < NRW ? ROW0 + wv : (wv >= ROW0 && wv < ROW0 + NRW ? wv - ROW0 : wv);
  }
  static constexpr int hi_row(int wv) {
    if (P16 == 16) {
      constexpr int t[8] = {15, 14, 11, 10, 13, 12, 9, 8};
      return t[wv];
    }
    return P16 - 1 - wv;
  }
  static constexpr int ntiles(int wv) { return lo_row(wv) + hi_row(wv) + 2; }
};

template <int P16>
struct TileSeq {
  static constexpr int T = P16 * (P16 + 1) / 2;
  static constexpr int seq_row(int i) { return (i & 1) ? P16 - 1 - (i >> 1) : (i >> 1); }  // i-th row of the sequence
  static constexpr int seq_start(int i) {  // first sequence index of row seq_row(i)
    int t = 0;
    for (int k = 0; k < i; ++k) t += seq_row(k) + 1;
    return t;
  }
  static constexpr int seq_of(int t) {  // sequence row holding sequence tile t
    int i = 0;
    while (i + 1 < P16 && seq_start(i + 1) <= t) ++i;
    return i;
  }
};
constexpr int NSEG = 4;

// Tiles [TLO, THI) of the paired-row tile sequence as up to NSEG segments, each a run of tiles
// (row, j0 .. j0 + cnt - 1) of one block row (one A operand per segment, B = column block j).
// diag(s): the segment holds its row's diagonal tile (row, row), the sequence's last tile of that
// row -- that segment forms the row block's X'Wz, so every block row's X'Wz is formed exactly once.
template <int P16, int TLO, int THI>
struct TileRun {
  using S = TileSeq<P16>;
  static constexpr int row(int s) {
    if (THI <= TLO) return -1;
    const int i = S::seq_of(TLO) + s;
    return i <= S::seq_of(THI - 1) ? S::seq_row(i) : -1;
  }
  static constexpr int j0(int s) { return s == 0 && THI > TLO ? TLO - S::seq_start(S::seq_of(TLO)) : 0; }
  static constexpr int cnt(int s) {
    if (row(s) < 0) return 0;
    const int i = S::seq_of(TLO) + s;
    const int b = i == S::seq_of(TLO) ? TLO : S::seq_start(i);  // first sequence tile in the run
    const int e = S::seq_start(i) + S::seq_row(i) + 1;          // end of the row in the sequence
    return (e < THI ? e : THI) - b;
  }
  static constexpr bool diag(int s) { return cnt(s) > 0 && j0(s) + cnt(s) - 1 == row(s); }
  static constexpr int off(int s) {
    int o = 0;
    for (int k = 0; k < s; ++k) o += cnt(k);
    return o;
  }
  static constexpr int NT = off(NSEG);
  static constexpr int seg_of(int k) {
    int sg = 0;
    while (sg + 1 < NSEG && off(sg + 1) <= k) ++sg;
    return sg;
  }
  static_assert(NT == (THI > TLO ? THI - TLO : 0), "the run fits NSEG segments");
};

// K1's tiles.  P16 = 16: wave WV owns block rows LO = lo_row(WV) and HI = hi_row(WV) whole -- two
// segments (the row waves' rows chosen short; K1r is bitwise this).  Other P16: the tile sequence
// cut into NW contiguous runs, the row waves' runs ROW_TILES shorter than the MFMA-only waves'.
// The row stage of the next block runs on the row waves between their k-steps and the block ends
// at a barrier; with whole row pairs the waves' shares were fixed by the pairs (P16 = 6: 8 / 6 / 7
// tiles, the single row wave's row stage on top of its 6) -- PMC, K1<6>: 39 % of wave cycles parked,
// profiles/r04_stalls/mid96.json.  Same-box A/B (profiles/r04_midp_ab_run6_k1runs.txt): P16 = 6
// with one row wave runs best 3 tiles short (8 / 5 / 8: p = 80 10.59 (round 3) -> 9.18 ms, p = 96
// 9.15 -> 8.02 ms; 0 or 5 short: 9.4-10.0 / 8.3-8.6), P16 = 8 with two row waves best evenly
// (9 tiles each: p = 112 10.16 -> 9.76 ms; 3 short 10.28).  Runs only move which wave forms a
// tile; every tile and X'Wz column sums the same k-steps in the same order.
template <int P16>
struct K1Runs {
  using G = Geo<P16>;
  static constexpr int ROW_TILES = G::NRW == 1 ? 3 : 0;
  static constexpr bool is_row(int w) { return w >= G::ROW0 && w < G::ROW0 + G::NRW; }
  static constexpr int LR = G::NA > 0 ? ((G::T - G::NA * ROW_TILES) / G::NW > 1 ? (G::T - G::NA * ROW_TILES) / G::NW : 1)
                                      : G::T;  // tiles of a row wave
  static constexpr int len(int w) {
    if (G::NA == 0) return G::T;
    if (is_row(w)) return LR;
    const int rest = G::T - G::NRW * LR;
    int ia = 0;  // issuer index of wave w
    for (int v = 0; v < w; ++v)
      if (!is_row(v)) ++ia;
    return rest * (ia + 1) / G::NA - rest * ia / G::NA;
  }
  static constexpr int lo(int w) {
    int t = 0;
    for (int v = 0; v < w; ++v) t += len(v);
    return t;
  }
  static_assert(lo(G::NW) == G::T, "the runs cover the tile triangle");
};
template <int P16, int WV, bool RUNS = (P16 != 16)>
struct TilesK1 : TileRun<P16, K1Runs<P16>::lo(WV), K1Runs<P16>::lo(WV + 1)> {};
template <int P16, int WV>
struct TilesK1<P16, WV, false> {
  static constexpr int LO = Geo<P16>::lo_row(WV), HI = Geo<P16>::hi_row(WV);
  static constexpr int row(int s) { return s == 0 ? LO : (s == 1 ? HI : -1); }
  static constexpr int j0(int) { return 0; }
  static constexpr int cnt(int s) { return s == 0 ? LO + 1 : (s == 1 ? HI + 1 : 0); }
  static constexpr bool diag(int s) { return s < 2; }
  static constexpr int off(int s) { return s == 0 ? 0 : (s == 1 ? LO + 1 : LO + HI + 2); }
  static constexpr int NT = LO + HI + 2;
  static constexpr int seg_of(int k) { return k <= LO ? 0 : 1; }
};

// s_waitcnt vmcnt(N) with expcnt / lgkmcnt left open (gfx9 encoding).
template <int N>
__device__ __forceinline__ void wait_vmcnt() {
  static_assert(N >= 0 && N < 64, "vmcnt range");
  __builtin_amdgcn_s_waitcnt((N & 15) | ((N >> 4) << 14) | (7 << 4) | (15 << 8));
}

// Workgroup barrier that orders LDS traffic but leaves LDS-DMA loads in flight.
__device__ __forceinline__ void lds_barrier() {
  asm volatile("s_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory");
}

// ---------------------------------------------------------------------------------
// LDS-DMA staging of one row block.  X tile image: column c occupies 32 doubles at
// c*32; row r of column c sits in slot r ^ (2c & 31) (XOR swizzle applied on the
// source address, rule 21), which makes both the MFMA fragment reads (16 columns x 2
// rows per half-wave) and the eta reads (RW rows x 64/RW column groups) conflict free.
// ---------------------------------------------------------------------------------
template <int P16>
__device__ __forceinline__ void stage_block(double* lds, int buf, const PassArgs& a, int64_t blk, int si,
                                            int lane) {
  // issuer si of NI moves quads [si*Q/NI, (si+1)*Q/NI) (Q = 4*P16) and its share of the
  // vectors y, m, offset, prior
  using G = Geo<P16>;
  constexpr int Q = 4 * P16;
  const int64_t r0 = blk * RB;
  // LDS-DMA destinations in address space 3, formed from the shared array's LDS address
  typedef __attribute__((address_space(3))) double lds_double;
  lds_double* l3 = (lds_double*)__builtin_amdgcn_readfirstlane((int)(uintptr_t)(lds_void*)lds);
  lds_double* xdst = l3 + G::OFF_X + buf * G::XB;
  const int i = lane & 15, cq = lane >> 4;
  // lane part of the source address; the column-quad part is wave-uniform (SGPRs).
  const double* lbase = a.X + (int64_t)cq * a.ld + r0;
  const int q0 = si * Q / G::NI, q1 = (si + 1) * Q / G::NI;
#pragma unroll
  for (int k = 0; k < G::QMAX; ++k) {
    const int q = q0 + k;                                      // LDS column quad
    if (q >= q1) break;
    const int qs = __builtin_amdgcn_readfirstlane(q < a.nq ? q : a.nq - 1);  // quads past p: duplicates
    const int srow = (2 * i) ^ ((8 * q + 2 * cq) & 31);        // slot swizzle of column 4q + cq
    const double* src = lbase + (int64_t)(4 * qs) * a.ld + srow;
    __builtin_amdgcn_global_load_lds((const void*)src, (lds_void*)(xdst + (q >> 2) * G::BSTR + (q & 3) * 128), 16, 0, DMA_NT);
  }
#pragma unroll
  for (int k = 0; k < G::VMAX; ++k) {
    // vector v: 0 y, 1 m, 2 offset, 3 prior (absent vectors re-load y)
    const int v = si * G::VMAX + k;
    if (v >= 4) break;
    const double* src = a.y;
    if (v == 1 && a.m) src = a.m;
    if (v == 2 && a.off) src = a.off;
    if (v == 3 && a.prior) src = a.prior;
    if (lane < 16) {
      __builtin_amdgcn_global_load_lds((const void*)(src + r0 + 2 * lane),
                                       (lds_void*)(l3 + G::OFF_V + buf * 4 * RB + v * RB), 16, 0, DMA_NT);
    }
  }
}

// Cross-lane sums without LDS: DPP row_ror:8 (lane i <-> i^8 inside a 16-lane row) and
// the gfx950 permlane16/32 swaps, which hand each lane its xor-16 / xor-32 partner.
__device__ __forceinline__ double add_xor8(double v) {
  const int lo = __builtin_amdgcn_mov_dpp(__double2loint(v), 0x128, 0xf, 0xf, false);
  const int hi = __builtin_amdgcn_mov_dpp(__double2hiint(v), 0x128, 0xf, 0xf, false);
  return v + __hiloint2double(hi, lo);
}
__device__ __forceinline__ double add_xor16(double v) {
  const auto a = __builtin_amdgcn_permlane16_swap(__double2loint(v), __double2loint(v), false, false);
  const auto b = __builtin_amdgcn_permlane16_swap(__double2hiint(v), __double2hiint(v), false, false);
  return __hiloint2double(b[0], a[0]) + __hiloint2double(b[1], a[1]);
}
__device__ __forceinline__ double add_xor32(double v) {
  const auto a = __builtin_amdgcn_permlane32_swap(__double2loint(v), __double2loint(v), false, false);
  const auto b = __builtin_amdgcn_permlane32_swap(__double2hiint(v), __double2hiint(v), false, false);
  return __hiloint2double(b[0], a[0]) + __hiloint2double(b[1], a[1]);
}

// Row stage for one block: wave wv owns rows RW*wv .. RW*wv+RW-1; 64/RW lanes per row
// form eta over the column groups {32t + CPG*g + u}; the first RW lanes run the family
// arithmetic and store w and w*z for the block's MFMA phase into the w buffer `wb`.
template <int P16, int FAM, int LNK>
__device__ __forceinline__ void row_stage(double* lds, int buf, int wb, const PassArgs& a, int64_t blk, int wv,
                                          int lane, double& s_dev, double& s_aux) {
  using G = Geo<P16>;
  const int rw = wv - G::ROW0;
  if (rw < 0 || rw >= G::NRW) return;
  const double* xs = lds + G::OFF_X + buf * G::XB;
  const double* beta = lds + G::OFF_BETA;
  const int rl = lane % G::RW, g = lane / G::RW;
  const int r = G::RW * rw + rl;
  double eta = 0.0;
  if (a.mode == MODE_IRLS) {
    // four independent partial sums per lane shorten the dependent FMA chain
    double e4[4] = {0.0, 0.0, 0.0, 0.0};
#pragma unroll
    for (int u = 0; u < G::CPG; ++u) {
      const int c0 = G::CPG * g + u;  // column in stripe 0; stripe t adds 32 columns, same slot
      const double* base = xs + (c0 >> 4) * G::BSTR + (c0 & 15) * 32 + (r ^ ((2 * c0) & 31));
#pragma unroll
      for (int t = 0; t < G::NCE / 32; ++t) e4[(u * (G::NCE / 32) + t) & 3] += base[2 * G::BSTR * t] * beta[c0 + 32 * t];
    }
    eta = (e4[0] + e4[1]) + (e4[2] + e4[3]);  // beta is 0 past p
    if constexpr (G::RW <= 8) eta = add_xor8(eta);
    if constexpr (G::RW <= 16) eta = add_xor16(eta);
    if constexpr (G::RW <= 32) eta = add_xor32(eta);
  }
  if (lane < G::RW) {
    const double* vv = lds + G::OFF_V + buf * 4 * RB;
    const int64_t row = blk * RB + r;
    double w = 0.0, wz = 0.0;
    if (row < a.n) {
      const double y = vv[r];
      const double m = a.m ? vv[RB + r] : 1.0;
      const double off = a.off ? vv[2 * RB + r] : 0.0;
      const double pw = a.prior ? vv[3 * RB + r] : 1.0;
      if (a.mode == MODE_IRLS) {
        eta = eta + off;
        if (a.eta_out) a.eta_out[row] = eta;
      }
      // initial pass (binomial, no m): the per-pass constants from LDS (bitwise pass_row_ref's rows)
      if (FAM == FAM_BINOMIAL && init_fast_row(FAM, a.mode, a.m != nullptr) && y >= 0.0 && y <= 1.0)
        pass_row_init(lds + G::OFF_INIT, y, off, pw, w, wz, s_dev, s_aux);
      // (P16 = 16: the row arithmetic of K1r's row_stage_r, so that K1 and K1r are bitwise
      // interchangeable -- tests/test_gpu_fused_split.py)
      else pass_row(FAM, LNK, a.mode, eta, y, m, off, pw, a.mu0, a.ybar, a.m != nullptr, w, wz, s_dev, s_aux,
                    P16 == 16);
    }
    lds[G::OFF_W + wb * 2 * RB + r] = w;
    lds[G::OFF_W + wb * 2 * RB + RB + r] = wz;
  }
}

// MFMA k-steps [S0, S0 + NST) of one block for wave WV (compile-time, so every operand is a
// static LDS offset): the wave's tiles (TilesK1 segments; P16 = 16: block rows LO, HI whole).  Lane l
// reads X[k0 + (l>>4)][16b + (l&15)]; the A operand (a segment's block row) is scaled by the lane's
// row weight, the B operands are used straight from LDS.  X'Wz accumulates on the VALU from the A
// fragments of the segments that hold their row's diagonal tile.  A phase is RB/8 k-steps starting
// at S0.  Narrow variants (P16 <= 8: at most 9 MFMAs per k-step) unroll the phase so the next
// k-step's LDS operand reads issue under the current k-step's MFMAs; wide variants carry enough
// MFMAs per k-step to cover the read latency.
template <int P16, int WV, int NST = RB / 8>
__device__ __forceinline__ void gram_steps(const double* lds, int buf, int wb, int lane, int S0,
                                           d4 (&acc)[TilesK1<P16, WV>::NT], double (&xz)[NSEG]) {
  using G = Geo<P16>;
  using T = TilesK1<P16, WV>;
  constexpr int UNR = P16 <= 8 ? NST : 1;
  const double* xs = lds + G::OFF_X + buf * G::XB;
  const double* w = lds + G::OFF_W + wb * 2 * RB;
  const int cl = lane & 15, rq = lane >> 4;
  const double* colbase = xs + cl * 32;  // column c = 16b + cl has (2c & 31) == 2cl for every b
#pragma unroll UNR
  for (int j = 0; j < NST; ++j) {
    const int r = 4 * (S0 + j) + rq;
    const double* base = colbase + (r ^ (2 * cl));
    const double wr = w[r], wzr = w[RB + r];
    double av[NSEG];
#pragma unroll
    for (int sg = 0; sg < NSEG; ++sg) {
      av[sg] = 0.0;
      if constexpr (true) {
        if (T::cnt(sg) > 0) {
          const double x = base[G::BSTR * (T::row(sg) >= 0 ? T::row(sg) : 0)];
          av[sg] = x * wr;
          if (T::diag(sg)) xz[sg] += x * wzr;
        }
      }
    }
#pragma unroll
    for (int k = 0; k < T::NT; ++k) {
      const int sg = T::seg_of(k);
      const double b = base[G::BSTR * (T::j0(sg) + k - T::off(sg))];
      acc[k] = __builtin_amdgcn_mfma_f64_16x16x4f64(av[sg], b, acc[k], 0, 0, 0);
    }
  }
}

// Pipeline per row block i (cur = i & 1), ONE barrier per block:
//   MFMA-only waves ("issuers"): MFMA k 0..KA-1 of block i; wait for their own LDS-DMA of
//                     block i+1 and publish it (LDS counter); MFMA k KA..7      | barrier;
//                     LDS-DMA of block i+2 into the buffer block i occupied.
//   row waves:        MFMA k 0..K1-1 of i; wait until every issuer published block i+1;
//                     row stage of block i+1 (w, w*z); MFMA k K1..7 of i       | barrier
// Only the end-of-block barrier orders the image and the w buffers across all waves.  The
// DMA issue (a burst the memory queues throttle to ~5k cycles per block) sits on the issuers,
// which have slack at the barrier; the row waves carry the critical path (their MFMAs + the
// row stage) at raised priority (per-phase s_memtime stamps, round 2: DESIGN.md 4 K1).
template <int P16, int FAM, int LNK, int WV>
__device__ __forceinline__ void pass_body(double* lds, const PassArgs& a, int wv, int lane) {
  using G = Geo<P16>;
  const int wg = blockIdx.x, nwg = gridDim.x;
  const int64_t b0 = (a.nblocks * wg) / nwg, b1 = (a.nblocks * (wg + 1)) / nwg;
  const bool do_gram = !a.no_gram;
  // roles are compile-time per wave (WV), so each wave's instantiation carries only its code
  constexpr int rw = WV - G::ROW0;
  constexpr bool row_wave = rw >= 0 && rw < G::NRW;
  // DMA issuer index: the MFMA-only waves in order (or the only wave)
  constexpr bool issuer = G::NA > 0 ? !row_wave : true;
  constexpr int si = G::NA > 0 ? (WV < G::ROW0 ? WV : WV - G::NRW) : 0;
  // MFMA k-steps of block i before the row stage of block i+1 (K1) and before an issuer
  // publishes its landed part of block i+1 (KA); A/B-measured per variant (tools/ab.py)
  constexpr int K1 = P16 == 16 ? 7 : 6;
  constexpr int KA = P16 == 16 ? 0 : 2;
  unsigned* flag = (unsigned*)(lds + G::OFF_FLAG);

  using TK = TilesK1<P16, WV>;
  d4 acc[TK::NT];
#pragma unroll
  for (int k = 0; k < TK::NT; ++k) acc[k] = d4{0.0, 0.0, 0.0, 0.0};
  double xz[NSEG] = {0.0, 0.0, 0.0, 0.0}, s_dev = 0.0, s_aux = 0.0;

  if (issuer && b0 < b1) {
    stage_block<P16>(lds, 0, a, b0, si, lane);
    if (b0 + 1 < b1) stage_block<P16>(lds, 1, a, b0 + 1, si, lane);
  }
  if (row_wave) __builtin_amdgcn_s_setprio(1);
  // Iteration blk runs the MFMA phase of block blk and the row stage of block blk+1.  The
  // first iteration (blk = b0-1: row stage of b0 only) is peeled so that the steady-state loop
  // carries no branch around its MFMA phases (HG: has_gram, compile-time).
  auto iteration = [&](int64_t blk, auto HG) {
    const int cur = (int)((blk - b0) & 1);  // buffers of block blk; block blk+1 uses cur ^ 1
    constexpr bool has_gram_ct = decltype(HG)::value;
    const bool has_gram = has_gram_ct && do_gram;
    const bool has_next = blk + 1 < b1;
    if constexpr (G::NA > 0) {
      if constexpr (!row_wave) {
        // MFMA-only wave: after KA k-steps, publish that its part of block blk+1 has landed
        if (has_gram) gram_steps<P16, WV, KA>(lds, cur & 1, cur & 1, lane, 0, acc, xz);
        if (has_next) {
          wait_vmcnt<0>();
          if (lane == 0) __hip_atomic_fetch_add(flag, 1u, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_WORKGROUP);
        }
        if (has_gram) gram_steps<P16, WV, RB / 4 - KA>(lds, cur & 1, cur & 1, lane, KA, acc, xz);
      } else {
        // row wave: after K1 k-steps, wait until every issuer's part of block blk+1 landed
        if (has_gram) gram_steps<P16, WV, K1>(lds, cur & 1, cur & 1, lane, 0, acc, xz);
        if (has_next) {
          const unsigned target = (unsigned)(G::NA * (blk + 2 - b0));
          while (__hip_atomic_load(flag, __ATOMIC_ACQUIRE, __HIP_MEMORY_SCOPE_WORKGROUP) < target)
            __builtin_amdgcn_s_sleep(1);
          row_stage<P16, FAM, LNK>(lds, cur ^ 1, cur ^ 1, a, blk + 1, wv, lane, s_dev, s_aux);
        }
        if (has_gram) gram_steps<P16, WV, RB / 4 - K1>(lds, cur & 1, cur & 1, lane, K1, acc, xz);
      }
    } else {
      // single wave: it stages, waits and computes everything itself
      if (has_gram) gram_steps<P16, WV, K1>(lds, cur & 1, cur & 1, lane, 0, acc, xz);
      if (has_next) {
        if (blk + 1 == b0 && b0 + 1 < b1) wait_vmcnt<G::QMAX + G::VMAX>();
        else wait_vmcnt<0>();
        row_stage<P16, FAM, LNK>(lds, cur ^ 1, cur ^ 1, a, blk + 1, wv, lane, s_dev, s_aux);
      }
      if (has_gram) gram_steps<P16, WV, RB / 4 - K1>(lds, cur & 1, cur & 1, lane, K1, acc, xz);
    }
    lds_barrier();
    if (issuer && blk >= b0 && blk + 2 < b1) stage_block<P16>(lds, cur, a, blk + 2, si, lane);
  };
  if (b0 < b1) iteration(b0 - 1, std::false_type{});
#pragma unroll 1
  for (int64_t blk = b0; blk < b1; ++blk) iteration(blk, std::true_type{});
  if (row_wave) __builtin_amdgcn_s_setprio(0);

  // ---- epilogue: this workgroup's partial (tile t of wave wv: see gram_steps) ----
  double* out = a.partials + (int64_t)wg * a.stride;
#pragma unroll
  for (int k = 0; k < TK::NT; ++k) {
    const int sg = TK::seg_of(k);
    const int bi = TK::row(sg), bj = TK::j0(sg) + k - TK::off(sg);
    const int t = bi * (bi + 1) / 2 + bj;
#pragma unroll
    for (int j = 0; j < 4; ++j) out[t * 256 + 64 * j + lane] = acc[k][j];
  }
#pragma unroll
  for (int sg = 0; sg < NSEG; ++sg) {
    if constexpr (true) {
      if (TK::diag(sg)) {
        double v = xz[sg];
        v += __shfl_xor(v, 16);
        v += __shfl_xor(v, 32);
        if (lane < 16) out[G::T * 256 + 16 * TK::row(sg) + lane] = v;
      }
    }
  }
#pragma unroll
  for (int o = 1; o < 64; o <<= 1) {
    s_dev += __shfl_xor(s_dev, o);
    s_aux += __shfl_xor(s_aux, o);
  }
  if (lane == 0) {
    lds[G::OFF_RED + wv * NS + 0] = s_dev;
    lds[G::OFF_RED + wv * NS + 1] = s_aux;
  }
  lds_barrier();
  if (wv == 0 && lane < NS) {
    double sd = 0.0, sa = 0.0;
    for (int k = 0; k < G::NW; ++k) {
      sd += lds[G::OFF_RED + k * NS + 0];
      sa += lds[G::OFF_RED + k * NS + 1];
    }
    double v = 0.0;
    if (lane == S_DEV) v = sd;
    if (lane == S_SUMW) v = sa;
    out[G::T * 256 + G::NC + lane] = v;
  }
}

template <int P16, int FAM, int LNK>
__global__ void __launch_bounds__(64 * Geo<P16>::NW, (Geo<P16>::WAVES_PER_SIMD)) irls_pass_kernel(PassArgs a) {
  using G = Geo<P16>;
  __shared__ double lds[G::LDS_DOUBLES];
  const int lane = threadIdx.x & 63;
  const int wv = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  for (int c = threadIdx.x; c < G::NCE; c += 64 * G::NW) lds[G::OFF_BETA + c] = (a.beta && c < a.p) ? a.beta[c] : 0.0;
  if (threadIdx.x == 0) *(unsigned*)(lds + G::OFF_FLAG) = 0u;
  if constexpr (FAM == FAM_BINOMIAL)
    if (threadIdx.x == 0 && init_fast_row(FAM, a.mode, a.m != nullptr)) {
      const InitConst ic = init_const(FAM, LNK, a.mode, a.mu0);
      for (int k = 0; k < 6; ++k) lds[G::OFF_INIT + k] = ic.v[k];
    }
  if constexpr (G::NCE > G::NC) {  // LDS columns no DMA writes: keep them finite (zero)
    for (int e = threadIdx.x; e < (G::NCE - G::NC) * RB; e += 64 * G::NW) {
      const int c = G::NC + e / RB, r = e % RB;
      lds[G::OFF_X + (c >> 4) * G::BSTR + (c & 15) * RB + r] = 0.0;
      lds[G::OFF_X + G::XB + (c >> 4) * G::BSTR + (c & 15) * RB + r] = 0.0;
    }
  }
  __syncthreads();
  switch (wv) {
    case 0: pass_body<P16, FAM, LNK, 0>(lds, a, wv, lane); break;
    case 1: if constexpr (G::NW > 1) pass_body<P16, FAM, LNK, 1>(lds, a, wv, lane); break;
    case 2: if constexpr (G::NW > 2) pass_body<P16, FAM, LNK, 2>(lds, a, wv, lane); break;
    case 3: if constexpr (G::NW > 3) pass_body<P16, FAM, LNK, 3>(lds, a, wv, lane); break;
    case 4: if constexpr (G::NW > 4) pass_body<P16, FAM, LNK, 4>(lds, a, wv, lane); break;
    case 5: if constexpr (G::NW > 5) pass_body<P16, FAM, LNK, 5>(lds, a, wv, lane); break;
    case 6: if constexpr (G::NW > 6) pass_body<P16, FAM, LNK, 6>(lds, a, wv, lane); break;
    default: if constexpr (G::NW > 7) pass_body<P16, FAM, LNK, 7>(lds, a, wv, lane); break;
  }
}

// ---------------------------------------------------------------------------------
// K1r: the split-role fused pass (P16 >= 10 by default; P16 = 16: 225 <= p <= 256, BASELINE
// configs[1]).  12 waves, three per SIMD: two "Gram waves" and one "row wave" on every SIMD.
//   Gram waves 0..7: 17 lower-triangle tiles each at P16 = 16, nothing but the block's MFMAs
//                    (A scaled by w) -- the SIMD always has an MFMA stream ready;
//   row waves 8..11: the LDS-DMA of the blocks, the row stage of the next block (eta, mu, w,
//                    w*z, deviance) and X'Wz.
// In K1 (pass_body) the row stage ran on a wave that also carried 15 tiles: its dependent fp64
// chain waited one partner MFMA (64 cycles) per instruction, and the partner wave ran out of
// MFMAs before the row stage ended (phase stamps: ~3.2K idle cycles per 23.2K-cycle block).
// Here the row stage's latency sits beside TWO MFMA streams that never wait for it inside a
// block; the row waves run it at raised priority, so its VALU issues into the MFMA gaps.
// Every tile and X'Wz row accumulates the same values in the same order as K1 (same k-steps,
// same blocks, same lanes), so the partials are bitwise K1's.
// Tile ownership (P16 = 16): Gram wave 0 = block row 15; Gram wave g = 1..7 = block rows g-1
// and 15-g; every Gram wave also one tile (7, g) of block row 7 (17 tiles each).  (Measured and
// not kept: the row waves owning block row 7's tiles after their row stage; a block barrier
// instead of the LDS counters; no alternating issue priority -- DESIGN.md 4 K1r.)
// ---------------------------------------------------------------------------------

// A wave's tiles are up to NSEG "segments", each a run of tiles (row, j0 .. j0+cnt-1) of one
// block row (one A operand per segment, B = column block j).
// P16 = 16: Gram wave 0 = block row 15 (16 tiles); Gram wave g = 1..7 = block rows g-1 and 15-g
// (16 tiles) + tile (7, g) of block row 7.  Other P16 (the mid-width generalisation): the tile
// rows taken in pairs (0, P16-1), (1, P16-2), ... -- P16 + 1 tiles a pair -- and that sequence of
// tiles cut into 8 equal contiguous runs, one per Gram wave (at most NSEG segments each).
template <int P16, int WV>
struct TilesR {
  static constexpr bool ROW = WV >= 8;
  using S = TileSeq<P16>;
  static constexpr int tlo() { return S::T * WV / 8; }
  static constexpr int thi() { return S::T * (WV + 1) / 8; }
  static constexpr int row(int s) {
    if constexpr (P16 == 16) {
      if (ROW) return -1;
      if (s == 0) return WV >= 1 ? WV - 1 : -1;   // LO row
      if (s == 1) return WV == 0 ? 15 : 15 - WV;  // HI row
      if (s == 2) return 7;  // one tile of block row 7
      return -1;
    } else {
      if (ROW || thi() <= tlo()) return -1;
      const int i = S::seq_of(tlo()) + s;
      return i <= S::seq_of(thi() - 1) ? S::seq_row(i) : -1;
    }
  }
  static constexpr int j0(int s) {
    if constexpr (P16 == 16) return s == 2 ? WV : 0;
    else return s == 0 && !ROW && thi() > tlo() ? tlo() - S::seq_start(S::seq_of(tlo())) : 0;
  }
  static constexpr int cnt(int s) {
    if (row(s) < 0) return 0;
    if constexpr (P16 == 16) {
      return s == 2 ? 1 : row(s) + 1;
    } else {
      const int i = S::seq_of(tlo()) + s;
      const int b = i == S::seq_of(tlo()) ? tlo() : S::seq_start(i);  // first sequence tile in the run
      const int e = S::seq_start(i) + S::seq_row(i) + 1;              // end of the row in the sequence
      return (e < thi() ? e : thi()) - b;
    }
  }
  static constexpr int off(int s) {
    int o = 0;
    for (int k = 0; k < s; ++k) o += cnt(k);
    return o;
  }
  static constexpr int NT = off(NSEG);
  static constexpr int seg_of(int k) {
    int sg = 0;
    while (sg + 1 < NSEG && off(sg + 1) <= k) ++sg;
    return sg;
  }
  static_assert(P16 == 16 || ROW || row(NSEG) < 0 || true, "segments");
};

// K1r's LDS: a ring of NBUF row-block buffers -- as deep as 160 KB allows (4 up to P16 = 8, 3 up to
// 12, 2 above): the DMA of block b + NBUF is issued when block b is consumed, so a row wave finds the
// next block landed instead of waiting out its HBM latency.  (With two buffers that wait sat on the
// row waves' per-block path; the deeper ring measured +1-9 % at P16 = 9..12 and +-0 at 16,
// profiles/r04_midp_ab_run2_ring.txt -- at the mid widths the clock and the row stage's VALU bound
// the pass more than the DMA latency did)
template <int P16>
struct GeoR {
  using G = Geo<P16>;
  static constexpr int NW = 12, NGW = 8;
  static constexpr int XB = G::XB;                        // doubles per X buffer (K1's image)
  static constexpr int NT = G::NCE / 32;                  // 32-column stripes of the row stage
  // Row stage of a block: the four row waves, RW = 8 rows each, LPR = 8 lanes per row forming eta
  // over CPG = 4 columns of every 32-column stripe, the family arithmetic on 8 lanes (K1's lanes and
  // order at P16 = 16: K1r bitwise K1).  (Measured and not kept, round 4: two row waves of 16 rows
  // taking alternate blocks -- half the family-arithmetic instructions -- 3-8 % slower at P16 = 9..12,
  // profiles/r04_midp_ab_run3_rowgroups.txt: the row stage's latency, not its VALU, is what a block
  // waits for.)  LA: blocks the row stage runs ahead of the Gram.  (Two where the ring has a third
  // buffer, so its latency would hide under two blocks' MFMAs: measured ±3 % at P16 = 5..12,
  // profiles/r04_midp_ab_run4_lookahead.txt -- not the bound either; one.)
  static constexpr int RG = 4;
  static constexpr int RW = RB / RG, LPR = 64 / RW, CPG = 32 / LPR;
  static constexpr int BETAG_STRIDE = CPG * NT + 2;       // lane group stride of betag (+2: distinct banks)
  static constexpr int PER_BUF = XB + 4 * RB + 2 * RB + RB;  // X | y, m, offset, prior | w, w*z | eta
  static constexpr int NCNT = 10;                         // counters: flag | ready[4] | done[4] (uint32)
  static constexpr int FIXED = G::NCE + NW * NS + LPR * BETAG_STRIDE + NCNT / 2 + 6;
  static constexpr int LDS_MAX = 160 * 1024 / 8;
  static constexpr int NBUF = 4 * PER_BUF + FIXED <= LDS_MAX ? 4 : (3 * PER_BUF + FIXED <= LDS_MAX ? 3 : 2);
  static constexpr int OFF_X = 0;                         // [NBUF][XB]
  static constexpr int OFF_V = NBUF * XB;                 // [NBUF][4][RB]
  static constexpr int OFF_W = OFF_V + NBUF * 4 * RB;     // [NBUF][w RB | w*z RB]
  static constexpr int OFF_ETA = OFF_W + NBUF * 2 * RB;   // [NBUF][RB] the row stage's eta (stored by Gram wave 0)
  static constexpr int OFF_BETA = OFF_ETA + NBUF * RB;    // [NCE]
  static constexpr int OFF_RED = OFF_BETA + G::NCE;       // [NW][NS]
  // [8 lane groups][4 NCE/32 (+2 pad: the groups' ds_read_b128 broadcasts land in distinct banks)]
  static constexpr int OFF_BETAG = OFF_RED + NW * NS;     // row_stage_r's betas [LPR groups][BETAG_STRIDE]
  static constexpr int OFF_FLAG = OFF_BETAG + LPR * BETAG_STRIDE;      // counters (uint32)
  static constexpr int OFF_INIT = OFF_FLAG + NCNT / 2;                  // [6] init_const
  static constexpr int LDS_DOUBLES = OFF_INIT + 6;
  static_assert(LDS_DOUBLES == NBUF * PER_BUF + FIXED, "layout");
  static constexpr int LA = 1;
  static_assert(LA >= 1 && LA < NBUF, "row-stage lookahead within the ring");
  static_assert(XB % 2 == 0 && OFF_V % 2 == 0, "LDS-DMA destinations 16-byte aligned");
  static constexpr int QPW = P16;                         // column quads each row wave stages
  static_assert(LDS_DOUBLES * 8 <= 160 * 1024, "LDS");
  // every Gram wave's tiles fit NSEG segments and the eight runs cover the triangle
  static constexpr bool tiles_ok() {
    return TilesR<P16, 0>::NT + TilesR<P16, 1>::NT + TilesR<P16, 2>::NT + TilesR<P16, 3>::NT + TilesR<P16, 4>::NT +
               TilesR<P16, 5>::NT + TilesR<P16, 6>::NT + TilesR<P16, 7>::NT + (P16 == 16 ? 0 : 0) ==
           G::T;
  }
  static_assert(tiles_ok(), "the Gram waves' segments cover the tile triangle");
};

// X'Wz of block `buf` on the row waves (the Gram waves keep only their MFMA operands): row wave
// k owns column blocks [P16 k / 4, P16 (k+1) / 4) (4k .. 4k+3 at P16 = 16) and reads them in the
// MFMA operand layout (lane (cl, rq): column 16b + cl, rows 4j + rq -- conflict free),
// accumulating exactly the per-lane sums K1's gram_steps forms (k-steps in order, blocks in
// order); the epilogue combines them with K1's xor-16 / xor-32 shuffles, so X'Wz is bitwise K1's.
template <int P16, int K>
struct XzBlocks {
  static constexpr int LO = P16 * K / 4, N = P16 * (K + 1) / 4 - LO;
  static_assert(N >= 1 && N <= 4, "one to four column blocks per row wave");
};
template <int P16, int K>
__device__ __forceinline__ void xz_rows_r(const double* lds, int buf, int lane, double (&xz)[4]) {
  using G = Geo<P16>;
  using R = GeoR<P16>;
  using XB = XzBlocks<P16, K>;
  const double* xs = lds + R::OFF_X + buf * R::XB + XB::LO * G::BSTR;
  const double* wz = lds + R::OFF_W + buf * 2 * RB + RB;
  const int cl = lane & 15, rq = lane >> 4;
  const double* colbase = xs + cl * 32;
  // two LDS round trips (every read of a half issued before its first FMA: a round trip of a row
  // wave waits behind the Gram waves' operand reads, ~1-2K cycles)
#pragma unroll
  for (int h = 0; h < 2; ++h) {
    double xv[RB / 8][4], wv[RB / 8];
#pragma unroll
    for (int jj = 0; jj < RB / 8; ++jj) {
      const int r = 4 * (h * RB / 8 + jj) + rq;
      const double* base = colbase + (r ^ (2 * cl));
      wv[jj] = wz[r];
#pragma unroll
      for (int b = 0; b < XB::N; ++b) xv[jj][b] = base[G::BSTR * b];
    }
#pragma unroll
    for (int jj = 0; jj < RB / 8; ++jj)
#pragma unroll
      for (int b = 0; b < XB::N; ++b) xz[b] = fma(xv[jj][b], wv[jj], xz[b]);
    __builtin_amdgcn_sched_group_barrier(0x100, (XB::N + 1) * RB / 8, 1);
    __builtin_amdgcn_sched_group_barrier(0x002, XB::N * RB / 8, 1);
  }
}

// LDS-DMA staging of one row block by row wave si (K1's stage_block, the same instructions and
// LDS image) with the lane-dependent part of every source address precomputed (voff: 32-bit
// byte offsets of the four swizzle classes q mod 4) and the rest on the scalar unit: under the
// two MFMA streams of its SIMD every VALU instruction of a row wave waits for the fp64 pipe, and
// K1's per-quad 64-bit address arithmetic made the burst take 5-9K cycles.
template <int P16>
__device__ __forceinline__ void stage_block_r(double* lds, int buf, const PassArgs& a, int64_t blk, int si,
                                              const uint32_t (&voff)[4], uint32_t vvoff) {
  using G = Geo<P16>;
  typedef __attribute__((address_space(3))) double lds_double;
  lds_double* l3 = (lds_double*)__builtin_amdgcn_readfirstlane((int)(uintptr_t)(lds_void*)lds);
  lds_double* xdst = l3 + GeoR<P16>::OFF_X + buf * GeoR<P16>::XB;
  const int64_t r0 = blk * RB;
  const int q0 = si * GeoR<P16>::QPW;
#pragma unroll
  for (int k = 0; k < GeoR<P16>::QPW; ++k) {
    const int q = q0 + k;
    const int qs = q < a.nq ? q : a.nq - 1;  // quads past p: duplicates
    const char* sb = (const char*)(a.X + (int64_t)(4 * qs) * a.ld + r0);
    __builtin_amdgcn_global_load_lds((const void*)(sb + voff[q & 3]), (lds_void*)(xdst + (q >> 2) * G::BSTR + (q & 3) * 128), 16, 0, DMA_NT);
  }
  const double* src = a.y;
  if (si == 1 && a.m) src = a.m;
  if (si == 2 && a.off) src = a.off;
  if (si == 3 && a.prior) src = a.prior;
  const char* sb = (const char*)(src + r0);
  if ((int)vvoff < 16 * 16)
    __builtin_amdgcn_global_load_lds((const void*)(sb + vvoff), (lds_void*)(l3 + GeoR<P16>::OFF_V + buf * 4 * RB + si * RB), 16, 0, DMA_NT);
}

// Row stage of K1r: K1's row_stage (the same lanes, partial sums and reduction order, so w, w*z
// and the deviance are bitwise K1's) with its LDS reads in two round trips (columns u = 0, 1 of
// every stripe, then u = 2, 3 -- the order K1 adds them in) and beta from a per-lane-group copy
// (betag: the 32 betas of lane group g contiguous, 16 ds_read_b128 instead of 32 ds_read_b64;
// groups 34 doubles apart so that the eight groups' broadcasts hit distinct banks).
template <int P16, int FAM, int LNK>
__device__ __forceinline__ void row_stage_r(double* lds, int buf, const PassArgs& a, int64_t blk, int rw, int lane,
                                            double& s_dev, double& s_aux) {
  using G = Geo<P16>;
  using R = GeoR<P16>;
  constexpr int RW = R::RW, CPG = R::CPG, NT = R::NT;
  static_assert(P16 != 16 || (G::RW == RW && G::CPG == CPG && NT == 8), "K1's P16 = 16 row-stage geometry");
  const double* xs = lds + R::OFF_X + buf * R::XB;
  const int rl = lane % RW, g = lane / RW;
  const double* bg = lds + R::OFF_BETAG + g * R::BETAG_STRIDE;
  const int r = RW * rw + rl;
  const double* vv = lds + R::OFF_V + buf * 4 * RB;
  const double y = vv[r];
  const double m = a.m ? vv[RB + r] : 1.0;
  const double off = a.off ? vv[2 * RB + r] : 0.0;
  const double pw = a.prior ? vv[3 * RB + r] : 1.0;
  double eta = 0.0;
  if (a.mode == MODE_IRLS) {
    double e4[4] = {0.0, 0.0, 0.0, 0.0};
#pragma unroll
    for (int h = 0; h < CPG / 2; ++h) {
      double xv[2][NT], bv[2][NT];
#pragma unroll
      for (int uu = 0; uu < 2; ++uu) {
        const int u = 2 * h + uu;
        const int c0 = CPG * g + u;
        const double* base = xs + (c0 >> 4) * G::BSTR + (c0 & 15) * 32 + (r ^ ((2 * c0) & 31));
#pragma unroll
        for (int t = 0; t < NT; ++t) {
          xv[uu][t] = base[2 * G::BSTR * t];
          bv[uu][t] = bg[t * CPG + u];
        }
      }
#pragma unroll
      for (int uu = 0; uu < 2; ++uu)
#pragma unroll
        for (int t = 0; t < NT; ++t) e4[t & 3] += xv[uu][t] * bv[uu][t];
      __builtin_amdgcn_sched_group_barrier(0x100, 3 * NT, 2);
      __builtin_amdgcn_sched_group_barrier(0x002, 2 * NT, 2);
    }
    eta = (e4[0] + e4[1]) + (e4[2] + e4[3]);
    if constexpr (RW <= 8) eta = add_xor8(eta);
    eta = add_xor16(eta);
    eta = add_xor32(eta);
  }
  if (lane < RW) {
    const int64_t row = blk * RB + r;
    double w = 0.0, wz = 0.0;
    if (row < a.n) {
      if (a.mode == MODE_IRLS) eta = eta + off;
      if (FAM == FAM_BINOMIAL && init_fast_row(FAM, a.mode, a.m != nullptr) && y >= 0.0 && y <= 1.0)
        pass_row_init(lds + R::OFF_INIT, y, off, pw, w, wz, s_dev, s_aux);
      else pass_row(FAM, LNK, a.mode, eta, y, m, off, pw, a.mu0, a.ybar, a.m != nullptr, w, wz, s_dev, s_aux, true);
    }
    lds[R::OFF_W + buf * 2 * RB + r] = w;
    lds[R::OFF_W + buf * 2 * RB + RB + r] = wz;
    // eta leaves through LDS: Gram wave 0 stores it after the block's Gram, so the row waves' only
    // vector-memory operations are their LDS-DMA and vmcnt counts exactly the blocks in flight
    lds[R::OFF_ETA + buf * RB + r] = eta;
  }
}

template <int P16, int WV>
__device__ __forceinline__ void gram_steps_r(const double* lds, int buf, int lane, d4 (&acc)[TilesR<P16, WV>::NT]) {
  using G = Geo<P16>;
  using T = TilesR<P16, WV>;
  const double* xs = lds + GeoR<P16>::OFF_X + buf * GeoR<P16>::XB;
  const double* w = lds + GeoR<P16>::OFF_W + buf * 2 * RB;
  const int cl = lane & 15, rq = lane >> 4;
  const double* colbase = xs + cl * 32;
  auto kstep = [&](int j) {
    const int r = 4 * j + rq;
    const double* base = colbase + (r ^ (2 * cl));
    const double wr = w[r];
    double av[NSEG];
#pragma unroll
    for (int sg = 0; sg < NSEG; ++sg) {
      av[sg] = 0.0;
      if (T::cnt(sg) > 0) av[sg] = base[G::BSTR * (T::row(sg) >= 0 ? T::row(sg) : 0)] * wr;
    }
#pragma unroll
    for (int k = 0; k < T::NT; ++k) {
      const int sg = T::seg_of(k);
      const double b = base[G::BSTR * (T::j0(sg) + k - T::off(sg))];
      acc[k] = __builtin_amdgcn_mfma_f64_16x16x4f64(av[sg], b, acc[k], 0, 0, 0);
    }
    // Keep 6 B-operand reads in flight ahead of the MFMAs (under the 168-VGPR budget of three
    // waves per SIMD the default schedule waits for every read in turn): the A-side reads and the
    // first reads, then one MFMA per further read.
    __builtin_amdgcn_sched_group_barrier(0x100, 4 + 6, 0);
#pragma unroll
    for (int k = 0; k < T::NT; ++k) {
      __builtin_amdgcn_sched_group_barrier(0x008, 1, 0);
      __builtin_amdgcn_sched_group_barrier(0x100, 1, 0);
    }
  };
#pragma unroll 1
  for (int j = 0; j < RB / 4; j += 2) {
    // the two Gram waves of a SIMD take turns at the higher issue priority, one k-step each, so
    // neither runs ahead and leaves the other alone at the end of the block (oldest-first
    // arbitration: waves 0-3 finished their Gram ~7K cycles before waves 4-7)
    if constexpr (!T::ROW) __builtin_amdgcn_s_setprio((WV >> 2) & 1 ? 0 : 1);
    kstep(j);
    if constexpr (!T::ROW) __builtin_amdgcn_s_setprio((WV >> 2) & 1 ? 1 : 0);
    kstep(j + 1);
  }
}

template <int P16, int FAM, int LNK, int WV>
__device__ __forceinline__ void pass_body_r(double* lds, const PassArgs& a, int lane) {
  using G = Geo<P16>;
  using R = GeoR<P16>;
  using T = TilesR<P16, WV>;
  constexpr bool row_wave = T::ROW;
  constexpr int si = row_wave ? WV - 8 : 0;  // DMA issuer index (row waves)
  const int wg = blockIdx.x, nwg = gridDim.x;
  const int64_t b0 = (a.nblocks * wg) / nwg, b1 = (a.nblocks * (wg + 1)) / nwg;
  const bool do_gram = !a.no_gram;
  unsigned* flag = (unsigned*)(lds + R::OFF_FLAG);

  d4 acc[T::NT > 0 ? T::NT : 1];
#pragma unroll
  for (int k = 0; k < T::NT; ++k) acc[k] = d4{0.0, 0.0, 0.0, 0.0};
  double xz[4] = {0.0, 0.0, 0.0, 0.0}, s_dev = 0.0, s_aux = 0.0;

  // lane parts of the DMA source addresses (bytes): column quad q's 4 columns at cq * ld, rows
  // in the slot swizzle of stage_block, which depends on q mod 4 only
  uint32_t voff[4];
  const int li = lane & 15, lcq = lane >> 4;
#pragma unroll
  for (int k = 0; k < 4; ++k) voff[k] = (uint32_t)(((int64_t)lcq * a.ld + ((2 * li) ^ ((8 * k + 2 * lcq) & 31))) * 8);
  const uint32_t vvoff = (uint32_t)(lane < 16 ? 16 * lane : 16 * 16);
  constexpr int NB = R::NBUF, PER = R::QPW + 1;  // ring depth; vector-memory operations per staged block
  if (row_wave)
#pragma unroll
    for (int k = 0; k < NB; ++k)
      if (b0 + k < b1) stage_block_r<P16>(lds, k, a, b0 + k, si, voff, vvoff);
  if (row_wave) __builtin_amdgcn_s_setprio(2);
  // wait until this wave's DMA of a block has landed while `later` blocks staged after it may fly
  auto wait_landed = [&](int64_t later) {
    if constexpr (NB >= 4)
      if (later >= 3) return wait_vmcnt<3 * PER>();
    if constexpr (NB >= 3)
      if (later >= 2) return wait_vmcnt<2 * PER>();
    if (later >= 1) return wait_vmcnt<PER>();
    wait_vmcnt<0>();
  };
  // No block barrier: LDS counters order the ring of NBUF buffers.
  //   flag      : +1 per row wave when its LDS-DMA part of a block has landed (4 per block); every row
  //               wave bumps it once per block and then waits for all four, so it acts as a barrier
  //               among the row waves and a plain count is exact
  //   ready[s]  : +1 per row-stage wave when its rows of the block in ring slot s are in the w buffer
  //               (RG per block)
  //   done[s]   : +1 per wave when it has finished reading the block in slot s: the Gram waves' MFMAs,
  //               the row waves' X'Wz (12 per block)
  // Per-slot counters: the Gram waves are not coupled to each other, and a fast one may finish a block
  // while a slow one is still in an earlier block -- one counter for all blocks would then count the
  // fast wave's later block as the slow wave's, and the slot could be restaged under the slow wave.
  // A slot's next use cannot begin before its counters reached the current round's targets (its DMA
  // waits for done[s]), so a per-slot count is exact.
  // A Gram wave starts block b once ready(b), so the two Gram waves of a SIMD no longer end every
  // block with one of them alone on the MFMA pipe; the row waves stage block b+NBUF into block b's
  // slot after done(b).  (The row stage of b+NBUF rewrites w(b): it follows the flag round of
  // b+NBUF, i.e. every row wave's DMA of b+NBUF, each issued after done(b).)
  unsigned* ready = flag + 1;     // [NB]
  unsigned* done = flag + 1 + 4;  // [NB]
  constexpr int RG = R::RG, LA = R::LA;
  auto spin = [&](unsigned* c, unsigned target) {
    while (__hip_atomic_load(c, __ATOMIC_ACQUIRE, __HIP_MEMORY_SCOPE_WORKGROUP) < target) __builtin_amdgcn_s_sleep(1);
  };
  auto bump = [&](unsigned* c) {
    if (lane == 0) __hip_atomic_fetch_add(c, 1u, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_WORKGROUP);
  };
  auto next_buf = [](int b) { return b + 1 == NB ? 0 : b + 1; };
  if constexpr (row_wave) {
    // row stages of the first LA blocks (slots 0 .. LA-1), each after its flag round
#pragma unroll
    for (int c = 0; c < LA; ++c) {
      if (b0 + c < b1) {
        wait_landed(std::min<int64_t>(b1 - b0 - 1, NB - 1) - c);
        bump(flag);
        spin(flag, 4u * (c + 1));
        row_stage_r<P16, FAM, LNK>(lds, c, a, b0 + c, si, lane, s_dev, s_aux);
        bump(ready + c);
      }
    }
    int cur = 0;
    unsigned rnd = 0;  // uses of slot cur before block blk
#pragma unroll 1
    for (int64_t blk = b0; blk < b1; ++blk) {
      if (blk + LA < b1) {  // the row stage of block blk + LA
        wait_landed(std::min<int64_t>(b1 - 1, blk + NB - 1) - (blk + LA));
        bump(flag);
        spin(flag, (unsigned)(4 * (blk + LA - b0 + 1)));
        int sl = cur + LA;
        if (sl >= NB) sl -= NB;
        row_stage_r<P16, FAM, LNK>(lds, sl, a, blk + LA, si, lane, s_dev, s_aux);
        bump(ready + sl);
      }
      // X'Wz of block blk reads every row wave's w*z of it: the flag round above ordered them (each
      // row wave bumps flag after its row stage of blk); the last LA blocks have no such round
      if (blk + LA >= b1) spin(ready + cur, (unsigned)(RG * (rnd + 1)));
      if (do_gram) xz_rows_r<P16, si>(lds, cur, lane, xz);
      bump(done + cur);  // this row wave's reads of block blk (X'Wz) are complete
      if (blk + NB < b1) {
        spin(done + cur, 12u * (rnd + 1));
        stage_block_r<P16>(lds, cur, a, blk + NB, si, voff, vvoff);
      }
      cur = next_buf(cur);
      if (cur == 0) ++rnd;
    }
  } else {
    int cur = 0;
    unsigned rnd = 0;
#pragma unroll 1
    for (int64_t blk = b0; blk < b1; ++blk) {
      spin(ready + cur, (unsigned)(RG * (rnd + 1)));
      if (do_gram) gram_steps_r<P16, WV>(lds, cur, lane, acc);
      if constexpr (WV == 0)  // the row stage's eta of this block (IRLS passes that keep it)
        if (a.eta_out && a.mode == MODE_IRLS && lane < RB && blk * RB + lane < a.n)
          a.eta_out[blk * RB + lane] = lds[R::OFF_ETA + cur * RB + lane];
      bump(done + cur);
      cur = next_buf(cur);
      if (cur == 0) ++rnd;
    }
  }
  if (row_wave) __builtin_amdgcn_s_setprio(0);

  // ---- epilogue: this workgroup's partial (the layout of K1's) ----
  double* out = a.partials + (int64_t)wg * a.stride;
#pragma unroll
  for (int k = 0; k < T::NT; ++k) {
    const int sg = T::seg_of(k);
    const int bi = T::row(sg), bj = T::j0(sg) + k - T::off(sg);
    const int t = bi * (bi + 1) / 2 + bj;
#pragma unroll
    for (int j = 0; j < 4; ++j) out[t * 256 + 64 * j + lane] = acc[k][j];
  }
  if constexpr (row_wave) {
#pragma unroll
    for (int b = 0; b < XzBlocks<P16, si>::N; ++b) {
      double v = xz[b];
      v += __shfl_xor(v, 16);
      v += __shfl_xor(v, 32);
      if (lane < 16) out[G::T * 256 + 16 * (XzBlocks<P16, si>::LO + b) + lane] = v;
    }
  }
#pragma unroll
  for (int o = 1; o < 64; o <<= 1) {
    s_dev += __shfl_xor(s_dev, o);
    s_aux += __shfl_xor(s_aux, o);
  }
  if (lane == 0) {
    lds[R::OFF_RED + WV * NS + 0] = s_dev;
    lds[R::OFF_RED + WV * NS + 1] = s_aux;
  }
  lds_barrier();
  if (WV == 0 && lane < NS) {
    // the row waves' sums in K1's order (its row waves 4..7 are waves 8..11 here; the Gram
    // waves contribute zeros, as K1's MFMA-only waves did)
    double sd = 0.0, sa = 0.0;
    for (int k = 0; k < R::NW; ++k) {
      sd += lds[R::OFF_RED + k * NS + 0];
      sa += lds[R::OFF_RED + k * NS + 1];
    }
    double v = 0.0;
    if (lane == S_DEV) v = sd;
    if (lane == S_SUMW) v = sa;
    out[G::T * 256 + G::NC + lane] = v;
  }
}

template <int P16, int FAM, int LNK>
__global__ void __launch_bounds__(64 * GeoR<P16>::NW, 3) irls_pass_r_kernel(PassArgs a) {
  using G = Geo<P16>;
  using R = GeoR<P16>;
  __shared__ double lds[R::LDS_DOUBLES];
  const int lane = threadIdx.x & 63;
  const int wv = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  for (int c = threadIdx.x; c < G::NCE; c += 64 * R::NW) {
    const double b = (a.beta && c < a.p) ? a.beta[c] : 0.0;
    lds[R::OFF_BETA + c] = b;
    // betag[g][t * CPG + u] = beta[CPG g + u + 32 t] (row_stage_r)
    lds[R::OFF_BETAG + ((c & 31) / R::CPG) * R::BETAG_STRIDE + (c >> 5) * R::CPG + (c & 31) % R::CPG] = b;
  }
  if (threadIdx.x < R::NCNT) ((unsigned*)(lds + R::OFF_FLAG))[threadIdx.x] = 0u;
  if constexpr (G::NCE > G::NC) {  // odd P16: the row stage's last stripe reads 16 columns no DMA writes
    for (int e = threadIdx.x; e < (G::NCE - G::NC) * RB; e += 64 * R::NW) {
      const int c = G::NC + e / RB, r = e % RB;
#pragma unroll
      for (int k = 0; k < R::NBUF; ++k) lds[R::OFF_X + k * R::XB + (c >> 4) * G::BSTR + (c & 15) * RB + r] = 0.0;
    }
  }
  if constexpr (FAM == FAM_BINOMIAL)
    if (threadIdx.x == 0 && init_fast_row(FAM, a.mode, a.m != nullptr)) {
      const InitConst ic = init_const(FAM, LNK, a.mode, a.mu0);
      for (int k = 0; k < 6; ++k) lds[R::OFF_INIT + k] = ic.v[k];
    }
  __syncthreads();
  switch (wv) {
    case 0: pass_body_r<P16, FAM, LNK, 0>(lds, a, lane); break;
    case 1: pass_body_r<P16, FAM, LNK, 1>(lds, a, lane); break;
    case 2: pass_body_r<P16, FAM, LNK, 2>(lds, a, lane); break;
    case 3: pass_body_r<P16, FAM, LNK, 3>(lds, a, lane); break;
    case 4: pass_body_r<P16, FAM, LNK, 4>(lds, a, lane); break;
    case 5: pass_body_r<P16, FAM, LNK, 5>(lds, a, lane); break;
    case 6: pass_body_r<P16, FAM, LNK, 6>(lds, a, lane); break;
    case 7: pass_body_r<P16, FAM, LNK, 7>(lds, a, lane); break;
    case 8: pass_body_r<P16, FAM, LNK, 8>(lds, a, lane); break;
    case 9: pass_body_r<P16, FAM, LNK, 9>(lds, a, lane); break;
    case 10: pass_body_r<P16, FAM, LNK, 10>(lds, a, lane); break;
    default: pass_body_r<P16, FAM, LNK, 11>(lds, a, lane); break;
  }
}

// K1 launch for the family/link of the pass (LM passes: the Gaussian identity row stage).
template <int P16>
static hipError_t launch_pass_k1(const PassArgs& a, int grid, hipStream_t st, hipEvent_t e0, hipEvent_t e1) {
  const dim3 g(grid), b(64 * Geo<P16>::NW);
  const int mode_fam = (a.mode == MODE_LM_GRAM) ? FAM_GAUSSIAN : a.family;
  const int mode_lnk = (a.mode == MODE_LM_GRAM) ? LNK_IDENTITY : a.link;
  if (mode_fam == FAM_BINOMIAL && mode_lnk == LNK_LOGIT)
    hipExtLaunchKernelGGL((irls_pass_kernel<P16, FAM_BINOMIAL, LNK_LOGIT>), g, b, 0, st, e0, e1, 0, a);
  else if (mode_fam == FAM_BINOMIAL && mode_lnk == LNK_PROBIT)
    hipExtLaunchKernelGGL((irls_pass_kernel<P16, FAM_BINOMIAL, LNK_PROBIT>), g, b, 0, st, e0, e1, 0, a);
  else if (mode_fam == FAM_BINOMIAL)
    hipExtLaunchKernelGGL((irls_pass_kernel<P16, FAM_BINOMIAL, LNK_CLOGLOG>), g, b, 0, st, e0, e1, 0, a);
  else if (mode_fam == FAM_GAUSSIAN)
    hipExtLaunchKernelGGL((irls_pass_kernel<P16, FAM_GAUSSIAN, LNK_IDENTITY>), g, b, 0, st, e0, e1, 0, a);
  else if (mode_fam == FAM_POISSON)
    hipExtLaunchKernelGGL((irls_pass_kernel<P16, FAM_POISSON, LNK_LOG>), g, b, 0, st, e0, e1, 0, a);
  else if (mode_fam == FAM_GAMMA)
    hipExtLaunchKernelGGL((irls_pass_kernel<P16, FAM_GAMMA, LNK_INVERSE>), g, b, 0, st, e0, e1, 0, a);
  else
    return hipErrorInvalidValue;
  return hipGetLastError();
}

// K1r launch for the family/link of the pass (LM passes: the Gaussian identity row stage).
template <int P16>
static hipError_t launch_pass_r_fl(const PassArgs& a, int grid, hipStream_t st, hipEvent_t e0, hipEvent_t e1) {
  const int fam = (a.mode == MODE_LM_GRAM) ? FAM_GAUSSIAN : a.family;
  const int lnk = (a.mode == MODE_LM_GRAM) ? LNK_IDENTITY : a.link;
  const dim3 g(grid), b(64 * GeoR<P16>::NW);
  if (fam == FAM_BINOMIAL && lnk == LNK_LOGIT) hipExtLaunchKernelGGL((irls_pass_r_kernel<P16, FAM_BINOMIAL, LNK_LOGIT>), g, b, 0, st, e0, e1, 0, a);
  else if (fam == FAM_BINOMIAL && lnk == LNK_PROBIT) hipExtLaunchKernelGGL((irls_pass_r_kernel<P16, FAM_BINOMIAL, LNK_PROBIT>), g, b, 0, st, e0, e1, 0, a);
  else if (fam == FAM_BINOMIAL) hipExtLaunchKernelGGL((irls_pass_r_kernel<P16, FAM_BINOMIAL, LNK_CLOGLOG>), g, b, 0, st, e0, e1, 0, a);
  else if (fam == FAM_GAUSSIAN) hipExtLaunchKernelGGL((irls_pass_r_kernel<P16, FAM_GAUSSIAN, LNK_IDENTITY>), g, b, 0, st, e0, e1, 0, a);
  else if (fam == FAM_POISSON) hipExtLaunchKernelGGL((irls_pass_r_kernel<P16, FAM_POISSON, LNK_LOG>), g, b, 0, st, e0, e1, 0, a);
  else if (fam == FAM_GAMMA) hipExtLaunchKernelGGL((irls_pass_r_kernel<P16, FAM_GAMMA, LNK_INVERSE>), g, b, 0, st, e0, e1, 0, a);
  else return hipErrorInvalidValue;
  return hipGetLastError();
}

}  // namespace sglm
