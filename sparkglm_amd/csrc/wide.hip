// wide.hip -- the wide-design (p > 256) IRLS pass for gfx950.
//
// A p x p Gramian no longer fits in one workgroup's registers beyond p = 256 (the fused
// kernel keeps all 136 tiles of a 256-column Gram resident), so the pass splits in two
// streaming kernels plus a fixed-order reduction:
//
//   wide_rows_kernel   eta = X beta + offset (etaCreate, GLM.scala:321-332), mu, g', V,
//                      w and w*z (zwCreateBinomial, GLM.scala:359-395) and the deviance
//                      partials; one coalesced read of X (thread per row), w / w*z
//                      written to two n-vectors.                       -> HBM-bound
//   wide_gram_kernel   X'WX over 128 x 128 column "super-tiles" (panel pairs I >= J) of
//                      16x16 fp64 MFMA tiles; persistent, two 4-wave workgroups per CU,
//                      each running a cost-balanced list of (super-tile, row range)
//                      pieces; diagonal super-tiles also form X'Wz.  Panels stream
//                      through LDS by LDS-DMA, double-buffered.        -> MFMA-bound
//   wide_reduce_kernel fixed-order sum of the work-item partials and the row partials
//                      into the packed wire format (deterministic).
//
// (partitionComponents / wlsComponents, utils.scala:84-126.)
#include <hip/hip_runtime.h>

#include <cstdint>

#include "common.hpp"
#include "kernels.hpp"
#include "procx.hpp"
#include "rowmath.hpp"

namespace sglm {

typedef double d4 __attribute__((ext_vector_type(4)));
typedef double dv2 __attribute__((ext_vector_type(2)));
typedef __attribute__((address_space(3))) void lds_void;

namespace {

// s_waitcnt vmcnt(N) with expcnt / lgkmcnt left open (gfx9 encoding).
template <int N>
__device__ __forceinline__ void wait_vm() {
  static_assert(N >= 0 && N < 64, "vmcnt range");
  __builtin_amdgcn_s_waitcnt((N & 15) | ((N >> 4) << 14) | (7 << 4) | (15 << 8));
}

__device__ __forceinline__ void lds_bar() { asm volatile("s_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory"); }

// LDS image (doubles) of one 16-row block of one 128-column panel: column c at (c >> 4) TB +
// 16 (c & 15), row r
// in slot r ^ f(c), f(c) = 2((c >> 1) & 7).  The XOR is applied on the DMA source address
// (the LDS-DMA destination is lane-linear; f even keeps each lane's 16-byte row pair
// contiguous) and makes the MFMA fragment reads (ds_read_b64, lanes (rq, cl) reading row
// 4s+rq of column 16b+cl) bank-conflict free: within each 32-lane group the 32 reads hit
// 16*(cl & 1) + ((4s + rq) ^ 2(cl >> 1)) mod 32, all distinct.
constexpr int PANEL = WIDE_PANEL;          // columns per panel
constexpr int PT = PANEL / 16;             // 16-column tile blocks per panel (8)
constexpr int WRB = WIDE_RB;               // rows per block (16)
// 16-column tile blocks TB = 16 WRB + 2 doubles apart: the pad keeps the MFMA operand reads of
// the four tiles of a wave row plain ds_read_b64 -- at 256 doubles apart the compiler pairs them
// into ds_read2st64_b64 (8 LDS cycles, and 2-way bank conflicts under the row swizzle: PMC
// SQ_LDS_BANK_CONFLICT was 48 % of the Gram kernels' LDS cycles).  (+2 keeps the LDS-DMA
// destinations 16-byte aligned.)
constexpr int TB = 16 * WRB + 2;           // doubles per 16-column tile block, padded (258)
constexpr int PB = PT * TB;                // doubles per panel block image (2064)
constexpr int OFF_X = 0;                   // [2 buffers][2 panels (I, J)][PB]
constexpr int OFF_V = 4 * PB;              // [2 buffers][w, w*z][WRB]
constexpr int LDS_DOUBLES = OFF_V + 4 * WRB;
// diagonal-super-tile kernel: [2 buffers][PB] | [2 buffers][w, w*z][WRB]
constexpr int OFF_VD = 2 * PB;
constexpr int LDS_DIAG = OFF_VD + 4 * WRB;
constexpr int NWAVE = 4;                   // one wave per SIMD; two workgroups per CU
// Workgroups per CU of the diagonal-super-tile kernel.  Its LDS image is one panel per buffer
// (33.5 KB), so three fit beside each other; measured: three waves per SIMD instead of two change
// nothing (p = 512 -0.3 %) and spill a few VGPRs, so two.
constexpr int DIAG_WG = 2;

__device__ __forceinline__ int swz(int c) { return 2 * ((c >> 1) & 7); }

// Stage block blk of panels I (and J unless DIAG) into buffer buf: one global_load_lds of
// 16 bytes per lane moves an "octet" of 8 columns x 16 rows; 16 octets per panel.  The
// source address is a wave-uniform part (octet column, block row: SGPRs) plus one of two
// per-lane offsets (column within the octet, swizzled row pair; swz depends only on the
// octet's parity), so no per-octet addresses stay live in VGPRs.  Octets past the stored
// columns (a multiple of 8) are skipped: they only feed tiles beyond p.
// PROC: the octet is generated (procx.hpp) and written by ds_write_b128 into the slots the
// DMA would fill (the pipeline's lgkmcnt(0) + barrier orders it like the DMA's vmcnt wait).
template <bool DIAG, bool PROC, int K0 = 0, int K1 = (DIAG ? 4 : 8)>
__device__ __forceinline__ void wstage(double* lds, int buf, const WideGramArgs& a, int64_t blk, int I, int J, int wv,
                                       const int64_t (&loff)[2], int lane) {
  constexpr int OW = DIAG ? 4 : 8;  // octets per wave; this call stages octets [K0, K1)
  const double* xb = a.X + blk * WRB;
#pragma unroll
  for (int k = K0; k < K1; ++k) {
    const int qq = wv * OW + k;  // 0..15 panel I, 16..31 panel J
    const int ps = qq >> 4, ol = qq & 15;
    const int c0 = (ps ? J : I) * PANEL + ol * 8;  // first column of the octet (uniform)
    if (c0 < a.ncols) {
      if constexpr (PROC) {
        const int oc = lane >> 3, i = lane & 7;
        const int64_t r = blk * WRB + ((2 * i) ^ swz(8 * (ol & 1) + oc));
        const double2 v = {proc_x(a.proc, r, c0 + oc), proc_x(a.proc, r + 1, c0 + oc)};
        *(double2*)(lds + OFF_X + (buf * 2 + ps) * PB + (ol >> 1) * TB + (ol & 1) * 128 + 2 * lane) = v;
      } else {
        __builtin_amdgcn_global_load_lds((const void*)(xb + (int64_t)c0 * a.ld + loff[ol & 1]),
                                         (lds_void*)(lds + OFF_X + (buf * 2 + ps) * PB + (ol >> 1) * TB + (ol & 1) * 128), 16, 0, 0);
      }
    }
  }
  if (K0 == 0) {
    const int v = wv & 1;  // waves alternate w / w*z (identical redundant copies)
    const double* vsrc = (v ? a.wz : a.w) + blk * WRB + 2 * lane;
    if (lane < WRB / 2)
      __builtin_amdgcn_global_load_lds((const void*)vsrc, (lds_void*)(lds + OFF_V + (buf * 2 + v) * WRB), 16, 0, 0);
  }
}

// Diagonal super-tiles: stage block blk of panel I into buffer buf of the one-panel image --
// four octets per wave, and w (wave 0) / w*z (wave 1) of the block.  Each panel is read by exactly
// one diagonal workgroup per block, so these loads are non-temporal (DMA_NT: 20M x 512 Gram pass
// -3.8 % on a same-box A/B, 3M x 2048 +-0); the off-diagonal staging above re-reads every panel
// from L2 / MALL across super-tiles and keeps the default policy (nt there measured +7 %).
template <bool PROC>
__device__ __forceinline__ void wstage_diag(double* lds, int buf, const WideGramArgs& a, int64_t blk, int I, int wv,
                                            const int64_t (&loff)[2], int lane) {
  const double* xb = a.X + blk * WRB;
  double* dst = lds + buf * PB;
#pragma unroll
  for (int k = 0; k < 4; ++k) {
    const int ol = wv * 4 + k;
    const int c0 = I * PANEL + ol * 8;
    if (c0 < a.ncols) {
      if constexpr (PROC) {
        const int oc = lane >> 3, i = lane & 7;
        const int64_t r = blk * WRB + ((2 * i) ^ swz(8 * (ol & 1) + oc));
        const double2 v = {proc_x(a.proc, r, c0 + oc), proc_x(a.proc, r + 1, c0 + oc)};
        *(double2*)(dst + (ol >> 1) * TB + (ol & 1) * 128 + 2 * lane) = v;
      } else {
        __builtin_amdgcn_global_load_lds((const void*)(xb + (int64_t)c0 * a.ld + loff[ol & 1]),
                                         (lds_void*)(dst + (ol >> 1) * TB + (ol & 1) * 128), 16, 0, DMA_NT);
      }
    }
  }
  if (wv < 2) {
    const double* vsrc = (wv ? a.wz : a.w) + blk * WRB + 2 * lane;
    if (lane < WRB / 2)
      __builtin_amdgcn_global_load_lds((const void*)vsrc, (lds_void*)(lds + OFF_VD + (buf * 2 + wv) * WRB), 16, 0, DMA_NT);
  }
}

// Per-lane DMA offsets (doubles) for even / odd octets: column oc = lane >> 3 of the octet,
// rows (2i, 2i+1) ^ swz(column), i = lane & 7.
__device__ __forceinline__ void lane_offsets(const WideGramArgs& a, int lane, int64_t (&loff)[2]) {
  const int i = lane & 7, oc = lane >> 3;
#pragma unroll
  for (int par = 0; par < 2; ++par) loff[par] = (int64_t)oc * a.ld + ((2 * i) ^ swz(8 * par + oc));
}

// Off-diagonal super-tile: wave wv owns tile rows 4(wv>>1)+{0..3} of panel I and tile
// columns 4(wv&1)+{0..3} of panel J (16 tiles).  A = X_I * w (row-scaled), B = X_J.  The
// operands of k-step s+1 are read from LDS while the 16 MFMAs of step s issue.
// hook(s) runs after the MFMAs of k-step s are issued (the procedural mode generates the next
// block's octets there, so the integer hashing interleaves with the MFMA stream).
template <typename Hook>
__device__ __forceinline__ void offdiag_block(const double* lds, int buf, int wv, int lane, d4 (&acc)[16],
                                              Hook&& hook) {
  const int cl = lane & 15, rq = lane >> 4;
  const int f = 2 * (cl >> 1);
  const double* xI = lds + OFF_X + (buf * 2 + 0) * PB + cl * WRB + TB * (4 * (wv >> 1));
  const double* xJ = lds + OFF_X + (buf * 2 + 1) * PB + cl * WRB + TB * (4 * (wv & 1));
  const double* w = lds + OFF_V + (buf * 2 + 0) * WRB;
  double av[2][4], bv[2][4], wr[2];
  auto load = [&](int s, int slot) {
    const int r = 4 * s + rq;
    const int o = r ^ f;
    wr[slot] = w[r];
#pragma unroll
    for (int t = 0; t < 4; ++t) av[slot][t] = xI[o + TB * t];
#pragma unroll
    for (int u = 0; u < 4; ++u) bv[slot][u] = xJ[o + TB * u];
  };
  load(0, 0);
#pragma unroll
  for (int s = 0; s < WRB / 4; ++s) {
    const int cur = s & 1;
    if (s + 1 < WRB / 4) load(s + 1, cur ^ 1);
    double as[4];
#pragma unroll
    for (int t = 0; t < 4; ++t) as[t] = av[cur][t] * wr[cur];
#pragma unroll
    for (int t = 0; t < 4; ++t)
#pragma unroll
      for (int u = 0; u < 4; ++u)
        acc[4 * t + u] = __builtin_amdgcn_mfma_f64_16x16x4f64(as[t], bv[cur][u], acc[4 * t + u], 0, 0, 0);
    hook(s);
  }
}

// Diagonal super-tile: wave q owns tile rows LO = q and HI = 7-q of the lower tile grid,
// tiles (LO,0..LO) and (HI,0..HI): 9 tiles, 36 over the four waves; X'Wz on the VALU.
template <int Q>
__device__ __forceinline__ void diag_block(const double* lds, int buf, int lane, d4 (&acc)[9], double& xz_lo,
                                           double& xz_hi) {
  constexpr int LO = Q, HI = PT - 1 - Q;  // HI >= LO: the B operands are tile columns 0..HI
  const int cl = lane & 15, rq = lane >> 4;
  const int f = 2 * (cl >> 1);
  const double* xs = lds + buf * PB + cl * WRB;
  const double* w = lds + OFF_VD + (buf * 2 + 0) * WRB;
  const double* wz = lds + OFF_VD + (buf * 2 + 1) * WRB;
  // operands of k-step s + 1 (all operands of a block first, then its 36 MFMAs: +0.6 %, not kept) are read from LDS while the 9 MFMAs of step s issue
  double xv[2][HI + 1], wr[2], wzr[2];
  auto load = [&](int s, int slot) {
    const int r = 4 * s + rq;
    const int o = r ^ f;
    wr[slot] = w[r];
    wzr[slot] = wz[r];
#pragma unroll
    for (int c = 0; c <= HI; ++c) xv[slot][c] = xs[o + TB * c];
  };
  load(0, 0);
#pragma unroll
  for (int s = 0; s < WRB / 4; ++s) {
    const int cur = s & 1;
    if (s + 1 < WRB / 4) load(s + 1, cur ^ 1);
    const double x_lo = xv[cur][LO], x_hi = xv[cur][HI];
    const double a_lo = x_lo * wr[cur], a_hi = x_hi * wr[cur];
    xz_lo += x_lo * wzr[cur];
    xz_hi += x_hi * wzr[cur];
#pragma unroll
    for (int k = 0; k <= PT; ++k)
      acc[k] = __builtin_amdgcn_mfma_f64_16x16x4f64(k <= LO ? a_lo : a_hi, xv[cur][k <= LO ? k : k - LO - 1], acc[k],
                                                    0, 0, 0);
  }
}

// Pipeline per piece (two LDS buffers, one barrier per block):
//   wait for this wave's DMA of block blk; barrier (every wave's DMA of blk has landed and
//   every wave is done reading the other buffer); DMA block blk+1 into the other buffer;
//   MFMAs of block blk.  The DMA of blk+1 flies under blk's MFMAs, and the second
//   workgroup on the CU covers whatever latency is left.
template <int Q, bool PROC>
__device__ void diag_piece(double* lds, const WideGramArgs& a, int I, int64_t b0, int64_t b1, int64_t bs, int wv,
                           int lane, double* out) {
  d4 acc[9];
#pragma unroll
  for (int k = 0; k < 9; ++k) acc[k] = d4{0.0, 0.0, 0.0, 0.0};
  double xz_lo = 0.0, xz_hi = 0.0;
  int64_t loff[2];
  lane_offsets(a, lane, loff);
  int cur = 0;
  if (b0 < b1) wstage_diag<PROC>(lds, 0, a, b0, I, wv, loff, lane);
#pragma unroll 1
  for (int64_t blk = b0; blk < b1; blk += bs, cur ^= 1) {
    wait_vm<0>();
    lds_bar();
    if (blk + bs < b1) wstage_diag<PROC>(lds, cur ^ 1, a, blk + bs, I, wv, loff, lane);
    diag_block<Q>(lds, cur, lane, acc, xz_lo, xz_hi);
  }
  constexpr int LO = Q, HI = PT - 1 - Q;
#pragma unroll
  for (int k = 0; k <= PT; ++k) {
    const int bi = k <= LO ? LO : HI, bj = k <= LO ? k : k - LO - 1;
    const int t = bi * PT + bj;
#pragma unroll
    for (int j = 0; j < 4; ++j) out[t * 256 + 64 * j + lane] = acc[k][j];
  }
  xz_lo += __shfl_xor(xz_lo, 16);
  xz_lo += __shfl_xor(xz_lo, 32);
  xz_hi += __shfl_xor(xz_hi, 16);
  xz_hi += __shfl_xor(xz_hi, 32);
  if (lane < 16) {
    out[PT * PT * 256 + 16 * LO + lane] = xz_lo;
    out[PT * PT * 256 + 16 * HI + lane] = xz_hi;
  }
}

template <bool PROC>
__device__ void offdiag_piece(double* lds, const WideGramArgs& a, int I, int J, int64_t b0, int64_t b1, int64_t bs,
                              int wv, int lane, double* out) {
  d4 acc[16];
#pragma unroll
  for (int k = 0; k < 16; ++k) acc[k] = d4{0.0, 0.0, 0.0, 0.0};
  int64_t loff[2];
  lane_offsets(a, lane, loff);
  if (b0 < b1) wstage<false, PROC>(lds, 0, a, b0, I, J, wv, loff, lane);
  int cur = 0;
#pragma unroll 1
  for (int64_t blk = b0; blk < b1; blk += bs, cur ^= 1) {
    const int64_t nb = blk + bs;
    wait_vm<0>();
    lds_bar();
    const bool next = nb < b1;
    if constexpr (PROC) {  // generate block blk+1 two octets per k-step, under the MFMAs
      offdiag_block(lds, cur, wv, lane, acc, [&](int s) {
        if (!next) return;
        if (s == 0) wstage<false, true, 0, 2>(lds, cur ^ 1, a, nb, I, J, wv, loff, lane);
        if (s == 1) wstage<false, true, 2, 4>(lds, cur ^ 1, a, nb, I, J, wv, loff, lane);
        if (s == 2) wstage<false, true, 4, 6>(lds, cur ^ 1, a, nb, I, J, wv, loff, lane);
        if (s == 3) wstage<false, true, 6, 8>(lds, cur ^ 1, a, nb, I, J, wv, loff, lane);
      });
    } else {  // issue block blk+1's DMA two octets per k-step, under the MFMAs
      offdiag_block(lds, cur, wv, lane, acc, [&](int s) {
        if (!next) return;
        if (s == 0) wstage<false, false, 0, 2>(lds, cur ^ 1, a, nb, I, J, wv, loff, lane);
        if (s == 1) wstage<false, false, 2, 4>(lds, cur ^ 1, a, nb, I, J, wv, loff, lane);
        if (s == 2) wstage<false, false, 4, 6>(lds, cur ^ 1, a, nb, I, J, wv, loff, lane);
        if (s == 3) wstage<false, false, 6, 8>(lds, cur ^ 1, a, nb, I, J, wv, loff, lane);
      });
    }
  }
  const int tr0 = 4 * (wv >> 1), tc0 = 4 * (wv & 1);
#pragma unroll
  for (int t = 0; t < 4; ++t)
#pragma unroll
    for (int u = 0; u < 4; ++u) {
      const int ti = (tr0 + t) * PT + tc0 + u;
#pragma unroll
      for (int j = 0; j < 4; ++j) out[ti * 256 + 64 * j + lane] = acc[4 * t + u][j];
    }
}

}  // namespace

// Persistent Gram kernels (one for the off-diagonal, one for the diagonal super-tiles, so
// each gets the whole register file): workgroup g runs the pieces [wg_begin[g],
// wg_begin[g+1]) of the cost-balanced schedule built on the host (engine.cpp).
template <bool DIAG, bool PROC>
__global__ void __launch_bounds__(64 * NWAVE, DIAG ? DIAG_WG : 2) wide_gram_kernel(WideGramArgs a) {
  __shared__ double lds[DIAG ? LDS_DIAG : LDS_DOUBLES];
  const int lane = threadIdx.x & 63;
  const int wv = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int pb = a.wg_begin[blockIdx.x], pe = a.wg_begin[blockIdx.x + 1];
#pragma unroll 1
  for (int pc = pb; pc < pe; ++pc) {
    const WidePiece pz = a.pieces[pc];
    const int64_t b1 = pz.b1 < a.nb_lim ? pz.b1 : a.nb_lim;  // a shorter last chunk clips the schedule
    const int st = pz.st;
    int I = 0;
    while ((I + 1) * (I + 2) / 2 <= st) ++I;
    const int J = st - I * (I + 1) / 2;
    double* out = a.partials + (int64_t)pz.slot * a.stride;
    if constexpr (!DIAG) {
      offdiag_piece<PROC>(lds, a, I, J, pz.b0, b1, pz.bs, wv, lane, out);
    } else {
      switch (wv) {
        case 0: diag_piece<0, PROC>(lds, a, I, pz.b0, b1, pz.bs, wv, lane, out); break;
        case 1: diag_piece<1, PROC>(lds, a, I, pz.b0, b1, pz.bs, wv, lane, out); break;
        case 2: diag_piece<2, PROC>(lds, a, I, pz.b0, b1, pz.bs, wv, lane, out); break;
        default: diag_piece<3, PROC>(lds, a, I, pz.b0, b1, pz.bs, wv, lane, out); break;
      }
    }
    lds_bar();  // every wave is done with both buffers before the next piece stages
  }
}

// Row stage: thread per row QUAD (two 16-byte loads of four adjacent rows of each column: a
// wave reads 2 KiB contiguous per column), columns streamed in order with four partial sums
// per row (the per-row summation order does not depend on the rows per thread).
template <int FAM, int LNK, int RPT, bool NT = false>
__device__ __forceinline__ void wide_rows_body(const WideRowArgs& a) {
  static_assert(RPT % 2 == 0 && 32 % RPT == 0, "rows per thread: even, divides 32");
  __shared__ double red[4][2];
  const int64_t q0 = a.r_begin / RPT, nq = (a.r_end - a.r_begin) / RPT;  // row quads of this launch
  const int64_t per = (nq + gridDim.x - 1) / gridDim.x;
  const int64_t lo = q0 + per * blockIdx.x, hi = (per * blockIdx.x + per < nq) ? lo + per : q0 + nq;
  double s_dev = 0.0, s_aux = 0.0;
  for (int64_t iq = lo + threadIdx.x; iq < hi; iq += blockDim.x) {
    const int64_t i = RPT * iq;
    double eta[RPT] = {};
    if (a.xs_out) {  // procedural chunk: generate the rows once, store them for the Gram kernels
      double* xo = a.xs_out + (i - a.r_begin);
      double e[RPT][4] = {};
      for (int j = 0; j < a.p; ++j) {
        const double b = (a.mode == MODE_IRLS) ? a.beta[j] : 0.0;
        double x[RPT];
#pragma unroll
        for (int r = 0; r < RPT; ++r) {
          x[r] = (i + r < a.n) ? proc_x(a.proc, i + r, j) : 0.0;
          e[r][j & 3] += x[r] * b;  // the resident path's partial-sum order (j + q, q = j & 3)
        }
#pragma unroll
        for (int h = 0; h < RPT / 2; ++h) *(double2*)(xo + (int64_t)j * a.xs_ld + 2 * h) = double2{x[2 * h], x[2 * h + 1]};
      }
      if (a.mode == MODE_IRLS) {
        const int pt = a.p & ~3;  // columns past the last whole quad went to e[r][0] in the resident order
#pragma unroll
        for (int r = 0; r < RPT; ++r) {
          double t[4] = {0.0, 0.0, 0.0, 0.0};
          // recompute in the resident order only when p is not a multiple of 4 (exactness)
          if (pt != a.p) {
            int j = 0;
            for (; j + 4 <= a.p; j += 4)
#pragma unroll
              for (int q = 0; q < 4; ++q) t[q] += xo[(int64_t)(j + q) * a.xs_ld + r] * a.beta[j + q];
            for (; j < a.p; ++j) t[0] += xo[(int64_t)j * a.xs_ld + r] * a.beta[j];
            eta[r] = (t[0] + t[1]) + (t[2] + t[3]);
          } else {
            eta[r] = (e[r][0] + e[r][1]) + (e[r][2] + e[r][3]);
          }
        }
      }
    } else if (a.mode == MODE_IRLS && a.eta_in) {  // procedural chunk, X beta from proc_gen_kernel
#pragma unroll
      for (int r = 0; r < RPT; ++r) eta[r] = (i + r < a.n) ? a.eta_in[i + r] : 0.0;
    } else if (a.mode == MODE_IRLS) {
      double e[RPT][4] = {};
      if (a.proc.on) {  // procedural design: same partial-sum order as the resident image
#pragma unroll
        for (int r = 0; r < RPT; ++r) {
          int j = 0;
          for (; j + 4 <= a.p; j += 4)
#pragma unroll
            for (int q = 0; q < 4; ++q) e[r][q] += proc_x(a.proc, i + r, j + q) * a.beta[j + q];
          for (; j < a.p; ++j) e[r][0] += proc_x(a.proc, i + r, j) * a.beta[j];
        }
      } else {
        const double* xc = a.X + i;
        int j = 0;
        for (; j + 4 <= a.p; j += 4)
#pragma unroll
          for (int q = 0; q < 4; ++q) {
            const double b = a.beta[j + q];
#pragma unroll
            for (int h = 0; h < RPT / 2; ++h) {
              const double2* src = (const double2*)(xc + (int64_t)(j + q) * a.ld + 2 * h);
              double2 v;
              if constexpr (NT) {
                const dv2 t = __builtin_nontemporal_load((const dv2*)src);
                v = double2{t.x, t.y};
              } else {
                v = *src;
              }
              e[2 * h][q] += v.x * b;
              e[2 * h + 1][q] += v.y * b;
            }
          }
        for (; j < a.p; ++j) {
#pragma unroll
          for (int h = 0; h < RPT / 2; ++h) {
            const double2 v = *(const double2*)(xc + (int64_t)j * a.ld + 2 * h);
            e[2 * h][0] += v.x * a.beta[j];
            e[2 * h + 1][0] += v.y * a.beta[j];
          }
        }
      }
#pragma unroll
      for (int r = 0; r < RPT; ++r) eta[r] = (e[r][0] + e[r][1]) + (e[r][2] + e[r][3]);
    }
    double w[RPT] = {}, wz[RPT] = {};
#pragma unroll
    for (int r = 0; r < RPT; ++r) {
      const int64_t row = i + r;
      if (row < a.n) {
        const double y = a.y[row];
        const double m = a.m ? a.m[row] : 1.0;
        const double off = a.off ? a.off[row] : 0.0;
        const double pw = a.prior ? a.prior[row] : 1.0;
        double et = eta[r];
        if (a.mode == MODE_IRLS) {
          et = et + off;
          if (a.eta_out) a.eta_out[row] = et;
        }
        pass_row(FAM, LNK, a.mode, et, y, m, off, pw, a.mu0, a.ybar, a.m != nullptr, w[r], wz[r], s_dev, s_aux);
      }
    }
#pragma unroll
    for (int h = 0; h < RPT / 2; ++h) {
      *(double2*)(a.w + i + 2 * h) = double2{w[2 * h], w[2 * h + 1]};
      *(double2*)(a.wz + i + 2 * h) = double2{wz[2 * h], wz[2 * h + 1]};
    }
  }
  for (int o = 1; o < 64; o <<= 1) {
    s_dev += __shfl_xor(s_dev, o);
    s_aux += __shfl_xor(s_aux, o);
  }
  if ((threadIdx.x & 63) == 0) {
    red[threadIdx.x >> 6][0] = s_dev;
    red[threadIdx.x >> 6][1] = s_aux;
  }
  __syncthreads();
  if (threadIdx.x < NS) {
    const int k = threadIdx.x;
    double v = 0.0;
    if (k == S_DEV) v = ((red[0][0] + red[1][0]) + red[2][0]) + red[3][0];
    if (k == S_SUMW) v = ((red[0][1] + red[1][1]) + red[2][1]) + red[3][1];
    a.row_partials[(int64_t)blockIdx.x * NS + k] = v;
  }
}

template <int FAM, int LNK>
__global__ void __launch_bounds__(256) wide_rows_kernel(WideRowArgs a) {
  wide_rows_body<FAM, LNK, 4>(a);
}

// The same row stage for the overlapped chunks (engine.cpp enqueue_pass): one workgroup per CU
// beside the two persistent Gram workgroups, so at most 96 VGPRs (2 x 208 + 96 = the SIMD's
// 512) and two rows per thread (no spills at that budget).  Per-row arithmetic and order are the
// full kernel's, bit for bit.  Non-temporal X loads keep the Gram's rows in the caches.
// Procedural chunks (xs_out: the design generated into the scratch beside the previous chunk's
// off-diagonal Gram launch) run at raised issue priority: the generator's integer chain is the
// longer of the two there (round 5, 250M x 512: 1284.5 -> 1266.9 ms per pass against no overlap;
// at normal priority 1285.7, the row kernels spanning 862 ms beside 1124 ms of Gram).
template <int FAM, int LNK>
__global__ void __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(5))) wide_rows_ov_kernel(WideRowArgs a) {
  if (a.xs_out) __builtin_amdgcn_s_setprio(1);
  wide_rows_body<FAM, LNK, 2, true>(a);
}

// Procedural chunks >= 1, the generator on its own (engine.cpp enqueue_pass): X rows [r_begin, r_end)
// into the scratch and X beta into eta_raw, a thread per row, nothing else -- so that it fits in 48
// VGPRs and two waves per SIMD run beside the two 208-VGPR off-diagonal Gram workgroups (the
// generating wide_rows_ov_kernel, with the family arithmetic in it, holds 87 VGPRs: one wave).  The
// family stage then runs from eta_raw (WideRowArgs::eta_in).  Partial sums in the resident order:
// whole column quads into e[j & 3], the tail columns into e[0] (wide_rows_body), so eta is bitwise.
// beta and the scratch are __restrict__ kernel arguments and the row loop has a uniform trip count:
// beta is then read through the scalar cache, not by vector loads, whose vmcnt wait would also wait
// for every scratch store in flight.  GUARD: the workgroup's rows reach past the chunk or past n.
template <bool POS, bool GUARD>
__device__ __forceinline__ void proc_gen_row(const ProcGenArgs& a, const double* __restrict__ beta,
                                             double* __restrict__ xs, int64_t t) {
  const int p = a.proc.p, pt = p & ~3;
  const double scale = a.proc.scale;
  const int64_t row = a.r_begin + t, ld = a.xs_ld;
  const bool in = !GUARD || t < a.r_end - a.r_begin, valid = !GUARD || row < a.proc.n;
  const uint64_t kb = a.proc.kx + (uint64_t)(a.proc.row0 + row) * (uint64_t)p;
  auto gx = [&](int j) {
    const double x = gen_x_row<POS>(kb, j, scale);
    return valid ? x : 0.0;
  };
  double* xo = xs + t;
  double e0 = 0.0, e1 = 0.0, e2 = 0.0, e3 = 0.0;
  int j = 0;
  for (; j < pt; j += 4) {  // two columns at a time (two hash chains in flight: the VGPR budget)
    const double x0 = gx(j), x1 = gx(j + 1);
    if (in) {
      xo[(int64_t)j * ld] = x0;
      xo[(int64_t)(j + 1) * ld] = x1;
    }
    if (beta) {
      e0 += x0 * beta[j];
      e1 += x1 * beta[j + 1];
    }
    __builtin_amdgcn_sched_barrier(0);
    const double x2 = gx(j + 2), x3 = gx(j + 3);
    if (in) {
      xo[(int64_t)(j + 2) * ld] = x2;
      xo[(int64_t)(j + 3) * ld] = x3;
    }
    if (beta) {
      e2 += x2 * beta[j + 2];
      e3 += x3 * beta[j + 3];
    }
    __builtin_amdgcn_sched_barrier(0);
  }
  for (; j < p; ++j) {
    const double x = gx(j);
    if (in) xo[(int64_t)j * ld] = x;
    if (beta) e0 += x * beta[j];
  }
  if (beta && in && valid) a.eta_raw[row] = (e0 + e1) + (e2 + e3);
}

template <bool POS>
__global__ void __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(8)))
proc_gen_kernel(ProcGenArgs a, const double* __restrict__ beta, double* __restrict__ xs) {
  __builtin_amdgcn_s_setprio(1);
  const int64_t nr = a.r_end - a.r_begin;
  for (int64_t t0 = blockIdx.x * (int64_t)blockDim.x; t0 < nr; t0 += (int64_t)gridDim.x * blockDim.x) {
    if (t0 + (int64_t)blockDim.x <= nr && a.r_begin + t0 + (int64_t)blockDim.x <= a.proc.n)
      proc_gen_row<POS, false>(a, beta, xs, t0 + threadIdx.x);
    else
      proc_gen_row<POS, true>(a, beta, xs, t0 + threadIdx.x);
  }
}

// Packed output: lower-tri X'WX row-major | X'Wz | NS scalars, summed in a fixed order.
__global__ void wide_reduce_kernel(const double* __restrict__ part, int64_t stride, const int* __restrict__ st_range,
                                   int p, const double* __restrict__ rowpart, int nrow, double* __restrict__ out) {
  const int64_t tri = (int64_t)p * (p + 1) / 2;
  const int64_t total = tri + p + NS;
  for (int64_t e = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; e < total; e += (int64_t)gridDim.x * blockDim.x) {
    double s = 0.0;
    if (e < tri + p) {
      int64_t st, src;
      if (e < tri) {
        int64_t i = (int64_t)((sqrt(8.0 * (double)e + 1.0) - 1.0) * 0.5);
        while (i * (i + 1) / 2 > e) --i;
        while ((i + 1) * (i + 2) / 2 <= e) ++i;
        const int64_t j = e - i * (i + 1) / 2;
        const int64_t I = i / PANEL, J = j / PANEL;
        st = I * (I + 1) / 2 + J;
        src = (((i % PANEL) >> 4) * PT + ((j % PANEL) >> 4)) * 256 + (i & 15) * 16 + (j & 15);
      } else {
        const int64_t c = e - tri, I = c / PANEL;
        st = I * (I + 1) / 2 + I;
        src = PT * PT * 256 + (c % PANEL);
      }
      const int g0 = st_range[2 * st], g1 = st_range[2 * st + 1];
      const double* ps = part + src;
      for (int g = g0; g < g1; ++g) s += ps[(int64_t)g * stride];
    } else {
      const int k = (int)(e - tri - p);  // scalars: compensated (rowmath.hpp neumaier_add)
      double c = 0.0;
      int g = 0;
      for (; g + 32 <= nrow; g += 32) {
        double v[32];
#pragma unroll
        for (int u = 0; u < 32; ++u) v[u] = rowpart[(int64_t)(g + u) * NS + k];
#pragma unroll
        for (int u = 0; u < 32; ++u) neumaier_add(s, c, v[u]);
      }
      for (; g < nrow; ++g) neumaier_add(s, c, rowpart[(int64_t)g * NS + k]);
      s += c;
    }
    out[e] = s;
  }
}

// Sum of the per-chunk packed results of a chunked procedural pass, in chunk order (scalars
// compensated, as wide_reduce_kernel's).
__global__ void sum_chunks_kernel(const double* __restrict__ chunks, int nch, int64_t len, double* __restrict__ out,
                                  int64_t scal0) {
  for (int64_t e = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; e < len; e += (int64_t)gridDim.x * blockDim.x) {
    double s = 0.0, c = 0.0;
    for (int k = 0; k < nch; ++k) {
      const double v = chunks[(int64_t)k * len + e];
      if (e >= scal0) neumaier_add(s, c, v);
      else s += v;
    }
    out[e] = s + c;
  }
}

// Packed lower triangle (row-major) -> column-major p x p lower triangle (for potrf; both
// triangles when `full`, for getrf) and X'Wz.
__global__ void unpack_lower_kernel(const double* __restrict__ packed, int p, double* __restrict__ A,
                                    double* __restrict__ b, int full) {
  const int64_t tri = (int64_t)p * (p + 1) / 2;
  for (int64_t e = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; e < tri + p; e += (int64_t)gridDim.x * blockDim.x) {
    if (e < tri) {
      int64_t i = (int64_t)((sqrt(8.0 * (double)e + 1.0) - 1.0) * 0.5);
      while (i * (i + 1) / 2 > e) --i;
      while ((i + 1) * (i + 2) / 2 <= e) ++i;
      const int64_t j = e - i * (i + 1) / 2;
      A[i + j * (int64_t)p] = packed[e];
      if (full) A[j + i * (int64_t)p] = packed[e];
    } else {
      b[e - tri] = packed[e];
    }
  }
}

// coefs = XtWXi * XtWy (utils.scala:104, 135) from the explicit inverse of the LU route: one
// thread per coefficient, the product summed over k in ascending order without contraction --
// the order of the oracle's wls_solve and of the host solver.  Column-major A: the threads of a
// wave read consecutive elements of column k.
__global__ void inv_gemv_kernel(const double* __restrict__ A, int p, const double* __restrict__ b,
                                double* __restrict__ x) {
#pragma clang fp contract(off)
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= p) return;
  double s = 0.0;
  for (int k = 0; k < p; ++k) s += A[i + (int64_t)k * p] * b[k];
  x[i] = s;
}

// ---------------------------------------------------------------------------------
// Host launchers
// ---------------------------------------------------------------------------------
int wide_panels(int p) { return (p + PANEL - 1) / PANEL; }
int64_t wide_stride() { return (int64_t)PT * PT * 256 + PANEL; }

#define SGLM_ROW_LAUNCH(KN)                                                                    \
  template <int F, int L>                                                                      \
  struct KN##_t {                                                                              \
    static void go(dim3 g, dim3 b, hipStream_t st, const WideRowArgs& a) {                     \
      hipLaunchKernelGGL((KN<F, L>), g, b, 0, st, a);                                          \
    }                                                                                          \
  };
SGLM_ROW_LAUNCH(wide_rows_kernel)
SGLM_ROW_LAUNCH(wide_rows_ov_kernel)
#undef SGLM_ROW_LAUNCH

template <template <int, int> class K>
static hipError_t launch_rows_fl(int fam, int lnk, dim3 g, dim3 b, hipStream_t st, const WideRowArgs& a) {
  if (fam == FAM_BINOMIAL && lnk == LNK_LOGIT)
    K<FAM_BINOMIAL, LNK_LOGIT>::go(g, b, st, a);
  else if (fam == FAM_BINOMIAL && lnk == LNK_PROBIT)
    K<FAM_BINOMIAL, LNK_PROBIT>::go(g, b, st, a);
  else if (fam == FAM_BINOMIAL)
    K<FAM_BINOMIAL, LNK_CLOGLOG>::go(g, b, st, a);
  else if (fam == FAM_GAUSSIAN)
    K<FAM_GAUSSIAN, LNK_IDENTITY>::go(g, b, st, a);
  else if (fam == FAM_POISSON)
    K<FAM_POISSON, LNK_LOG>::go(g, b, st, a);
  else if (fam == FAM_GAMMA)
    K<FAM_GAMMA, LNK_INVERSE>::go(g, b, st, a);
  else
    return hipErrorInvalidValue;
  return hipGetLastError();
}

hipError_t launch_wide_rows(const WideRowArgs& a, int grid, hipStream_t st, bool ov) {
  const dim3 g(grid), b(256);
  const int fam = (a.mode == MODE_LM_GRAM) ? FAM_GAUSSIAN : a.family;
  const int lnk = (a.mode == MODE_LM_GRAM) ? LNK_IDENTITY : a.link;
  return ov ? launch_rows_fl<wide_rows_ov_kernel_t>(fam, lnk, g, b, st, a)
            : launch_rows_fl<wide_rows_kernel_t>(fam, lnk, g, b, st, a);
}

hipError_t launch_proc_gen(const ProcGenArgs& a, int grid, hipStream_t st) {
  if (a.proc.kind == 3)
    hipLaunchKernelGGL(proc_gen_kernel<true>, dim3(grid), dim3(256), 0, st, a, a.beta, a.xs);
  else
    hipLaunchKernelGGL(proc_gen_kernel<false>, dim3(grid), dim3(256), 0, st, a, a.beta, a.xs);
  return hipGetLastError();
}

int wide_gram_wg_per_cu(bool diag) { return diag ? DIAG_WG : 2; }

hipError_t launch_wide_gram(const WideGramArgs& a, bool diag, int grid, hipStream_t st) {
  if (diag && a.proc.on)
    hipLaunchKernelGGL((wide_gram_kernel<true, true>), dim3(grid), dim3(64 * NWAVE), 0, st, a);
  else if (diag)
    hipLaunchKernelGGL((wide_gram_kernel<true, false>), dim3(grid), dim3(64 * NWAVE), 0, st, a);
  else if (a.proc.on)
    hipLaunchKernelGGL((wide_gram_kernel<false, true>), dim3(grid), dim3(64 * NWAVE), 0, st, a);
  else
    hipLaunchKernelGGL((wide_gram_kernel<false, false>), dim3(grid), dim3(64 * NWAVE), 0, st, a);
  return hipGetLastError();
}

hipError_t launch_wide_reduce(const double* part, int64_t stride, const int* st_range, int p, const double* rowpart,
                              int nrow, double* out, hipStream_t st) {
  const int64_t total = (int64_t)p * (p + 1) / 2 + p + NS;
  int blocks = (int)((total + 255) / 256);
  if (blocks > 8192) blocks = 8192;
  hipLaunchKernelGGL(wide_reduce_kernel, dim3(blocks), dim3(256), 0, st, part, stride, st_range, p, rowpart, nrow, out);
  return hipGetLastError();
}

hipError_t launch_sum_chunks(const double* chunks, int nch, int p, double* out, hipStream_t st) {
  const int64_t len = (int64_t)p * (p + 1) / 2 + p + NS;
  int blocks = (int)((len + 255) / 256);
  if (blocks > 8192) blocks = 8192;
  hipLaunchKernelGGL(sum_chunks_kernel, dim3(blocks), dim3(256), 0, st, chunks, nch, len, out, len - NS);
  return hipGetLastError();
}

hipError_t launch_unpack_lower(const double* packed, int p, double* A, double* b, hipStream_t st, bool full) {
  const int64_t total = (int64_t)p * (p + 1) / 2 + p;
  int blocks = (int)((total + 255) / 256);
  if (blocks > 8192) blocks = 8192;
  hipLaunchKernelGGL(unpack_lower_kernel, dim3(blocks), dim3(256), 0, st, packed, p, A, b, full ? 1 : 0);
  return hipGetLastError();
}

hipError_t launch_inv_gemv(const double* A, int p, const double* b, double* x, hipStream_t st) {
  hipLaunchKernelGGL(inv_gemv_kernel, dim3((p + 63) / 64), dim3(64), 0, st, A, p, b, x);
  return hipGetLastError();
}

}  // namespace sglm
