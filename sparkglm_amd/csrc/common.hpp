// common.hpp -- shared definitions for the sparkGLM MI355X engine (host + device).
#pragma once
#include <cstdint>

namespace sglm {

// Rows per LDS row block of the fused pass (one DMA'd tile of X).
constexpr int RB = 32;
// Scalar slots appended to every packed partial / reduced buffer.
constexpr int NS = 8;
enum Scalar : int { S_DEV = 0, S_PEARSON = 1, S_LL = 2, S_BAD = 3, S_AUX0 = 4, S_AUX1 = 5, S_AUX2 = 6, S_SUMW = 7 };

// Pass modes (shared with sglm_backend.pass in include/sglm.h).
enum PassMode : int {
  MODE_IRLS = 0,        // eta = X beta + offset (etaCreate, GLM.scala:321-332)
  MODE_INIT_SINGLE = 1, // eta = link(mu0, m), mu = mu0            (GLM.scala:263-270)
  MODE_INIT_MULTI = 2,  // eta = link(mu0, m), mu = unlink(eta, m) (GLM.scala:429-442, 370)
  MODE_LM_GRAM = 3,     // w = 1, z = y: X'X and X'y (LM.scala:142-155)
  MODE_LM_RESID = 4     // no Gram: SSE/SSR/SST at beta (LM.scala:160-188)
};

enum Family : int { FAM_BINOMIAL = 0, FAM_GAUSSIAN = 1, FAM_POISSON = 2, FAM_GAMMA = 3 };
enum Link : int { LNK_LOGIT = 0, LNK_PROBIT = 1, LNK_CLOGLOG = 2, LNK_IDENTITY = 3, LNK_LOG = 4, LNK_INVERSE = 5 };

// Which families carry their final statistics in the narrow pass (PassArgs::stats_in_pass;
// rowmath.hpp pass_row_stats): binomial / logit (without m), Poisson / log, Gamma / inverse.
constexpr bool stats_in_pass_family(int fam, int lnk) {
  return (fam == FAM_BINOMIAL && lnk == LNK_LOGIT) || (fam == FAM_POISSON && lnk == LNK_LOG) ||
         (fam == FAM_GAMMA && lnk == LNK_INVERSE);
}

// Cache policy of the design-streaming LDS-DMA (global_load_lds aux): non-temporal.  Every byte of X
// is read once per pass, so it should not displace what the caches hold (round 5, same box: 1B x 32
// logit pass 45.92 -> 44.84 ms, 200M x 32 -1.0 %, 125M x 64 Poisson -0.4 %, 30M x 256 -0.6 %,
// bitwise the default policy).  The wide path's panels are re-read by several super-tiles: default there.
constexpr int DMA_NT = 2;

// Largest column-block count of the fused (single-panel) kernel: p <= 16*16 = 256.
constexpr int MAX_P16 = 16;

inline int64_t tri_count(int64_t p) { return p * (p + 1) / 2; }
inline int64_t packed_len(int64_t p) { return tri_count(p) + p + NS; }

// Arguments of one fused pass launch.
struct PassArgs {
  const double* X;      // col-major, leading dimension ld, 4*nq columns (zero past p)
  int64_t ld;
  int p;
  int nq;               // column quads stored: ceil(p / 4)
  const double* y;
  const double* m;      // may be null (binomial trials = 1)
  const double* off;    // may be null
  const double* prior;  // may be null
  const double* beta;   // device, >= p entries (MODE_IRLS / MODE_LM_RESID)
  int64_t n;            // valid rows
  int64_t nblocks;      // row blocks of RB rows (ld == nblocks*RB)
  int family, link, mode;
  double mu0;           // init modes
  double ybar;          // LM resid mode
  double* partials;     // [grid][stride]
  int64_t stride;
  double* eta_out;      // optional [n]: eta of MODE_IRLS rows (for the final statistics)
  int stats_in_pass;    // narrow binomial/logit IRLS pass without m: pearson / loglik / bad in the
                        // pass's scalars instead of the eta store + stats_kernel
  int no_gram;          // deviance-only pass (glm_drive's speculative last pass): row stage, no Gram
  int fused_split;      // split-role kernel K1r (irls_pass_r_kernel) from P16 >= threshold: 1 default, 0 never, N: P16 >= N
  int lm_extras;        // narrow LM Gram pass of the one-round-trip LM.fit: X'1 after the scalars, y'y in S_PEARSON
};

// ---- wide-design path (p > 16*MAX_P16): row kernel + panel-pair Gram kernel ----
constexpr int WIDE_PANEL = 128;  // columns per Gram panel (8 tile blocks of 16)
constexpr int MAX_P_WIDE = 8192;

// Procedural design (sglm_synth_procedural): X is regenerated in the kernels, never stored.
struct ProcX {
  int on;               // 0: X is the resident image
  int kind, p;
  int64_t row0, n;      // global row of local row 0; valid rows
  uint64_t kx;          // splitmix64(seed)
  double scale;         // 1/sqrt(p)
};

struct WideRowArgs {
  const double* X;
  int64_t ld;
  int p;
  const double* y;
  const double* m;
  const double* off;
  const double* prior;
  const double* beta;   // device [p] (MODE_IRLS)
  int64_t n, n_pad;
  int family, link, mode;
  double mu0, ybar;
  double* w;            // [n_pad] working weights (0 on padding rows)
  double* wz;           // [n_pad] w * z
  double* eta_out;      // optional [n]
  double* row_partials; // [grid][NS]
  ProcX proc;
  int64_t r_begin, r_end;  // rows [r_begin, r_end) of this launch (multiples of 4; r_end may pass n_pad)
  double* xs_out;       // procedural chunks: the generated X rows stored here (column-major,
  int64_t xs_ld;        //   leading dimension xs_ld, local row = row - r_begin), else null
  const double* eta_in; // procedural chunks after proc_gen_kernel: X beta of rows < n (MODE_IRLS), else null
};

// Procedural chunks: the lean generator (wide.hip proc_gen_kernel) -- X rows [r_begin, r_end) into
// the scratch and X beta (no offset) of the rows < proc.n into eta_raw.
struct ProcGenArgs {
  ProcX proc;
  const double* beta;   // device [p], or null (no eta: the initial pass)
  double* xs;           // scratch, column-major, leading dimension xs_ld, local row = row - r_begin
  int64_t xs_ld;
  int64_t r_begin, r_end;
  double* eta_raw;      // [n], global row index
};

// One run of 16-row blocks of one super-tile, processed by one workgroup of the persistent
// Gram kernel and written to partial slot `slot`: blocks b0, b0 + bs, b0 + 2 bs, ... < b1
// (bs = 1: consecutive blocks; bs = k: the k workgroups of a super-tile interleave block by
// block, so every workgroup of the launch sweeps the same rows at the same time).
struct WidePiece {
  int64_t b0, b1;       // blocks of WIDE_RB rows
  int st;               // super-tile I(I+1)/2 + J
  int slot;             // partial slot (slots of one super-tile are consecutive)
  int64_t bs;           // block stride
};
constexpr int WIDE_RB = 16;   // rows per Gram-kernel LDS block

struct WideGramArgs {
  const double* X;
  int64_t ld;
  int ncols;            // columns stored (multiple of 8, zero past p)
  const double* w;
  const double* wz;
  const WidePiece* pieces;
  const int* wg_begin;  // [grid + 1]: pieces of workgroup g are [wg_begin[g], wg_begin[g+1])
  double* partials;     // [slots][stride]
  int64_t stride;
  ProcX proc;
  int64_t nb_lim;       // blocks of this launch's rows: pieces are clipped to [b0, min(b1, nb_lim))
};

// Arguments of the final-statistics pass (stats_kernel).
struct StatsArgs {
  const double* y;
  const double* m;
  const double* prior;
  const double* eta;    // MODE_IRLS: eta of the last pass; MODE_LM_RESID: X*coefs (or X != null below)
  const double* X;      // MODE_LM_RESID on a resident shard: eta = X*beta formed in the kernel
  int64_t ld;           //   (predict_kernel's order), so the residual pass reads X once and
  int p;                //   writes no eta
  const double* beta;
  int64_t n;
  int family, link, mode;
  double mu0, ybar;
  double* partials;     // [grid][NS]
  const double* ybar_dev;  // non-null: ybar read from the device (the LM device round trip, lm_chol_kernel)
  int beta_by_value;    // p <= STATS_BETA_MAX: beta travels in the kernel arguments (no H2D copy)
  double bv[32];        //   beta_by_value: beta[0..p)
};
constexpr int STATS_BETA_MAX = 32;

}  // namespace sglm
