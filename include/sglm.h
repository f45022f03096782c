/*
 * sglm.h -- C ABI of the MI355X fitting engine for sparkGLM's lm()/glm() hot path.
 *
 * This is the drop-in boundary.  The reference (cafreeman/sparkGLM, Scala/Spark) has no
 * FFI of its own; the seam is internal: the fit drivers return PreGLM / PreLM and the
 * unchanged model code (GLM.createObj, new LM) builds the user-visible objects.  Each
 * entry point below replaces one reference function body, reached from Scala over JNI
 * (binding stubs in INTEGRATION.md):
 *
 *   sglm_set_data        replaces utils.dataFrameToMatrix / dfToDenseMatrix
 *                        (utils.scala:36-49) + the per-action re-conversion: one upload,
 *                        X stays resident in HBM across iterations and fits.
 *   sglm_reserve +       the same, partition by partition (dataFrameToMatrix builds one
 *   sglm_set_rows        DenseMatrix per partition, utils.scala:36-39; GLM.scala:576-578):
 *                        blocks of rows -- each within a JVM array's 2^31 elements -- staged
 *                        through pinned buffers into the reserved shard.
 *   sglm_fit_glm         replaces GLM.fitSingleBinomial (GLM.scala:254-315) and
 *                        GLM.fitMultipleBinomial (GLM.scala:410-468); output = PreGLM
 *                        (GLM.scala:25-33).
 *   sglm_fit_lm          replaces LM.fitSingle / LM.fitMultiple (LM.scala:191-237) and
 *                        the stderr tail of LM.fit (LM.scala:260-263); output = PreLM
 *                        (LM.scala:10-14) + stdErr/sigma.
 *   sglm_irls_pass       one IRLS pass (zwCreateBinomial + wlsComponents, GLM.scala:
 *                        359-395, utils.scala:110-126) for tests and benchmarks.
 *   sglm_predict_new     replaces LM.predictSingle/predictMultiple's newX * coefs
 *                        (LM.scala:39-61) on new rows, without evicting the resident shard;
 *                        response scale (mu = unlink(eta)) for GLMs.
 *   sglm_create          SURVEY 8(b)'s constructor over devs[0..ndev): one device, or one
 *                        process owning several GPUs (the single Spark driver that calls
 *                        GLM.fit / LM.fit, GLM.scala:587, LM.scala:254): row shards per device,
 *                        one RCCL group all-reduce (ncclCommInitAll) per iteration.
 *   sglm_glm_summary / sglm_lm_summary
 *                        the printed summaries of GLM.summary (GLM.scala:998-1025) and
 *                        SummaryLM (LM.scala:66-137), produced host-side in C++.
 *
 * Conventions
 *   - Status codes: 0 ok; SGLM_EINVAL maps to IllegalArgumentException (the reference's
 *     require(...)); SGLM_ESINGULAR to breeze MatrixSingularException; SGLM_EHIP /
 *     SGLM_ECOMM to RuntimeException.  sglm_last_error() returns a thread-local message.
 *   - Matrices are column-major fp64 (Breeze DenseMatrix layout): element (i,j) at
 *     X[i + j*ldx].  The caller keeps ownership of every pointer it passes; the engine
 *     copies into device memory it owns until sglm_destroy.
 *   - A handle from sglm_create with ndev = 1 (or sglm_create_device) drives one HIP device;
 *     with ndev > 1 it drives several (row shards, Spark's slicing [d n/D, (d+1) n/D)).  Across processes (or host
 *     threads, one handle each) shards join a communicator: RCCL over xGMI, a caller-supplied
 *     all-reduce, or the in-process sglm_local_allreduce.  Every rank receives identical results.
 *   - Handles are not thread-safe; distinct handles may be used concurrently.
 */
#ifndef SGLM_H
#define SGLM_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define SGLM_ABI_VERSION 8  /* 3: sglm_stats.dev_passes; 4: sglm_stats.overlap_chunks; 5: sglm_set_comm_rank,
                              sglm_stats.comm_path / rank_blocks / pass_kernel_ms_min / proc_chunks /
                              proc_chunk_rows / solve_path; 6: sglm_stats.pass_kernel / pass_kernel_name,
                              sglm_set_comm_rank collective; 7: sglm_stats.lm_device_fits /
                              lm_device_reruns; 8: sglm_create(devs, ndev) as SURVEY 8(b) names it,
                              the one-device form renamed sglm_create_device (sglm_create_multi stays:
                              the group handle at any ndev), SGLM_KERNEL_NARROW_SPLIT retired,
                              sglm_stats.lm_onepass_fits */

enum sglm_status {
  SGLM_OK = 0,
  SGLM_EINVAL = 1,    /* require(...) failed -> IllegalArgumentException */
  SGLM_ESINGULAR = 2, /* inv() of a singular matrix -> MatrixSingularException */
  SGLM_EHIP = 3,      /* HIP runtime / device error */
  SGLM_ECOMM = 4,     /* RCCL or caller all-reduce failure */
  SGLM_ENOMEM = 5     /* device or host allocation failed */
};

/* Families: the reference fits only binomial (GLM.scala:486-590); the rest follow R's
 * family objects on the reference's IRLS skeleton. */
enum sglm_family { SGLM_BINOMIAL = 0, SGLM_GAUSSIAN = 1, SGLM_POISSON = 2, SGLM_GAMMA = 3 };
enum sglm_link {
  SGLM_LOGIT = 0, SGLM_PROBIT = 1, SGLM_CLOGLOG = 2, /* binomial (GLM.scala:190-251) */
  SGLM_IDENTITY = 3, SGLM_LOG = 4, SGLM_INVERSE = 5   /* gaussian / poisson / gamma */
};

/* How mu is formed on the first iteration. */
enum sglm_init {
  SGLM_INIT_SINGLE = 0,  /* fitSingleBinomial: mu = mean(y) directly (GLM.scala:263, 282-290) */
  SGLM_INIT_MULTIPLE = 1 /* fitMultipleBinomial: mu = unlink(link(mean(y))) (GLM.scala:370-371) */
};

/* How the last p x p solve ran (sglm_stats.solve_path). */
enum sglm_solve_path {
  SGLM_SOLVE_HOST_CHOL = 0,   /* host Cholesky (p <= 256, well conditioned) */
  SGLM_SOLVE_HOST_LU = 1,     /* host LU + explicit inverse: Breeze inv (utils.scala:103-105) */
  SGLM_SOLVE_DEVICE_CHOL = 2, /* wide p (default): rocSOLVER potrf / potrs / potri */
  SGLM_SOLVE_DEVICE_LU = 3    /* wide p, SGLM_WIDE_SOLVE=lu (or ill-conditioned above p = 1024):
                                 rocSOLVER getrf + getri, coefs = inv * X'Wz */
};

/* Where a pass's all-reduce ran (sglm_stats.comm_path). */
enum sglm_comm_path {
  SGLM_COMM_NONE = 0,         /* one shard, no communicator */
  SGLM_COMM_CALLER_HOST = 1,  /* sglm_set_comm, host buffers (gloo, sglm_local_allreduce, ...) */
  SGLM_COMM_CALLER_DEVICE = 2,/* sglm_set_comm, device buffers (e.g. a torch RCCL group) */
  SGLM_COMM_RCCL = 3,         /* sglm_set_comm_rccl: the engine's own RCCL communicator (xGMI) */
  SGLM_COMM_GROUP_RCCL = 4,   /* multi-device handle: one RCCL group call over ncclCommInitAll */
  SGLM_COMM_GROUP_HOST = 5    /* multi-device handle with a repeated device: host sums in shard order */
};

/* The kernel that ran the last pass (sglm_stats.pass_kernel; the roofline line's `kernel`). */
enum sglm_pass_kernel {
  SGLM_KERNEL_NONE = 0,
  SGLM_KERNEL_FUSED = 1,       /* irls_pass_kernel<P16, fam, link>: 65 <= p <= 256 below the K1r threshold */
  SGLM_KERNEL_FUSED_SPLIT = 2, /* irls_pass_r_kernel<P16, fam, link> (K1r, split roles) */
  SGLM_KERNEL_NARROW = 3,      /* irls_narrow_kernel<P16, fam, link, irls, stats>: p <= 64 */
  SGLM_KERNEL_WIDE = 4,        /* wide_rows_kernel + wide_gram_kernel: p > 256 (resident X) */
  SGLM_KERNEL_WIDE_PROC = 5    /* the same over procedural X (generated chunks or in-kernel) */
  /* 6 (SGLM_KERNEL_NARROW_SPLIT, ABI <= 7): retired with its kernel, never returned */
};

/* Prediction scale (R's predict(type = "link" | "response")). */
enum sglm_predict_type { SGLM_PREDICT_LINK = 0, SGLM_PREDICT_RESPONSE = 1 };

typedef struct sglm_engine sglm_engine;

typedef struct {
  int family;      /* enum sglm_family */
  int link;        /* enum sglm_link */
  double tol;      /* absolute |delta deviance| stopping tolerance; reference default 1e-6 */
  int verbose;     /* print "iter\tdeltad" per iteration (GLM.scala:304, 461) */
  int max_iter;    /* 0 = unbounded, as in the reference (extension guard otherwise) */
  int init_mode;   /* enum sglm_init */
  int npart;       /* value reported in PreGLM.npart (reference: Spark partition count); 0 = #ranks */
} sglm_glm_opts;

typedef struct { /* PreGLM (GLM.scala:25-33) */
  double *coefs;        /* [p] caller-allocated */
  double *std_err;      /* [p] caller-allocated: sqrt(diag(inv(X'WX))) of the last solve */
  double deviance;
  double null_deviance;
  double pearson;
  double loglik;
  int iter;
  double nrow;
  int npart;
  double *dev_trace;    /* optional [max_trace]: deviance after each iteration, [0] = null */
  int max_trace;
} sglm_preglm;

typedef struct { /* PreLM (LM.scala:10-14) + LM.fit's derived stdErr / sigma */
  double *coefs;        /* [p] */
  double *xtxi;         /* [p*p] col-major inv(X'X), may be NULL */
  double *std_err;      /* [p] sqrt(sse/(n-p) * diag(xtxi)) (LM.scala:260-263) */
  double sse;
  double r2;            /* SSR/SST, as the reference (LM.scala:185) */
  double fstat;
  double sigma;
  double nrow;
  int npart;
} sglm_prelm;

/* Per-handle timing counters (HIP events on the engine stream). */
typedef struct {
  int64_t passes;           /* fused IRLS / LM passes launched */
  double pass_kernel_ms;    /* total time of the fused pass kernel (sum over passes) */
  double reduce_kernel_ms;  /* total time of the partial-reduction kernel */
  double last_pass_ms;      /* fused kernel time of the last pass */
  double comm_ms;           /* host wall time in the all-reduce */
  double solve_ms;          /* host wall time in the p x p solves */
  int64_t n_local;          /* rows resident on this device */
  int64_t p;
  int workgroups;           /* fused-kernel grid size (wide path: Gram work items) */
  int kernel_variant;       /* fused path: column-block count P16; wide path: 0 */
  int path;                 /* 0 fused single-panel pass (p <= 256), 1 wide panel-pair pass */
  int wide_panels;          /* wide path: 128-column panels */
  double row_kernel_ms;     /* wide path: total time of the row kernel (eta, w, w*z) */
  double gram_kernel_ms;    /* wide path: total time of the panel-pair Gram kernel */
  double load_ms;           /* host wall time of set_data / set_rows (pinned staging + H2D) */
  int64_t load_bytes;       /* bytes those calls moved to the device */
  int ndev;                 /* devices driven by this handle */
  int rccl_group;           /* multi-device handle reducing over RCCL (1) or on the host (0) */
  int64_t dev_passes;       /* deviance-only passes: iterations the fit predicted to be its last
                               (quadratic convergence) ran without the unused Gram; bitwise the
                               scalars of the full pass (SGLM_SPECULATE=0 disables) */
  int overlap_chunks;       /* wide path, resident X: chunks per pass whose row kernel runs on a
                               second stream beside the previous chunk's Gram (0: not overlapped;
                               SGLM_WIDE_OVERLAP sets the count, SGLM_WIDE_OV_MIN the fewest rows) */
  int comm_path;            /* enum sglm_comm_path */
  int rank_blocks;          /* 1: the scalars (deviance, ...) are summed across ranks / shards in rank
                               order with compensation from per-rank blocks (needs the own rank: RCCL,
                               the in-process communicator, or sglm_set_comm_rank); 0: plain sum */
  double pass_kernel_ms_min;/* multi-device handle: pass_kernel_ms of the fastest shard (the max is
                               pass_kernel_ms); one device: = pass_kernel_ms.  comm_ms there is
                               the collective after the last shard arrived (RCCL: device events) */
  int proc_chunks;          /* procedural shard: chunks of X generated per pass (0: in-kernel) */
  int64_t proc_chunk_rows;  /* rows per chunk (SGLM_PROC_SCRATCH_MAX caps the scratch, GiB) */
  int solve_path;           /* enum sglm_solve_path of the last solve, -1 before any */
  int pass_kernel;          /* enum sglm_pass_kernel of the last pass (the engine's own choice: the K1 / K1r
                               threshold, its row limit, the narrow / wide paths) */
  char pass_kernel_name[64];/* that kernel's name as rocprofv3 lists it, e.g. "irls_pass_r_kernel<16,binomial,logit>" */
  int64_t lm_device_fits;   /* LM fits done in one device round trip (Gram pass, device Cholesky, residual pass;
                               resident p <= 64 shards without a communicator; SGLM_LM_DEVICE=0 disables) */
  int64_t lm_device_reruns; /* of those, fits whose device coefficients were not the host solve's bit for bit (the
                               host left Cholesky for LU) or whose one-pass statistics were flagged: the residual
                               pass reran at the host's coefficients */
  int64_t lm_onepass_fits;  /* of the device fits, those whose SSE / R^2 / F came from the Gram pass's sums (X'X,
                               X'y, X'1, y'y, sum y) -- one pass over X -- instead of a residual pass */
} sglm_stats;

/* Caller-supplied all-reduce (sum, fp64, in place).  on_device != 0: buf is a device
 * pointer and stream the engine's hipStream_t; otherwise buf is host memory.
 * THREAD: with a deadline (SGLM_COMM_TIMEOUT_S > 0, the default 300 s, read when the communicator
 * is set) the callback runs on a communicator thread the handle owns (its device current), not on
 * the thread that called sglm_fit_* / sglm_irls_*, which waits with the deadline; a callback still
 * running at the deadline is abandoned on that thread.  Callbacks bound to the calling thread
 * (MPI_THREAD_SINGLE / FUNNELED, thread-local JNI or torch state) need SGLM_COMM_TIMEOUT_S=0: the
 * callback then runs inline on the caller's thread, without a deadline.  sglm_local_allreduce
 * always runs inline (it bounds its own wait). */
typedef int (*sglm_allreduce_fn)(void *ctx, double *buf, int64_t count, void *stream, int on_device);

/* ---- lifecycle ---------------------------------------------------------------- */
int sglm_abi_version(void);
const char *sglm_last_error(void);
int sglm_device_count(int *count);
/* One handle over devs[0..ndev).  ndev = 1: a single-device handle, exactly
 * sglm_create_device(devs[0]).  ndev > 1: rows are sharded contiguously across the devices; each
 * iteration's packed partials are all-reduced by one RCCL group call over communicators from
 * ncclCommInitAll (distinct devices) or summed on the host in device order (a device listed
 * twice: rehearsal on fewer GPUs).  Every call below accepts a multi-device handle, except
 * sglm_set_data_device, sglm_set_comm and sglm_set_comm_rccl. */
int sglm_create(const int *devs, int ndev, sglm_engine **out);
/* One device by ordinal (the ABI <= 7 sglm_create(int, ...)). */
int sglm_create_device(int device, sglm_engine **out);
/* Always the multi-device (group) handle, for ndev = 1 too: a one-device group runs the RCCL
 * group all-reduce path (ncclCommInitAll over one device) -- how tests execute it on one GPU. */
int sglm_create_multi(const int *devs, int ndev, sglm_engine **out);
int sglm_handle_devices(sglm_engine *h, int *ndev);
void sglm_destroy(sglm_engine *h);

/* ---- data (utils.dataFrameToMatrix replacement) ------------------------------ */
/* Host arrays.  m (binomial trials), offset and prior (weights) may be NULL. */
int sglm_set_data(sglm_engine *h, const double *X, int64_t n, int64_t p, int64_t ldx,
                  const double *y, const double *m, const double *offset, const double *prior);
/* Same, from device memory already on this engine's device. */
int sglm_set_data_device(sglm_engine *h, const double *dX, int64_t n, int64_t p, int64_t ldx,
                         const double *dy, const double *dm, const double *doffset,
                         const double *dprior);
/* Partition-wise ingest.  sglm_reserve allocates the shard (n rows x p columns, plus the
 * optional vectors) without filling it; sglm_set_rows then copies rows [row0, row0+nrows)
 * from a host column-major block (leading dimension ldx >= nrows; vectors of nrows) through
 * two pinned staging buffers (pageable memory never reaches the DMA engine).  Blocks may
 * arrive in any order and must not overlap; a fit requires every reserved row written.
 * m / offset / prior must be passed exactly when reserved. */
int sglm_reserve(sglm_engine *h, int64_t n, int64_t p, int has_m, int has_offset, int has_prior);
int sglm_set_rows(sglm_engine *h, int64_t row0, int64_t nrows, const double *X, int64_t ldx,
                  const double *y, const double *m, const double *offset, const double *prior);
/* Generate this rank's row shard [row0, row0+n) of the seeded synthetic design directly
 * in HBM (bench / scale tests).  kind: 0 = logit design (y in {0,1}), 1 = gaussian (LM),
 * 2 = poisson counts + offset + prior, 3 = gamma design (positive X, y > 0).  Column 0
 * is the intercept.  Bit-identical to sparkglm_amd.synth on the host. */
int sglm_synth(sglm_engine *h, int kind, int64_t row0, int64_t n, int64_t p, uint64_t seed);
/* Procedural shard of the same synthetic design: y (+ offset / prior for kind 2) are
 * generated and stored, X is NOT -- the (wide-path) pass kernels regenerate every X[i, j]
 * from the counter-based generator where they would have read it, bit-identical to the
 * resident image of sglm_synth.  For designs larger than HBM (BASELINE configs[4]:
 * 2B x 512 = 8.19 TB).  Fits, LM, predict and stats work as on a resident shard;
 * sglm_get_data cannot return X. */
int sglm_synth_procedural(sglm_engine *h, int kind, int64_t row0, int64_t n, int64_t p, uint64_t seed);
/* Copy back the resident design (tests; X col-major with ldx = n). */
int sglm_get_data(sglm_engine *h, double *X, double *y, double *m, double *offset, double *prior);

/* ---- communicators (Spark treeReduce replacement) ----------------------------- */
/* fn runs on the handle's communicator thread unless SGLM_COMM_TIMEOUT_S=0 (see sglm_allreduce_fn).
 * RCCL (sglm_set_comm_rccl) and group handles: the deadline of an all-reduce starts when the work
 * this rank queued before it (its pass kernels) has finished, so it bounds the wait for the peers only. */
int sglm_set_comm(sglm_engine *h, sglm_allreduce_fn fn, void *ctx, int on_device);
/* This handle's rank in the communicator just set by sglm_set_comm (0 <= rank < its rank count;
 * known without this call for RCCL and sglm_local_allreduce).  With it the per-iteration scalars
 * (deviance, Pearson, loglik) are summed across ranks in rank order with compensation, so the
 * convergence test does not depend on the rank count beyond ~1 ulp.  COLLECTIVE: every rank of the
 * communicator calls it (it changes the length of every later all-reduce); one all-reduce checks
 * that all ranks joined with distinct ranks, else SGLM_EINVAL on every rank. */
int sglm_set_comm_rank(sglm_engine *h, int rank);
/* Native RCCL communicator over xGMI.  unique_id: 128 bytes from
 * sglm_rccl_unique_id() on rank 0, broadcast by the caller. */
int sglm_rccl_unique_id(void *out128);
int sglm_set_comm_rccl(sglm_engine *h, int nranks, int rank, const void *unique_id128);

/* ---- fits ---------------------------------------------------------------------- */
int sglm_fit_glm(sglm_engine *h, const sglm_glm_opts *opts, sglm_preglm *out);
int sglm_fit_lm(sglm_engine *h, sglm_prelm *out);

/* One IRLS pass at beta (beta == NULL: the initial constant-eta pass at mu0),
 * all-reduced over the communicator.  Outputs (any may be NULL): gram [p*p] col-major
 * full symmetric X'WX, xtwz [p], scalars [8] = {deviance-sum, pearson, loglik-part, bad,
 * aux0, aux1, aux2, sum prior}. */
int sglm_irls_pass(sglm_engine *h, const sglm_glm_opts *opts, const double *beta, double mu0,
                   double *gram, double *xtwz, double *scalars);

/* The test-level step of SURVEY.md 8(b): the pass at beta (beta != NULL) with the deviance at
 * beta (family factor applied, as GLM.scala:397 createBinomialDeviance sums it).  Outputs may be
 * NULL: xtwx [p*p] col-major full symmetric X'WX, xtwz [p], dev. */
int sglm_irls_step(sglm_engine *h, const sglm_glm_opts *opts, const double *beta, double *xtwx, double *xtwz,
                   double *dev);

/* `iters` IRLS iterations from beta (in/out): each is one fused pass at beta followed by
 * the p x p solve -- the unit the benchmark times.  last_dev (may be NULL) receives the
 * deviance at the last input beta. */
int sglm_irls_iterations(sglm_engine *h, const sglm_glm_opts *opts, double *beta, int iters,
                         double *last_dev);

/* eta = X * beta (+ offset if add_offset) for the resident rows, written to out [n_local]. */
int sglm_predict(sglm_engine *h, const double *beta, int add_offset, double *out);
/* The same on the link (eta) or response (mu = unlink(eta, m), m = the resident trials or 1)
 * scale of family/link: fitted values of the resident rows. */
int sglm_predict_glm(sglm_engine *h, const double *beta, int family, int link, int type, int add_offset,
                     double *out);
/* Score NEW rows (LM.predict, LM.scala:29-61; GLM response-scale prediction): X column-major
 * n x p (ldx >= n), optional offset / m (NULL: 0 / 1).  Streams X through a device scratch in
 * chunks; the resident training shard is untouched. */
int sglm_predict_new(sglm_engine *h, const double *X, int64_t n, int64_t p, int64_t ldx,
                     const double *beta, const double *offset, const double *m, int family, int link,
                     int type, double *out);

int sglm_get_stats(sglm_engine *h, sglm_stats *out);
/* The kernel an engine would run a pass of an n x p shard with (enum sglm_pass_kernel, -1 on bad
 * arguments) and its name into name[namelen] -- the engine's own dispatch rule, for callers and CPU
 * tests.  fused_split: SGLM_FUSED_SPLIT's meaning (1 default threshold, 0 never K1r, N from P16 = N);
 * flags: 1 procedural shard, 2 forced wide path (SGLM_FORCE_WIDE).  No device is touched. */
int sglm_pass_kernel_for(int64_t n, int64_t p, int fused_split, int flags, int family, int link, char *name,
                         int64_t namelen);
int sglm_reset_stats(sglm_engine *h);

/* ---- external backend: the same IRLS driver over caller-computed partials ---------
 * Lets a host (or a test) run the engine's driver, solve and convergence logic over
 * partial sums produced elsewhere (e.g. a CPU shard).  pass() must write the packed
 * wire format: lower-triangular X'WX row-major (i>=j: i*(i+1)/2+j), then X'Wz [p], then
 * 8 scalars.  mode: 0 irls(beta), 1 init-single, 2 init-multiple, 3 lm-gram, 4 lm-resid. */
typedef struct {
  void *ctx;
  int64_t p;
  int (*local_sums)(void *ctx, double *out2 /* {sum y, n_local} */);
  int (*pass)(void *ctx, int mode, const double *beta, double mu0, double ybar, double *packed);
} sglm_backend;

/* fn: as sglm_set_comm's (the communicator thread unless SGLM_COMM_TIMEOUT_S=0). */
int sglm_fit_glm_external(const sglm_backend *be, sglm_allreduce_fn fn, void *comm_ctx,
                          const sglm_glm_opts *opts, sglm_preglm *out);
int sglm_fit_lm_external(const sglm_backend *be, sglm_allreduce_fn fn, void *comm_ctx,
                         sglm_prelm *out);

/* ---- in-process communicator: N host threads in one process, one handle each ---------
 * (a JVM driver's thread pool over N single-device handles; the alternative to
 * sglm_create_multi).  Pass sglm_local_allreduce with sglm_local_comm_rank(c, r) as the
 * context of rank r to sglm_set_comm (on_device = 0) or sglm_fit_*_external.  The sum runs
 * in rank order, so every rank gets bitwise the same result. */
typedef struct sglm_local_comm sglm_local_comm;
int sglm_local_comm_create(int nranks, sglm_local_comm **out);
void sglm_local_comm_destroy(sglm_local_comm *c);
void *sglm_local_comm_rank(sglm_local_comm *c, int rank);
int sglm_local_allreduce(void *ctx, double *buf, int64_t count, void *stream, int on_device);

/* ---- model objects and printed summaries (host-side, C++) ---------------------- */
/* GLM.createObj (GLM.scala:59-88) derived fields. */
typedef struct {
  double df_residual, df_null, p_dispersion, aic;
} sglm_glm_derived;
int sglm_glm_create_obj(const sglm_preglm *pre, int64_t p, sglm_glm_derived *out);
/* GLM.summary text (GLM.scala:998-1025). xnames: p C strings. Returns bytes needed. */
int64_t sglm_glm_summary(const sglm_preglm *pre, int64_t p, const char *const *xnames,
                         const char *yname, const char *family, const char *link, char *buf,
                         int64_t buflen);
/* SummaryLM.print text (LM.scala:128-136). */
int64_t sglm_lm_summary(const sglm_prelm *pre, int64_t p, const char *const *xnames,
                        const char *yname, char *buf, int64_t buflen);
/* Helpers reproduced from utils.scala:146-169 and java.lang.Double.toString. */
double sglm_sig_digits(double num, int digits);
double sglm_round_digits(double num, int digits);
int64_t sglm_java_double_string(double x, char *buf, int64_t buflen);
/* 2*(1-Phi(|z|)) and 2*(1-T_df(|t|)) as used by the summaries. */
double sglm_pval_normal(double z);
double sglm_pval_t(double t, double df);

#ifdef __cplusplus
}
#endif
#endif /* SGLM_H */
