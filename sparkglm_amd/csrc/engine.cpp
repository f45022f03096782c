// engine.cpp -- the C ABI (include/sglm.h) over the HIP backend.
//
// One sglm_engine drives one HIP device: it owns the row shard resident in HBM (X
// column-major with a leading dimension padded to the 32-row block, y / m / offset /
// prior, the last pass's eta), the fused-pass workspace and a communicator.  A pass is
//   H2D beta -> irls_pass_kernel (one read of X) -> reduce_partials_kernel (fixed order)
//   -> [device all-reduce: RCCL over xGMI] -> D2H packed -> [host all-reduce callback]
// replacing one zwCreateBinomial + wlsComponents + treeReduce round of the reference
// (GLM.scala:453-458, utils.scala:110-126).
//
// Wide designs (p > 256, or SGLM_FORCE_WIDE=1) run the panel-pair path of wide.hip
// instead: wide_rows_kernel (eta, w, w*z) -> wide_gram_kernel (X'WX over 128x128 column
// super-tiles) -> wide_reduce_kernel, and the p x p system is solved on the device
// (rocSOLVER potrf/potrs, potri for the standard errors) from the reduced buffer.
#include <hip/hip_runtime.h>
#include <rccl/rccl.h>
#include <rocblas/rocblas.h>
#include <rocsolver/rocsolver.h>

#include <algorithm>
#include <chrono>
#include <cmath>
#include <condition_variable>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <memory>
#include <mutex>
#include <string>
#include <thread>
#include <vector>

#include "../../include/sglm.h"
#include "common.hpp"
#include "driver.hpp"
#include "kernels.hpp"
#include "solve.hpp"

using namespace sglm;

namespace {

std::string hip_msg(hipError_t e, const char* what) {
  return std::string("HIP error in ") + what + ": " + hipGetErrorString(e);
}

#define HIPCHK(expr)                                  \
  do {                                                \
    hipError_t _e = (expr);                           \
    if (_e != hipSuccess) {                           \
      set_error(hip_msg(_e, #expr));                  \
      return SGLM_EHIP;                               \
    }                                                 \
  } while (0)

// Compensated (Neumaier) accumulation of the scalar partials (host side of rowmath.hpp's
// neumaier_add): the deviance sum decides the iteration count against an absolute 1e-6.
inline void neumaier_add(double& s, double& c, double x) {
  const double t = s + x;
  c += (std::fabs(s) >= std::fabs(x)) ? (s - t) + x : (x - t) + s;
  s = t;
}

double now_ms() {
  using namespace std::chrono;
  return duration<double, std::milli>(steady_clock::now().time_since_epoch()).count();
}

// ---- bounded waits on the per-iteration all-reduce (utils.scala:110-126's treeReduce seam) ----
// A rank that dies or stalls must not hang the others until an outside time limit: every wait on
// a collective has a deadline, SGLM_COMM_TIMEOUT_S seconds (default 300; 0 = unbounded), read when
// the communicator is set.  On expiry (or an asynchronous RCCL error) the call returns SGLM_ECOMM
// naming the rank and what it waited for, and the communicator is unusable from then on.
double comm_timeout_ms_env() {
  const char* e = std::getenv("SGLM_COMM_TIMEOUT_S");
  if (!e || !*e) return 300e3;
  const double s = std::atof(e);
  return s > 0.0 ? s * 1e3 : 0.0;
}

std::string rank_str(int rank) { return rank >= 0 ? "rank " + std::to_string(rank) : "this rank"; }

// Wait for the streams whose last work is a collective over `comms` (the engine's RCCL
// communicator, or a multi-device handle's ncclCommInitAll group): poll hipStreamQuery and every
// communicator's asynchronous error until the streams drain or the deadline passes.  On a remote
// error or expiry the communicators are aborted (ncclCommAbort makes their kernels exit) and
// nulled, and SGLM_ECOMM is returned -- never a silent hang.  `starts`: events recorded on those
// streams just before the collective (this rank's own pass done); the deadline counts from the
// moment all of them have completed, so it bounds the wait for the peers, never this rank's own
// pass kernels (a long pass on a large shard cannot expire it).
int wait_collective(const std::vector<hipStream_t>& sts, std::vector<ncclComm_t*> comms, double timeout_ms,
                    int rank, const char* what, const std::vector<hipEvent_t>& starts = {}) {
  for (hipEvent_t ev : starts) {  // this rank's pass kernels: no deadline (they need no peer)
    hipError_t e;
    while ((e = hipEventQuery(ev)) == hipErrorNotReady) std::this_thread::yield();
    if (e != hipSuccess) {
      set_error(hip_msg(e, "hipEventQuery (the pass before the all-reduce)"));
      return SGLM_EHIP;
    }
  }
  const double t0 = now_ms();
  std::vector<char> done(sts.size(), 0);
  size_t left = sts.size();
  auto abort_all = [&](const std::string& why) {
    for (ncclComm_t* c : comms)
      if (*c) {
        (void)ncclCommAbort(*c);
        *c = nullptr;
      }
    set_error(why);
    return SGLM_ECOMM;
  };
  for (uint64_t it = 0; left > 0; ++it) {
    for (size_t i = 0; i < sts.size(); ++i) {
      if (done[i]) continue;
      const hipError_t e = hipStreamQuery(sts[i]);
      if (e == hipSuccess) {
        done[i] = 1;
        --left;
      } else if (e != hipErrorNotReady) {
        set_error(hip_msg(e, "hipStreamQuery (wait on the all-reduce)"));
        return SGLM_EHIP;
      }
    }
    if (left == 0) break;
    if ((it & 255) == 255) {
      for (ncclComm_t* c : comms) {
        ncclResult_t ae = ncclSuccess;
        if (*c && ncclCommGetAsyncError(*c, &ae) == ncclSuccess && ae != ncclSuccess && ae != ncclInProgress)
          return abort_all(std::string("RCCL asynchronous error on ") + rank_str(rank) + " during " + what + ": " +
                           ncclGetErrorString(ae) + "; communicator aborted");
      }
      if (timeout_ms > 0.0 && now_ms() - t0 > timeout_ms)
        return abort_all(rank_str(rank) + ": " + what + " did not complete within SGLM_COMM_TIMEOUT_S = " +
                         std::to_string(timeout_ms * 1e-3) + " s (a peer rank died, stalled or never joined); "
                         "communicator aborted");
    }
    std::this_thread::yield();
  }
  return SGLM_OK;
}

// Caller-supplied all-reduce callbacks (sglm_set_comm, sglm_fit_*_external) run on a communicator
// thread owned by the handle -- one thread for the handle's life, with the handle's device
// current -- while the calling thread waits with the deadline.  A callback that never returns is
// abandoned (its thread detached with its own copy of a host buffer) and the handle's communicator
// is marked broken.  sglm_local_allreduce is bounded by itself and runs inline.
class CallbackRunner {
 public:
  explicit CallbackRunner(int device = -1) : device_(device) {}
  ~CallbackRunner() {
    if (!st_) return;
    {
      std::lock_guard<std::mutex> lk(st_->mu);
      st_->stop = true;
    }
    st_->cv.notify_all();
    if (th_.joinable()) th_.join();
  }
  CallbackRunner(const CallbackRunner&) = delete;
  CallbackRunner& operator=(const CallbackRunner&) = delete;

  bool broken() const { return !broken_msg_.empty(); }
  // a timed-out device-buffer callback may still write its buffer: the owner must not free it
  bool leaked_device_buffer() const { return leaked_dev_; }
  void reset() {  // a new communicator
    broken_msg_.clear();
    leaked_dev_ = false;
  }
  int call(sglm_allreduce_fn fn, void* ctx, double* buf, int64_t count, void* stream, int on_device, double timeout_ms,
           int rank) {
    if (broken()) {
      set_error(broken_msg_);
      return SGLM_ECOMM;
    }
    if (timeout_ms <= 0.0 || fn == &sglm_local_allreduce) {
      if (fn(ctx, buf, count, stream, on_device) != 0) {
        set_error(fn == &sglm_local_allreduce
                      ? "in-process all-reduce failed on " + rank_str(rank) +
                            " (ranks passed different lengths, or a rank did not arrive within SGLM_COMM_TIMEOUT_S)"
                      : "caller all-reduce failed on " + rank_str(rank));
        return SGLM_ECOMM;
      }
      return SGLM_OK;
    }
    start();
    std::unique_lock<std::mutex> lk(st_->mu);
    st_->fn = fn;
    st_->ctx = ctx;
    st_->count = count;
    st_->stream = stream;
    st_->on_device = on_device;
    if (on_device) {
      st_->buf = buf;
    } else {
      st_->host.assign(buf, buf + count);
      st_->buf = st_->host.data();
    }
    st_->done = false;
    st_->has_job = true;
    st_->cv.notify_all();
    const bool ok = st_->cv.wait_for(lk, std::chrono::duration<double, std::milli>(timeout_ms), [&] { return st_->done; });
    if (!ok) {
      lk.unlock();
      broken_msg_ = rank_str(rank) + ": the caller all-reduce did not return within SGLM_COMM_TIMEOUT_S = " +
                    std::to_string(timeout_ms * 1e-3) + " s (a peer rank died, stalled or never joined); the "
                    "communicator is broken -- set a new one";
      leaked_dev_ = on_device != 0;
      th_.detach();  // the thread keeps its state (and the host copy) alive by itself
      st_.reset();
      set_error(broken_msg_);
      return SGLM_ECOMM;
    }
    if (!on_device) std::memcpy(buf, st_->host.data(), sizeof(double) * (size_t)count);
    if (st_->rc != 0) {
      set_error("caller all-reduce failed on " + rank_str(rank));
      return SGLM_ECOMM;
    }
    return SGLM_OK;
  }

 private:
  struct State {
    std::mutex mu;
    std::condition_variable cv;
    bool has_job = false, done = false, stop = false;
    sglm_allreduce_fn fn = nullptr;
    void* ctx = nullptr;
    double* buf = nullptr;
    int64_t count = 0;
    void* stream = nullptr;
    int on_device = 0, rc = 0;
    std::vector<double> host;
  };
  void start() {
    if (st_) return;
    st_ = std::make_shared<State>();
    std::shared_ptr<State> s = st_;
    const int dev = device_;
    th_ = std::thread([s, dev] {
      if (dev >= 0) (void)hipSetDevice(dev);
      std::unique_lock<std::mutex> lk(s->mu);
      for (;;) {
        s->cv.wait(lk, [&] { return s->has_job || s->stop; });
        if (s->stop) return;
        s->has_job = false;
        lk.unlock();
        const int rc = s->fn(s->ctx, s->buf, s->count, s->stream, s->on_device);
        lk.lock();
        s->rc = rc;
        s->done = true;
        s->cv.notify_all();
      }
    });
  }
  int device_;
  std::shared_ptr<State> st_;
  std::thread th_;
  std::string broken_msg_;
  bool leaked_dev_ = false;
};

struct Comm {
  int kind = 0;  // 0 none, 1 callback, 2 rccl
  sglm_allreduce_fn fn = nullptr;
  void* ctx = nullptr;
  int on_device = 0;
  ncclComm_t nccl = nullptr;
  int nranks = 1;
  int rank = -1;  // this handle's rank (RCCL, the in-process communicator, sglm_set_comm_rank); -1 unknown
  double ms = 0.0;
  double timeout_ms = 300e3;  // SGLM_COMM_TIMEOUT_S when the communicator was set (0: unbounded)
};

// Cross-rank sums of the NS scalars (deviance, Pearson, loglik ingredients, ...) in rank order
// with compensation.  The all-reduce buffer carries, after the packed result, one block of
// `count` slots per rank in which only the owner's block is non-zero, so the all-reduce -- in
// whatever order RCCL or the caller adds -- delivers every rank's scalars exactly (x + 0 = x),
// and each rank then sums them itself, in rank order, Neumaier-compensated: the fit's deviance
// trajectory no longer depends on how many ranks the rows are spread over beyond ~1 ulp.  A plain
// all-reduce of the deviance adds up to G - 1 uncompensated roundings of up to half an ulp each
// (2.4e-7 at 1e9 rows, beside GLM.scala:452's absolute tol 1e-6).  The partition-order sum of the
// reference (GLM.scala:404-407) is the order used here; only the rounding is compensated.
void compensated_rank_sum(const double* blocks, int nranks, int64_t count, double* out) {
  for (int64_t k = 0; k < count; ++k) {
    double s = 0.0, c = 0.0;
    for (int r = 0; r < nranks; ++r) neumaier_add(s, c, blocks[(int64_t)r * count + k]);
    out[k] = s + c;
  }
}

// Copy a column-major host block (rows x cols, leading dimension sld) into a packed buffer,
// on several threads for large blocks (the pageable -> pinned leg of the ingest path).
void pack_cols(double* dst, const double* src, int64_t sld, int64_t rows, int64_t cols) {
  const int64_t total = rows * cols;
  const int hw = (int)std::max(1u, std::min(8u, std::thread::hardware_concurrency()));
  const int nt = total >= ((int64_t)2 << 20) ? hw : 1;  // >= 16 MiB: split the copy
  auto part = [&](int t) {
    if (cols >= nt) {
      for (int64_t c = t; c < cols; c += nt) std::memcpy(dst + c * rows, src + c * sld, sizeof(double) * rows);
    } else {
      const int64_t r0 = rows * t / nt, r1 = rows * (t + 1) / nt;
      for (int64_t c = 0; c < cols; ++c)
        std::memcpy(dst + c * rows + r0, src + c * sld + r0, sizeof(double) * (size_t)(r1 - r0));
    }
  };
  if (nt == 1) {
    part(0);
    return;
  }
  std::vector<std::thread> th;
  for (int t = 1; t < nt; ++t) th.emplace_back(part, t);
  part(0);
  for (auto& x : th) x.join();
}

}  // namespace

// Which kernel a pass runs (enum sglm_pass_kernel) and its name: the dispatch rules of
// ensure_workspace / launch_pass / launch_narrow / the wide path, in one place (the engine labels
// its passes with it; sglm_pass_kernel_for exposes it for a CPU test of the mapping).
namespace {
int pass_kernel_choice(int64_t n_pad, int P16, bool narrow, bool wide, bool proc, int fused_split, int family,
                       int link, char* name, size_t len) {
  static const char* fam[] = {"binomial", "gaussian", "poisson", "gamma"};
  static const char* lnk[] = {"logit", "probit", "cloglog", "identity", "log", "inverse"};
  const char* f = (family >= 0 && family < 4) ? fam[family] : "?";
  const char* l = (link >= 0 && link < 6) ? lnk[link] : "?";
  int k;
  if (wide) {
    k = proc ? SGLM_KERNEL_WIDE_PROC : SGLM_KERNEL_WIDE;
    std::snprintf(name, len, "wide_gram_kernel<%s>", proc ? "procedural" : "resident");
  } else if (narrow) {
    k = SGLM_KERNEL_NARROW;
    std::snprintf(name, len, "irls_narrow_kernel<%d,%s,%s>", P16, f, l);
  } else if (pass_uses_split(P16, fused_split, n_pad)) {
    k = SGLM_KERNEL_FUSED_SPLIT;
    std::snprintf(name, len, "irls_pass_r_kernel<%d,%s,%s>", P16, f, l);
  } else {
    k = SGLM_KERNEL_FUSED;
    std::snprintf(name, len, "irls_pass_kernel<%d,%s,%s>", P16, f, l);
  }
  return k;
}
}  // namespace

// ---- in-process communicator: N host threads, one handle each (a JVM driver's thread pool) ----
// Every rank's call blocks until all N have arrived; the last to arrive sums the N buffers in
// rank order (deterministic, independent of arrival order) and writes the sum into all of them.
struct sglm_local_comm {
  int nranks = 0;
  std::mutex mu;
  std::condition_variable cv;
  int arrived = 0;
  uint64_t generation = 0;
  std::vector<double*> bufs;
  int64_t count = -1;
  bool failed = false;  // this round: a rank passed another count
  bool result = false;  // the last completed round failed (read by its waiters only)
  double timeout_ms = 0.0;  // SGLM_COMM_TIMEOUT_S, read once by sglm_local_comm_create
  struct Rank {
    sglm_local_comm* c;
    int rank;
  };
  std::vector<Rank> ranks;
};

namespace {
// The rank a caller-supplied communicator context stands for, when the engine can tell: the
// in-process communicator's rank contexts (sglm_local_comm_rank); -1 otherwise.
int known_rank(sglm_allreduce_fn fn, void* ctx) {
  if (fn == &sglm_local_allreduce && ctx) return static_cast<sglm_local_comm::Rank*>(ctx)->rank;
  return -1;
}
}  // namespace

struct sglm_engine : public Backend {
  int device = 0;
  hipStream_t st = nullptr;
  hipEvent_t ev0 = nullptr, ev1 = nullptr, ev2 = nullptr;
  hipEvent_t evc = nullptr;  // end of the pass's device all-reduce (comm time = ev2 -> evc)
  hipEvent_t evpre = nullptr;  // before a small RCCL all-reduce: where its deadline starts
  int ncu = 256;
  // resident shard
  int64_t n = 0, p = 0, n_pad = 0, nblocks = 0;
  double *dX = nullptr, *dy = nullptr, *dm = nullptr, *doff = nullptr, *dprior = nullptr, *deta = nullptr;
  // pass workspace
  int P16 = 0, grid = 0;
  int64_t stride = 0;
  double *dbeta = nullptr, *dpart = nullptr, *dred = nullptr, *dsmall = nullptr;
  double *hbeta = nullptr, *hred = nullptr;
  int64_t part_cap = 0, red_cap = 0;
  Comm comm;
  bool red_on_device = false;  // dred holds the all-reduced result of the last pass
  bool lp_stats = false;       // the last pass carried the final statistics (PassArgs::stats_in_pass)
  double stats_const = 0.0;    // the fit's initial-pass S_AUX2: constant part of in-pass Poisson / Gamma statistics
  int consts_family = -1;      // family whose initial pass produced stats_const on this data (-1: none)
  // deviance-only passes (Backend::pass_dev): the next enqueue_pass runs the row stage and the
  // scalar reduction but no Gram -- bitwise the scalars of the full pass.  SGLM_SPECULATE=0 off.
  bool dev_only = false, allow_spec = true;
  // wide path (wide.hip)
  bool wide = false, force_wide = false;
  // narrow path (narrow.hip, p <= 64): barrier-free per-wave pipelines
  bool narrow = false;
  // procedural shard (sglm_synth_procedural): X regenerated in the wide kernels, not stored
  ProcX procx{};
  // procedural shards in chunks (setup_proc_chunks): each pass generates C rows of X at a time
  // into an HBM scratch (the row kernel, while it forms eta) and runs the resident Gram kernels
  // over it -- X is generated once per pass instead of once per super-tile that reads it
  int64_t ch_rows = 0;  // rows per chunk (multiple of 32); 0: in-kernel generation (PROC kernels)
  int nch = 0;
  std::vector<hipEvent_t> evch;  // [4 * nch + 1]: row span, Gram span per chunk; st -> st2 fork
  double *dxsc = nullptr, *dchunks = nullptr;
  bool allow_chunks = true;  // SGLM_PROC_CHUNKS=0 disables
  // SGLM_PROC_OVERLAP: chunks of an overlapped procedural pass (<= 1: one buffer, serial).  Round 2
  // measured it slower beside both Gram launches (250M x 512 logit: 1257 ms per pass serial, 1420 /
  // 1480 at 8 / 16 chunks -- the generator's integer + fp64 VALU slowed the Gram by 31-38 %).  Round 5
  // (VERDICT r4 item 6): gated to the off-diagonal launches (then SGLM_PROC_OV_GATE; the diagonal launch
  // goes first) and the generating row kernel at raised priority, 8 chunks: 1284.5 -> 1266.9 ms on one
  // box (ungated 1466.3, gated at normal priority 1285.7).  Round 5 then split the
  // generator off (proc_gen_kernel, 48 VGPRs) and let it start beside each chunk's diagonal launch,
  // which goes first; round 6 measured the other launch orders +4.5 % (generator held until the
  // diagonal launch is done) and +5.5 % (off-diagonal launch first) and retired them.
  int proc_ov_want = 8;
  bool proc_ov = false;      // double-buffered scratch, row kernels on st2 (as the resident overlap below)
  int64_t proc_ov_min = (int64_t)1 << 20;  // SGLM_PROC_OV_MIN: fewest rows per overlapped chunk
  // resident wide shards, overlapped passes: the rows are cut into nov chunks; the row kernel of
  // chunk c + 1 runs on a second stream (st2) beside the Gram kernels of chunk c, so only chunk 0's
  // row stage is exposed.  Each chunk is reduced into dchunks[c]; the chunks are summed in order.
  int ov_want = 16;                // SGLM_WIDE_OVERLAP: chunks per pass (<= 1: off)
  int64_t ov_min = (int64_t)1 << 16;  // SGLM_WIDE_OV_MIN: fewest rows per chunk (fewer chunks on small shards)
  int nov = 0;
  int64_t ov_rows = 0;             // rows per chunk (multiple of 32; the last chunk may be shorter)
  int rgrid_ov = 0;                // row-kernel grid of chunks >= 1 (one workgroup per CU)
  hipStream_t st2 = nullptr;
  std::vector<hipEvent_t> evov;    // [4 * nov + 1]: row span, Gram span per chunk; st -> st2 fork
  double *dw = nullptr, *dwz = nullptr, *dgp = nullptr, *drp = nullptr;
  int64_t gp_cap = 0, rp_cap = 0, wstride = 0;
  int npan = 0, nst = 0, nslots = 0, ggrid = 0, rgrid = 0;
  int ggk[2] = {0, 0};  // persistent grid of the off-diagonal / diagonal Gram kernels
  WidePiece* dpieces[2] = {nullptr, nullptr};  // [0] off-diagonal, [1] diagonal super-tiles
  int* dwgb[2] = {nullptr, nullptr};
  int* dstr = nullptr;                          // [nst][2] partial slot range per super-tile
  bool has_sched[2] = {false, false};
  hipEvent_t evm = nullptr;
  rocblas_handle blas = nullptr;
  // wide-path device solve (SGLM_WIDE_SOLVE): 0 Cholesky (potrf / potrs / potri, the default),
  // 1 LU + explicit inverse (Breeze inv's algorithm: dgetrf + dgetri, utils.scala:103-105)
  int wide_lu = 0;
  int64_t proc_scratch_max = 0;  // SGLM_PROC_SCRATCH_MAX (GiB): cap on the procedural chunk scratch (0: none)
  // stats
  int64_t passes = 0, dev_passes = 0;
  double pass_ms = 0.0, reduce_ms = 0.0, last_pass_ms = 0.0, last_reduce_ms = 0.0, row_ms = 0.0, gram_ms = 0.0;
  int fused_split = 1;  // SGLM_FUSED_SPLIT: 1 K1r from its default column-block count up, 0 never (K1), N >= 2 from P16 = N
  bool allow_lm_device = true;  // SGLM_LM_DEVICE=0: LM fits take the two host round trips (tests)
  bool lm_extras_pass = false;  // the next LM Gram pass also sums X'1 and y'y (lm_device, one pass)
  int64_t lm_device_fits = 0;
  int64_t lm_onepass_fits = 0;  // of those, fits whose statistics came from the Gram pass's sums
  int last_kernel = SGLM_KERNEL_NONE;  // the kernel of the last pass (enum sglm_pass_kernel) and its name
  char last_kernel_name[64] = "";
  // ingest (sglm_reserve / sglm_set_rows): two pinned staging buffers, double-buffered
  static constexpr int64_t STAGE_DOUBLES = (int64_t)8 << 20;  // 64 MiB each
  double* hstage[2] = {nullptr, nullptr};
  hipEvent_t evstage[2] = {nullptr, nullptr};
  int stage_k = 0;
  int64_t rows_loaded = 0;  // rows covered by the blocks written since the shard was reserved
  std::vector<std::pair<int64_t, int64_t>> written;  // those blocks' row ranges, disjoint, sorted
  double load_ms = 0.0;     // host wall time in set_data / set_rows (staging + H2D)
  int64_t load_bytes = 0;
  // new-row scoring (sglm_predict_new): a device scratch, separate from the resident shard
  double *dxs = nullptr, *dvs = nullptr, *dms = nullptr, *dos = nullptr;
  int64_t xs_cap = 0, vs_cap = 0;
  // single-process multi-device handle (sglm_create_multi): the shards' engines; this handle
  // then only routes and reduces (one process owns all GPUs, as SURVEY 8(b) asks)
  std::vector<sglm_engine*> subs;
  std::vector<int64_t> sub_lo;       // first global row of each shard
  std::vector<ncclComm_t> gcomms;    // ncclCommInitAll over distinct devices (else host sums)
  bool group_aborted = false;        // a group all-reduce missed its deadline (wait_collective)
  int64_t g_n = 0;                   // group: total rows
  bool group() const { return !subs.empty(); }

  ~sglm_engine() override {
    for (sglm_engine* s : subs) delete s;
    for (ncclComm_t c : gcomms)
      if (c) (void)ncclCommDestroy(c);
    subs.clear();
    gcomms.clear();
    release();
  }

  void free_data() {
    for (double** ptr : {&dX, &dy, &dm, &doff, &dprior, &deta, &dw, &dwz}) {
      if (*ptr) (void)hipFree(*ptr);
      *ptr = nullptr;
    }
    n = p = n_pad = nblocks = 0;
    lm_last_pass_ms = -1.0;  // a new shard: the next device LM fit is timed
    rows_loaded = 0;
    written.clear();
    consts_family = -1;
    procx = ProcX{};
    for (double** ptr : {&dxsc, &dchunks}) {
      if (*ptr) (void)hipFree(*ptr);
      *ptr = nullptr;
    }
    ch_rows = 0;
    nch = 0;
    proc_ov = false;
    nov = 0;
    ov_rows = 0;
  }
  void release() {
    (void)hipSetDevice(device);
    free_data();
    for (double** ptr : {&dbeta, &dpart, &dred, &dsmall, &dgp, &drp, &dxs, &dvs, &dms, &dos}) {
      if (*ptr) (void)hipFree(*ptr);
      *ptr = nullptr;
    }
    xs_cap = vs_cap = 0;
    dsmall_cap = 0;
    for (int k = 0; k < 2; ++k) {
      if (hstage[k]) (void)hipHostFree(hstage[k]);
      if (evstage[k]) (void)hipEventDestroy(evstage[k]);
      hstage[k] = nullptr;
      evstage[k] = nullptr;
    }
    free_schedule();
    part_cap = red_cap = gp_cap = rp_cap = 0;
    if (blas) (void)rocblas_destroy_handle(blas);
    blas = nullptr;
    if (evm) (void)hipEventDestroy(evm);
    evm = nullptr;
    for (double** ptr : {&hbeta, &hred, &hsmall}) {
      if (*ptr) (void)hipHostFree(*ptr);
      *ptr = nullptr;
    }
    if (comm.nccl) (void)ncclCommDestroy(comm.nccl);
    comm.nccl = nullptr;
    for (hipEvent_t e : evch) (void)hipEventDestroy(e);
    evch.clear();
    for (hipEvent_t e : evov) (void)hipEventDestroy(e);
    evov.clear();
    if (st2) (void)hipStreamDestroy(st2);
    st2 = nullptr;
    if (ev0) (void)hipEventDestroy(ev0);
    if (ev1) (void)hipEventDestroy(ev1);
    if (ev2) (void)hipEventDestroy(ev2);
    if (evpre) (void)hipEventDestroy(evpre);
    if (evc) (void)hipEventDestroy(evc);
    if (st) (void)hipStreamDestroy(st);
    ev0 = ev1 = ev2 = evc = evpre = nullptr;
    st = nullptr;
  }

  int64_t ncols() const override { return group() ? subs[0]->p : p; }
  bool pass_has_stats() const override { return group() ? subs[0]->lp_stats : lp_stats; }
  int npart() const override { return group() ? (int)subs.size() : comm.nranks; }

  // ---- communicator helpers ----
  // after_pass: dbuf is the pass just enqueued (ev2 marks its end on st); the RCCL time is then
  // ev2 -> evc on the device (this rank's wait for the others included), not the host wall time
  // of a synchronize that would also cover the pass kernels.
  std::unique_ptr<CallbackRunner> cbr;  // caller callbacks with a deadline (CallbackRunner)
  CallbackRunner& runner() {
    if (!cbr) cbr.reset(new CallbackRunner(device));
    return *cbr;
  }
  // a caller callback abandoned at its deadline may still write the device buffer it was given:
  // those buffers are leaked, never freed under it
  void leak_comm_buffers() {
    dred = dsmall = nullptr;
    red_cap = dsmall_cap = 0;
  }
  int call_comm(double* buf, int64_t count, int on_device) {
    const int rc = runner().call(comm.fn, comm.ctx, buf, count, (void*)st, on_device, comm.timeout_ms, comm.rank);
    if (rc && runner().leaked_device_buffer()) leak_comm_buffers();
    return rc;
  }
  int allreduce_device(double* dbuf, int64_t count, bool after_pass = false) {
    if (comm.kind == 2) {
      if (!comm.nccl) {
        set_error(rank_str(comm.rank) + ": the RCCL communicator was aborted by an earlier failure; set a new one");
        return SGLM_ECOMM;
      }
      const double t0 = now_ms();
      // the deadline starts when everything this rank queued before the collective is done: the pass
      // (ev2, recorded at its end) or, for the small all-reduces, whatever precedes them on st
      if (!after_pass) {
        if (!evpre) HIPCHK(hipEventCreateWithFlags(&evpre, hipEventDisableTiming));
        HIPCHK(hipEventRecord(evpre, st));
      }
      ncclResult_t r = ncclAllReduce(dbuf, dbuf, (size_t)count, ncclFloat64, ncclSum, comm.nccl, st);
      if (r != ncclSuccess) {
        set_error(std::string("RCCL ncclAllReduce on ") + rank_str(comm.rank) + ": " + ncclGetErrorString(r));
        return SGLM_ECOMM;
      }
      if (after_pass) HIPCHK(hipEventRecord(evc, st));
      if (int rc = wait_collective({st}, {&comm.nccl}, comm.timeout_ms, comm.rank, "ncclAllReduce",
                                   {after_pass ? ev2 : evpre}))
        return rc;
      if (after_pass) {
        float ms = 0.f;
        HIPCHK(hipEventElapsedTime(&ms, ev2, evc));
        comm.ms += ms;
      } else {
        comm.ms += now_ms() - t0;
      }
    } else if (comm.kind == 1 && comm.on_device) {
      HIPCHK(hipStreamSynchronize(st));
      const double t0 = now_ms();
      if (int rc = call_comm(dbuf, count, 1)) return rc;
      comm.ms += now_ms() - t0;
    }
    return SGLM_OK;
  }
  int allreduce_host(double* hbuf, int64_t count) {
    if (comm.kind == 1 && !comm.on_device) {
      const double t0 = now_ms();
      if (int rc = call_comm(hbuf, count, 0)) return rc;
      comm.ms += now_ms() - t0;
    }
    return SGLM_OK;
  }
  bool comm_on_device() const { return comm.kind == 2 || (comm.kind == 1 && comm.on_device); }
  // scalars summed across ranks through rank blocks (compensated_rank_sum): needs >1 rank and a
  // known own rank; otherwise the communicator's plain sum
  bool gather_ranks() const { return comm.kind != 0 && comm.nranks > 1 && comm.rank >= 0 && comm.rank < comm.nranks; }
  int64_t dsmall_cap = 0;
  double* hsmall = nullptr;  // pinned [64]: the final statistics' sums (stats)
  int ensure_small(int64_t count) {
    if (!hsmall) HIPCHK(hipHostMalloc(&hsmall, sizeof(double) * 64, hipHostMallocDefault));
    if (count <= dsmall_cap && dsmall) return SGLM_OK;
    if (dsmall) HIPCHK(hipFree(dsmall));
    dsmall = nullptr;
    dsmall_cap = std::max<int64_t>(64, count);
    HIPCHK(hipMalloc(&dsmall, sizeof(double) * dsmall_cap));
    return SGLM_OK;
  }
  // all-reduce a small host vector (count scalar sums) through whichever path the communicator uses
  int allreduce_small(double* h, int64_t count) {
    if (comm.kind == 0) return SGLM_OK;
    std::vector<double> blocks;
    double* b = h;
    int64_t len = count;
    if (gather_ranks()) {  // this rank's values in its own block, zeros elsewhere
      blocks.assign((size_t)(count * comm.nranks), 0.0);
      std::memcpy(blocks.data() + (int64_t)comm.rank * count, h, sizeof(double) * count);
      b = blocks.data();
      len = count * comm.nranks;
    }
    if (comm_on_device()) {
      if (int rc = ensure_small(len)) return rc;
      HIPCHK(hipMemcpyAsync(dsmall, b, sizeof(double) * len, hipMemcpyHostToDevice, st));
      int rc = allreduce_device(dsmall, len);
      if (rc) return rc;
      HIPCHK(hipMemcpyAsync(b, dsmall, sizeof(double) * len, hipMemcpyDeviceToHost, st));
      HIPCHK(hipStreamSynchronize(st));
    } else if (int rc = allreduce_host(b, len)) {
      return rc;
    }
    if (b != h) compensated_rank_sum(b, comm.nranks, count, h);
    return SGLM_OK;
  }
  // dred / hred hold at least len doubles (the packed result + the rank blocks of its scalars)
  int ensure_red_len(int64_t len) {
    if (len <= red_cap && dred) return SGLM_OK;
    if (dred) HIPCHK(hipFree(dred));
    if (hred) HIPCHK(hipHostFree(hred));
    dred = hred = nullptr;
    HIPCHK(hipMalloc(&dred, sizeof(double) * len));
    HIPCHK(hipHostMalloc(&hred, sizeof(double) * len, hipHostMallocDefault));
    if (dbeta) HIPCHK(hipFree(dbeta));
    if (hbeta) HIPCHK(hipHostFree(hbeta));
    dbeta = hbeta = nullptr;
    HIPCHK(hipMalloc(&dbeta, sizeof(double) * len));
    HIPCHK(hipHostMalloc(&hbeta, sizeof(double) * len, hipHostMallocDefault));
    red_cap = len;
    return SGLM_OK;
  }
  // this shard's scalars into rank block `r` of the nr blocks after the packed result, zeros in the
  // others (device buffer, on st)
  int stage_rank_block(int r, int nr) {
    const int64_t plen = packed_len(p), sc = tri_count(p) + p;
    HIPCHK(hipMemsetAsync(dred + plen, 0, sizeof(double) * (size_t)(NS * nr), st));
    HIPCHK(hipMemcpyAsync(dred + plen + (int64_t)r * NS, dred + sc, sizeof(double) * NS, hipMemcpyDeviceToDevice, st));
    return SGLM_OK;
  }

  void free_schedule() {
    for (int k = 0; k < 2; ++k) {
      if (dpieces[k]) (void)hipFree(dpieces[k]);
      if (dwgb[k]) (void)hipFree(dwgb[k]);
      dpieces[k] = nullptr;
      dwgb[k] = nullptr;
      has_sched[k] = false;
    }
    if (dstr) (void)hipFree(dstr);
    dstr = nullptr;
  }

  // Cost-balanced static schedules of the persistent Gram kernels.  For each kernel (off-
  // diagonal / diagonal super-tiles) the (super-tile, block) line, super-tile major, is cut
  // into ggrid equal segments; a segment's runs inside one super-tile are its pieces.
  // Pieces are numbered in line order, so the partial slots of a super-tile are consecutive.
  //
  // Banded schedule: the k = ggrid / S workgroups of each of the S super-tiles take
  // its blocks round-robin (block stride k), so all S k workgroups sweep the rows together and a
  // block read by one super-tile's workgroup is read by the others' while it is still in the
  // Infinity Cache / L2 (the workgroups that read the same blocks are numbered onto the same XCD,
  // blockIdx % 8).  The E = ggrid - S k workgroups left over take the rows' tail, a fraction
  // E / ggrid of every super-tile's blocks cut into E equal contiguous segments, so no workgroup
  // idles and each carries the same work.  Slots of a super-tile: its k strided pieces, then its
  // tail pieces in row order (the fixed reduction order).
  // (shards too short to give every super-tile two workgroups keep the contiguous pieces)
  bool banded_kind(int S, int64_t nb, int G) const { return S > 0 && G / S >= 2 && nb >= 2; }
  int build_wide_schedule() {
    const int64_t nb = (nch > 0 ? ch_rows : nov > 0 ? ov_rows : n_pad) / WIDE_RB;
    std::vector<int> str((size_t)nst * 2, 0);
    free_schedule();
    int slot = 0;
    for (int kind = 0; kind < 2; ++kind) {
      std::vector<int> sts;
      for (int I = 0; I < npan; ++I)
        for (int J = 0; J <= I; ++J)
          if ((I == J) == (kind == 1)) sts.push_back(I * (I + 1) / 2 + J);
      if (sts.empty()) continue;
      const int G = ggk[kind];
      const int64_t total = nb * (int64_t)sts.size();
      std::vector<WidePiece> pieces;
      std::vector<int> wgb((size_t)G + 1, 0);
      if (banded_kind((int)sts.size(), nb, G)) {
        const int S = (int)sts.size();
        const int k = G / S, E = G - S * k;
        const int64_t tail = nb * E / G, nbm = nb - tail;  // banded blocks [0, nbm), tail [nbm, nb)
        const int per_xcd = std::max(1, G / 8);
        std::vector<int> gq((size_t)S * k), extra;  // pair q = j S + s -> workgroup; the left-over workgroups
        std::vector<char> used((size_t)G, 0);
        for (int q = 0; q < S * k; ++q) {
          const int g = (G % 8 == 0) ? (q % per_xcd) * 8 + q / per_xcd : q;
          gq[(size_t)q] = g;
          used[(size_t)g] = 1;
        }
        for (int g = 0; g < G; ++g)
          if (!used[(size_t)g]) extra.push_back(g);
        struct Pc { int g; int64_t b0, b1, bs; };
        std::vector<std::vector<Pc>> per_st((size_t)S);
        for (int j = 0; j < k; ++j)
          for (int s2 = 0; s2 < S; ++s2)
            if (j < nbm) per_st[(size_t)s2].push_back(Pc{gq[(size_t)j * S + s2], j, nbm, k});
        const int64_t tl = (int64_t)S * tail;  // tail line, super-tile major
        for (int e = 0; e < E && tl > 0; ++e) {
          int64_t pos = tl * e / E;
          const int64_t end = tl * (e + 1) / E;
          while (pos < end) {
            const int s2 = (int)(pos / tail);
            const int64_t b = pos % tail, len = std::min(tail - b, end - pos);
            per_st[(size_t)s2].push_back(Pc{extra[(size_t)e], nbm + b, nbm + b + len, 1});
            pos += len;
          }
        }
        std::vector<std::vector<WidePiece>> per_g((size_t)G);
        for (int s2 = 0; s2 < S; ++s2) {
          const int st = sts[(size_t)s2];
          str[(size_t)st * 2] = slot;
          for (const Pc& c : per_st[(size_t)s2]) per_g[(size_t)c.g].push_back(WidePiece{c.b0, c.b1, st, slot++, c.bs});
          str[(size_t)st * 2 + 1] = slot;
        }
        for (int g = 0; g < G; ++g) {
          wgb[(size_t)g] = (int)pieces.size();
          for (const WidePiece& w : per_g[(size_t)g]) pieces.push_back(w);
        }
        wgb[(size_t)G] = (int)pieces.size();
      } else {
        int64_t pos = 0, b = 0;
        size_t si = 0;
        for (int g = 0; g < G; ++g) {
          wgb[(size_t)g] = (int)pieces.size();
          const int64_t end = (int64_t)((__int128)total * (g + 1) / G);
          while (si < sts.size() && pos < end) {
            const int64_t k = std::min(nb - b, end - pos);
            const int st = sts[si];
            if (b == 0) str[(size_t)st * 2] = slot;
            pieces.push_back(WidePiece{b, b + k, st, slot++, 1});
            str[(size_t)st * 2 + 1] = slot;
            pos += k;
            b += k;
            if (b == nb) {
              ++si;
              b = 0;
            }
          }
        }
        wgb[(size_t)G] = (int)pieces.size();
      }
      HIPCHK(hipMalloc(&dpieces[kind], sizeof(WidePiece) * pieces.size()));
      HIPCHK(hipMalloc(&dwgb[kind], sizeof(int) * wgb.size()));
      HIPCHK(hipMemcpy(dpieces[kind], pieces.data(), sizeof(WidePiece) * pieces.size(), hipMemcpyHostToDevice));
      HIPCHK(hipMemcpy(dwgb[kind], wgb.data(), sizeof(int) * wgb.size(), hipMemcpyHostToDevice));
      has_sched[kind] = true;
    }
    nslots = slot;
    HIPCHK(hipMalloc(&dstr, sizeof(int) * str.size()));
    HIPCHK(hipMemcpy(dstr, str.data(), sizeof(int) * str.size(), hipMemcpyHostToDevice));
    return SGLM_OK;
  }

  // chunks whose row kernels run beside the Gram (resident or procedural), 0 if none
  int ov_chunks() const { return nov > 1 ? nov : (proc_ov ? nch : 0); }
  double* rowpart(int c) const { return drp + (c == 0 ? 0 : ((int64_t)rgrid + (int64_t)(c - 1) * rgrid_ov) * NS); }

  int ensure_wide_workspace() {
    npan = wide_panels((int)p);
    nst = npan * (npan + 1) / 2;
    wstride = wide_stride();
    ggk[0] = ncu * wide_gram_wg_per_cu(false);
    ggk[1] = ncu * wide_gram_wg_per_cu(true);
    ggrid = ggk[0];
    nov = 0;
    ov_rows = 0;
    if (!procx.on && dX && ov_want > 1 && n_pad >= 2 * ov_min) {
      ov_rows = (std::max<int64_t>(ov_min, (n_pad + ov_want - 1) / ov_want) + 31) / 32 * 32;
      nov = (int)((n_pad + ov_rows - 1) / ov_rows);
      if (nov < 2) nov = 0, ov_rows = 0;
    }
    if (nov > 1) {
      if (!st2) HIPCHK(hipStreamCreateWithFlags(&st2, hipStreamNonBlocking));
      while (evov.size() < (size_t)4 * nov + 1) {
        hipEvent_t e = nullptr;
        HIPCHK(hipEventCreate(&e));
        evov.push_back(e);
      }
      if (dchunks) HIPCHK(hipFree(dchunks));
      dchunks = nullptr;
      HIPCHK(hipMalloc(&dchunks, sizeof(double) * (size_t)nov * (size_t)packed_len(p)));
    }
    int rc = build_wide_schedule();
    if (rc) return rc;
    grid = nslots;
    rgrid = (int)std::max<int64_t>(1, std::min<int64_t>(8 * (int64_t)ncu, ((nov > 0 ? ov_rows : n_pad) + 255) / 256));
    rgrid_ov = std::min(rgrid, ncu);
    const int64_t need_gp = (int64_t)std::max(nslots, 1) * wstride;
    if (need_gp > gp_cap) {
      if (dgp) HIPCHK(hipFree(dgp));
      dgp = nullptr;
      HIPCHK(hipMalloc(&dgp, sizeof(double) * need_gp));
      gp_cap = need_gp;
    }
    // overlapped passes keep every chunk's row partials until its reduce (the next chunk's row
    // kernel runs meanwhile): chunk 0 at [0, rgrid), chunk c >= 1 at rgrid + (c - 1) rgrid_ov
    const int64_t need_rp = ((int64_t)rgrid + (int64_t)(std::max(ov_chunks(), 1) - 1) * rgrid_ov) * NS;
    if (need_rp > rp_cap) {
      if (drp) HIPCHK(hipFree(drp));
      drp = nullptr;
      HIPCHK(hipMalloc(&drp, sizeof(double) * need_rp));
      rp_cap = need_rp;
    }
    if (!evm) HIPCHK(hipEventCreate(&evm));
    return SGLM_OK;
  }

  // Chunked procedural passes: the largest chunk the free HBM holds (minus a margin), balanced
  // over the chunks; w / w*z cover nch * ch_rows rows (zero past n_pad).  Called once procx is set.
  int setup_proc_chunks() {
    if (!procx.on || !allow_chunks) return SGLM_OK;
    size_t fr = 0, tot = 0;
    HIPCHK(hipMemGetInfo(&fr, &tot));
    const int64_t ncols8 = (p + 7) / 8 * 8;
    const size_t margin = (size_t)4 << 30;
    size_t room = fr > margin ? fr - margin : 0;
    if (proc_scratch_max > 0) room = std::min(room, (size_t)proc_scratch_max << 30);
    const int64_t cap_rows = (int64_t)(room / (sizeof(double) * (size_t)ncols8));
    int64_t c = std::min<int64_t>(n_pad, cap_rows / 32 * 32);
    if (c < std::min<int64_t>(n_pad, (int64_t)1 << 20)) return SGLM_OK;  // too little room: in-kernel generation
    int64_t k = (n_pad + c - 1) / c;
    // overlapped: two scratch buffers, the row kernel of chunk c + 1 generates into one while the
    // Gram kernels of chunk c read the other; at least proc_ov_want chunks of >= 1M rows
    const int64_t half = cap_rows / 2 / 32 * 32, kmin = proc_ov_min;
    proc_ov = false;
    if (proc_ov_want > 1 && half >= kmin && n_pad >= 2 * kmin) {
      k = std::max<int64_t>((n_pad + half - 1) / half, std::min<int64_t>(proc_ov_want, n_pad / kmin));
      proc_ov = k >= 2;
    }
    c = ((n_pad + k - 1) / k + 31) / 32 * 32;
    ch_rows = c;
    nch = (int)((n_pad + c - 1) / c);
    const size_t sc = sizeof(double) * (size_t)c * (size_t)ncols8 * (proc_ov ? 2 : 1);
    HIPCHK(hipMalloc(&dxsc, sc));
    HIPCHK(hipMemsetAsync(dxsc, 0, sc, st));
    if (proc_ov && !st2) HIPCHK(hipStreamCreateWithFlags(&st2, hipStreamNonBlocking));
    const int64_t span = (int64_t)nch * c;  // w / w*z rows the chunks address
    if (span > n_pad) {
      for (double** q : {&dw, &dwz}) {
        if (*q) HIPCHK(hipFree(*q));
        *q = nullptr;
        HIPCHK(hipMalloc(q, sizeof(double) * (size_t)span));
        HIPCHK(hipMemsetAsync(*q, 0, sizeof(double) * (size_t)span, st));
      }
    }
    HIPCHK(hipMalloc(&dchunks, sizeof(double) * (size_t)nch * (size_t)packed_len(p)));
    while (evch.size() < (size_t)4 * nch + 1) {
      hipEvent_t e = nullptr;
      HIPCHK(hipEventCreate(&e));
      evch.push_back(e);
    }
    HIPCHK(hipStreamSynchronize(st));
    return ensure_wide_workspace();  // the Gram schedule for ch_rows-row chunks
  }

  int ensure_workspace() {
    if (wide) {
      P16 = 0;
      int rc = ensure_wide_workspace();
      if (rc) return rc;
    }
    narrow = !wide && p <= 64;
    if (narrow) {
      P16 = narrow_variant((int)p);
      stride = narrow_stride(P16);
      const int64_t want_grid = (int64_t)ncu * narrow_wg_per_cu();
      const int64_t per_wg = narrow_rows_per_wg(P16);
      const int64_t need = (nblocks * RB + per_wg - 1) / per_wg;
      grid = (int)std::max<int64_t>(1, std::min(need, want_grid));
    } else {
      if (!wide) P16 = pass_variant((int)p, fused_split, n_pad);
      stride = wide ? 0 : pass_stride(P16);
      if (!wide) {
        const int64_t want_grid = (int64_t)ncu * (pass_uses_split(P16, fused_split, n_pad) ? 1 : pass_wg_per_cu(P16));
        grid = (int)(nblocks < want_grid ? (nblocks > 0 ? nblocks : 1) : want_grid);
      }
    }
    const int64_t need_part = std::max<int64_t>((int64_t)grid * stride, 4096 * NS);
    if (need_part > part_cap) {
      if (dpart) HIPCHK(hipFree(dpart));
      dpart = nullptr;
      HIPCHK(hipMalloc(&dpart, sizeof(double) * need_part));
      part_cap = need_part;
    }
    const int64_t need_red = packed_len(p) + 16 * std::max(P16, 1);
    if (need_red > red_cap) {
      if (dred) HIPCHK(hipFree(dred));
      if (dbeta) HIPCHK(hipFree(dbeta));
      if (hred) HIPCHK(hipHostFree(hred));
      if (hbeta) HIPCHK(hipHostFree(hbeta));
      dred = dbeta = hred = hbeta = nullptr;
      HIPCHK(hipMalloc(&dred, sizeof(double) * need_red));
      HIPCHK(hipMalloc(&dbeta, sizeof(double) * need_red));
      HIPCHK(hipHostMalloc(&hred, sizeof(double) * need_red, hipHostMallocDefault));
        HIPCHK(hipHostMalloc(&hbeta, sizeof(double) * need_red, hipHostMallocDefault));
      red_cap = need_red;
    }
    return ensure_small(64);
  }

  int alloc_data(int64_t n_, int64_t p_, bool has_m, bool has_off, bool has_prior, bool proc = false) {
    HIPCHK(hipSetDevice(device));
    free_data();
    if (n_ < 0 || p_ <= 0) {
      set_error("requirement failed: n >= 0 and p >= 1");
      return SGLM_EINVAL;
    }
    if (p_ > MAX_P_WIDE) {
      set_error("requirement failed: p <= " + std::to_string(MAX_P_WIDE) + " columns");
      return SGLM_EINVAL;
    }
    n = n_;
    p = p_;
    wide = force_wide || proc || p > 16 * MAX_P16;
    nblocks = (n + RB - 1) / RB;
    n_pad = std::max<int64_t>(nblocks, 1) * RB;
    const size_t vb = sizeof(double) * (size_t)n_pad;
    const size_t ncols = (size_t)((p + 7) / 8 * 8);  // whole column octets for the LDS-DMA staging
    hipError_t e = hipSuccess;
    if (!proc) {
      e = hipMalloc(&dX, vb * ncols);
      if (e != hipSuccess) {
        set_error(hip_msg(e, "hipMalloc(X)"));
        free_data();
        return SGLM_ENOMEM;
      }
      HIPCHK(hipMemsetAsync(dX, 0, vb * ncols, st));
    }
    for (auto pr : {std::make_pair(&dy, true), std::make_pair(&dm, has_m), std::make_pair(&doff, has_off),
                    std::make_pair(&dprior, has_prior), std::make_pair(&deta, true), std::make_pair(&dw, wide),
                    std::make_pair(&dwz, wide)}) {
      if (!pr.second) continue;
      e = hipMalloc(pr.first, vb);
      if (e != hipSuccess) {
        set_error(hip_msg(e, "hipMalloc(vector)"));
        free_data();
        return SGLM_ENOMEM;
      }
      HIPCHK(hipMemsetAsync(*pr.first, 0, vb, st));
    }
    return ensure_workspace();
  }

  // ---- ingest: pageable host -> pinned staging -> HBM ----
  int ensure_staging() {
    if (hstage[0]) return SGLM_OK;
    for (int k = 0; k < 2; ++k) {
      HIPCHK(hipHostMalloc(&hstage[k], sizeof(double) * STAGE_DOUBLES, hipHostMallocDefault));
      HIPCHK(hipEventCreateWithFlags(&evstage[k], hipEventDisableTiming));
      HIPCHK(hipEventRecord(evstage[k], st));
    }
    return SGLM_OK;
  }
  // Column-major host block (rows x cols, leading dimension sld) -> device (leading dimension
  // dld) through the two pinned buffers: the CPU packs one while the DMA engine drains the
  // other.  Pageable memory is never handed to the DMA engine directly.
  int h2d_block(double* dst, int64_t dld, const double* src, int64_t sld, int64_t rows, int64_t cols) {
    if (rows <= 0 || cols <= 0) return SGLM_OK;
    int rc = ensure_staging();
    if (rc) return rc;
    const int64_t rchunk = std::min<int64_t>(rows, STAGE_DOUBLES);
    for (int64_t r0 = 0; r0 < rows; r0 += rchunk) {
      const int64_t rr = std::min(rchunk, rows - r0);
      const int64_t cchunk = std::max<int64_t>(1, STAGE_DOUBLES / rr);
      for (int64_t c0 = 0; c0 < cols; c0 += cchunk) {
        const int64_t cc = std::min(cchunk, cols - c0);
        const int k = stage_k;
        stage_k ^= 1;
        HIPCHK(hipEventSynchronize(evstage[k]));  // the copy that last read this buffer is done
        pack_cols(hstage[k], src + r0 + c0 * sld, sld, rr, cc);
        HIPCHK(hipMemcpy2DAsync(dst + r0 + c0 * dld, sizeof(double) * (size_t)dld, hstage[k], sizeof(double) * rr,
                                sizeof(double) * rr, (size_t)cc, hipMemcpyHostToDevice, st));
        HIPCHK(hipEventRecord(evstage[k], st));
      }
    }
    return SGLM_OK;
  }

  // Rows [row0, row0 + nr) of the reserved shard from host memory (sglm_set_rows).
  int set_rows(int64_t row0, int64_t nr, const double* X, int64_t ldx, const double* yv, const double* mv,
               const double* ov, const double* pv) {
    HIPCHK(hipSetDevice(device));
    if (p <= 0 || procx.on) {
      set_error("requirement failed: sglm_reserve the shard before sglm_set_rows");
      return SGLM_EINVAL;
    }
    if (row0 < 0 || nr < 0 || row0 + nr > n || (nr > 0 && (!X || !yv || ldx < nr))) {
      set_error("requirement failed: 0 <= row0, row0 + nrows <= reserved rows, X and y non-null, ldx >= nrows");
      return SGLM_EINVAL;
    }
    if ((mv != nullptr) != (dm != nullptr) || (ov != nullptr) != (doff != nullptr) ||
        (pv != nullptr) != (dprior != nullptr)) {
      set_error("requirement failed: m / offset / prior must be given exactly when they were reserved");
      return SGLM_EINVAL;
    }
    if (nr == 0) return SGLM_OK;
    // blocks must not overlap (sglm.h): a repeated or overlapping block would count its rows twice
    // and let a fit run over reserved rows that were never written (zero X, y)
    auto it = std::lower_bound(written.begin(), written.end(), std::make_pair(row0, row0));
    if ((it != written.end() && it->first < row0 + nr) || (it != written.begin() && std::prev(it)->second > row0)) {
      set_error("requirement failed: rows [" + std::to_string(row0) + ", " + std::to_string(row0 + nr) +
                ") overlap a block already written (sglm_set_rows blocks must not overlap)");
      return SGLM_EINVAL;
    }
    const double t0 = now_ms();
    int rc = h2d_block(dX + row0, n_pad, X, ldx, nr, p);
    for (auto pr : {std::make_pair(dy, yv), std::make_pair(dm, mv), std::make_pair(doff, ov),
                    std::make_pair(dprior, pv)})
      if (!rc && pr.second) rc = h2d_block(pr.first + row0, n_pad, pr.second, nr, nr, 1);
    if (rc) return rc;
    HIPCHK(hipStreamSynchronize(st));
    load_ms += now_ms() - t0;
    const int nvec = 1 + (mv != nullptr) + (ov != nullptr) + (pv != nullptr);
    load_bytes += (int64_t)sizeof(double) * nr * (p + nvec);
    it = written.insert(std::lower_bound(written.begin(), written.end(), std::make_pair(row0, row0)),
                        std::make_pair(row0, row0 + nr));
    if (std::next(it) != written.end() && std::next(it)->first == it->second) {  // merge touching neighbours
      it->second = std::next(it)->second;
      written.erase(std::next(it));
    }
    if (it != written.begin() && std::prev(it)->second == it->first) {
      std::prev(it)->second = it->second;
      written.erase(it);
    }
    rows_loaded += nr;
    return SGLM_OK;
  }

  int check_loaded() const {
    if (p <= 0) {
      set_error("requirement failed: no data set (sglm_set_data)");
      return SGLM_EINVAL;
    }
    if (!procx.on && rows_loaded < n) {
      set_error("requirement failed: " + std::to_string(n - rows_loaded) +
                " reserved rows were never written (sglm_set_rows)");
      return SGLM_EINVAL;
    }
    return SGLM_OK;
  }

  // ---- scoring of new rows (sglm_predict_new): its own scratch, the shard stays resident ----
  int predict_new(const double* X, int64_t nn, int64_t pp, int64_t ldx, const double* beta, const double* off,
                  const double* mv, int family, int link, int type, double* out) {
    HIPCHK(hipSetDevice(device));
    const int64_t chunk = std::max<int64_t>(1, std::min<int64_t>(nn, ((int64_t)1 << 27) / std::max<int64_t>(pp, 1)));
    if (pp * chunk > xs_cap) {
      if (dxs) HIPCHK(hipFree(dxs));
      dxs = nullptr;
      HIPCHK(hipMalloc(&dxs, sizeof(double) * (size_t)(pp * chunk)));
      xs_cap = pp * chunk;
    }
    if (chunk > vs_cap) {
      for (double** q : {&dvs, &dms, &dos}) {
        if (*q) HIPCHK(hipFree(*q));
        *q = nullptr;
        HIPCHK(hipMalloc(q, sizeof(double) * (size_t)chunk));
      }
      vs_cap = chunk;
    }
    int rc = ensure_beta(pp);
    if (rc) return rc;
    std::memcpy(hbeta, beta, sizeof(double) * pp);
    HIPCHK(hipMemcpyAsync(dbeta, hbeta, sizeof(double) * pp, hipMemcpyHostToDevice, st));
    for (int64_t r0 = 0; r0 < nn; r0 += chunk) {
      const int64_t nr = std::min(chunk, nn - r0);
      rc = h2d_block(dxs, nr, X + r0, ldx, nr, pp);
      if (!rc && off) rc = h2d_block(dos, nr, off + r0, nr, nr, 1);
      if (!rc && mv) rc = h2d_block(dms, nr, mv + r0, nr, nr, 1);
      if (rc) return rc;
      HIPCHK(launch_predict(dxs, nr, (int)pp, nr, dbeta, off ? dos : nullptr, dvs, st, ProcX{}));
      if (type == SGLM_PREDICT_RESPONSE) HIPCHK(launch_unlink(dvs, mv ? dms : nullptr, nr, family, link, st));
      HIPCHK(hipMemcpyAsync(out + r0, dvs, sizeof(double) * nr, hipMemcpyDeviceToHost, st));
      HIPCHK(hipStreamSynchronize(st));
    }
    return SGLM_OK;
  }
  // hbeta / dbeta hold at least pp doubles (scoring before any shard exists)
  int ensure_beta(int64_t pp) {
    if (red_cap >= pp && dbeta) return SGLM_OK;
    const int64_t need = std::max<int64_t>(pp, red_cap);
    if (dred) HIPCHK(hipFree(dred));
    if (dbeta) HIPCHK(hipFree(dbeta));
    if (hred) HIPCHK(hipHostFree(hred));
    if (hbeta) HIPCHK(hipHostFree(hbeta));
    dred = dbeta = hred = hbeta = nullptr;
    HIPCHK(hipMalloc(&dred, sizeof(double) * need));
    HIPCHK(hipMalloc(&dbeta, sizeof(double) * need));
    HIPCHK(hipHostMalloc(&hred, sizeof(double) * need, hipHostMallocDefault));
    HIPCHK(hipHostMalloc(&hbeta, sizeof(double) * need, hipHostMallocDefault));
    red_cap = need;
    return SGLM_OK;
  }

  // ---- Backend ----
  int global_sums(double* out2) override {
    if (group()) {  // shard order, as the reference sums partitions (GLM.scala:420-423), compensated
      std::vector<double> blocks(2 * subs.size());
      for (size_t d = 0; d < subs.size(); ++d)
        if (int rc = subs[d]->global_sums(blocks.data() + 2 * d)) return rc;
      compensated_rank_sum(blocks.data(), (int)subs.size(), 2, out2);
      return SGLM_OK;
    }
    HIPCHK(hipSetDevice(device));
    if (int rc = check_loaded()) return rc;
    const int nparts = 1024;
    HIPCHK(launch_ysum(dy, n, dpart, nparts, st));
    std::vector<double> h(nparts);
    HIPCHK(hipMemcpyAsync(h.data(), dpart, sizeof(double) * nparts, hipMemcpyDeviceToHost, st));
    HIPCHK(hipStreamSynchronize(st));
    double s = 0.0, c = 0.0;
    for (int i = 0; i < nparts; ++i) neumaier_add(s, c, h[i]);
    out2[0] = s + c;
    out2[1] = (double)n;
    return allreduce_small(out2, 2);
  }

  bool has_dev_pass() const override { return allow_spec; }
  int pass_dev(int mode, const double* beta, double mu0, double ybar, int family, int link, double* packed) override {
    for (sglm_engine* s : subs) s->dev_only = true;
    dev_only = true;
    const int rc = pass(mode, beta, mu0, ybar, family, link, packed);
    for (sglm_engine* s : subs) s->dev_only = false;
    dev_only = false;
    dev_passes += 1;
    return rc;
  }

  int pass(int mode, const double* beta, double mu0, double ybar, int family, int link, double* packed) override {
    if (group()) return group_pass(mode, beta, mu0, ybar, family, link, packed);
    const int64_t plen = packed_len(p), sc = tri_count(p) + p;
    const int R = gather_ranks() ? comm.nranks : 0;  // rank blocks of the scalars (compensated_rank_sum)
    const int64_t len = plen + (int64_t)NS * R;
    if (int rc = ensure_red_len(len)) return rc;
    int rc = enqueue_pass(mode, beta, mu0, ybar, family, link);
    if (rc) return rc;
    if (comm_on_device()) {
      if (R && (rc = stage_rank_block(comm.rank, R))) return rc;
      rc = allreduce_device(dred, len, true);
      if (rc) return rc;
    }
    HIPCHK(hipMemcpyAsync(hred, dred, sizeof(double) * (comm_on_device() ? len : plen), hipMemcpyDeviceToHost, st));
    HIPCHK(hipStreamSynchronize(st));
    rc = pass_timing();
    if (rc) return rc;
    red_on_device = comm_on_device() || comm.kind == 0;
    if (!comm_on_device()) {
      if (R) {
        std::fill(hred + plen, hred + len, 0.0);
        std::memcpy(hred + plen + (int64_t)comm.rank * NS, hred + sc, sizeof(double) * NS);
      }
      rc = allreduce_host(hred, comm.kind == 0 ? plen : len);
      if (rc) return rc;
    }
    if (R) compensated_rank_sum(hred + plen, R, NS, hred + sc);
    std::memcpy(packed, hred, sizeof(double) * plen);
    finish_scalars(mode, family, packed + sc);
    return SGLM_OK;
  }

  // The narrow pass's in-pass Poisson / Gamma statistics lack their per-fit constants (rowmath.hpp
  // init_stats_const), which the fit's initial pass sums into S_AUX2: kept here, applied to every
  // later pass that carried the statistics -- R's dpois loglik sum pw (y log mu - mu) minus
  // sum pw lgamma(y + 1); Gamma's S_LL = sum pw log y and S_AUX1 = sum pw log mu = sum pw log y -
  // sum pw log(y eta).  Applied once, on the all-reduced scalars.
  // (The statistics ride only in passes of a fit, after its initial pass: enqueue_pass.)
  void finish_scalars(int mode, int family, double* s) {
    if (family != FAM_POISSON && family != FAM_GAMMA) return;
    if (mode == MODE_INIT_SINGLE || mode == MODE_INIT_MULTI) {
      stats_const = s[S_AUX2];
      s[S_AUX2] = 0.0;
      consts_family = family;
      for (sglm_engine* sub : subs) sub->consts_family = family;
      return;
    }
    if (mode != MODE_IRLS || !pass_has_stats()) return;
    if (family == FAM_POISSON) {
      s[S_LL] -= stats_const;
    } else {
      s[S_LL] = stats_const;
      s[S_AUX1] = stats_const - s[S_AUX1];
    }
  }

  // Kernel times of the pass just synchronised (HIP events on this engine's stream).
  int pass_timing() {
    float k1 = 0.f, k2 = 0.f;
    HIPCHK(hipEventElapsedTime(&k1, ev0, ev1));
    HIPCHK(hipEventElapsedTime(&k2, ev1, ev2));
    if (wide) {
      float km = 0.f;
      if (nov > 0 || nch > 0) {  // chunked pass: row spans and Gram spans per chunk
        const std::vector<hipEvent_t>& ev = nov > 0 ? evov : evch;
        float kg = 0.f;
        for (int c = 0; c < (nov > 0 ? nov : nch); ++c) {
          float kr = 0.f, kc = 0.f;
          HIPCHK(hipEventElapsedTime(&kr, ev[(size_t)4 * c], ev[(size_t)4 * c + 1]));
          HIPCHK(hipEventElapsedTime(&kc, ev[(size_t)4 * c + 2], ev[(size_t)4 * c + 3]));
          km += kr;
          kg += kc;
        }
        row_ms += km;
        gram_ms += kg;
      } else {
        HIPCHK(hipEventElapsedTime(&km, ev0, evm));
        row_ms += km;
        gram_ms += k1 - km;
      }
    }
    passes += 1;
    pass_ms += k1;
    reduce_ms += k2;
    last_pass_ms = k1;
    last_reduce_ms = k2;
    return SGLM_OK;
  }
  // An untimed pass (enqueue_pass timed = false: LM.fit on the device, see lm_device) counts the
  // kernel times of the last timed one.
  // (LM fits keep their own last timing: another pass kind in between must not be booked as LM time)
  double lm_last_pass_ms = -1.0, lm_last_reduce_ms = 0.0;
  void pass_untimed() {
    passes += 1;
    pass_ms += lm_last_pass_ms;
    reduce_ms += lm_last_reduce_ms;
  }

  // H2D beta, the pass kernels and the fixed-order partial reduction into dred -- all
  // asynchronous on this engine's stream (a multi-device handle enqueues every shard first).
  int enqueue_pass(int mode, const double* beta, double mu0, double ybar, int family, int link, bool timed = true) {
    HIPCHK(hipSetDevice(device));
    if (int rc = check_loaded()) return rc;
    if (beta) {
      std::memcpy(hbeta, beta, sizeof(double) * p);
      HIPCHK(hipMemcpyAsync(dbeta, hbeta, sizeof(double) * p, hipMemcpyHostToDevice, st));
    }
    PassArgs a{};
    a.X = dX;
    a.ld = n_pad;
    a.p = (int)p;
    a.nq = (int)((p + 3) / 4);
    a.y = dy;
    a.m = dm;
    a.off = doff;
    a.prior = dprior;
    a.beta = beta ? dbeta : nullptr;
    a.n = n;
    a.nblocks = nblocks;
    a.family = family;
    a.link = link;
    a.mode = mode;
    a.mu0 = mu0;
    a.ybar = ybar;
    a.partials = dpart;
    a.stride = stride;
    // Final statistics in the narrow pass, no eta store (rowmath.hpp stats_in_pass_family):
    // binomial / logit (m = 1) in every IRLS pass -- measured faster than the lean variant, the
    // statistics hide under the stream (DESIGN 4 K1') -- and Poisson / Gamma in the deviance-only
    // pass only, the pass glm_drive predicts to end the fit: at p = 64 their statistics rows cost
    // +14 % per pass (125M x 64 Poisson: 17.4 against 15.3 ms, tools/ab_stats.py; the family
    // arithmetic runs on 16 of 64 lanes there), while the deviance-only pass has no Gram to slow.
    // (Poisson / Gamma: only after this data's initial pass has summed the statistics' constants.)
    a.stats_in_pass = (narrow && mode == MODE_IRLS && stats_in_pass_family(family, link) &&
                       !(family == FAM_BINOMIAL && dm) &&
                       (family == FAM_BINOMIAL || (dev_only && consts_family == family))) ? 1 : 0;
    lp_stats = a.stats_in_pass != 0;
    note_kernel(mode == MODE_LM_GRAM ? FAM_GAUSSIAN : family, mode == MODE_LM_GRAM ? LNK_IDENTITY : link);
    a.eta_out = (mode == MODE_IRLS && !a.stats_in_pass) ? deta : nullptr;
    a.no_gram = dev_only ? 1 : 0;
    a.fused_split = fused_split;
    a.lm_extras = (mode == MODE_LM_GRAM && narrow && lm_extras_pass) ? 1 : 0;
    if (wide) {
      HIPCHK(hipEventRecord(ev0, st));
      WideRowArgs r{};
      r.X = dX;
      r.ld = n_pad;
      r.p = (int)p;
      r.y = dy;
      r.m = dm;
      r.off = doff;
      r.prior = dprior;
      r.beta = beta ? dbeta : nullptr;
      r.n = n;
      r.n_pad = n_pad;
      r.family = family;
      r.link = link;
      r.mode = mode;
      r.mu0 = mu0;
      r.ybar = ybar;
      r.w = dw;
      r.wz = dwz;
      r.eta_out = (mode == MODE_IRLS) ? deta : nullptr;
      r.row_partials = drp;
      r.proc = procx;
      r.r_begin = 0;
      r.r_end = n_pad;
      WideGramArgs g{};
      g.X = dX;
      g.ld = n_pad;
      g.ncols = (int)((p + 7) / 8 * 8);
      g.w = dw;
      g.wz = dwz;
      g.partials = dgp;
      g.stride = wstride;
      g.proc = procx;
      g.nb_lim = INT64_MAX;
      if (nch > 0) {  // procedural shard in chunks: generate C rows into the scratch, resident Gram over it
        const int64_t plen = packed_len(p);
        const int64_t bufd = ch_rows * (int64_t)g.ncols;  // doubles per scratch buffer
        g.ld = ch_rows;
        g.proc = ProcX{};
        r.xs_ld = ch_rows;
        hipStream_t rs = proc_ov ? st2 : st;  // row kernels
        if (proc_ov) {
          HIPCHK(hipEventRecord(evch[(size_t)4 * nch], st));  // fork: beta uploaded, the last pass done
          HIPCHK(hipStreamWaitEvent(st2, evch[(size_t)4 * nch], 0));
        }
        for (int c = 0; c < nch; ++c) {
          double* xs = dxsc + (proc_ov ? (int64_t)(c & 1) * bufd : 0);
          r.r_begin = (int64_t)c * ch_rows;
          r.r_end = r.r_begin + ch_rows;
          r.xs_out = dev_only ? nullptr : xs;  // deviance only: eta from the generator, no scratch
          r.row_partials = proc_ov ? rowpart(c) : drp;
          // buffer c & 1 is free once the Gram kernels of chunk c - 2 are done with it: chunk c's
          // generator then starts beside chunk c - 1's diagonal launch (which goes first, below)
          if (proc_ov && c >= 2) HIPCHK(hipStreamWaitEvent(st2, evch[(size_t)4 * (c - 2) + 3], 0));
          HIPCHK(hipEventRecord(evch[(size_t)4 * c], rs));
          if (!dev_only && proc_ov && c > 0) {
            // the lean generator (X into the scratch, X beta into deta), then the family stage from deta
            ProcGenArgs pg{};
            pg.proc = procx;
            pg.beta = mode == MODE_IRLS ? r.beta : nullptr;
            pg.xs = xs;
            pg.xs_ld = ch_rows;
            pg.r_begin = r.r_begin;
            pg.r_end = r.r_end;
            pg.eta_raw = deta;
            HIPCHK(launch_proc_gen(pg, c > 0 ? 2 * ncu : rgrid, rs));
            WideRowArgs rf = r;
            rf.xs_out = nullptr;
            rf.proc = ProcX{};
            rf.eta_in = mode == MODE_IRLS ? deta : nullptr;
            HIPCHK(launch_wide_rows(rf, c > 0 ? rgrid_ov : rgrid, rs, c > 0));
          } else {
            HIPCHK(launch_wide_rows(r, proc_ov && c > 0 ? rgrid_ov : rgrid, rs, proc_ov && c > 0));
          }
          HIPCHK(hipEventRecord(evch[(size_t)4 * c + 1], rs));
          if (proc_ov) HIPCHK(hipStreamWaitEvent(st, evch[(size_t)4 * c + 1], 0));
          HIPCHK(hipEventRecord(evch[(size_t)4 * c + 2], st));
          g.X = xs;
          g.w = dw + r.r_begin;
          g.wz = dwz + r.r_begin;
          for (int q = 0; q < 2 && !dev_only; ++q) {
            const int kind = proc_ov ? 1 - q : q;  // overlapped: the diagonal launch first
            if (has_sched[kind]) {
              g.pieces = dpieces[kind];
              g.wg_begin = dwgb[kind];
              HIPCHK(launch_wide_gram(g, kind == 1, ggk[kind], st));
            }
          }
          HIPCHK(hipEventRecord(evch[(size_t)4 * c + 3], st));
          HIPCHK(launch_wide_reduce(dgp, wstride, dstr, (int)p, r.row_partials, proc_ov && c > 0 ? rgrid_ov : rgrid,
                                    dchunks + (int64_t)c * plen, st));
        }
        HIPCHK(hipEventRecord(evm, st));  // unused in chunked timing (pass_timing sums evch)
        HIPCHK(hipEventRecord(ev1, st));
        HIPCHK(launch_sum_chunks(dchunks, nch, (int)p, dred, st));
        HIPCHK(hipEventRecord(ev2, st));
        return SGLM_OK;
      }
      if (nov > 0) {  // overlapped chunks: row kernels on st2, chunk c's Gram on st once its rows are done
        const int64_t plen = packed_len(p);
        auto rows_of = [&](int c, int64_t& r0, int64_t& r1) {
          r0 = (int64_t)c * ov_rows;
          r1 = std::min<int64_t>(n_pad, r0 + ov_rows);
        };
        HIPCHK(hipEventRecord(evov[(size_t)4 * nov], st));  // fork: beta uploaded, the last pass's Gram done
        HIPCHK(hipStreamWaitEvent(st2, evov[(size_t)4 * nov], 0));
        for (int c = 0; c < nov; ++c) {
          rows_of(c, r.r_begin, r.r_end);
          r.row_partials = rowpart(c);
          HIPCHK(hipEventRecord(evov[(size_t)4 * c], st2));
          HIPCHK(launch_wide_rows(r, c == 0 ? rgrid : rgrid_ov, st2, c > 0));
          HIPCHK(hipEventRecord(evov[(size_t)4 * c + 1], st2));
        }
        for (int c = 0; c < nov; ++c) {
          int64_t r0 = 0, r1 = 0;
          rows_of(c, r0, r1);
          HIPCHK(hipStreamWaitEvent(st, evov[(size_t)4 * c + 1], 0));
          HIPCHK(hipEventRecord(evov[(size_t)4 * c + 2], st));
          g.X = dX + r0;
          g.w = dw + r0;
          g.wz = dwz + r0;
          g.nb_lim = (r1 - r0) / WIDE_RB;
          for (int kind = 0; kind < 2 && !dev_only; ++kind) {
            if (!has_sched[kind]) continue;
            g.pieces = dpieces[kind];
            g.wg_begin = dwgb[kind];
            HIPCHK(launch_wide_gram(g, kind == 1, ggk[kind], st));
          }
          HIPCHK(hipEventRecord(evov[(size_t)4 * c + 3], st));
          HIPCHK(launch_wide_reduce(dgp, wstride, dstr, (int)p, rowpart(c), c == 0 ? rgrid : rgrid_ov,
                                    dchunks + (int64_t)c * plen, st));
        }
        HIPCHK(hipEventRecord(ev1, st));
        HIPCHK(launch_sum_chunks(dchunks, nov, (int)p, dred, st));
        HIPCHK(hipEventRecord(ev2, st));
        return SGLM_OK;
      }
      HIPCHK(launch_wide_rows(r, rgrid, st));
      HIPCHK(hipEventRecord(evm, st));
      for (int kind = 0; kind < 2 && !dev_only; ++kind) {
        if (!has_sched[kind]) continue;
        g.pieces = dpieces[kind];
        g.wg_begin = dwgb[kind];
        HIPCHK(launch_wide_gram(g, kind == 1, ggk[kind], st));
      }
      HIPCHK(hipEventRecord(ev1, st));
      HIPCHK(launch_wide_reduce(dgp, wstride, dstr, (int)p, drp, rgrid, dred, st));
    } else {
      // the pass kernel and the reduce record ev0 / ev1 / ev2 as part of their dispatches
      // (hipExtLaunchKernel): separate event records put a ~5 us marker between the kernels,
      // a tenth of an LM.fit on configs[0]
      hipEvent_t e0 = timed ? ev0 : nullptr, e1 = timed ? ev1 : nullptr, e2 = timed ? ev2 : nullptr;
      if (nblocks > 0) {
        if (narrow) HIPCHK(launch_narrow(P16, a, grid, st, e0, e1));
        else HIPCHK(launch_pass(P16, a, grid, st, e0, e1));
      } else {
        HIPCHK(hipEventRecord(ev0, st));
        HIPCHK(hipMemsetAsync(dpart, 0, sizeof(double) * stride, st));
        HIPCHK(hipEventRecord(ev1, st));
        e2 = ev2;
      }
      HIPCHK(launch_reduce(dpart, stride, nblocks > 0 ? grid : 1, (int)p, P16, dred, st, e2, a.lm_extras ? (int)p : 0));
      return SGLM_OK;
    }
    HIPCHK(hipEventRecord(ev2, st));
    return SGLM_OK;
  }

  // The kernel this shard's passes run (sglm_stats.pass_kernel / pass_kernel_name): the engine's
  // own dispatch decision -- narrow / fused / wide, and K1 against K1r by pass_uses_split with its
  // row limit -- so a roofline line is labelled by what ran, not by a re-derived threshold.
  void note_kernel(int family, int link) {
    last_kernel = pass_kernel_choice(n_pad, P16, narrow, wide, procx.on != 0, fused_split, family, link,
                                     last_kernel_name, sizeof last_kernel_name);
  }

  // ---- multi-device handle: every shard's pass enqueued, then one reduction ----
  // Distinct devices: ncclAllReduce of the packed buffers in one RCCL group call (xGMI), every
  // shard ends with the sum.  Repeated devices (rehearsal on fewer GPUs): host sums in shard
  // order.  Either way the wide-path device solver reads shard 0's buffers.
  // The scalars are summed in shard order with compensation either way (compensated_rank_sum).
  // comm_ms: RCCL -- the shortest span from a shard's pass end (ev2) to its all-reduce end (evc),
  // i.e. the collective after the last shard arrived; host sums -- the host time of the sum.
  int group_pass(int mode, const double* beta, double mu0, double ybar, int family, int link, double* packed) {
    const int64_t pp = subs[0]->p, plen = packed_len(pp), sc = tri_count(pp) + pp;
    const int D = (int)subs.size();
    const int64_t len = plen + (int64_t)NS * D;
    if (group_aborted) {
      set_error("the multi-device handle's RCCL group was aborted by an earlier failure; create a new handle");
      return SGLM_ECOMM;
    }
    for (sglm_engine* s : subs) {
      HIPCHK(hipSetDevice(s->device));
      if (int rc = s->ensure_red_len(len)) return rc;
    }
    for (sglm_engine* s : subs)
      if (int rc = s->enqueue_pass(mode, beta, mu0, ybar, family, link)) return rc;
    if (!gcomms.empty()) {
      for (int d = 0; d < D; ++d) {
        HIPCHK(hipSetDevice(subs[d]->device));
        if (int rc = subs[d]->stage_rank_block(d, D)) return rc;
      }
      ncclResult_t r = ncclGroupStart();
      for (int d = 0; d < D && r == ncclSuccess; ++d)
        r = ncclAllReduce(subs[d]->dred, subs[d]->dred, (size_t)len, ncclFloat64, ncclSum, gcomms[d], subs[d]->st);
      ncclResult_t r2 = ncclGroupEnd();
      if (r != ncclSuccess || r2 != ncclSuccess) {
        set_error(std::string("RCCL ncclAllReduce (group): ") + ncclGetErrorString(r != ncclSuccess ? r : r2));
        return SGLM_ECOMM;
      }
      for (sglm_engine* s : subs) {
        HIPCHK(hipSetDevice(s->device));
        HIPCHK(hipEventRecord(s->evc, s->st));
      }
      sglm_engine* s0 = subs[0];
      HIPCHK(hipSetDevice(s0->device));
      HIPCHK(hipMemcpyAsync(s0->hred, s0->dred, sizeof(double) * len, hipMemcpyDeviceToHost, s0->st));
      {  // every shard's stream drains, or the group is aborted at the deadline (wait_collective)
        std::vector<hipStream_t> sts;
        std::vector<ncclComm_t*> cs;
        std::vector<hipEvent_t> evs;  // every shard's pass done: the deadline starts there
        for (int d = 0; d < D; ++d) {
          sts.push_back(subs[d]->st);
          cs.push_back(&gcomms[d]);
          evs.push_back(subs[d]->ev2);
        }
        if (int rc = wait_collective(sts, cs, comm.timeout_ms, -1, "the multi-device ncclAllReduce group", evs)) {
          group_aborted = true;  // the handle's communicators are gone: every later pass fails
          return rc;
        }
      }
      double cms = -1.0;
      for (sglm_engine* s : subs) {
        HIPCHK(hipSetDevice(s->device));
        if (int rc = s->pass_timing()) return rc;
        float ms = 0.f;
        HIPCHK(hipEventElapsedTime(&ms, s->ev2, s->evc));
        cms = cms < 0.0 ? ms : std::min(cms, (double)ms);
      }
      comm.ms += std::max(cms, 0.0);
      compensated_rank_sum(s0->hred + plen, D, NS, s0->hred + sc);
      std::memcpy(packed, s0->hred, sizeof(double) * plen);
      s0->red_on_device = true;
    } else {
      for (sglm_engine* s : subs) {
        HIPCHK(hipSetDevice(s->device));
        HIPCHK(hipMemcpyAsync(s->hred, s->dred, sizeof(double) * plen, hipMemcpyDeviceToHost, s->st));
      }
      for (sglm_engine* s : subs) {
        HIPCHK(hipSetDevice(s->device));
        HIPCHK(hipStreamSynchronize(s->st));
        if (int rc = s->pass_timing()) return rc;
      }
      const double t0 = now_ms();
      std::memcpy(packed, subs[0]->hred, sizeof(double) * sc);
      for (int d = 1; d < D; ++d)
        for (int64_t k = 0; k < sc; ++k) packed[k] += subs[(size_t)d]->hred[k];
      std::vector<double> blocks((size_t)(NS * D));
      for (int d = 0; d < D; ++d) std::memcpy(blocks.data() + (int64_t)d * NS, subs[(size_t)d]->hred + sc, sizeof(double) * NS);
      compensated_rank_sum(blocks.data(), D, NS, packed + sc);
      subs[0]->red_on_device = false;
      comm.ms += now_ms() - t0;
    }
    finish_scalars(mode, family, packed + sc);
    return SGLM_OK;
  }

  // blocks (= partials) of the statistics pass; the LM device round trip and the host path alike
  // (LM 1M x 20: 2048 blocks measured equal, 4096 +5 %: profiles/r04_lm_stats_blocks.txt)
  static int stats_blocks(int64_t rows) {
    return (int)std::min<int64_t>(4096, std::max<int64_t>(1024, rows / 131072));
  }

  // LM.fit in one round trip (driver.hpp Backend::lm_device): a resident narrow shard with no
  // communicator -- the Gram pass, which also sums X'1 and y'y (narrow LMX), then lm_chol_kernel:
  // the host Cholesky, bitwise, on the device, and the residual statistics of LM.scala:160-188 from
  // those sums (SSE = y'y - 2 b'X'y + b'X'X b, ...; kernels.hip lm_chol_kernel), written with the
  // whole result to pinned host memory -- ONE pass over X and one synchronisation.  Where the sums
  // cancel too far (LM_ONEPASS_MAX_RATIO) the statistics come back flagged (S_BAD) and lm_drive runs
  // the residual pass, the reference's own form; so does a device Cholesky that is not the host's.
  // configs[0] (1M x 20) is launch- and latency-bound: round 5 removed the host round trip between
  // the two passes, round 6 the second pass.
  int lm_device(double* packed, double* dev_coefs, double* s, bool& done) override {
    done = false;
    if (!allow_lm_device || group() || comm.kind != 0 || wide || procx.on || !narrow || p > 64 || nblocks <= 0)
      return SGLM_OK;
    HIPCHK(hipSetDevice(device));
    // one device buffer, copied back in one piece: packed Gram | X'1 [p] | statistics [NS] | coefs [p]
    const int64_t plen = packed_len(p);
    if (int rc = ensure_red_len(plen + p + NS + p)) return rc;
    if (int rc = ensure_small(64)) return rc;
    // a kernel that carries a completion event ends ~4.5 us later than one that does not (its
    // end-of-kernel signal; measured on the configs[0] timeline): LM fits time their Gram pass on
    // every 16th fit and count that time for the others (pass_untimed)
    const bool timed = (lm_device_fits % 16) == 0 || lm_last_pass_ms < 0.0;
    lm_extras_pass = true;
    const int prc = enqueue_pass(MODE_LM_GRAM, nullptr, 0.0, 0.0, FAM_GAUSSIAN, LNK_IDENTITY, timed);
    lm_extras_pass = false;
    if (prc) return prc;
    double* aux = dsmall + NS;  // {ybar, leave-Cholesky flag}
    double* dstat = dred + plen + p;
    double* dcoef = dred + plen + p + NS;
    double* hred_dev = nullptr;  // the pinned result buffer as the device sees it (no copy blit)
    HIPCHK(hipHostGetDevicePointer((void**)&hred_dev, hred, 0));
    LmOnePass op;
    op.x1 = dred + plen;
    op.stats = dstat;
    op.host = hred_dev;
    op.ncopy = plen + p;
    HIPCHK(launch_lm_chol(dred, (int)p, LU_SWITCH_RATIO, dcoef, aux, st, op));
    HIPCHK(hipStreamSynchronize(st));  // (a spin on hipStreamQuery measured slower: 0.124 against 0.115 ms)
    if (timed) {
      if (int rc = pass_timing()) return rc;
      lm_last_pass_ms = last_pass_ms;
      lm_last_reduce_ms = last_reduce_ms;
    } else {
      pass_untimed();
    }
    red_on_device = true;
    std::memcpy(packed, hred, sizeof(double) * plen);
    std::memcpy(s, hred + plen + p, sizeof(double) * NS);
    std::memcpy(dev_coefs, hred + plen + p + NS, sizeof(double) * p);
    done = true;
    lm_device_fits += 1;
    lm_onepass_fits += s[S_BAD] == 0.0 ? 1 : 0;
    return SGLM_OK;
  }

  std::unique_ptr<SolverIface> make_solver(int64_t pp) override;
  int blas_handle() {
    if (!blas) {
      if (rocblas_create_handle(&blas) != rocblas_status_success) {
        blas = nullptr;
        set_error("rocblas_create_handle failed");
        return SGLM_EHIP;
      }
    }
    if (rocblas_set_stream(blas, st) != rocblas_status_success) {
      set_error("rocblas_set_stream failed");
      return SGLM_EHIP;
    }
    return SGLM_OK;
  }

  int stats(int mode, const double* beta, double mu0, double ybar, int family, int link, double* s) override {
    if (group()) {  // shard order, compensated (compensated_rank_sum)
      std::vector<double> blocks((size_t)NS * subs.size());
      for (size_t d = 0; d < subs.size(); ++d)
        if (int rc = subs[d]->stats(mode, beta, mu0, ybar, family, link, blocks.data() + NS * d)) return rc;
      compensated_rank_sum(blocks.data(), (int)subs.size(), NS, s);
      return SGLM_OK;
    }
    HIPCHK(hipSetDevice(device));
    StatsArgs a{};
    // LM residuals of a narrow resident design: beta rides in the kernel arguments (no H2D copy on
    // the fit's critical path, configs[0] is launch- and latency-bound)
    const bool by_value = mode == MODE_LM_RESID && !procx.on && p <= STATS_BETA_MAX;
    if (mode == MODE_LM_RESID && !by_value) {  // pred = X * coefs into the eta buffer
      std::memcpy(hbeta, beta, sizeof(double) * p);
      HIPCHK(hipMemcpyAsync(dbeta, hbeta, sizeof(double) * p, hipMemcpyHostToDevice, st));
      if (procx.on) HIPCHK(launch_predict(dX, n_pad, (int)p, n, dbeta, nullptr, deta, st, procx));
    }
    if (mode == MODE_LM_RESID && !procx.on) {  // one read of X, no eta round trip
      a.X = dX;
      a.ld = n_pad;
      a.p = (int)p;
      a.beta = dbeta;
      a.beta_by_value = by_value ? 1 : 0;
      if (by_value) std::memcpy(a.bv, beta, sizeof(double) * p);
    }
    a.y = dy;
    a.m = (mode == MODE_LM_RESID) ? nullptr : dm;
    a.prior = (mode == MODE_LM_RESID) ? nullptr : dprior;
    a.eta = deta;
    a.n = n;
    a.family = family;
    a.link = link;
    a.mode = mode;
    a.mu0 = mu0;
    a.ybar = ybar;
    a.partials = dpart;
    // one wave per SIMD leaves the per-row chain latency-bound on large shards; small ones
    // (LM 1M x 20) keep 1024 partials; they are summed on the device (reduce_stats_kernel,
    // compensated) and only the NS sums come back
    const int nb = stats_blocks(n);
    HIPCHK(launch_stats(a, nb, st));
    if (int rc = ensure_small(64)) return rc;
    HIPCHK(launch_reduce_stats(dpart, nb, dsmall, st));
    HIPCHK(hipMemcpyAsync(hsmall, dsmall, sizeof(double) * NS, hipMemcpyDeviceToHost, st));
    HIPCHK(hipStreamSynchronize(st));
    std::memcpy(s, hsmall, sizeof(double) * NS);
    return allreduce_small(s, NS);
  }
};

// =====================================================================================
// Device solver for wide p, from the reduced buffer on the GPU.
// Default: Cholesky (rocSOLVER potrf / potrs, potri for the standard errors).  A matrix potrf
// rejects or whose pivots flag it ill-conditioned (solve.hpp LU_SWITCH_RATIO) takes the
// reference's own algorithm, LU with partial pivoting and the explicit inverse (Breeze inv =
// LAPACK dgetrf + dgetri, utils.scala:103-105, 134-136): on the host -- the oracle's unblocked
// order, as the narrow path -- up to p = HOST_LU_MAX_P, by rocSOLVER getrf / getri above it (a
// host LU at p = 2048 is ~10 s).  SGLM_WIDE_SOLVE=lu runs the rocSOLVER LU route always, coefs =
// inv * X'Wz summed in the reference's order (inv_gemv_kernel), stdErr from diag(inv).
// Measured against the oracle's unblocked LU (tests/test_gpu_wide.py, oracle/lu_floor.py):
// Cholesky lands closer than rocSOLVER's blocked getrf + getri on ill-conditioned gamma designs
// (p = 520, cond ~1e7: 1e-9 against 1e-7 elementwise on the smallest coefficient), which is why
// it stays the default; norm-wise both agree to ~1e-12.  Exact singularity (a zero pivot of
// dgetrf) -> MatrixSingularException, as Breeze's inv.
// =====================================================================================
namespace {

constexpr int64_t HOST_LU_MAX_P = 1024;

struct DeviceSolver : public SolverIface {
  sglm_engine* e;
  int64_t p;
  double *dA = nullptr, *dB = nullptr, *dAi = nullptr, *dpk = nullptr, *dx = nullptr;
  rocblas_int *dinfo = nullptr, *dipiv = nullptr;
  std::vector<double> ldiag;
  std::unique_ptr<HostSolver> host;
  int kind = 0;  // 0 none, 1 Cholesky factor in dA, 2 explicit inverse in dA (LU route), 3 host solver
  DeviceSolver(sglm_engine* eng, int64_t pp) : e(eng), p(pp) {}
  int path() const override {
    return kind == 1 ? SGLM_SOLVE_DEVICE_CHOL : kind == 2 ? SGLM_SOLVE_DEVICE_LU : kind == 3 ? host->path() : -1;
  }
  ~DeviceSolver() override {
    (void)hipSetDevice(e->device);
    for (double* ptr : {dA, dB, dAi, dpk, dx})
      if (ptr) (void)hipFree(ptr);
    if (dinfo) (void)hipFree(dinfo);
    if (dipiv) (void)hipFree(dipiv);
  }
  int alloc() {
    if (dA) return SGLM_OK;
    HIPCHK(hipMalloc(&dA, sizeof(double) * (size_t)(p * p)));
    HIPCHK(hipMalloc(&dAi, sizeof(double) * (size_t)(p * p)));
    HIPCHK(hipMalloc(&dB, sizeof(double) * (size_t)p));
    HIPCHK(hipMalloc(&dx, sizeof(double) * (size_t)p));
    HIPCHK(hipMalloc(&dinfo, sizeof(rocblas_int)));
    HIPCHK(hipMalloc(&dipiv, sizeof(rocblas_int) * (size_t)p));
    return SGLM_OK;
  }
  int read_info(rocblas_int* info) {
    HIPCHK(hipMemcpyAsync(info, dinfo, sizeof *info, hipMemcpyDeviceToHost, e->st));
    HIPCHK(hipStreamSynchronize(e->st));
    return SGLM_OK;
  }
  int solve(const double* packed, double* x) override {
    HIPCHK(hipSetDevice(e->device));
    int rc = alloc();
    if (!rc) rc = e->blas_handle();
    if (rc) return rc;
    const double* src = e->dred;
    if (!e->red_on_device) {  // the reduction ended on the host: upload it
      if (!dpk) HIPCHK(hipMalloc(&dpk, sizeof(double) * (size_t)packed_len(p)));
      HIPCHK(hipMemcpyAsync(dpk, packed, sizeof(double) * (size_t)packed_len(p), hipMemcpyHostToDevice, e->st));
      src = dpk;
    }
    kind = 0;
    if (e->wide_lu) return solve_lu(src, x);
    HIPCHK(launch_unpack_lower(src, (int)p, dA, dB, e->st));
    if (rocsolver_dpotrf(e->blas, rocblas_fill_lower, (rocblas_int)p, dA, (rocblas_int)p, dinfo) !=
        rocblas_status_success) {
      set_error("rocsolver_dpotrf failed");
      return SGLM_EHIP;
    }
    rocblas_int info = 0;
    HIPCHK(hipMemcpyAsync(&info, dinfo, sizeof info, hipMemcpyDeviceToHost, e->st));
    if (info == 0) {  // diag(L) for the collinearity check (solve.hpp chol_pivot_ratio)
      ldiag.resize((size_t)p);
      HIPCHK(hipMemcpy2DAsync(ldiag.data(), sizeof(double), dA, sizeof(double) * (size_t)(p + 1), sizeof(double),
                              (size_t)p, hipMemcpyDeviceToHost, e->st));
    }
    HIPCHK(hipStreamSynchronize(e->st));
    if (info == 0) {
      double r = 1.0;
      for (int64_t j = 0; j < p; ++j) {
        const double a = packed[j * (j + 1) / 2 + j];
        if (a > 0.0) r = std::fmin(r, ldiag[(size_t)j] * ldiag[(size_t)j] / a);
      }
      if (r < LU_SWITCH_RATIO) info = -1;  // ill-conditioned: the reference's LU inverse
    }
    if (info != 0) {  // not positive definite / ill-conditioned: the reference's LU inverse
      if (p > HOST_LU_MAX_P) return solve_lu(src, x);
      if (!host) host = std::make_unique<HostSolver>(p);
      kind = 3;
      return host->solve(packed, x);
    }
    if (rocsolver_dpotrs(e->blas, rocblas_fill_lower, (rocblas_int)p, 1, dA, (rocblas_int)p, dB, (rocblas_int)p) !=
        rocblas_status_success) {
      set_error("rocsolver_dpotrs failed");
      return SGLM_EHIP;
    }
    HIPCHK(hipMemcpyAsync(x, dB, sizeof(double) * (size_t)p, hipMemcpyDeviceToHost, e->st));
    HIPCHK(hipStreamSynchronize(e->st));
    kind = 1;
    return SGLM_OK;
  }
  // inv(A) by dgetrf + dgetri in dA, x = inv(A) b (utils.scala:103-104)
  int solve_lu(const double* src, double* x) {
    HIPCHK(launch_unpack_lower(src, (int)p, dA, dB, e->st, true));
    if (rocsolver_dgetrf(e->blas, (rocblas_int)p, (rocblas_int)p, dA, (rocblas_int)p, dipiv, dinfo) !=
        rocblas_status_success) {
      set_error("rocsolver_dgetrf failed");
      return SGLM_EHIP;
    }
    rocblas_int info = 0;
    if (int rc = read_info(&info)) return rc;
    if (info != 0) {
      set_error("breeze.linalg.MatrixSingularException: X'WX is singular");
      return SGLM_ESINGULAR;
    }
    if (rocsolver_dgetri(e->blas, (rocblas_int)p, dA, (rocblas_int)p, dipiv, dinfo) != rocblas_status_success) {
      set_error("rocsolver_dgetri failed");
      return SGLM_EHIP;
    }
    HIPCHK(launch_inv_gemv(dA, (int)p, dB, dx, e->st));
    HIPCHK(hipMemcpyAsync(x, dx, sizeof(double) * (size_t)p, hipMemcpyDeviceToHost, e->st));
    if (int rc = read_info(&info)) return rc;
    if (info != 0) {
      set_error("breeze.linalg.MatrixSingularException: X'WX is singular");
      return SGLM_ESINGULAR;
    }
    kind = 2;
    return SGLM_OK;
  }
  // inv(A) (lower triangle) into dAi from the kept Cholesky factor
  int device_inverse() {
    HIPCHK(hipMemcpyAsync(dAi, dA, sizeof(double) * (size_t)(p * p), hipMemcpyDeviceToDevice, e->st));
    if (rocsolver_dpotri(e->blas, rocblas_fill_lower, (rocblas_int)p, dAi, (rocblas_int)p, dinfo) !=
        rocblas_status_success) {
      set_error("rocsolver_dpotri failed");
      return SGLM_EHIP;
    }
    return SGLM_OK;
  }
  int inv_diag(double* d) override {
    if (kind == 3) return host->inv_diag(d);
    if (kind == 0) {
      for (int64_t i = 0; i < p; ++i) d[i] = 0.0;
      return SGLM_OK;
    }
    HIPCHK(hipSetDevice(e->device));
    if (kind == 1)
      if (int rc = device_inverse()) return rc;
    HIPCHK(hipMemcpy2DAsync(d, sizeof(double), kind == 1 ? dAi : dA, sizeof(double) * (size_t)(p + 1), sizeof(double),
                            (size_t)p, hipMemcpyDeviceToHost, e->st));
    HIPCHK(hipStreamSynchronize(e->st));
    return SGLM_OK;
  }
  int inverse(double* Ainv) override {
    if (kind == 3) return host->inverse(Ainv);
    if (kind == 0) return SGLM_OK;
    HIPCHK(hipSetDevice(e->device));
    if (kind == 1)
      if (int rc = device_inverse()) return rc;
    HIPCHK(hipMemcpyAsync(Ainv, kind == 1 ? dAi : dA, sizeof(double) * (size_t)(p * p), hipMemcpyDeviceToHost, e->st));
    HIPCHK(hipStreamSynchronize(e->st));
    if (kind == 1)
      for (int64_t j = 0; j < p; ++j)
        for (int64_t i = 0; i < j; ++i) Ainv[i + j * p] = Ainv[j + i * p];
    return SGLM_OK;
  }
};

}  // namespace

std::unique_ptr<SolverIface> sglm_engine::make_solver(int64_t pp) {
  if (group()) return subs[0]->make_solver(pp);
  if (wide) return std::make_unique<DeviceSolver>(this, pp);
  return std::make_unique<HostSolver>(pp);
}

// =====================================================================================
// External backend adapter (caller-computed partials)
// =====================================================================================
namespace {

struct ExternalBackend : public Backend {
  const sglm_backend* be;
  sglm_allreduce_fn fn;
  void* ctx;
  int nranks = 1;
  int rank = -1;  // known for the in-process communicator: scalars then summed in rank blocks
  double timeout_ms = comm_timeout_ms_env();
  CallbackRunner runner;  // the callback on a communicator thread, waited for with the deadline
  ExternalBackend(const sglm_backend* b, sglm_allreduce_fn f, void* c) : be(b), fn(f), ctx(c), rank(known_rank(f, c)) {}
  int64_t ncols() const override { return be->p; }
  int npart() const override { return nranks; }
  int reduce_raw(double* buf, int64_t count) {
    return fn ? runner.call(fn, ctx, buf, count, nullptr, 0, timeout_ms, rank) : SGLM_OK;
  }
  // buf[0, count): the last nsc entries are scalar sums -- through rank blocks when the rank is known
  int reduce(double* buf, int64_t count, int64_t nsc) {
    if (!(fn && rank >= 0 && rank < nranks && nranks > 1)) return reduce_raw(buf, count);
    std::vector<double> b((size_t)(count + nsc * nranks), 0.0);
    std::memcpy(b.data(), buf, sizeof(double) * count);
    std::memcpy(b.data() + count + (int64_t)rank * nsc, buf + count - nsc, sizeof(double) * nsc);
    if (int rc = reduce_raw(b.data(), (int64_t)b.size())) return rc;
    std::memcpy(buf, b.data(), sizeof(double) * (count - nsc));
    compensated_rank_sum(b.data() + count, nranks, nsc, buf + count - nsc);
    return SGLM_OK;
  }
  int global_sums(double* out2) override {
    if (be->local_sums(be->ctx, out2) != 0) {
      set_error("external backend local_sums failed");
      return SGLM_EINVAL;
    }
    double one[1] = {1.0};
    int rc = reduce_raw(one, 1);  // counts the ranks joined by the communicator
    if (rc) return rc;
    nranks = (int)std::lround(one[0]);
    return reduce(out2, 2, 2);
  }
  int pass(int mode, const double* beta, double mu0, double ybar, int family, int link, double* packed) override {
    (void)family;
    (void)link;
    if (be->pass(be->ctx, mode, beta, mu0, ybar, packed) != 0) {
      set_error("external backend pass failed");
      return SGLM_EINVAL;
    }
    return reduce(packed, packed_len(be->p), NS);
  }
  int stats(int mode, const double* beta, double mu0, double ybar, int family, int link, double* s) override {
    std::vector<double> packed((size_t)packed_len(be->p));
    int rc = pass(mode, beta, mu0, ybar, family, link, packed.data());
    if (rc) return rc;
    std::memcpy(s, packed.data() + tri_count(be->p) + be->p, sizeof(double) * NS);
    return SGLM_OK;
  }
};

int check_handle(sglm_engine* h) {
  if (!h) {
    set_error("requirement failed: null engine handle");
    return SGLM_EINVAL;
  }
  return SGLM_OK;
}

}  // namespace

// =====================================================================================
// C ABI
// =====================================================================================
extern "C" {

int sglm_abi_version(void) { return SGLM_ABI_VERSION; }
const char* sglm_last_error(void) { return get_error(); }

int sglm_device_count(int* count) {
  int c = 0;
  hipError_t e = hipGetDeviceCount(&c);
  if (e != hipSuccess) {
    *count = 0;
    set_error(hip_msg(e, "hipGetDeviceCount"));
    return SGLM_EHIP;
  }
  *count = c;
  return SGLM_OK;
}

int sglm_create_device(int device, sglm_engine** out) {
  if (!out) {
    set_error("requirement failed: out handle pointer");
    return SGLM_EINVAL;
  }
  *out = nullptr;
  int count = 0;
  hipError_t e = hipGetDeviceCount(&count);
  if (e != hipSuccess || count <= 0) {
    set_error(e != hipSuccess ? hip_msg(e, "hipGetDeviceCount") : std::string("no HIP device visible"));
    return SGLM_EHIP;
  }
  if (device < 0 || device >= count) {
    set_error("requirement failed: device ordinal out of range");
    return SGLM_EINVAL;
  }
  auto* h = new sglm_engine();
  h->device = device;
  auto fail = [&](hipError_t err, const char* what) {
    set_error(hip_msg(err, what));
    delete h;
    return SGLM_EHIP;
  };
  if ((e = hipSetDevice(device)) != hipSuccess) return fail(e, "hipSetDevice");
  if ((e = hipStreamCreateWithFlags(&h->st, hipStreamNonBlocking)) != hipSuccess) return fail(e, "hipStreamCreate");
  if ((e = hipEventCreate(&h->ev0)) != hipSuccess) return fail(e, "hipEventCreate");
  if ((e = hipEventCreate(&h->ev1)) != hipSuccess) return fail(e, "hipEventCreate");
  if ((e = hipEventCreate(&h->ev2)) != hipSuccess) return fail(e, "hipEventCreate");
  if ((e = hipEventCreate(&h->evc)) != hipSuccess) return fail(e, "hipEventCreate");
  hipDeviceProp_t prop;
  if ((e = hipGetDeviceProperties(&prop, device)) != hipSuccess) return fail(e, "hipGetDeviceProperties");
  h->ncu = prop.multiProcessorCount > 0 ? prop.multiProcessorCount : 256;
  if (const char* fw = std::getenv("SGLM_FORCE_WIDE")) h->force_wide = std::atoi(fw) != 0;
  if (const char* pc = std::getenv("SGLM_PROC_CHUNKS")) h->allow_chunks = std::atoi(pc) != 0;
  if (const char* po = std::getenv("SGLM_PROC_OVERLAP")) h->proc_ov_want = std::atoi(po);
  if (const char* pm = std::getenv("SGLM_PROC_OV_MIN")) h->proc_ov_min = std::max<int64_t>(32, std::atoll(pm));
  if (const char* ov = std::getenv("SGLM_WIDE_OVERLAP")) h->ov_want = std::atoi(ov);
  if (const char* om = std::getenv("SGLM_WIDE_OV_MIN")) h->ov_min = std::max<int64_t>(32, std::atoll(om));
  if (const char* sp = std::getenv("SGLM_SPECULATE")) h->allow_spec = std::atoi(sp) != 0;
  if (const char* ld = std::getenv("SGLM_LM_DEVICE")) h->allow_lm_device = std::atoi(ld) != 0;
  if (const char* fs = std::getenv("SGLM_FUSED_SPLIT")) h->fused_split = std::max(0, std::atoi(fs));
  if (const char* ws = std::getenv("SGLM_WIDE_SOLVE")) h->wide_lu = std::strcmp(ws, "lu") == 0;
  if (const char* pm = std::getenv("SGLM_PROC_SCRATCH_MAX")) h->proc_scratch_max = std::max<int64_t>(0, std::atoll(pm));
  *out = h;
  return SGLM_OK;
}

void sglm_destroy(sglm_engine* h) { delete h; }

// SURVEY 8(b)'s constructor: one handle over devs[0..ndev).  One device: the single-device handle
// (sglm_create_device); several: the group handle (sglm_create_multi).
int sglm_create(const int* devs, int ndev, sglm_engine** out) {
  if (!out || !devs || ndev < 1) {
    set_error("requirement failed: devs[ndev], ndev >= 1, out handle pointer");
    return SGLM_EINVAL;
  }
  *out = nullptr;
  return ndev == 1 ? sglm_create_device(devs[0], out) : sglm_create_multi(devs, ndev, out);
}

// The group handle: one shard engine per listed device, one RCCL communicator per device from
// ncclCommInitAll when they are distinct -- for one device too (a one-device group runs the RCCL
// group all-reduce path: the tests' way to execute it on a one-GPU box).
int sglm_create_multi(const int* devs, int ndev, sglm_engine** out) {
  if (!out || !devs || ndev < 1) {
    set_error("requirement failed: devs[ndev], ndev >= 1, out handle pointer");
    return SGLM_EINVAL;
  }
  *out = nullptr;
  auto* g = new sglm_engine();
  g->device = devs[0];
  for (int d = 0; d < ndev; ++d) {
    sglm_engine* s = nullptr;
    int rc = sglm_create_device(devs[d], &s);
    if (rc) {
      delete g;
      return rc;
    }
    g->subs.push_back(s);
  }
  g->allow_spec = g->subs[0]->allow_spec;  // the group handle drives the fit (SGLM_SPECULATE)
  bool distinct = true;
  for (int a = 0; a < ndev; ++a)
    for (int b = 0; b < a; ++b) distinct = distinct && devs[a] != devs[b];
  g->comm.timeout_ms = comm_timeout_ms_env();  // the group all-reduce's deadline (wait_collective)
  if (distinct) {  // one communicator per device, one process (ncclCommInitAll)
    g->gcomms.assign((size_t)ndev, nullptr);
    ncclResult_t r = ncclCommInitAll(g->gcomms.data(), ndev, devs);
    if (r != ncclSuccess) {
      g->gcomms.clear();
      set_error(std::string("ncclCommInitAll: ") + ncclGetErrorString(r));
      delete g;
      return SGLM_ECOMM;
    }
  }
  *out = g;
  return SGLM_OK;
}

int sglm_handle_devices(sglm_engine* h, int* ndev) {
  if (int rc = check_handle(h)) return rc;
  *ndev = h->group() ? (int)h->subs.size() : 1;
  return SGLM_OK;
}

// Row ranges of a multi-device handle's shards: Spark's slicing [d n / D, (d+1) n / D).
static void group_split(sglm_engine* h, int64_t n) {
  const int64_t D = (int64_t)h->subs.size();
  h->sub_lo.assign((size_t)D + 1, 0);
  for (int64_t d = 0; d <= D; ++d) h->sub_lo[(size_t)d] = (int64_t)((__int128)d * n / D);
  h->g_n = n;
}

static int reserve_impl(sglm_engine* h, int64_t n, int64_t p, int has_m, int has_off, int has_prior) {
  h->consts_family = -1;
  if (n <= 0 || p <= 0) {
    set_error("requirement failed: n >= 1, p >= 1");
    return SGLM_EINVAL;
  }
  if (h->group()) {
    if (n < (int64_t)h->subs.size()) {
      set_error("requirement failed: at least one row per device");
      return SGLM_EINVAL;
    }
    group_split(h, n);
    for (size_t d = 0; d < h->subs.size(); ++d)
      if (int rc = reserve_impl(h->subs[d], h->sub_lo[d + 1] - h->sub_lo[d], p, has_m, has_off, has_prior)) return rc;
    return SGLM_OK;
  }
  return h->alloc_data(n, p, has_m != 0, has_off != 0, has_prior != 0);
}

int sglm_reserve(sglm_engine* h, int64_t n, int64_t p, int has_m, int has_offset, int has_prior) {
  if (int rc = check_handle(h)) return rc;
  return reserve_impl(h, n, p, has_m, has_offset, has_prior);
}

static int set_rows_impl(sglm_engine* h, int64_t row0, int64_t nr, const double* X, int64_t ldx, const double* y,
                         const double* m, const double* off, const double* prior) {
  h->consts_family = -1;
  if (!h->group()) return h->set_rows(row0, nr, X, ldx, y, m, off, prior);
  if (h->g_n <= 0 || row0 < 0 || nr < 0 || row0 + nr > h->g_n) {
    set_error("requirement failed: sglm_reserve first; 0 <= row0, row0 + nrows <= reserved rows");
    return SGLM_EINVAL;
  }
  for (size_t d = 0; d < h->subs.size(); ++d) {  // the block's intersection with each shard
    const int64_t a = std::max(row0, h->sub_lo[d]), b = std::min(row0 + nr, h->sub_lo[d + 1]);
    if (a >= b) continue;
    const int64_t o = a - row0;
    auto sh = [&](const double* v) { return v ? v + o : nullptr; };
    if (int rc = h->subs[d]->set_rows(a - h->sub_lo[d], b - a, X + o, ldx, sh(y), sh(m), sh(off), sh(prior)))
      return rc;
  }
  return SGLM_OK;
}

int sglm_set_rows(sglm_engine* h, int64_t row0, int64_t nrows, const double* X, int64_t ldx, const double* y,
                  const double* m, const double* offset, const double* prior) {
  if (int rc = check_handle(h)) return rc;
  return set_rows_impl(h, row0, nrows, X, ldx, y, m, offset, prior);
}

int sglm_set_data(sglm_engine* h, const double* X, int64_t n, int64_t p, int64_t ldx, const double* y,
                  const double* m, const double* offset, const double* prior) {
  if (int rc = check_handle(h)) return rc;
  if (!X || !y || ldx < n || n <= 0 || p <= 0) {
    set_error("requirement failed: X, y non-null, n >= 1, p >= 1, ldx >= n");
    return SGLM_EINVAL;
  }
  int rc = reserve_impl(h, n, p, m != nullptr, offset != nullptr, prior != nullptr);
  if (rc) return rc;
  return set_rows_impl(h, 0, n, X, ldx, y, m, offset, prior);
}

int sglm_set_data_device(sglm_engine* h, const double* dX, int64_t n, int64_t p, int64_t ldx, const double* dy,
                         const double* dm, const double* doffset, const double* dprior) {
  if (int rc = check_handle(h)) return rc;
  if (h->group()) {
    set_error("requirement failed: sglm_set_data_device takes one device's memory; use a single-device handle");
    return SGLM_EINVAL;
  }
  if (!dX || !dy || ldx < n || n <= 0 || p <= 0) {
    set_error("requirement failed: X, y non-null, n >= 1, p >= 1, ldx >= n");
    return SGLM_EINVAL;
  }
  int rc = h->alloc_data(n, p, dm != nullptr, doffset != nullptr, dprior != nullptr);
  if (rc) return rc;
  const size_t vb = sizeof(double) * (size_t)n;
  const hipMemcpyKind kind = hipMemcpyDeviceToDevice;
  HIPCHK(hipMemcpy2DAsync(h->dX, sizeof(double) * h->n_pad, dX, sizeof(double) * ldx, vb, (size_t)p, kind, h->st));
  HIPCHK(hipMemcpyAsync(h->dy, dy, vb, kind, h->st));
  if (dm) HIPCHK(hipMemcpyAsync(h->dm, dm, vb, kind, h->st));
  if (doffset) HIPCHK(hipMemcpyAsync(h->doff, doffset, vb, kind, h->st));
  if (dprior) HIPCHK(hipMemcpyAsync(h->dprior, dprior, vb, kind, h->st));
  HIPCHK(hipStreamSynchronize(h->st));
  h->rows_loaded = n;
  h->written.assign(1, std::make_pair((int64_t)0, n));
  return SGLM_OK;
}

static int synth_impl(sglm_engine* h, int kind, int64_t row0, int64_t n, int64_t p, uint64_t seed, bool proc) {
  h->consts_family = -1;
  if (kind < 0 || kind > 3 || n <= 0 || p <= 0 || row0 < 0) {
    set_error("requirement failed: synth kind in {0,1,2,3}, n >= 1, p >= 1");
    return SGLM_EINVAL;
  }
  if (h->group()) {
    if (n < (int64_t)h->subs.size()) {
      set_error("requirement failed: at least one row per device");
      return SGLM_EINVAL;
    }
    group_split(h, n);
    for (size_t d = 0; d < h->subs.size(); ++d)
      if (int rc = synth_impl(h->subs[d], kind, row0 + h->sub_lo[d], h->sub_lo[d + 1] - h->sub_lo[d], p, seed, proc))
        return rc;
    return SGLM_OK;
  }
  int rc = h->alloc_data(n, p, false, kind == 2, kind == 2, proc);
  if (rc) return rc;
  const double scale = 1.0 / std::sqrt((double)p);
  // procedural: y (and offset / prior) from the same generator; X itself is not stored
  HIPCHK(launch_synth(kind, row0, n, (int)p, seed, scale, proc ? nullptr : h->dX, h->n_pad, h->dy, nullptr, h->doff,
                      h->dprior, h->st));
  HIPCHK(hipStreamSynchronize(h->st));
  h->rows_loaded = n;
  h->written.assign(1, std::make_pair((int64_t)0, n));
  if (proc) {
    h->procx.on = 1;
    h->procx.kind = kind;
    h->procx.p = (int)p;
    h->procx.row0 = row0;
    h->procx.n = n;
    h->procx.kx = splitmix64_host(seed);
    h->procx.scale = scale;
    if (int rc2 = h->setup_proc_chunks()) return rc2;
  }
  return SGLM_OK;
}

int sglm_synth(sglm_engine* h, int kind, int64_t row0, int64_t n, int64_t p, uint64_t seed) {
  if (int rc = check_handle(h)) return rc;
  return synth_impl(h, kind, row0, n, p, seed, false);
}

int sglm_synth_procedural(sglm_engine* h, int kind, int64_t row0, int64_t n, int64_t p, uint64_t seed) {
  if (int rc = check_handle(h)) return rc;
  return synth_impl(h, kind, row0, n, p, seed, true);
}

static int get_data_impl(sglm_engine* h, double* X, int64_t ldx, double* y, double* m, double* offset,
                         double* prior) {
  if (h->group()) {
    for (size_t d = 0; d < h->subs.size(); ++d) {
      const int64_t o = h->sub_lo[d];
      auto sh = [&](double* v) { return v ? v + o : nullptr; };
      if (int rc = get_data_impl(h->subs[d], X ? X + o : nullptr, ldx, sh(y), sh(m), sh(offset), sh(prior)))
        return rc;
    }
    return SGLM_OK;
  }
  if (X && h->procx.on) {
    set_error("requirement failed: a procedural shard stores no X");
    return SGLM_EINVAL;
  }
  HIPCHK(hipSetDevice(h->device));
  const size_t vb = sizeof(double) * (size_t)h->n;
  if (X)
    HIPCHK(hipMemcpy2DAsync(X, sizeof(double) * (size_t)ldx, h->dX, sizeof(double) * h->n_pad, vb, (size_t)h->p,
                            hipMemcpyDeviceToHost, h->st));
  if (y) HIPCHK(hipMemcpyAsync(y, h->dy, vb, hipMemcpyDeviceToHost, h->st));
  if (m && h->dm) HIPCHK(hipMemcpyAsync(m, h->dm, vb, hipMemcpyDeviceToHost, h->st));
  if (offset && h->doff) HIPCHK(hipMemcpyAsync(offset, h->doff, vb, hipMemcpyDeviceToHost, h->st));
  if (prior && h->dprior) HIPCHK(hipMemcpyAsync(prior, h->dprior, vb, hipMemcpyDeviceToHost, h->st));
  HIPCHK(hipStreamSynchronize(h->st));
  return SGLM_OK;
}

int sglm_get_data(sglm_engine* h, double* X, double* y, double* m, double* offset, double* prior) {
  if (int rc = check_handle(h)) return rc;
  return get_data_impl(h, X, h->group() ? h->g_n : h->n, y, m, offset, prior);
}

static int no_group(sglm_engine* h, const char* what) {
  if (!h->group()) return SGLM_OK;
  set_error(std::string("requirement failed: ") + what +
            " joins one device to other processes; a multi-device handle already reduces over its devices");
  return SGLM_EINVAL;
}

int sglm_set_comm(sglm_engine* h, sglm_allreduce_fn fn, void* ctx, int on_device) {
  if (int rc = check_handle(h)) return rc;
  if (int rc = no_group(h, "sglm_set_comm")) return rc;
  h->comm.kind = fn ? 1 : 0;
  h->comm.fn = fn;
  h->comm.ctx = ctx;
  h->comm.on_device = on_device;
  h->comm.nranks = 1;
  h->comm.rank = known_rank(fn, ctx);
  h->comm.timeout_ms = comm_timeout_ms_env();
  if (h->cbr) h->cbr->reset();
  if (fn) {  // count the ranks joined by the caller's communicator
    double one[1] = {1.0};
    if (on_device) {
      HIPCHK(hipSetDevice(h->device));
      if (int rc = h->ensure_small(64)) return rc;
      HIPCHK(hipMemcpy(h->dsmall, one, sizeof(double), hipMemcpyHostToDevice));
      HIPCHK(hipStreamSynchronize(h->st));
      if (int rc = h->call_comm(h->dsmall, 1, 1)) return rc;
      HIPCHK(hipStreamSynchronize(h->st));
      HIPCHK(hipMemcpy(one, h->dsmall, sizeof(double), hipMemcpyDeviceToHost));
    } else if (int rc = h->call_comm(one, 1, 0)) {
      return rc;
    }
    h->comm.nranks = (int)std::lround(one[0]);
  }
  return SGLM_OK;
}

int sglm_rccl_unique_id(void* out128) {
  static_assert(sizeof(ncclUniqueId) == 128, "ncclUniqueId is 128 bytes");
  ncclUniqueId id;
  ncclResult_t r = ncclGetUniqueId(&id);
  if (r != ncclSuccess) {
    set_error(std::string("ncclGetUniqueId: ") + ncclGetErrorString(r));
    return SGLM_ECOMM;
  }
  std::memcpy(out128, &id, sizeof id);
  return SGLM_OK;
}

int sglm_set_comm_rccl(sglm_engine* h, int nranks, int rank, const void* unique_id128) {
  if (int rc = check_handle(h)) return rc;
  if (int rc = no_group(h, "sglm_set_comm_rccl")) return rc;
  if (nranks < 1 || rank < 0 || rank >= nranks || !unique_id128) {
    set_error("requirement failed: 0 <= rank < nranks, unique id");
    return SGLM_EINVAL;
  }
  HIPCHK(hipSetDevice(h->device));
  if (h->comm.nccl) (void)ncclCommDestroy(h->comm.nccl);
  ncclUniqueId id;
  std::memcpy(&id, unique_id128, sizeof id);
  ncclResult_t r = ncclCommInitRank(&h->comm.nccl, nranks, id, rank);
  if (r != ncclSuccess) {
    h->comm.nccl = nullptr;
    set_error(std::string("ncclCommInitRank: ") + ncclGetErrorString(r));
    return SGLM_ECOMM;
  }
  h->comm.kind = 2;
  h->comm.nranks = nranks;
  h->comm.rank = rank;
  h->comm.timeout_ms = comm_timeout_ms_env();
  if (int rc = h->ensure_small(64)) return rc;
  return SGLM_OK;
}

int sglm_set_comm_rank(sglm_engine* h, int rank) {
  if (int rc = check_handle(h)) return rc;
  if (int rc = no_group(h, "sglm_set_comm_rank")) return rc;
  if (h->comm.kind == 0) {  // no communicator: no other rank to wait for
    set_error("requirement failed: a communicator joined first (sglm_set_comm), 0 <= rank < its rank count");
    return SGLM_EINVAL;
  }
  // Collective: with a rank the scalars travel in per-rank blocks, which lengthens every later
  // all-reduce, so every rank must opt in -- with distinct ranks -- or the ranks would post
  // collectives of different sizes.  Every rank joins one plain all-reduce of [bad | one-hot of
  // its rank], a rank whose own check fails with bad = 1 (never returning before the collective,
  // which would leave the others waiting in it): the ranks are valid and distinct iff bad sums to
  // 0 and every one-hot slot to exactly 1.
  HIPCHK(hipSetDevice(h->device));
  h->comm.rank = -1;
  const int nr = h->comm.nranks;
  const bool local_ok = rank >= 0 && rank < nr;
  std::vector<double> chk((size_t)nr + 1, 0.0);
  chk[0] = local_ok ? 0.0 : 1.0;
  if (local_ok) chk[(size_t)rank + 1] = 1.0;
  if (int rc = h->allreduce_small(chk.data(), (int64_t)chk.size())) return rc;
  bool ok = chk[0] == 0.0;
  for (int k = 0; k < nr; ++k) ok = ok && chk[(size_t)k + 1] == 1.0;
  if (!ok) {
    set_error("requirement failed: sglm_set_comm_rank must be called by every rank of the communicator, each with "
              "its own distinct rank in [0, " + std::to_string(h->comm.nranks) + ")");
    return SGLM_EINVAL;
  }
  h->comm.rank = rank;
  return SGLM_OK;
}

// The handle holds a complete design: every reserved row written (or generated).
static int check_ready(sglm_engine* h) {
  if (h->group()) {
    for (sglm_engine* s : h->subs)
      if (int rc = s->check_loaded()) return rc;
    return SGLM_OK;
  }
  return h->check_loaded();
}

int sglm_fit_glm(sglm_engine* h, const sglm_glm_opts* opts, sglm_preglm* out) {
  if (int rc = check_handle(h)) return rc;
  if (!opts || !out || !out->coefs || !out->std_err) {
    set_error("requirement failed: opts, out, out->coefs, out->std_err");
    return SGLM_EINVAL;
  }
  if (int rc = check_ready(h)) return rc;
  return glm_drive(*h, *opts, out);
}

int sglm_fit_lm(sglm_engine* h, sglm_prelm* out) {
  if (int rc = check_handle(h)) return rc;
  if (!out || !out->coefs || !out->std_err) {
    set_error("requirement failed: out, out->coefs, out->std_err");
    return SGLM_EINVAL;
  }
  if (int rc = check_ready(h)) return rc;
  return lm_drive(*h, out);
}

int sglm_irls_pass(sglm_engine* h, const sglm_glm_opts* opts, const double* beta, double mu0, double* gram,
                   double* xtwz, double* scalars) {
  if (int rc = check_handle(h)) return rc;
  if (!opts || !family_link_valid(opts->family, opts->link)) {
    set_error("requirement failed: opts with a supported family/link");
    return SGLM_EINVAL;
  }
  if (int rc = check_ready(h)) return rc;
  const int64_t p = h->ncols();
  std::vector<double> packed((size_t)packed_len(p)), g((size_t)(p * p)), x((size_t)p);
  const int mode = beta ? MODE_IRLS : (opts->init_mode == SGLM_INIT_MULTIPLE ? MODE_INIT_MULTI : MODE_INIT_SINGLE);
  int rc = h->pass(mode, beta, mu0, 0.0, opts->family, opts->link, packed.data());
  if (rc) return rc;
  unpack_gram(packed.data(), p, g.data(), x.data());
  if (gram) std::memcpy(gram, g.data(), sizeof(double) * g.size());
  if (xtwz) std::memcpy(xtwz, x.data(), sizeof(double) * x.size());
  if (scalars) std::memcpy(scalars, packed.data() + tri_count(p) + p, sizeof(double) * NS);
  return SGLM_OK;
}

int sglm_irls_step(sglm_engine* h, const sglm_glm_opts* opts, const double* beta, double* xtwx, double* xtwz,
                   double* dev) {
  if (!beta) {
    set_error("requirement failed: beta");
    return SGLM_EINVAL;
  }
  double s[NS];
  if (int rc = sglm_irls_pass(h, opts, beta, 0.0, xtwx, xtwz, s)) return rc;
  if (dev) *dev = family_dev_factor(opts->family) * s[S_DEV];
  return SGLM_OK;
}

int sglm_irls_iterations(sglm_engine* h, const sglm_glm_opts* opts, double* beta, int iters, double* last_dev) {
  if (int rc = check_handle(h)) return rc;
  if (!opts || !beta || iters < 0) {
    set_error("requirement failed: opts, beta, iters >= 0");
    return SGLM_EINVAL;
  }
  if (int rc = check_ready(h)) return rc;
  return irls_iterate(*h, *opts, beta, iters, last_dev);
}

// eta (+ offset) of the resident rows -- or, type SGLM_PREDICT_RESPONSE, mu = unlink(eta, m) --
// into out [n_local]; a multi-device handle concatenates its shards in row order.
static int predict_resident(sglm_engine* h, const double* beta, int add_offset, int family, int link, int type,
                            double* out) {
  if (h->group()) {
    for (size_t d = 0; d < h->subs.size(); ++d)
      if (int rc = predict_resident(h->subs[d], beta, add_offset, family, link, type, out + h->sub_lo[d])) return rc;
    return SGLM_OK;
  }
  if (int rc = h->check_loaded()) return rc;
  HIPCHK(hipSetDevice(h->device));
  std::memcpy(h->hbeta, beta, sizeof(double) * h->p);
  HIPCHK(hipMemcpyAsync(h->dbeta, h->hbeta, sizeof(double) * h->p, hipMemcpyHostToDevice, h->st));
  HIPCHK(launch_predict(h->dX, h->n_pad, (int)h->p, h->n, h->dbeta, add_offset ? h->doff : nullptr, h->deta, h->st,
                        h->procx));
  if (type == SGLM_PREDICT_RESPONSE) HIPCHK(launch_unlink(h->deta, h->dm, h->n, family, link, h->st));
  HIPCHK(hipMemcpyAsync(out, h->deta, sizeof(double) * h->n, hipMemcpyDeviceToHost, h->st));
  HIPCHK(hipStreamSynchronize(h->st));
  return SGLM_OK;
}

int sglm_predict(sglm_engine* h, const double* beta, int add_offset, double* out) {
  if (int rc = check_handle(h)) return rc;
  if (!beta || !out) {
    set_error("requirement failed: beta, out");
    return SGLM_EINVAL;
  }
  return predict_resident(h, beta, add_offset, FAM_GAUSSIAN, LNK_IDENTITY, SGLM_PREDICT_LINK, out);
}

int sglm_predict_glm(sglm_engine* h, const double* beta, int family, int link, int type, int add_offset,
                     double* out) {
  if (int rc = check_handle(h)) return rc;
  if (!beta || !out || !family_link_valid(family, link) || (type != SGLM_PREDICT_LINK && type != SGLM_PREDICT_RESPONSE)) {
    set_error("requirement failed: beta, out, a supported family/link, type link or response");
    return SGLM_EINVAL;
  }
  return predict_resident(h, beta, add_offset, family, link, type, out);
}

int sglm_predict_new(sglm_engine* h, const double* X, int64_t n, int64_t p, int64_t ldx, const double* beta,
                     const double* offset, const double* m, int family, int link, int type, double* out) {
  if (int rc = check_handle(h)) return rc;
  if (!X || !beta || !out || n < 0 || p <= 0 || ldx < n || !family_link_valid(family, link) ||
      (type != SGLM_PREDICT_LINK && type != SGLM_PREDICT_RESPONSE)) {
    set_error("requirement failed: X, beta, out, n >= 0, p >= 1, ldx >= n, a supported family/link, type link "
              "or response");
    return SGLM_EINVAL;
  }
  if (n == 0) return SGLM_OK;
  sglm_engine* e = h->group() ? h->subs[0] : h;  // new rows are scored on the first device
  return e->predict_new(X, n, p, ldx, beta, offset, m, family, link, type, out);
}

int sglm_pass_kernel_for(int64_t n, int64_t p, int fused_split, int flags, int family, int link, char* name,
                         int64_t namelen) {
  if (n < 1 || p < 1 || fused_split < 0 || !family_link_valid(family, link)) {
    set_error("requirement failed: n >= 1, p >= 1, fused_split >= 0, a supported family/link");
    return -1;
  }
  const int64_t n_pad = (n + RB - 1) / RB * RB;  // alloc_data's leading dimension
  const bool proc = (flags & 1) != 0, wide = proc || (flags & 2) || p > 16 * MAX_P16, narrow = !wide && p <= 64;
  const int P16 = wide ? 0 : narrow ? narrow_variant((int)p) : pass_variant((int)p, fused_split, n_pad);
  char buf[64];
  const int k = pass_kernel_choice(n_pad, P16, narrow, wide, proc, fused_split, family, link, buf, sizeof buf);
  if (name && namelen > 0) std::snprintf(name, (size_t)namelen, "%s", buf);
  return k;
}

int sglm_get_stats(sglm_engine* h, sglm_stats* out) {
  if (int rc = check_handle(h)) return rc;
  if (h->group()) {  // kernel times: the slowest shard; rows and bytes: all shards
    if (int rc = sglm_get_stats(h->subs[0], out)) return rc;
    for (size_t d = 1; d < h->subs.size(); ++d) {
      sglm_stats s{};
      (void)sglm_get_stats(h->subs[d], &s);
      out->pass_kernel_ms = std::max(out->pass_kernel_ms, s.pass_kernel_ms);
      out->reduce_kernel_ms = std::max(out->reduce_kernel_ms, s.reduce_kernel_ms);
      out->last_pass_ms = std::max(out->last_pass_ms, s.last_pass_ms);
      out->row_kernel_ms = std::max(out->row_kernel_ms, s.row_kernel_ms);
      out->gram_kernel_ms = std::max(out->gram_kernel_ms, s.gram_kernel_ms);
      out->n_local += s.n_local;
      out->load_ms += s.load_ms;
      out->load_bytes += s.load_bytes;
    }
    out->pass_kernel_ms_min = out->pass_kernel_ms;
    for (size_t d = 1; d < h->subs.size(); ++d)
      out->pass_kernel_ms_min = std::min(out->pass_kernel_ms_min, h->subs[d]->pass_ms);
    out->comm_ms = h->comm.ms;
    out->solve_ms = h->solve_ms;
    out->ndev = (int)h->subs.size();
    out->rccl_group = h->gcomms.empty() ? 0 : 1;
    out->dev_passes = h->dev_passes;
    out->overlap_chunks = h->subs.empty() ? 0 : h->subs[0]->ov_chunks();
    out->comm_path = h->gcomms.empty() ? SGLM_COMM_GROUP_HOST : SGLM_COMM_GROUP_RCCL;
    out->rank_blocks = 1;
    out->solve_path = h->solve_path;
    return SGLM_OK;  // pass_kernel / pass_kernel_name: shard 0's (every shard runs the same variant)
  }
  out->passes = h->passes;
  out->pass_kernel_ms = h->pass_ms;
  out->reduce_kernel_ms = h->reduce_ms;
  out->last_pass_ms = h->last_pass_ms;
  out->comm_ms = h->comm.ms;
  out->solve_ms = h->solve_ms;
  out->n_local = h->n;
  out->p = h->p;
  out->workgroups = h->grid;
  out->kernel_variant = h->P16;
  out->path = h->wide ? 1 : (h->narrow ? 2 : 0);
  out->wide_panels = h->wide ? h->npan : 0;
  out->row_kernel_ms = h->row_ms;
  out->gram_kernel_ms = h->wide ? h->gram_ms : h->pass_ms;
  out->load_ms = h->load_ms;
  out->load_bytes = h->load_bytes;
  out->ndev = 1;
  out->rccl_group = 0;
  out->dev_passes = h->dev_passes;
  out->overlap_chunks = h->ov_chunks();
  out->comm_path = h->comm.kind == 2   ? SGLM_COMM_RCCL
                   : h->comm.kind == 1 ? (h->comm.on_device ? SGLM_COMM_CALLER_DEVICE : SGLM_COMM_CALLER_HOST)
                                       : SGLM_COMM_NONE;
  out->rank_blocks = h->gather_ranks() ? 1 : 0;
  out->pass_kernel_ms_min = h->pass_ms;
  out->proc_chunks = h->nch;
  out->proc_chunk_rows = h->ch_rows;
  out->solve_path = h->solve_path;
  out->pass_kernel = h->last_kernel;
  out->lm_device_fits = h->lm_device_fits;
  out->lm_device_reruns = h->lm_device_reruns;
  out->lm_onepass_fits = h->lm_onepass_fits;
  std::memcpy(out->pass_kernel_name, h->last_kernel_name, sizeof out->pass_kernel_name);
  return SGLM_OK;
}

int sglm_reset_stats(sglm_engine* h) {
  if (int rc = check_handle(h)) return rc;
  for (sglm_engine* s : h->subs) (void)sglm_reset_stats(s);
  h->passes = h->dev_passes = h->lm_device_fits = h->lm_device_reruns = h->lm_onepass_fits = 0;
  h->pass_ms = h->reduce_ms = h->last_pass_ms = h->last_reduce_ms = h->row_ms = h->gram_ms = 0.0;
  h->comm.ms = 0.0;
  h->solve_ms = 0.0;
  h->load_ms = 0.0;
  h->load_bytes = 0;
  return SGLM_OK;
}

int sglm_fit_glm_external(const sglm_backend* be, sglm_allreduce_fn fn, void* comm_ctx, const sglm_glm_opts* opts,
                          sglm_preglm* out) {
  if (!be || !be->pass || !be->local_sums || be->p <= 0 || !opts || !out || !out->coefs || !out->std_err) {
    set_error("requirement failed: backend callbacks, p >= 1, opts, out");
    return SGLM_EINVAL;
  }
  ExternalBackend eb(be, fn, comm_ctx);
  return glm_drive(eb, *opts, out);
}

int sglm_fit_lm_external(const sglm_backend* be, sglm_allreduce_fn fn, void* comm_ctx, sglm_prelm* out) {
  if (!be || !be->pass || !be->local_sums || be->p <= 0 || !out || !out->coefs || !out->std_err) {
    set_error("requirement failed: backend callbacks, p >= 1, out");
    return SGLM_EINVAL;
  }
  ExternalBackend eb(be, fn, comm_ctx);
  double sums[2];
  if (int rc = eb.global_sums(sums)) return rc;  // establishes the rank count
  return lm_drive(eb, out);
}


int sglm_local_comm_create(int nranks, sglm_local_comm** out) {
  if (!out || nranks < 1) {
    set_error("requirement failed: nranks >= 1, out");
    return SGLM_EINVAL;
  }
  auto* c = new sglm_local_comm();
  c->nranks = nranks;
  c->timeout_ms = comm_timeout_ms_env();  // once, here: no getenv on the rank threads' all-reduces
  c->bufs.assign((size_t)nranks, nullptr);
  for (int r = 0; r < nranks; ++r) c->ranks.push_back({c, r});
  *out = c;
  return SGLM_OK;
}

void sglm_local_comm_destroy(sglm_local_comm* c) { delete c; }

void* sglm_local_comm_rank(sglm_local_comm* c, int rank) {
  if (!c || rank < 0 || rank >= c->nranks) return nullptr;
  return &c->ranks[(size_t)rank];
}

int sglm_local_allreduce(void* ctx, double* buf, int64_t count, void* stream, int on_device) {
  (void)stream;
  auto* rk = static_cast<sglm_local_comm::Rank*>(ctx);
  if (!rk || on_device) return 1;  // host buffers only
  sglm_local_comm* c = rk->c;
  std::unique_lock<std::mutex> lk(c->mu);
  const uint64_t gen = c->generation;
  if (c->arrived == 0) {
    c->count = count;
    c->failed = false;
  } else if (count != c->count) {
    c->failed = true;
  }
  c->bufs[(size_t)rk->rank] = buf;
  if (++c->arrived == c->nranks) {
    if (!c->failed) {
      std::vector<double> sum(c->bufs[0], c->bufs[0] + count);
      for (int r = 1; r < c->nranks; ++r)
        for (int64_t k = 0; k < count; ++k) sum[(size_t)k] += c->bufs[(size_t)r][k];
      for (int r = 0; r < c->nranks; ++r) std::memcpy(c->bufs[(size_t)r], sum.data(), sizeof(double) * count);
    }
    c->result = c->failed;
    c->arrived = 0;
    ++c->generation;
    c->cv.notify_all();
  } else {
    // bounded (SGLM_COMM_TIMEOUT_S): a rank that never arrives fails the round for everyone
    // instead of leaving the others blocked; the one timing out withdraws its buffer
    const double tmo = c->timeout_ms;
    auto arrived = [&] { return c->generation != gen; };
    if (tmo > 0.0) {
      if (!c->cv.wait_for(lk, std::chrono::duration<double, std::milli>(tmo), arrived)) {
        c->bufs[(size_t)rk->rank] = nullptr;
        --c->arrived;
        c->failed = true;
        return 1;
      }
    } else {
      c->cv.wait(lk, arrived);
    }
  }
  return c->result ? 1 : 0;
}

}  // extern "C"
