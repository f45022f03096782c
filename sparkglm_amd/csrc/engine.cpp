// engine.cpp -- the C ABI (include/sglm.h) over the HIP backend.
//
// One sglm_engine drives one HIP device: it owns the row shard resident in HBM (X
// column-major with a leading dimension padded to the 32-row block, y / m / offset /
// prior, the last pass's eta), the fused-pass workspace and a communicator.  A pass is
//   H2D beta -> irls_pass_kernel (one read of X) -> reduce_partials_kernel (fixed order)
//   -> [device all-reduce: RCCL over xGMI] -> D2H packed -> [host all-reduce callback]
// replacing one zwCreateBinomial + wlsComponents + treeReduce round of the reference
// (GLM.scala:453-458, utils.scala:110-126).
#include <hip/hip_runtime.h>
#include <rccl/rccl.h>

#include <chrono>
#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <string>
#include <vector>

#include "../../include/sglm.h"
#include "common.hpp"
#include "driver.hpp"
#include "kernels.hpp"

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

double now_ms() {
  using namespace std::chrono;
  return duration<double, std::milli>(steady_clock::now().time_since_epoch()).count();
}

struct Comm {
  int kind = 0;  // 0 none, 1 callback, 2 rccl
  sglm_allreduce_fn fn = nullptr;
  void* ctx = nullptr;
  int on_device = 0;
  ncclComm_t nccl = nullptr;
  int nranks = 1;
  double ms = 0.0;
};

}  // namespace

struct sglm_engine : public Backend {
  int device = 0;
  hipStream_t st = nullptr;
  hipEvent_t ev0 = nullptr, ev1 = nullptr, ev2 = nullptr;
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
  // stats
  int64_t passes = 0;
  double pass_ms = 0.0, reduce_ms = 0.0, last_pass_ms = 0.0;
  int dbg = 0;  // profiling ablations (SGLM_DEBUG_ABLATE), never set in production

  ~sglm_engine() override { release(); }

  void free_data() {
    for (double** ptr : {&dX, &dy, &dm, &doff, &dprior, &deta}) {
      if (*ptr) (void)hipFree(*ptr);
      *ptr = nullptr;
    }
    n = p = n_pad = nblocks = 0;
  }
  void release() {
    (void)hipSetDevice(device);
    free_data();
    for (double** ptr : {&dbeta, &dpart, &dred, &dsmall}) {
      if (*ptr) (void)hipFree(*ptr);
      *ptr = nullptr;
    }
    for (double** ptr : {&hbeta, &hred}) {
      if (*ptr) (void)hipHostFree(*ptr);
      *ptr = nullptr;
    }
    if (comm.nccl) (void)ncclCommDestroy(comm.nccl);
    comm.nccl = nullptr;
    if (ev0) (void)hipEventDestroy(ev0);
    if (ev1) (void)hipEventDestroy(ev1);
    if (ev2) (void)hipEventDestroy(ev2);
    if (st) (void)hipStreamDestroy(st);
    ev0 = ev1 = ev2 = nullptr;
    st = nullptr;
  }

  int64_t ncols() const override { return p; }
  int npart() const override { return comm.nranks; }

  // ---- communicator helpers ----
  int allreduce_device(double* dbuf, int64_t count) {
    if (comm.kind == 2) {
      const double t0 = now_ms();
      ncclResult_t r = ncclAllReduce(dbuf, dbuf, (size_t)count, ncclFloat64, ncclSum, comm.nccl, st);
      if (r != ncclSuccess) {
        set_error(std::string("RCCL ncclAllReduce: ") + ncclGetErrorString(r));
        return SGLM_ECOMM;
      }
      HIPCHK(hipStreamSynchronize(st));
      comm.ms += now_ms() - t0;
    } else if (comm.kind == 1 && comm.on_device) {
      HIPCHK(hipStreamSynchronize(st));
      const double t0 = now_ms();
      if (comm.fn(comm.ctx, dbuf, count, (void*)st, 1) != 0) {
        set_error("caller all-reduce failed");
        return SGLM_ECOMM;
      }
      comm.ms += now_ms() - t0;
    }
    return SGLM_OK;
  }
  int allreduce_host(double* hbuf, int64_t count) {
    if (comm.kind == 1 && !comm.on_device) {
      const double t0 = now_ms();
      if (comm.fn(comm.ctx, hbuf, count, (void*)st, 0) != 0) {
        set_error("caller all-reduce failed");
        return SGLM_ECOMM;
      }
      comm.ms += now_ms() - t0;
    }
    return SGLM_OK;
  }
  bool comm_on_device() const { return comm.kind == 2 || (comm.kind == 1 && comm.on_device); }
  // all-reduce a small host vector through whichever path the communicator uses
  int allreduce_small(double* h, int64_t count) {
    if (comm_on_device()) {
      HIPCHK(hipMemcpyAsync(dsmall, h, sizeof(double) * count, hipMemcpyHostToDevice, st));
      int rc = allreduce_device(dsmall, count);
      if (rc) return rc;
      HIPCHK(hipMemcpyAsync(h, dsmall, sizeof(double) * count, hipMemcpyDeviceToHost, st));
      HIPCHK(hipStreamSynchronize(st));
      return SGLM_OK;
    }
    return allreduce_host(h, count);
  }

  int ensure_workspace() {
    P16 = pass_variant((int)p);
    stride = pass_stride(P16);
    const int64_t want_grid = (int64_t)ncu * pass_wg_per_cu(P16);
    grid = (int)(nblocks < want_grid ? (nblocks > 0 ? nblocks : 1) : want_grid);
    const int64_t need_part = std::max<int64_t>((int64_t)grid * stride, 4096 * NS);
    if (need_part > part_cap) {
      if (dpart) HIPCHK(hipFree(dpart));
      dpart = nullptr;
      HIPCHK(hipMalloc(&dpart, sizeof(double) * need_part));
      part_cap = need_part;
    }
    const int64_t need_red = packed_len(p) + 16 * P16;
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
    if (!dsmall) HIPCHK(hipMalloc(&dsmall, sizeof(double) * 64));
    return SGLM_OK;
  }

  int alloc_data(int64_t n_, int64_t p_, bool has_m, bool has_off, bool has_prior) {
    HIPCHK(hipSetDevice(device));
    free_data();
    if (n_ < 0 || p_ <= 0) {
      set_error("requirement failed: n >= 0 and p >= 1");
      return SGLM_EINVAL;
    }
    if (p_ > 16 * MAX_P16) {
      set_error("requirement failed: p <= 256 in this engine build (wide-p panels not yet enabled)");
      return SGLM_EINVAL;
    }
    n = n_;
    p = p_;
    nblocks = (n + RB - 1) / RB;
    n_pad = std::max<int64_t>(nblocks, 1) * RB;
    const size_t vb = sizeof(double) * (size_t)n_pad;
    const size_t ncols = (size_t)((p + 3) / 4 * 4);  // whole column quads for the LDS-DMA staging
    hipError_t e = hipMalloc(&dX, vb * ncols);
    if (e != hipSuccess) {
      set_error(hip_msg(e, "hipMalloc(X)"));
      free_data();
      return SGLM_ENOMEM;
    }
    HIPCHK(hipMemsetAsync(dX, 0, vb * ncols, st));
    for (auto pr : {std::make_pair(&dy, true), std::make_pair(&dm, has_m), std::make_pair(&doff, has_off),
                    std::make_pair(&dprior, has_prior), std::make_pair(&deta, true)}) {
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

  // ---- Backend ----
  int global_sums(double* out2) override {
    HIPCHK(hipSetDevice(device));
    const int nparts = 1024;
    HIPCHK(launch_ysum(dy, n, dpart, nparts, st));
    std::vector<double> h(nparts);
    HIPCHK(hipMemcpyAsync(h.data(), dpart, sizeof(double) * nparts, hipMemcpyDeviceToHost, st));
    HIPCHK(hipStreamSynchronize(st));
    double s = 0.0;
    for (int i = 0; i < nparts; ++i) s += h[i];
    out2[0] = s;
    out2[1] = (double)n;
    return allreduce_small(out2, 2);
  }

  int pass(int mode, const double* beta, double mu0, double ybar, int family, int link, double* packed) override {
    HIPCHK(hipSetDevice(device));
    if (p <= 0) {
      set_error("requirement failed: no data set (sglm_set_data)");
      return SGLM_EINVAL;
    }
    const int64_t plen = packed_len(p);
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
    a.eta_out = (mode == MODE_IRLS) ? deta : nullptr;
    a.dbg = dbg;
    HIPCHK(hipEventRecord(ev0, st));
    if (nblocks > 0) {
      HIPCHK(launch_pass(P16, a, grid, st));
    } else {
      HIPCHK(hipMemsetAsync(dpart, 0, sizeof(double) * stride, st));
    }
    HIPCHK(hipEventRecord(ev1, st));
    HIPCHK(launch_reduce(dpart, stride, nblocks > 0 ? grid : 1, (int)p, P16, dred, st));
    HIPCHK(hipEventRecord(ev2, st));
    int rc = SGLM_OK;
    if (comm_on_device()) {
      rc = allreduce_device(dred, plen);
      if (rc) return rc;
    }
    HIPCHK(hipMemcpyAsync(hred, dred, sizeof(double) * plen, hipMemcpyDeviceToHost, st));
    HIPCHK(hipStreamSynchronize(st));
    float k1 = 0.f, k2 = 0.f;
    HIPCHK(hipEventElapsedTime(&k1, ev0, ev1));
    HIPCHK(hipEventElapsedTime(&k2, ev1, ev2));
    passes += 1;
    pass_ms += k1;
    reduce_ms += k2;
    last_pass_ms = k1;
    if (!comm_on_device()) {
      rc = allreduce_host(hred, plen);
      if (rc) return rc;
    }
    std::memcpy(packed, hred, sizeof(double) * plen);
    return SGLM_OK;
  }

  int stats(int mode, const double* beta, double mu0, double ybar, int family, int link, double* s) override {
    HIPCHK(hipSetDevice(device));
    if (mode == MODE_LM_RESID) {  // pred = X * coefs into the eta buffer
      std::memcpy(hbeta, beta, sizeof(double) * p);
      HIPCHK(hipMemcpyAsync(dbeta, hbeta, sizeof(double) * p, hipMemcpyHostToDevice, st));
      HIPCHK(launch_predict(dX, n_pad, (int)p, n, dbeta, nullptr, deta, st));
    }
    StatsArgs a{};
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
    const int nb = 1024;
    HIPCHK(launch_stats(a, nb, st));
    std::vector<double> h((size_t)nb * NS);
    HIPCHK(hipMemcpyAsync(h.data(), dpart, sizeof(double) * h.size(), hipMemcpyDeviceToHost, st));
    HIPCHK(hipStreamSynchronize(st));
    for (int k = 0; k < NS; ++k) {
      double v = 0.0;
      for (int b = 0; b < nb; ++b) v += h[(size_t)b * NS + k];
      s[k] = v;
    }
    return allreduce_small(s, NS);
  }
};

// =====================================================================================
// External backend adapter (caller-computed partials)
// =====================================================================================
namespace {

struct ExternalBackend : public Backend {
  const sglm_backend* be;
  sglm_allreduce_fn fn;
  void* ctx;
  int nranks = 1;
  ExternalBackend(const sglm_backend* b, sglm_allreduce_fn f, void* c) : be(b), fn(f), ctx(c) {}
  int64_t ncols() const override { return be->p; }
  int npart() const override { return nranks; }
  int reduce(double* buf, int64_t count) {
    if (fn && fn(ctx, buf, count, nullptr, 0) != 0) {
      set_error("caller all-reduce failed");
      return SGLM_ECOMM;
    }
    return SGLM_OK;
  }
  int global_sums(double* out2) override {
    if (be->local_sums(be->ctx, out2) != 0) {
      set_error("external backend local_sums failed");
      return SGLM_EINVAL;
    }
    double one[1] = {1.0};
    int rc = reduce(one, 1);  // counts the ranks joined by the communicator
    if (rc) return rc;
    nranks = (int)std::lround(one[0]);
    return reduce(out2, 2);
  }
  int pass(int mode, const double* beta, double mu0, double ybar, int family, int link, double* packed) override {
    (void)family;
    (void)link;
    if (be->pass(be->ctx, mode, beta, mu0, ybar, packed) != 0) {
      set_error("external backend pass failed");
      return SGLM_EINVAL;
    }
    return reduce(packed, packed_len(be->p));
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

int sglm_create(int device, sglm_engine** out) {
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
  hipDeviceProp_t prop;
  if ((e = hipGetDeviceProperties(&prop, device)) != hipSuccess) return fail(e, "hipGetDeviceProperties");
  h->ncu = prop.multiProcessorCount > 0 ? prop.multiProcessorCount : 256;
  if (const char* ab = std::getenv("SGLM_DEBUG_ABLATE")) h->dbg = std::atoi(ab);
  *out = h;
  return SGLM_OK;
}

void sglm_destroy(sglm_engine* h) { delete h; }

static int set_data_impl(sglm_engine* h, const double* X, int64_t n, int64_t p, int64_t ldx, const double* y,
                         const double* m, const double* off, const double* prior, hipMemcpyKind kind) {
  if (int rc = check_handle(h)) return rc;
  if (!X || !y || ldx < n || n <= 0 || p <= 0) {
    set_error("requirement failed: X, y non-null, n >= 1, p >= 1, ldx >= n");
    return SGLM_EINVAL;
  }
  int rc = h->alloc_data(n, p, m != nullptr, off != nullptr, prior != nullptr);
  if (rc) return rc;
  const size_t vb = sizeof(double) * (size_t)n;
  HIPCHK(hipMemcpy2DAsync(h->dX, sizeof(double) * h->n_pad, X, sizeof(double) * ldx, vb, (size_t)p, kind, h->st));
  HIPCHK(hipMemcpyAsync(h->dy, y, vb, kind, h->st));
  if (m) HIPCHK(hipMemcpyAsync(h->dm, m, vb, kind, h->st));
  if (off) HIPCHK(hipMemcpyAsync(h->doff, off, vb, kind, h->st));
  if (prior) HIPCHK(hipMemcpyAsync(h->dprior, prior, vb, kind, h->st));
  HIPCHK(hipStreamSynchronize(h->st));
  return SGLM_OK;
}

int sglm_set_data(sglm_engine* h, const double* X, int64_t n, int64_t p, int64_t ldx, const double* y,
                  const double* m, const double* offset, const double* prior) {
  return set_data_impl(h, X, n, p, ldx, y, m, offset, prior, hipMemcpyHostToDevice);
}

int sglm_set_data_device(sglm_engine* h, const double* dX, int64_t n, int64_t p, int64_t ldx, const double* dy,
                         const double* dm, const double* doffset, const double* dprior) {
  return set_data_impl(h, dX, n, p, ldx, dy, dm, doffset, dprior, hipMemcpyDeviceToDevice);
}

int sglm_synth(sglm_engine* h, int kind, int64_t row0, int64_t n, int64_t p, uint64_t seed) {
  if (int rc = check_handle(h)) return rc;
  if (kind < 0 || kind > 2 || n <= 0 || p <= 0 || row0 < 0) {
    set_error("requirement failed: synth kind in {0,1,2}, n >= 1, p >= 1");
    return SGLM_EINVAL;
  }
  int rc = h->alloc_data(n, p, false, kind == 2, kind == 2);
  if (rc) return rc;
  const double scale = 1.0 / std::sqrt((double)p);
  HIPCHK(launch_synth(kind, row0, n, (int)p, seed, scale, h->dX, h->n_pad, h->dy, nullptr, h->doff, h->dprior, h->st));
  HIPCHK(hipStreamSynchronize(h->st));
  return SGLM_OK;
}

int sglm_get_data(sglm_engine* h, double* X, double* y, double* m, double* offset, double* prior) {
  if (int rc = check_handle(h)) return rc;
  HIPCHK(hipSetDevice(h->device));
  const size_t vb = sizeof(double) * (size_t)h->n;
  if (X)
    HIPCHK(hipMemcpy2DAsync(X, vb, h->dX, sizeof(double) * h->n_pad, vb, (size_t)h->p, hipMemcpyDeviceToHost, h->st));
  if (y) HIPCHK(hipMemcpyAsync(y, h->dy, vb, hipMemcpyDeviceToHost, h->st));
  if (m && h->dm) HIPCHK(hipMemcpyAsync(m, h->dm, vb, hipMemcpyDeviceToHost, h->st));
  if (offset && h->doff) HIPCHK(hipMemcpyAsync(offset, h->doff, vb, hipMemcpyDeviceToHost, h->st));
  if (prior && h->dprior) HIPCHK(hipMemcpyAsync(prior, h->dprior, vb, hipMemcpyDeviceToHost, h->st));
  HIPCHK(hipStreamSynchronize(h->st));
  return SGLM_OK;
}

int sglm_set_comm(sglm_engine* h, sglm_allreduce_fn fn, void* ctx, int on_device) {
  if (int rc = check_handle(h)) return rc;
  h->comm.kind = fn ? 1 : 0;
  h->comm.fn = fn;
  h->comm.ctx = ctx;
  h->comm.on_device = on_device;
  h->comm.nranks = 1;
  if (fn) {  // count the ranks joined by the caller's communicator
    double one[1] = {1.0};
    if (on_device) {
      HIPCHK(hipSetDevice(h->device));
      if (!h->dsmall) HIPCHK(hipMalloc(&h->dsmall, sizeof(double) * 64));
      HIPCHK(hipMemcpy(h->dsmall, one, sizeof(double), hipMemcpyHostToDevice));
      if (fn(ctx, h->dsmall, 1, (void*)h->st, 1) != 0) {
        set_error("caller all-reduce failed");
        return SGLM_ECOMM;
      }
      HIPCHK(hipStreamSynchronize(h->st));
      HIPCHK(hipMemcpy(one, h->dsmall, sizeof(double), hipMemcpyDeviceToHost));
    } else if (fn(ctx, one, 1, (void*)h->st, 0) != 0) {
      set_error("caller all-reduce failed");
      return SGLM_ECOMM;
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
  if (!h->dsmall) HIPCHK(hipMalloc(&h->dsmall, sizeof(double) * 64));
  return SGLM_OK;
}

int sglm_fit_glm(sglm_engine* h, const sglm_glm_opts* opts, sglm_preglm* out) {
  if (int rc = check_handle(h)) return rc;
  if (!opts || !out || !out->coefs || !out->std_err) {
    set_error("requirement failed: opts, out, out->coefs, out->std_err");
    return SGLM_EINVAL;
  }
  if (h->p <= 0) {
    set_error("requirement failed: no data set (sglm_set_data)");
    return SGLM_EINVAL;
  }
  return glm_drive(*h, *opts, out);
}

int sglm_fit_lm(sglm_engine* h, sglm_prelm* out) {
  if (int rc = check_handle(h)) return rc;
  if (!out || !out->coefs || !out->std_err) {
    set_error("requirement failed: out, out->coefs, out->std_err");
    return SGLM_EINVAL;
  }
  if (h->p <= 0) {
    set_error("requirement failed: no data set (sglm_set_data)");
    return SGLM_EINVAL;
  }
  return lm_drive(*h, out);
}

int sglm_irls_pass(sglm_engine* h, const sglm_glm_opts* opts, const double* beta, double mu0, double* gram,
                   double* xtwz, double* scalars) {
  if (int rc = check_handle(h)) return rc;
  if (!opts || !family_link_valid(opts->family, opts->link)) {
    set_error("requirement failed: opts with a supported family/link");
    return SGLM_EINVAL;
  }
  const int64_t p = h->p;
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

int sglm_irls_iterations(sglm_engine* h, const sglm_glm_opts* opts, double* beta, int iters, double* last_dev) {
  if (int rc = check_handle(h)) return rc;
  if (!opts || !beta || iters < 0) {
    set_error("requirement failed: opts, beta, iters >= 0");
    return SGLM_EINVAL;
  }
  return irls_iterate(*h, *opts, beta, iters, last_dev);
}

int sglm_predict(sglm_engine* h, const double* beta, int add_offset, double* out) {
  if (int rc = check_handle(h)) return rc;
  if (!beta || !out) {
    set_error("requirement failed: beta, out");
    return SGLM_EINVAL;
  }
  HIPCHK(hipSetDevice(h->device));
  std::memcpy(h->hbeta, beta, sizeof(double) * h->p);
  HIPCHK(hipMemcpyAsync(h->dbeta, h->hbeta, sizeof(double) * h->p, hipMemcpyHostToDevice, h->st));
  HIPCHK(launch_predict(h->dX, h->n_pad, (int)h->p, h->n, h->dbeta, add_offset ? h->doff : nullptr, h->deta, h->st));
  HIPCHK(hipMemcpyAsync(out, h->deta, sizeof(double) * h->n, hipMemcpyDeviceToHost, h->st));
  HIPCHK(hipStreamSynchronize(h->st));
  return SGLM_OK;
}

int sglm_get_stats(sglm_engine* h, sglm_stats* out) {
  if (int rc = check_handle(h)) return rc;
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
  return SGLM_OK;
}

int sglm_reset_stats(sglm_engine* h) {
  if (int rc = check_handle(h)) return rc;
  h->passes = 0;
  h->pass_ms = h->reduce_ms = h->last_pass_ms = 0.0;
  h->comm.ms = 0.0;
  h->solve_ms = 0.0;
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

}  // extern "C"
