// C ABI of libmlffpcg.so (declared in include/mlffpcg.h): context, kernel
// matrix, preconditioner builds and the scipy-1.7.3-compatible PCG driver.
//
// PCG driver (restating scipy.sparse.linalg.cg 1.7.3 = CGREVCOM template + python
// wrapper, as called at src/sGDML/sgdml/solvers/iterative_solver.py:995-1005):
//   atol = tol * ||b||                      (legacy atol=None; ||A x0 - b|| <= tol exits early)
//   r = b - A x0;  if ||r|| < atol: done
//   ITER = ITER + 1:  z = M r; rho = r.z; p = z + (rho/rho1) p (p = z at ITER 1)
//                     q = A p; alpha = rho / p.q; x += alpha p; r -= alpha q
//                     stop test ||r|| <= atol, re-checked with r = b - A x when ITER > 1
//                     ITER == maxiter -> info = maxiter
// Every iteration is 5-7 launches on one stream with all scalars kept on the
// device; the host polls the status word once per chunk of iterations, and
// kernels of iterations past convergence return immediately (status gating),
// so the iteration count is exact without a per-iteration host sync.
#include "common.h"

#include <cstdlib>

#include <algorithm>
#include <chrono>
#include <cmath>
#include <condition_variable>
#include <cstring>
#include <limits>
#include <map>
#include <mutex>

using namespace mlff;

static thread_local std::string g_last_error;

namespace mlff {

int set_error(mlff_ctx *ctx, int code, const std::string &msg) {
  if (ctx != nullptr) ctx->err = msg;
  g_last_error = msg;
  return code;
}

void local_abort(mlff_ctx *ctx);

int api_exception(mlff_ctx *ctx, int code, const char *what) {
  try {
    local_abort(ctx);
    return set_error(ctx, code, std::string("C++ exception in libmlffpcg: ") + (what ? what : ""));
  } catch (...) {
    return code;
  }
}

constexpr size_t kScratchChunk = size_t(64) << 20;

ScratchScope::ScratchScope(mlff_ctx *c) : ctx(c), chunk(c->scratch_cur), off(c->scratch_off) {
  ++ctx->scratch_depth;
}

// Closing the outermost scope returns every chunk but one standard-size chunk to the device
// (after the stream has drained the kernels that used them): build temporaries such as the
// k x k Woodbury Gram, eigensolver panels or split-K slabs do not stay allocated through the
// PCG that follows.
ScratchScope::~ScratchScope() {
  ctx->scratch_cur = chunk;
  ctx->scratch_off = off;
  if (--ctx->scratch_depth != 0) return;
  auto &ch = ctx->scratch_chunks;
  const bool keep_first = !ch.empty() && ch[0].size == kScratchChunk;
  if (ch.size() > (keep_first ? 1u : 0u)) {
    (void)hipStreamSynchronize(ctx->stream);
    for (size_t i = keep_first ? 1 : 0; i < ch.size(); ++i) (void)hipFree(ch[i].p);
    ch.resize(keep_first ? 1 : 0);
  }
  ctx->scratch_cur = 0;
  ctx->scratch_off = 0;
}

int scratch_get(mlff_ctx *ctx, size_t bytes, void **out) {
  constexpr size_t kAlign = 256, kChunk = kScratchChunk;
  bytes = (bytes + kAlign - 1) / kAlign * kAlign;
  auto &ch = ctx->scratch_chunks;
  while (true) {
    if (ctx->scratch_cur < ch.size()) {
      const auto &c = ch[ctx->scratch_cur];
      if (ctx->scratch_off + bytes <= c.size) {
        *out = c.p + ctx->scratch_off;
        ctx->scratch_off += bytes;
        return MLFF_OK;
      }
      ++ctx->scratch_cur;  // the rest of this chunk stays unused until the scope closes
      ctx->scratch_off = 0;
      continue;
    }
    void *p = nullptr;
    MLFF_HIP(ctx, hipMalloc(&p, std::max(bytes, kChunk)));
    ch.push_back({static_cast<char *>(p), std::max(bytes, kChunk)});
    ctx->scratch_cur = ch.size() - 1;
    ctx->scratch_off = 0;
  }
}

// A device failure on one rank of an in-process group aborts the group, so its peers
// return MLFF_ERR_COMM from their next collective instead of waiting forever.
int hip_check(mlff_ctx *ctx, hipError_t e, const char *what) {
  const int code = (e == hipErrorOutOfMemory) ? MLFF_ERR_NOMEM : MLFF_ERR_HIP;
  local_abort(ctx);
  return set_error(ctx, code, std::string(what) + ": " + hipGetErrorString(e));
}

int nccl_check(mlff_ctx *ctx, ncclResult_t e, const char *what) {
  return set_error(ctx, MLFF_ERR_COMM, std::string(what) + ": " + ncclGetErrorString(e));
}

// In-process transport: `world` contexts of one process (one host thread each,
// any devices) joined by a comm_id "LOCAL:<key>".  Collectives are host-staged
// and reduce in rank order.  Used to exercise the multi-rank code path on a
// single GPU (RCCL refuses two ranks on one device); production multi-GPU runs
// use RCCL.
struct LocalGroup {
  int world = 0;
  std::mutex m;
  std::condition_variable cv;
  int arrived = 0;
  long long gen = 0;
  bool aborted = false;
  std::vector<double> buf;  // world * count staging
  // false once any member has aborted the group
  bool barrier() {
    std::unique_lock<std::mutex> lk(m);
    if (aborted) return false;
    const long long g = gen;
    if (++arrived == world) {
      arrived = 0;
      ++gen;
      cv.notify_all();
    } else {
      cv.wait(lk, [&] { return gen != g || aborted; });
    }
    return !aborted;
  }
  void abort() {
    std::lock_guard<std::mutex> lk(m);
    aborted = true;
    cv.notify_all();
  }
};

void local_abort(mlff_ctx *ctx) {
  if (ctx != nullptr && ctx->local) ctx->local->abort();
}

#define LOCAL_BARRIER(ctx, g)                                                        \
  do {                                                                               \
    if (!(g).barrier())                                                              \
      return set_error((ctx), MLFF_ERR_COMM, "in-process group aborted by a peer rank"); \
  } while (0)

static std::mutex g_groups_m;
static std::map<std::string, std::weak_ptr<LocalGroup>> g_groups;

std::shared_ptr<LocalGroup> join_local_group(const std::string &key, int world) {
  std::lock_guard<std::mutex> lk(g_groups_m);
  auto it = g_groups.find(key);
  std::shared_ptr<LocalGroup> gp = (it != g_groups.end()) ? it->second.lock() : nullptr;
  if (!gp) {
    gp = std::make_shared<LocalGroup>();
    gp->world = world;
    g_groups[key] = gp;
  }
  return gp;
}

__global__ void k_selftest_fill(double *p, size_t n, double scale) {
  for (size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (size_t)gridDim.x * blockDim.x)
    p[i] = scale * (1.0 + 0.5 * (double)i);
}

// RCCL transport: the collectives are enqueued on the context's stream, so they are ordered
// after the kernels that produced `send` and before the ones that read `recv` with no host
// synchronisation.  Semantics are those of the LOCAL branches below: allreduce in place over
// n doubles; allgather of `count` doubles per rank into recv[rank*count ...] (in place when
// send == recv + rank*count); reduce-scatter of world*count doubles into this rank's `count`.
// mlff_comm_selftest drives these three functions on a one-rank communicator, the only RCCL
// configuration a one-GPU box can run.
static int rccl_allreduce(mlff_ctx *ctx, double *buf, size_t n) {
  MLFF_NCCL(ctx, ncclAllReduce(buf, buf, n, ncclDouble, ncclSum, ctx->comm, ctx->stream));
  return MLFF_OK;
}

static int rccl_allgather(mlff_ctx *ctx, const double *send, double *recv, size_t count) {
  MLFF_NCCL(ctx, ncclAllGather(send, recv, count, ncclDouble, ctx->comm, ctx->stream));
  return MLFF_OK;
}

static int rccl_reduce_scatter(mlff_ctx *ctx, const double *send, double *recv, size_t count) {
  MLFF_NCCL(ctx, ncclReduceScatter(send, recv, count, ncclDouble, ncclSum, ctx->comm, ctx->stream));
  return MLFF_OK;
}

// SOLO transport (comm_id "SOLO:..."): ONE rank of a W-way split runs alone and every
// collective keeps only this rank's own contribution (no data from peers, no wait).  The
// numbers are meaningless; the kernels, their sizes and their launch sequence are those of
// rank `rank` of W, so a one-GPU kernel trace shows the per-rank compute of the sharded
// iteration without the collectives (bench.py --solo-world).  Profiling only.
int comm_allreduce(mlff_ctx *ctx, double *buf, size_t n) {
  if (ctx->world <= 1 || n == 0 || ctx->solo) return MLFF_OK;
  if (ctx->comm != nullptr) return rccl_allreduce(ctx, buf, n);
  LocalGroup &g = *ctx->local;
  std::vector<double> mine(n), sum(n, 0.0);
  MLFF_HIP(ctx, hipMemcpyAsync(mine.data(), buf, sizeof(double) * n, hipMemcpyDeviceToHost, ctx->stream));
  MLFF_HIP(ctx, hipStreamSynchronize(ctx->stream));
  LOCAL_BARRIER(ctx, g);  // previous users of g.buf are done
  if (ctx->rank == 0) g.buf.assign((size_t)g.world * n, 0.0);
  LOCAL_BARRIER(ctx, g);
  std::memcpy(g.buf.data() + (size_t)ctx->rank * n, mine.data(), sizeof(double) * n);
  LOCAL_BARRIER(ctx, g);
  for (int r = 0; r < g.world; ++r)
    for (size_t i = 0; i < n; ++i) sum[i] += g.buf[(size_t)r * n + i];
  LOCAL_BARRIER(ctx, g);
  MLFF_HIP(ctx, hipMemcpyAsync(buf, sum.data(), sizeof(double) * n, hipMemcpyHostToDevice, ctx->stream));
  MLFF_HIP(ctx, hipStreamSynchronize(ctx->stream));
  return MLFF_OK;
}

int comm_allgather(mlff_ctx *ctx, const double *send, double *recv, size_t count) {
  if (ctx->world <= 1) {
    if (send != recv)
      MLFF_HIP(ctx, hipMemcpyAsync(recv, send, sizeof(double) * count, hipMemcpyDeviceToDevice, ctx->stream));
    return MLFF_OK;
  }
  if (ctx->solo) {
    double *own = recv + (size_t)ctx->rank * count;
    if (send != own)
      MLFF_HIP(ctx, hipMemcpyAsync(own, send, sizeof(double) * count, hipMemcpyDeviceToDevice, ctx->stream));
    return MLFF_OK;
  }
  if (ctx->comm != nullptr) return rccl_allgather(ctx, send, recv, count);
  LocalGroup &g = *ctx->local;
  std::vector<double> mine(count);
  MLFF_HIP(ctx, hipMemcpyAsync(mine.data(), send, sizeof(double) * count, hipMemcpyDeviceToHost, ctx->stream));
  MLFF_HIP(ctx, hipStreamSynchronize(ctx->stream));
  LOCAL_BARRIER(ctx, g);
  if (ctx->rank == 0) g.buf.assign((size_t)g.world * count, 0.0);
  LOCAL_BARRIER(ctx, g);
  std::memcpy(g.buf.data() + (size_t)ctx->rank * count, mine.data(), sizeof(double) * count);
  LOCAL_BARRIER(ctx, g);
  std::vector<double> all(g.buf);
  LOCAL_BARRIER(ctx, g);
  MLFF_HIP(ctx, hipMemcpyAsync(recv, all.data(), sizeof(double) * all.size(), hipMemcpyHostToDevice, ctx->stream));
  MLFF_HIP(ctx, hipStreamSynchronize(ctx->stream));
  return MLFF_OK;
}

int comm_reduce_scatter(mlff_ctx *ctx, const double *send, double *recv, size_t count) {
  if (ctx->world <= 1) {
    if (send != recv)
      MLFF_HIP(ctx, hipMemcpyAsync(recv, send, sizeof(double) * count, hipMemcpyDeviceToDevice, ctx->stream));
    return MLFF_OK;
  }
  if (ctx->solo) {
    MLFF_HIP(ctx, hipMemcpyAsync(recv, send + (size_t)ctx->rank * count, sizeof(double) * count,
                                 hipMemcpyDeviceToDevice, ctx->stream));
    return MLFF_OK;
  }
  if (ctx->comm != nullptr) return rccl_reduce_scatter(ctx, send, recv, count);
  LocalGroup &g = *ctx->local;
  const size_t n = count * (size_t)g.world;
  std::vector<double> mine(n), out(count, 0.0);
  MLFF_HIP(ctx, hipMemcpyAsync(mine.data(), send, sizeof(double) * n, hipMemcpyDeviceToHost, ctx->stream));
  MLFF_HIP(ctx, hipStreamSynchronize(ctx->stream));
  LOCAL_BARRIER(ctx, g);
  if (ctx->rank == 0) g.buf.assign((size_t)g.world * n, 0.0);
  LOCAL_BARRIER(ctx, g);
  std::memcpy(g.buf.data() + (size_t)ctx->rank * n, mine.data(), sizeof(double) * n);
  LOCAL_BARRIER(ctx, g);
  for (int r = 0; r < g.world; ++r)
    for (size_t i = 0; i < count; ++i) out[i] += g.buf[(size_t)r * n + (size_t)ctx->rank * count + i];
  LOCAL_BARRIER(ctx, g);
  MLFF_HIP(ctx, hipMemcpyAsync(recv, out.data(), sizeof(double) * count, hipMemcpyHostToDevice, ctx->stream));
  MLFF_HIP(ctx, hipStreamSynchronize(ctx->stream));
  return MLFF_OK;
}

}  // namespace mlff

namespace {

constexpr int kTimingPool = 4096;

int ensure_matrix(mlff_ctx *ctx) {
  if (ctx->K == nullptr) {
    MLFF_HIP(ctx, hipMalloc(&ctx->K, sizeof(double) * ctx->blk * ctx->ld));
  }
  return MLFF_OK;
}

int dev_free(void *p) {
  if (p != nullptr) (void)hipFree(p);
  return MLFF_OK;
}

void rbf_free(mlff_ctx *ctx) {
  dev_free(ctx->rbf.Xs);
  ctx->rbf = RbfData();
}

// the dense rows of the RBF source, generated on first use (DENSE storage, the masked
// eigen build); the symmetric tiles and every column access go without them
int ensure_rows(mlff_ctx *ctx) {
  if (ctx->has_matrix || !ctx->rbf.ready) return MLFF_OK;
  MLFF_TRY(ensure_matrix(ctx));
  if (ctx->blk > ctx->nrows)  // zero padding rows
    MLFF_HIP(ctx, hipMemsetAsync(ctx->K + ctx->nrows * ctx->ld, 0,
                                 sizeof(double) * (ctx->blk - ctx->nrows) * ctx->ld, ctx->stream));
  if (ctx->nrows > 0)
    launch_gen_rbf(ctx->K, ctx->ld, ctx->nrows, ctx->row0, ctx->rows_per, ctx->blk, ctx->N,
                   ctx->rbf.Xs, ctx->rbf.d, ctx->rbf.jitter, ctx->stream);
  MLFF_HIP(ctx, hipGetLastError());
  MLFF_HIP(ctx, hipStreamSynchronize(ctx->stream));
  ctx->has_matrix = true;
  return MLFF_OK;
}

// allreduce (sum) of n doubles in place, no-op on one rank
int allreduce(mlff_ctx *ctx, double *buf, size_t n) { return comm_allreduce(ctx, buf, n); }

// gather the rank blocks of an ld-long padded vector (in place)
int allgather_blocks(mlff_ctx *ctx, double *full) {
  if (ctx->world > 1)
    return comm_allgather(ctx, full + ctx->rank * ctx->blk, full, (size_t)ctx->blk);
  return MLFF_OK;
}

// scatter a global host vector (N) into a padded device vector (ld)
int scatter_global(mlff_ctx *ctx, const double *v, double *dev_full) {
  MLFF_HIP(ctx, hipMemsetAsync(dev_full, 0, sizeof(double) * ctx->ld, ctx->stream));
  for (int r = 0; r < ctx->world; ++r) {
    const int64_t g0 = (int64_t)r * ctx->rows_per;
    if (g0 >= ctx->N) break;
    const int64_t cnt = std::min<int64_t>(ctx->rows_per, ctx->N - g0);
    MLFF_HIP(ctx, hipMemcpyAsync(dev_full + (int64_t)r * ctx->blk, v + g0, sizeof(double) * cnt,
                                 hipMemcpyHostToDevice, ctx->stream));
  }
  return MLFF_OK;
}

// scalar = sum over ranks of a . b (local), synchronous
int dot_sync(mlff_ctx *ctx, const double *a, const double *b, double *out) {
  double *part = ctx->part;  // slot 0 region
  launch_dot_part(a, b, ctx->nrows, part, nullptr, ctx->stream);
  MLFF_TRY(allreduce(ctx, part, kVecGrid));
  launch_reduce_to(part, kVecGrid, &ctx->st->pad0, ctx->stream);
  MLFF_HIP(ctx, hipMemcpyAsync(out, &ctx->st->pad0, sizeof(double), hipMemcpyDeviceToHost,
                               ctx->stream));
  MLFF_HIP(ctx, hipStreamSynchronize(ctx->stream));
  return MLFF_OK;
}

// epoch of the next cluster-apply launch: never 0 (the value of a cleared hand-off slot)
unsigned next_lr_epoch(mlff_ctx *c) {
  if (++c->lr_epoch == 0) ++c->lr_epoch;
  return c->lr_epoch;
}

double *rho_part(mlff_ctx *c) { return c->part + 0 * kMaxPart; }
double *pq_part(mlff_ctx *c) { return c->part + 1 * kMaxPart; }
double *rr_part(mlff_ctx *c) { return c->part + 2 * kMaxPart; }

int alloc_panel(mlff_ctx *ctx, int64_t k) {
  if (ctx->T != nullptr) {
    (void)hipFree(ctx->T);
    ctx->T = nullptr;
  }
  if (ctx->tpart_base != nullptr) {
    (void)hipFree(ctx->tpart_base);
    ctx->tpart_base = nullptr;
    ctx->tpart = nullptr;
  }
  ctx->spec_t = false;
  MLFF_HIP(ctx, hipMalloc(&ctx->T, sizeof(double) * round_up(k, 8) * ctx->blk));
  MLFF_HIP(ctx, hipMemsetAsync(ctx->T, 0, sizeof(double) * round_up(k, 8) * ctx->blk, ctx->stream));
  ctx->tsplit = choose_tsplit(k, ctx->blk);
  if (const char *e = std::getenv("MLFF_TSPLIT")) ctx->tsplit = std::max(1, std::atoi(e));  // sweeps
  // [rr partials (kVecGrid) | tpart (k x tsplit)]: on several ranks the end-of-iteration
  // ||r||^2 reduction and the next iteration's T r reduction share one all-reduce
  MLFF_HIP(ctx, hipMalloc(&ctx->tpart_base, sizeof(double) * (kVecGrid + k * ctx->tsplit)));
  ctx->tpart = ctx->tpart_base + kVecGrid;
  if (ctx->zpart != nullptr) {
    (void)hipFree(ctx->zpart);
    ctx->zpart = nullptr;
  }
  ctx->zsplit = choose_zsplit(k, ctx->blk);
  if (const char *e = std::getenv("MLFF_ZSPLIT"))  // sweeps
    ctx->zsplit = (int)std::min<int64_t>(std::max(1, std::atoi(e)), (k + 15) / 16);
  MLFF_HIP(ctx, hipMalloc(&ctx->zpart, sizeof(double) * ctx->zsplit * ctx->blk));
  // one rank, rows that fit a workgroup's registers: the one-pass apply (at >= 7 rows per
  // workgroup its G partial vectors are <= 2/7 of a panel pass) from k = 768, and at any k on
  // short rows (N_loc <= 4096), where the launches it saves dominate the step: ethanol M = 111
  // (N = 2997), k = 50 / 150 / 398: PCG step 33.7 / 33.2 / 35.3 -> 29.5 / 29.5 / 30.1 us; M = 23
  // (N = 621), k = 30 / 132: 30.2 / 30.2 -> 28.7 / 28.4 us; at N = 15741, k = 300 the step is
  // the same either way (52.3 / 52.0 us), and k = 554 keeps the two-pass order its golden
  // fixture's crossings were measured with (profiles/r05/lr_small/).  MLFF_LR_ROWS=0 / 1
  // forces the two-pass / one-pass apply (A/B, tests)
  for (void **p : {(void **)&ctx->lr_zpart, (void **)&ctx->lr_slots, (void **)&ctx->lr_fault})
    if (*p != nullptr) {
      (void)hipFree(*p);
      *p = nullptr;
    }
  const char *lr_env = std::getenv("MLFF_LR_ROWS");
  const bool lr_on = lr_env == nullptr || std::atoi(lr_env) != 0;
  ctx->lr_rows = ctx->world == 1 && lr_rows_fits(ctx->blk) &&
                 (lr_env ? lr_on : (k >= 768 || ctx->blk <= 4096));
  // longer rows: clusters of workgroups share a row (lr_cluster_count of them resident);
  // worth it from ~4 rows per cluster (the Q partial vectors against the second pass)
  ctx->lr_cluster = false;
  if (ctx->world == 1 && !ctx->lr_rows && lr_on && lr_cluster_fits(ctx->blk)) {
    ctx->lr_q = lr_cluster_count(ctx->blk, ctx->device);
    if (const char *e = std::getenv("MLFF_LR_CLUSTERS"))  // A/B: fewer clusters
      ctx->lr_q = std::min(ctx->lr_q, std::max(1, std::atoi(e)));
    ctx->lr_cluster = ctx->lr_q >= 1 && k >= 4 * (int64_t)ctx->lr_q;
  }
  if (ctx->lr_rows)
    MLFF_HIP(ctx, hipMalloc(&ctx->lr_zpart, sizeof(double) * lr_rows_groups(k) * ctx->blk));
  if (ctx->lr_cluster) {
    const size_t ns = (size_t)k * lr_cluster_members(ctx->blk) * 2;
    MLFF_HIP(ctx, hipMalloc(&ctx->lr_zpart, sizeof(double) * ctx->lr_q * ctx->blk));
    MLFF_HIP(ctx, hipMalloc(&ctx->lr_slots, sizeof(unsigned long long) * ns));
    MLFF_HIP(ctx, hipMemsetAsync(ctx->lr_slots, 0, sizeof(unsigned long long) * ns, ctx->stream));
    MLFF_HIP(ctx, hipMalloc(&ctx->lr_fault, sizeof(int)));
    MLFF_HIP(ctx, hipMemsetAsync(ctx->lr_fault, 0, sizeof(int), ctx->stream));
    ctx->lr_epoch = 0;
  }
  return MLFF_OK;
}

// _cho_factor_stable (iterative_solver.py:555-583; :584-618 are unreachable after `if True:`):
// lo_eig = the smallest eigenvalue of M (eigh of the lower triangle, :577 -- here the
// device tridiagonalisation + Sturm bisection of kernels_syev.hip), M += (+1e-15 if lo_eig
// <= 0 else -1e-15) I (:578-579), then the Cholesky factor (:580-582; LinAlgError when it
// fails).  A (k x k, device) is overwritten with the lower factor; lo_eig_out: the value used.
//
// Inside the builds (lo_eig_out == nullptr) the downward shift is tried first: when M - 1e-15 I
// factors, M's smallest eigenvalue is above 1e-15 (to the factorisation's backward error), so
// the reference takes the lo_eig > 0 branch and factors this same matrix -- the same factor,
// without the eigenvalue (whose tridiagonalisation is most of a Nystrom build: 2 x 5.3 s of 13 s
// at k = 14670, profiles/r04/syev/).  Otherwise (lo_eig at or below 1e-15, where the sign
// decides) the eigenvalue path runs as before.  MLFF_CHO_FAST=0 (read at context creation):
// always the eigenvalue path.
int cho_factor_stable(mlff_ctx *ctx, double *A, int64_t k, double *lo_eig_out,
                      double *shift_out = nullptr) {
  if (shift_out) *shift_out = -1e-15;
  if (lo_eig_out == nullptr && ctx->cho_fast) {
    ScratchScope scope(ctx);
    double *B = nullptr;
    MLFF_TRY(scratch_alloc(ctx, &B, (size_t)(k * k)));
    MLFF_HIP(ctx, hipMemcpyAsync(B, A, sizeof(double) * k * k, hipMemcpyDeviceToDevice, ctx->stream));
    launch_add_diag(B, k, -1e-15, ctx->stream);
    bool ok = false;
    MLFF_TRY(potrf_lower(ctx, B, k, &ok));
    if (ok) {
      MLFF_HIP(ctx, hipMemcpyAsync(A, B, sizeof(double) * k * k, hipMemcpyDeviceToDevice, ctx->stream));
      ctx->last_lo_eig = std::numeric_limits<double>::quiet_NaN();  // above 1e-15, not computed
      return MLFF_OK;
    }
  }
  double lo = 0.0;
  std::vector<double> d((size_t)k), e((size_t)(k > 1 ? k - 1 : 0));
  MLFF_TRY(sym_min_eig(ctx, A, k, &lo, d.data(), e.data()));
  // |lo| <= 2 eps ||M|| (||M|| bounded by Gershgorin on the tridiagonal, which is similar to M):
  // eigh's own rounding (~eps ||M||, tests/golden/cho_stable_ethanol.npz delta = 0) decides the
  // sign there, so the device's sign may differ from LAPACK's.  When such a lo > 0 makes the
  // downward shift fail, the upward one the reference takes for lo <= 0 is tried before
  // LinAlgError.  (The fixture's lo = 1.26e-16 at ||M|| ~ 0.03 is 20x above the bound and still
  // raises like the reference.)  MLFF_CHO_TEST_NOISY_POSITIVE=1: a noisy lo is taken as > 0
  // (the test of this retry; never set in production).
  double gersh = 0.0;
  for (int64_t i = 0; i < k; ++i)
    gersh = std::max(gersh, std::fabs(d[i]) + (i > 0 ? std::fabs(e[i - 1]) : 0.0) +
                                (i + 1 < k ? std::fabs(e[i]) : 0.0));
  const bool noisy = std::fabs(lo) <= 2.0 * std::numeric_limits<double>::epsilon() * gersh;
  if (noisy && lo <= 0.0) {
    const char *t = std::getenv("MLFF_CHO_TEST_NOISY_POSITIVE");
    if (t != nullptr && std::atoi(t) == 1) lo = std::fabs(lo) > 0.0 ? std::fabs(lo) : 1e-300;
  }
  ctx->last_lo_eig = lo;
  if (lo_eig_out) *lo_eig_out = lo;
  if (!(noisy && lo > 0.0)) {
    launch_add_diag(A, k, lo <= 0.0 ? 1e-15 : -1e-15, ctx->stream);
    if (shift_out) *shift_out = lo <= 0.0 ? 1e-15 : -1e-15;
    return potrf_lower(ctx, A, k);
  }
  ScratchScope scope(ctx);
  double *keep = nullptr;
  MLFF_TRY(scratch_alloc(ctx, &keep, (size_t)(k * k)));
  MLFF_HIP(ctx, hipMemcpyAsync(keep, A, sizeof(double) * k * k, hipMemcpyDeviceToDevice, ctx->stream));
  launch_add_diag(A, k, -1e-15, ctx->stream);
  bool ok = false;
  MLFF_TRY(potrf_lower(ctx, A, k, &ok));
  if (ok) return MLFF_OK;
  MLFF_HIP(ctx, hipMemcpyAsync(A, keep, sizeof(double) * k * k, hipMemcpyDeviceToDevice, ctx->stream));
  launch_add_diag(A, k, 1e-15, ctx->stream);
  if (shift_out) *shift_out = 1e-15;
  ctx->cho_flipped = true;
  return potrf_lower(ctx, A, k);
}

// Woodbury panel from a wide factor W = L^T (k x blk) in place:
//   G = lam I + W W^T; L2 = chol(G); W <- L2^-1 W   (iterative_cholesky.py:141-143)
//
// ctx->wb_refine (MLFF_WB_REFINE): W is the top block of Q1 = A R1^-1, A = [L; sqrt(lam) I],
// R1 = L2^T -- one CholeskyQR step.  A second step re-orthogonalises it: G2 = Q1^T Q1 =
// W W^T + lam L2^-1 L2^-T (= I in exact arithmetic, so the preconditioner is unchanged),
// C C^T = G2, W <- C^-1 W.  At lam = 1e-10 the PCG count depends on how accurately the
// Woodbury apply's r - W^T W r cancels (DESIGN.md 2, configs[1] at full size).
// The second CholeskyQR step of a panel W = L2^-1 X^T (k x blk, this rank's columns) built
// from L2 L2^T = X^T X + mu I: W is the top block of Q1 = [X; sqrt(mu) I] L2^-T, so
// G2 = Q1^T Q1 = W W^T + mu L2^-1 L2^-T (= I in exact arithmetic), C C^T = G2, W <- C^-1 W.
// L2: the lower factor (k x k, the same on every rank).
// steps > 1 (MLFF_WB_REFINE=<steps>): CholeskyQR3 and beyond -- step s uses the accumulated
// factor (L2 C_1 ... C_{s-1}), whose inverse is C_{s-1}^-1 ... C_1^-1 L2^-1 (Li updated by one
// k x k triangular solve per step)
int reorthogonalise_panel(mlff_ctx *ctx, double *W, const double *L2, int64_t k, double mu,
                          int steps = 1) {
  ScratchScope scope(ctx);
  hipStream_t s = ctx->stream;
  double *Li = nullptr, *G2 = nullptr;
  MLFF_TRY(scratch_alloc(ctx, &Li, k * k));
  MLFF_TRY(scratch_alloc(ctx, &G2, k * k));
  MLFF_HIP(ctx, hipMemsetAsync(Li, 0, sizeof(double) * k * k, s));
  launch_add_diag(Li, k, 1.0, s);
  MLFF_TRY(trsm_lower_wide(ctx, L2, k, Li, k, k));  // Li = L2^-1
  for (int st = 0; st < steps; ++st) {
    if (ctx->wb_gram_dd)
      MLFF_TRY(gram_wide_dd(ctx, W, k, ctx->blk, ctx->blk, G2, ctx->wb_gram_dd == 2));
    else
      MLFF_TRY(syrk_wide(ctx, W, k, ctx->blk, ctx->blk, G2));
    MLFF_TRY(allreduce(ctx, G2, (size_t)(k * k)));
    launch_gemm(false, true, k, k, k, mu, Li, k, Li, k, 1.0, G2, k, s);  // + mu Li Li^T
    MLFF_TRY(potrf_lower(ctx, G2, k));
    MLFF_TRY(trsm_lower_wide(ctx, G2, k, W, ctx->blk, ctx->blk));
    if (st + 1 < steps) MLFF_TRY(trsm_lower_wide(ctx, G2, k, Li, k, k));  // Li <- C^-1 Li
  }
  return MLFF_OK;
}

int woodbury_inplace(mlff_ctx *ctx, double *W, int64_t k) {
  ScratchScope scope(ctx);
  hipStream_t s = ctx->stream;
  double *G = nullptr;
  MLFF_TRY(scratch_alloc(ctx, &G, k * k));
  if (ctx->wb_gram_dd)  // L^T L rounded once per entry (DESIGN.md 2, configs[1])
    MLFF_TRY(gram_wide_dd(ctx, W, k, ctx->blk, ctx->blk, G, ctx->wb_gram_dd == 2));
  else
    MLFF_TRY(syrk_wide(ctx, W, k, ctx->blk, ctx->blk, G));
  MLFF_TRY(allreduce(ctx, G, (size_t)(k * k)));
  launch_add_diag(G, k, ctx->lam, s);
  MLFF_TRY(potrf_lower(ctx, G, k));
  MLFF_TRY(trsm_lower_wide(ctx, G, k, W, ctx->blk, ctx->blk));
  if (ctx->wb_refine > 0) MLFF_TRY(reorthogonalise_panel(ctx, W, G, k, ctx->lam, ctx->wb_refine));
  MLFF_HIP(ctx, hipStreamSynchronize(s));
  return MLFF_OK;
}

__global__ void k_unit_idx(double *__restrict__ x, const int64_t *__restrict__ idx, int64_t j,
                           int64_t rows_per, int64_t blk, double val) {
  if (threadIdx.x == 0) {
    const int64_t g = idx[j];
    x[(g / rows_per) * blk + g % rows_per] = val;
  }
}

// W[j, i] = (sigma_K K)[row0 + i, idx_j] for the local rows: a gather from the
// dense rows, evaluated from the RBF points, or from the matrix-free sGDML operator (the
// reference's own column access, K_op.matvec(e_i), iterative_cholesky.py:152-156)
int fetch_cols(mlff_ctx *ctx, const int64_t *didx, int64_t k, double *W, int64_t ldw) {
  hipStream_t s = ctx->stream;
  if (ctx->has_matrix) {
    launch_gather_cols(ctx->K, ctx->ld, ctx->nrows, didx, k, ctx->rows_per, ctx->blk, ctx->sigma_K,
                       W, ldw, s);
    MLFF_HIP(ctx, hipGetLastError());
    return MLFF_OK;
  }
  if (ctx->rbf.ready) {
    launch_rbf_cols(ctx->rbf, ctx->N, ctx->row0, ctx->nrows, didx, k, nullptr, ctx->sigma_K, W, ldw, s);
    MLFF_HIP(ctx, hipGetLastError());
    return MLFF_OK;
  }
  if (!ctx->mf.ready) return set_error(ctx, MLFF_ERR_STATE, "no kernel matrix / operator set");
  if (mf_columns(ctx, didx, k, ctx->sigma_K, W, ldw)) {  // single-column path, one launch
    MLFF_HIP(ctx, hipGetLastError());
    return MLFF_OK;
  }
  MLFF_HIP(ctx, hipMemsetAsync(ctx->xg, 0, sizeof(double) * ctx->ld, s));
  for (int64_t j = 0; j < k; ++j) {
    hipLaunchKernelGGL(k_unit_idx, dim3(1), dim3(64), 0, s, ctx->xg, didx, j, ctx->rows_per,
                       ctx->blk, 1.0);
    launch_mf_operator(ctx, ctx->xg, W + j * ldw, nullptr, nullptr, ctx->sigma_K, 0.0);
    hipLaunchKernelGGL(k_unit_idx, dim3(1), dim3(64), 0, s, ctx->xg, didx, j, ctx->rows_per,
                       ctx->blk, 0.0);
    if ((j & 255) == 255) MLFF_HIP(ctx, hipGetLastError());
  }
  MLFF_HIP(ctx, hipGetLastError());
  return MLFF_OK;
}

// Nystrom panel (iterative_solver.py:112-283 for variant 0, :343-374 for variant 1,
// :489-550 for the leverage scores which follow variant 0).  W: k x blk, zeroed.
int nystrom_panel(mlff_ctx *ctx, const int64_t *idx_host, int64_t k, int variant, double lam,
                  double *W) {
  hipStream_t s = ctx->stream;
  ScratchScope scope(ctx);
  int64_t *didx = nullptr;
  double *Smm = nullptr, *G = nullptr;
  MLFF_TRY(scratch_alloc(ctx, &didx, k));
  MLFF_TRY(scratch_alloc(ctx, &Smm, k * k));
  MLFF_TRY(scratch_alloc(ctx, &G, k * k));
  MLFF_HIP(ctx, hipMemcpyAsync(didx, idx_host, sizeof(int64_t) * k, hipMemcpyHostToDevice, s));
  // K_nm^T (sign convention S = sigma_K K; sign flips cancel in B^T B)
  MLFF_TRY(fetch_cols(ctx, didx, k, W, ctx->blk));
  launch_gather_mm(W, ctx->blk, didx, k, ctx->row0, ctx->nrows, Smm, s);
  MLFF_TRY(allreduce(ctx, Smm, (size_t)(k * k)));
  int rc;
  if (variant == 0) {
    rc = cho_factor_stable(ctx, Smm, k, nullptr);  // U^T U = -K_mm (+-1e-15)
  } else {
    launch_add_diag(Smm, k, 1e-16, s);            // cholesky(K_mm + 1e-16 I, lower=True)
    rc = potrf_lower(ctx, Smm, k);
  }
  if (rc != MLFF_OK) return rc;
  MLFF_TRY(trsm_lower_wide(ctx, Smm, k, W, ctx->blk, ctx->blk));   // C^T = U^-T K_nm^T
  MLFF_TRY(syrk_wide(ctx, W, k, ctx->blk, ctx->blk, G));           // C^T C
  MLFF_TRY(allreduce(ctx, G, (size_t)(k * k)));
  launch_add_diag(G, k, lam, s);
  double shift = 0.0;
  if (variant == 0)
    rc = cho_factor_stable(ctx, G, k, nullptr, &shift);
  else
    rc = potrf_lower(ctx, G, k);
  if (rc != MLFF_OK) return rc;
  MLFF_TRY(trsm_lower_wide(ctx, G, k, W, ctx->blk, ctx->blk));     // B = V^-T C^T
  // B is the top block of [C; sqrt(lam + shift) I] V^-T: the same second CholeskyQR step as
  // the Woodbury panel (MLFF_NYS_REFINE)
  if (ctx->nys_refine) MLFF_TRY(reorthogonalise_panel(ctx, W, G, k, lam + shift));
  MLFF_HIP(ctx, hipStreamSynchronize(s));
  return MLFF_OK;
}

int check_idx(mlff_ctx *ctx, const int64_t *idx, int64_t k) {
  if (idx == nullptr || k < 1 || k > ctx->N) return set_error(ctx, MLFF_ERR_ARG, "bad column index set");
  for (int64_t j = 0; j < k; ++j) {
    if (idx[j] < 0 || idx[j] >= ctx->N) return set_error(ctx, MLFF_ERR_ARG, "column index out of range");
    if (j > 0 && idx[j] <= idx[j - 1])
      return set_error(ctx, MLFF_ERR_ARG, "column indices must be sorted and unique (train.py:1197-1201)");
  }
  return MLFF_OK;
}

// the operator needs K (dense rows), the RBF points or the matrix-free sGDML data
int require_operator(mlff_ctx *ctx) {
  if (!ctx->has_matrix && !ctx->mf.ready && !ctx->rbf.ready)
    return set_error(ctx, MLFF_ERR_STATE, "no kernel matrix / operator set");
  if (!ctx->has_operator) return set_error(ctx, MLFF_ERR_STATE, "mlff_set_operator not called");
  return MLFF_OK;
}

// preconditioner builds read columns of the dense K
int require_matrix(mlff_ctx *ctx) {
  MLFF_TRY(require_operator(ctx));
  MLFF_TRY(ensure_rows(ctx));
  if (!ctx->has_matrix)
    return set_error(ctx, MLFF_ERR_STATE,
                     "this build needs the dense kernel matrix (assemble it first)");
  return MLFF_OK;
}

// Decide the operator storage (mlff_set_storage) and build the symmetric tiles
// if they are to be used and not current.
int resolve_storage(mlff_ctx *ctx) {
  ctx->use_mf = false;
  if (ctx->exact_sums) {
    // the exact-sum anchor (kernels_dd.hip) is a dense-row operator on one rank: refused for
    // every other storage before any of them is chosen, so the fused matrix-free iteration
    // (which moves the x / r update into the next apply) can never run beside its apply
    if (ctx->world > 1 || ctx->storage == MLFF_STORAGE_MATFREE ||
        ctx->storage == MLFF_STORAGE_SYMTILE || (!ctx->has_matrix && !ctx->rbf.ready))
      return set_error(ctx, MLFF_ERR_STATE,
                       "MLFF_EXACT_SUMS: dense-row storage (a matrix or RBF points) on one rank only");
    MLFF_TRY(ensure_rows(ctx));
    ctx->use_sym = false;
    return MLFF_OK;
  }
  if (ctx->storage == MLFF_STORAGE_MATFREE) {
    if (!ctx->mf.ready)
      return set_error(ctx, MLFF_ERR_STATE, "MLFF_STORAGE_MATFREE needs mlff_sgdml_operator / mlff_assemble_sgdml");
    ctx->use_sym = false;
    ctx->use_mf = true;
    return MLFF_OK;
  }
  if (!ctx->has_matrix && !ctx->rbf.ready) {  // only the matrix-free operator exists
    ctx->use_sym = false;
    ctx->use_mf = true;
    return MLFF_OK;
  }
  if (ctx->storage == MLFF_STORAGE_AUTO && ctx->mf.ready) {
    // the matrix-free operator or the stored K (tiles, rows): whichever the time model of
    // the measured rates (mf_seconds) puts first for this rank's share
    const double Np = (double)round_up(ctx->ld, kSymTile);
    const double t_tiles = 10e-6 + 4.0 * Np * Np / ctx->world / 6.9e12;  // 2 launches + stream
    double t_mf = mf_seconds(ctx);
    if (ctx->world > 1) {
      // one decision for all ranks (each models its own share; the slowest rank paces the
      // iteration): the modelled times are all-reduced as a world-long vector and every rank
      // takes the same maximum -- ranks that chose differently would run mismatched collectives
      if (ctx->world > kMaxPart) return set_error(ctx, MLFF_ERR_ARG, "world too large");
      std::vector<double> t(ctx->world, 0.0);
      t[ctx->rank] = t_mf;
      double *buf = ctx->part + 3 * kMaxPart;
      MLFF_HIP(ctx, hipMemcpyAsync(buf, t.data(), sizeof(double) * ctx->world, hipMemcpyHostToDevice,
                                   ctx->stream));
      MLFF_TRY(comm_allreduce(ctx, buf, ctx->world));
      MLFF_HIP(ctx, hipMemcpyAsync(t.data(), buf, sizeof(double) * ctx->world, hipMemcpyDeviceToHost,
                                   ctx->stream));
      MLFF_HIP(ctx, hipStreamSynchronize(ctx->stream));
      t_mf = *std::max_element(t.begin(), t.end());
    }
    if (t_mf < t_tiles) {
      ctx->use_sym = false;
      ctx->use_mf = true;
      return MLFF_OK;
    }
  }
  if (ctx->storage == MLFF_STORAGE_DENSE) {
    MLFF_TRY(ensure_rows(ctx));
    ctx->use_sym = false;
    return MLFF_OK;
  }
  if (ctx->sym.ready) {
    ctx->use_sym = true;
    return MLFF_OK;
  }
  if (!ctx->has_matrix) {  // RBF source: the tiles are generated from the points
    bool symmetric = true;
    MLFF_TRY(sym_build(ctx, false, &symmetric));
    ctx->use_sym = true;
    return MLFF_OK;
  }
  const bool explicit_sym = ctx->storage == MLFF_STORAGE_SYMTILE;
  if (ctx->world > 1 && !ctx->K_symmetric && !explicit_sym) {
    ctx->use_sym = false;  // a sharded host matrix cannot be checked locally
    return MLFF_OK;
  }
  const bool check = !ctx->K_symmetric && ctx->world == 1;
  bool symmetric = true;
  int rc = sym_build(ctx, check, &symmetric);
  if (ctx->world > 1) {
    // every rank must take the same path (the tiled operator has a collective)
    const double fail_here = (rc != MLFF_OK || !symmetric) ? 1.0 : 0.0;
    double *flag = ctx->part + 3 * kMaxPart;
    MLFF_HIP(ctx, hipMemcpyAsync(flag, &fail_here, sizeof(double), hipMemcpyHostToDevice, ctx->stream));
    MLFF_TRY(comm_allreduce(ctx, flag, 1));
    double fails = 0.0;
    MLFF_HIP(ctx, hipMemcpyAsync(&fails, flag, sizeof(double), hipMemcpyDeviceToHost, ctx->stream));
    MLFF_HIP(ctx, hipStreamSynchronize(ctx->stream));
    if (fails > 0.0 && rc == MLFF_OK) symmetric = false;
  }
  if (rc != MLFF_OK || !symmetric) {
    sym_free(ctx->sym);
    (void)hipGetLastError();
    ctx->use_sym = false;
    if (explicit_sym) {
      if (rc != MLFF_OK) return rc;
      return set_error(ctx, MLFF_ERR_ARG, "MLFF_STORAGE_SYMTILE: K is not symmetric");
    }
    ctx->err.clear();
    return MLFF_OK;  // AUTO: dense row GEMV
  }
  ctx->use_sym = true;
  return MLFF_OK;
}

// y_loc = sigma_K K v_full + lam v_loc over this rank's rows (status gated).
// pq_part: also the v_loc . y_loc partials of the CG step (kVecGrid, k_dot_part's layout;
// fused into the last operator kernel where it can be)
int launch_operator(mlff_ctx *ctx, const double *v_full, double *y_loc, const double *v_loc,
                    const int *status, double *pq_part = nullptr, const PFuse *pf = nullptr) {
  hipStream_t s = ctx->stream;
  if (ctx->exact_sums) {  // measurement anchor (kernels_dd.hip): dense rows, one rank
    if (ctx->use_mf || ctx->use_sym || ctx->world > 1)
      return set_error(ctx, MLFF_ERR_STATE, "MLFF_EXACT_SUMS: dense-row storage on one rank only");
    launch_dd_gemv_rows(ctx->K, ctx->ld, ctx->nrows, ctx->N, v_full, y_loc, ctx->sigma_K, ctx->lam,
                        v_loc, status, s);
    if (pq_part != nullptr) launch_dot_part(v_loc, y_loc, ctx->nrows, pq_part, status, s);
    return MLFF_OK;
  }
  if (ctx->use_mf) {
    launch_mf_operator(ctx, v_full, y_loc, v_loc, status, ctx->sigma_K, ctx->lam, pq_part, pf);
    return MLFF_OK;
  }
  if (!ctx->use_sym) {
    launch_gemv_rows(ctx->K, ctx->ld, ctx->nrows, v_full, y_loc, ctx->sigma_K, ctx->lam, v_loc,
                     status, s);
    if (pq_part != nullptr) launch_dot_part(v_loc, y_loc, ctx->nrows, pq_part, status, s);
    return MLFF_OK;
  }
  if (pq_part != nullptr) return set_error(ctx, MLFF_ERR_STATE, "launch_operator: pq with tiles");
  SymPack &sp = ctx->sym;
  launch_symv(sp, v_full, sp.P, status, s);
  if (ctx->world == 1) {
    launch_sym_reduce(sp, ctx->nrows, y_loc, true, ctx->sigma_K, ctx->lam, v_loc, status, s);
    return MLFF_OK;
  }
  launch_sym_reduce_ranks(sp, ctx->rank, ctx->world, ctx->blk, nullptr, nullptr, nullptr, 0.0, 0.0,
                          status, s);
  MLFF_TRY(comm_reduce_scatter(ctx, sp.yg, sp.yr, (size_t)sp.ystride));
  launch_axpby_loc(sp.yr, y_loc, ctx->nrows, ctx->sigma_K, ctx->lam, v_loc, status, s);
  return MLFF_OK;
}

}  // namespace

// y_loc = S x = sigma_K K x (no ridge) for this rank's rows, x given as this rank's block
// of a distributed vector (blk entries, zero padded): the block is all-gathered into the
// operand xg first (one collective).  resolve_storage must have run.  Stream ordered.
int mlff::operator_apply_local(mlff_ctx *ctx, const double *x_loc, double *y_loc) {
  MLFF_HIP(ctx, hipMemcpyAsync(ctx->xg + (int64_t)ctx->rank * ctx->blk, x_loc,
                               sizeof(double) * ctx->blk, hipMemcpyDeviceToDevice, ctx->stream));
  MLFF_TRY(allgather_blocks(ctx, ctx->xg));
  return launch_operator(ctx, ctx->xg, y_loc, nullptr, nullptr);
}

int mlff::operator_prepare(mlff_ctx *ctx) {
  MLFF_TRY(require_operator(ctx));
  return resolve_storage(ctx);
}

int mlff::operator_diag(mlff_ctx *ctx, double *out) {
  if (ctx->has_matrix) {
    launch_diag_of(ctx->K, ctx->ld, ctx->nrows, ctx->row0, ctx->rows_per, ctx->blk, ctx->sigma_K,
                   out, ctx->stream);
    MLFF_HIP(ctx, hipGetLastError());
    return MLFF_OK;
  }
  if (ctx->rbf.ready) {  // K[i, i] = 1 + jitter
    launch_fill(out, ctx->nrows, ctx->sigma_K * (1.0 + ctx->rbf.jitter), ctx->stream);
    MLFF_HIP(ctx, hipGetLastError());
    return MLFF_OK;
  }
  if (!ctx->mf.ready) return set_error(ctx, MLFF_ERR_STATE, "no kernel matrix / operator set");
  return mf_diag(ctx, out);
}

namespace {

double operator_bytes(const mlff_ctx *ctx) {
  if (ctx->use_mf) return mf_bytes(ctx);
  if (ctx->use_sym)
    return 8.0 * (double)ctx->sym.ntiles * kSymTile * kSymTile + 16.0 * (double)ctx->nrows;
  return 8.0 * (double)ctx->nrows * (double)ctx->N + 16.0 * (double)ctx->nrows;
}

hipEvent_t timing_event(mlff_ctx *ctx) {
  Timing &t = ctx->timing;
  if (t.used >= t.ev.size()) {
    hipEvent_t e;
    if (hipEventCreateWithFlags(&e, timing_event_flags()) != hipSuccess) return nullptr;
    t.ev.push_back(e);
  }
  return t.ev[t.used++];
}

// a timed segment of one iteration: events ev0 -> ev1 of the pool; kind 0 = operator,
// 1 = low-rank preconditioner apply
struct GemvMark {
  size_t ev0, ev1;
  long long it;
  int kind;
};

constexpr size_t kNoMark = (size_t)-1;

size_t mark_begin(mlff_ctx *ctx, std::vector<GemvMark> *marks) {
  if (!ctx->timing.on || marks == nullptr || !ctx->timing.sample) return kNoMark;
  hipEvent_t e0 = timing_event(ctx);
  if (e0 == nullptr) return kNoMark;
  hipEventRecord(e0, ctx->stream);
  return ctx->timing.used - 1;
}

void mark_end(mlff_ctx *ctx, std::vector<GemvMark> *marks, size_t i0, long long it, int kind = 0) {
  if (i0 == kNoMark) return;
  hipEvent_t e1 = timing_event(ctx);
  if (e1) {
    hipEventRecord(e1, ctx->stream);
    marks->push_back({i0, ctx->timing.used - 1, it, kind});
  }
}

// One PCG iteration on several ranks: three collectives instead of five:
//   allgather(z_g | rho partials)  -> rho and the whole p on every rank
//   [symmetric tiles] reduce-scatter(K p partial rows | p.q shares) -> q rows and p.q
//   [other storages]  allreduce(p.q partials)
//   allreduce(rr partials | T r partials of the next iteration)   (low-rank precon)
// Same recurrence as launch_iteration; the sums are over the same terms in another
// (fixed) order, bitwise identical on all ranks.
int launch_iteration_ranks(mlff_ctx *ctx, long long it, std::vector<GemvMark> *marks,
                           bool fold_in, bool stop_out) {
  hipStream_t s = ctx->stream;
  const int *status = &ctx->st->status;
  double *p_loc = ctx->p_full + (int64_t)ctx->rank * ctx->blk;
  double *zg = ctx->gb + (int64_t)ctx->rank * ctx->gstride;  // this rank's gather block
  const bool lowrank = ctx->precon_kind != MLFF_PRECON_NONE;
  double *rrp = lowrank ? ctx->tpart_base : rr_part(ctx);
  StopFold fold;  // stop test of iteration it - 1 in this iteration's first kernel
  if (fold_in) fold = StopFold{rrp, ctx->st, ctx->trace, it - 1};
  if (lowrank) {
    if (!ctx->spec_t) {
      launch_gemv_split(ctx->T, ctx->blk, ctx->k, ctx->blk, ctx->tsplit, ctx->r, ctx->tpart, status, s,
                        fold);
      fold = StopFold{};
      MLFF_TRY(allreduce(ctx, ctx->tpart, (size_t)(ctx->k * ctx->tsplit)));
    }
    // the low-rank apply: T r (issued at the end of the previous iteration, kind 3) + z here
    const size_t pm = mark_begin(ctx, marks);
    launch_precon_z(ctx->T, ctx->blk, ctx->k, ctx->tsplit, ctx->tpart, ctx->r, zg, ctx->nrows,
                    ctx->sigma_p, 1.0 / ctx->lam, zg + ctx->blk, status, s, ctx->zpart, ctx->zsplit,
                    fold);
    mark_end(ctx, marks, pm, it, 1);
  } else {
    launch_copy_dot(ctx->r, ctx->nrows, zg, zg + ctx->blk, status, s, fold);
  }
  size_t c0 = mark_begin(ctx, marks);
  MLFF_TRY(comm_allgather(ctx, zg, ctx->gb, (size_t)ctx->gstride));
  mark_end(ctx, marks, c0, it, 2);
  // symmetric tiles (dynamic schedule): p = z + beta p formed by the tile workgroups from the
  // gathered z and written by the slot reduction (k_update_p_gathered's bits, one launch less)
  const bool fuse_pg = ctx->fuse_p && ctx->use_sym && ctx->sym.dyn > 0 && ctx->sym.ntiles > 0;
  // symmetric tiles + low-rank apply: k_update_xr_shares folded into the next T r pass
  const bool fold_xr = ctx->fuse_xr_ranks && ctx->use_sym && lowrank &&
                       xr_fold_fits(ctx->blk, ctx->tsplit, ctx->nrows);
  PGather pg;
  if (fuse_pg)
    pg = PGather{ctx->gb, ctx->gstride, ctx->blk, ctx->world, ctx->st, it};
  else
    launch_update_p_gathered(ctx->gb, ctx->gstride, ctx->blk, ctx->world, ctx->p_full, ctx->st, it,
                             status, s);
  const size_t e0 = mark_begin(ctx, marks);
  if (ctx->use_sym) {
    SymPack &sp = ctx->sym;
    launch_symv(sp, ctx->p_full, sp.P, status, s, pg);
    launch_sym_reduce_ranks(sp, ctx->rank, ctx->world, ctx->blk, ctx->p_full, pq_part(ctx),
                            pq_part(ctx) + kVecGrid, ctx->sigma_K, ctx->lam, status, s, pg,
                            ctx->pq_publish);
    mark_end(ctx, marks, e0, it);
    c0 = mark_begin(ctx, marks);
    MLFF_TRY(comm_reduce_scatter(ctx, sp.yg, sp.yr, (size_t)sp.ystride));
    mark_end(ctx, marks, c0, it, 2);
    if (!fold_xr)
      launch_update_xr_shares(ctx->x, ctx->r, p_loc, sp.yr, sp.yr + ctx->blk, ctx->world,
                              ctx->nrows, ctx->sigma_K, ctx->lam,
                              lowrank ? ctx->tpart_base : rr_part(ctx), ctx->st, status, s);
  } else {
    MLFF_TRY(launch_operator(ctx, ctx->p_full, ctx->q, p_loc, status, pq_part(ctx)));
    mark_end(ctx, marks, e0, it);
    c0 = mark_begin(ctx, marks);
    MLFF_TRY(allreduce(ctx, pq_part(ctx), kVecGrid));
    mark_end(ctx, marks, c0, it, 2);
    launch_update_xr(ctx->x, ctx->r, p_loc, ctx->q, ctx->nrows, pq_part(ctx),
                     lowrank ? ctx->tpart_base : rr_part(ctx), ctx->st, status, s);
  }
  if (lowrank) {
    // the T r half of iteration it + 1's apply: bracketed with that iteration (its
    // z half, kind 1) so a sampled apply is always timed whole
    ctx->timing.sample = (it + 1) % ctx->timing.every == 0;
    const size_t tm = mark_begin(ctx, marks);
    if (fold_xr) {
      // x, r update of this iteration inside the T r pass: r_new goes to the other buffer
      // (ctx->z, unused by the sharded iteration), which becomes r
      launch_gemv_xr(ctx->T, ctx->blk, ctx->k, ctx->blk, ctx->tsplit, ctx->r, ctx->z, ctx->x, p_loc,
                     ctx->sym.yr, ctx->sym.yr + ctx->blk, ctx->world, ctx->nrows, ctx->sigma_K,
                     ctx->lam, ctx->tpart_base, ctx->st, ctx->tpart, status, s);
      std::swap(ctx->r, ctx->z);
    } else {
      launch_gemv_split(ctx->T, ctx->blk, ctx->k, ctx->blk, ctx->tsplit, ctx->r, ctx->tpart, status,
                        s);
    }
    mark_end(ctx, marks, tm, it, 3);
    c0 = mark_begin(ctx, marks);
    MLFF_TRY(allreduce(ctx, ctx->tpart_base, (size_t)(kVecGrid + ctx->k * ctx->tsplit)));
    mark_end(ctx, marks, c0, it, 2);
    ctx->spec_t = true;
  } else {
    c0 = mark_begin(ctx, marks);
    MLFF_TRY(allreduce(ctx, rrp, kVecGrid));
    mark_end(ctx, marks, c0, it, 2);
  }
  if (stop_out) launch_stoptest(rrp, ctx->st, ctx->trace, it, s);
  return MLFF_OK;
}

// one PCG iteration (ITER = it), all launches status gated.  fold_in: the stop test of
// iteration it - 1 runs in this iteration's first kernel (StopFold); stop_out: the stop
// test of this iteration runs as its own launch (last iteration of a chunk)
int launch_iteration(mlff_ctx *ctx, long long it, std::vector<GemvMark> *marks, bool fold_in,
                     bool stop_out) {
  // events cost GPU time between the kernels they bracket: only every timing.every-th
  // iteration is bracketed (the averages are over the sampled iterations)
  ctx->timing.sample = it % ctx->timing.every == 0;
  if (ctx->world > 1) return launch_iteration_ranks(ctx, it, marks, fold_in, stop_out);
  hipStream_t s = ctx->stream;
  const int *status = &ctx->st->status;
  double *p_loc = ctx->p_full + (int64_t)ctx->rank * ctx->blk;
  const bool lowrank = ctx->precon_kind != MLFF_PRECON_NONE;
  StopFold fold;
  if (fold_in) fold = StopFold{rr_part(ctx), ctx->st, ctx->trace, it - 1};
  // matrix-free operator (default form): p = z + beta p formed inside the operator kernels;
  // with the one-pass apply also k_update_xr of iteration it - 1 folded into this
  // iteration's apply (x, r, rr partials written by k_lr_fin) and its stop test into the
  // operator's first kernel: 4 launches per iteration instead of 6
  const bool fuse_p = ctx->use_mf && mf_can_fuse_p(ctx);
  const bool fuse_xr = fuse_p && lowrank && ctx->lr_rows && ctx->fuse_xr;
  XrFold xf;
  StopFold fold_op;
  if (fuse_xr && fold_in) {  // iteration it - 1 left its x, r update to this iteration
    xf = XrFold{ctx->x, ctx->r, p_loc, ctx->q, pq_part(ctx), rr_part(ctx), ctx->st};
    fold_op = fold;
    fold = StopFold{};
  }
  // symmetric tiles + low-rank apply (configs[2]): p = z + beta p formed by the tile workgroups
  // (k_symv_dyn, PGather with one rank) and written by the slot reduction -- k_update_p's bits,
  // one launch less; the apply writes z and its rho partials into the gather block for it
  const bool fuse_p1 = ctx->fuse_p && ctx->use_sym && lowrank && ctx->sym.dyn > 0 &&
                       ctx->sym.ntiles > 0 && !ctx->exact_sums;
  double *zout = fuse_p1 ? ctx->gb : ctx->z;
  double *rhoout = fuse_p1 ? ctx->gb + ctx->blk : rho_part(ctx);
  const double *zsrc;
  if (lowrank) {
    const size_t pm = mark_begin(ctx, marks);
    if (ctx->exact_sums) {  // measurement anchor: two double-double passes, rho separately
      if (fold.st != nullptr) launch_stoptest(rr_part(ctx), ctx->st, ctx->trace, it - 1, s);
      launch_dd_lowrank(ctx->T, ctx->blk, ctx->k, ctx->r, ctx->z, ctx->nrows, ctx->sigma_p,
                        1.0 / ctx->lam, ctx->tpart, status, s);
      launch_dot_part(ctx->r, ctx->z, ctx->nrows, rho_part(ctx), status, s);
    } else if (ctx->lr_rows) {
      launch_lr_apply_rows(ctx->T, ctx->blk, ctx->k, ctx->r, zout, ctx->nrows, ctx->sigma_p,
                           1.0 / ctx->lam, rhoout, status, s, ctx->lr_zpart, fold, xf);
    } else if (ctx->lr_cluster) {
      launch_lr_apply_cluster(ctx->T, ctx->blk, ctx->k, ctx->lr_q, ctx->r, zout, ctx->nrows,
                              ctx->sigma_p, 1.0 / ctx->lam, rhoout, status, s,
                              ctx->lr_zpart, ctx->lr_slots, next_lr_epoch(ctx), &ctx->st->status,
                              fold);
    } else {
      launch_gemv_split(ctx->T, ctx->blk, ctx->k, ctx->blk, ctx->tsplit, ctx->r, ctx->tpart, status,
                        s, fold);
      launch_precon_z(ctx->T, ctx->blk, ctx->k, ctx->tsplit, ctx->tpart, ctx->r, zout, ctx->nrows,
                      ctx->sigma_p, 1.0 / ctx->lam, rhoout, status, s, ctx->zpart, ctx->zsplit);
    }
    mark_end(ctx, marks, pm, it, 1);
    zsrc = zout;
  } else {
    launch_dot_part(ctx->r, ctx->r, ctx->nrows, rho_part(ctx), status, s, fold);
    zsrc = ctx->r;
  }
  const PFuse pf{zsrc, rho_part(ctx), ctx->st, it, fold_op};
  if (!fuse_p && !fuse_p1)
    launch_update_p(zsrc, p_loc, ctx->nrows, rho_part(ctx), ctx->st, it, status, s);
  const size_t e0 = mark_begin(ctx, marks);
  if (ctx->use_sym) {
    // q = sigma K p + lam p and the p.q partials from the slot reduction (no dot launch)
    const PGather pg1 = fuse_p1 ? PGather{ctx->gb, ctx->gstride, ctx->blk, 1, ctx->st, it}
                                : PGather{};
    launch_symv(ctx->sym, ctx->p_full, ctx->sym.P, status, s, pg1);
    launch_sym_reduce_pq(ctx->sym, ctx->nrows, ctx->q, ctx->sigma_K, ctx->lam, p_loc,
                         pq_part(ctx), status, s, pg1);
    mark_end(ctx, marks, e0, it);
  } else {
    MLFF_TRY(launch_operator(ctx, ctx->p_full, ctx->q, p_loc, status, pq_part(ctx),
                             fuse_p ? &pf : nullptr));
    mark_end(ctx, marks, e0, it);
  }
  if (!fuse_xr || stop_out)  // else: done by iteration it + 1 (same chunk, fold_in)
    launch_update_xr(ctx->x, ctx->r, p_loc, ctx->q, ctx->nrows, pq_part(ctx), rr_part(ctx), ctx->st,
                     status, s);
  if (stop_out) launch_stoptest(rr_part(ctx), ctx->st, ctx->trace, it, s);
  return MLFF_OK;
}

// true-residual recheck of the python wrapper: r = b - A x, resid = ||r||
int do_recheck(mlff_ctx *ctx) {
  hipStream_t s = ctx->stream;
  MLFF_HIP(ctx, hipMemcpyAsync(ctx->xg + (int64_t)ctx->rank * ctx->blk, ctx->x,
                               sizeof(double) * ctx->blk, hipMemcpyDeviceToDevice, s));
  MLFF_TRY(allgather_blocks(ctx, ctx->xg));
  MLFF_TRY(launch_operator(ctx, ctx->xg, ctx->q, ctx->x, nullptr));
  launch_residual(ctx->b, ctx->q, ctx->r, ctx->nrows, rr_part(ctx), s);
  MLFF_TRY(allreduce(ctx, rr_part(ctx), kVecGrid));
  launch_recheck_finish(rr_part(ctx), ctx->st, ctx->trace, s);
  MLFF_HIP(ctx, hipGetLastError());
  return MLFF_OK;
}

int poll_state(mlff_ctx *ctx) {
  MLFF_HIP(ctx, hipMemcpyAsync(ctx->h_st, ctx->st, sizeof(DevState), hipMemcpyDeviceToHost,
                               ctx->stream));
  MLFF_HIP(ctx, hipStreamSynchronize(ctx->stream));
  return MLFF_OK;
}

}  // namespace

extern "C" {

int mlff_version(void) { return 100; }

int mlff_device_count(int *n_out) {
  MLFF_API_BEGIN
  if (n_out == nullptr) return set_error(nullptr, MLFF_ERR_ARG, "null pointer");
  int n = 0;
  const hipError_t e = hipGetDeviceCount(&n);
  if (e != hipSuccess) {
    *n_out = 0;
    return hip_check(nullptr, e, "hipGetDeviceCount");
  }
  *n_out = n;
  return MLFF_OK;
  MLFF_API_END(nullptr)
}

int mlff_comm_unique_id(unsigned char id_out[128]) {
  MLFF_API_BEGIN
  if (id_out == nullptr) return set_error(nullptr, MLFF_ERR_ARG, "null pointer");
  ncclUniqueId id;
  MLFF_NCCL(nullptr, ncclGetUniqueId(&id));
  static_assert(sizeof(ncclUniqueId) == 128, "ncclUniqueId size");
  std::memcpy(id_out, &id, 128);
  return MLFF_OK;
  MLFF_API_END(nullptr)
}

int mlff_comm_selftest(int device, int64_t count, double *max_err_out) {
  MLFF_API_BEGIN
  if (max_err_out == nullptr || count < 1) return set_error(nullptr, MLFF_ERR_ARG, "bad arguments");
  *max_err_out = -1.0;
  int ndev = 0;
  if (hipGetDeviceCount(&ndev) != hipSuccess || device < 0 || device >= ndev)
    return set_error(nullptr, MLFF_ERR_ARG, "bad device id");
  // every exit (error returns of the MLFF_HIP checks, exceptions caught by MLFF_API_END)
  // releases the buffers, the communicator, the stream and the context
  struct Owned {
    mlff_ctx *ctx = new mlff_ctx();
    double *a = nullptr, *b = nullptr;
    ~Owned() {
      dev_free(a);
      dev_free(b);
      mlff_ctx_destroy(ctx);
    }
  } own;
  mlff_ctx *ctx = own.ctx;
  ctx->device = device;
  ctx->rank = 0;
  ctx->world = 1;
  double *&a = own.a, *&b = own.b;
  if (hipSetDevice(device) != hipSuccess || hipStreamCreateWithFlags(&ctx->stream, hipStreamNonBlocking) != hipSuccess)
    return set_error(nullptr, MLFF_ERR_HIP, "stream create failed");
  ncclUniqueId id;
  ncclResult_t e = ncclGetUniqueId(&id);
  if (e == ncclSuccess) e = ncclCommInitRank(&ctx->comm, 1, id, 0);
  if (e != ncclSuccess) {
    ctx->comm = nullptr;
    return set_error(nullptr, MLFF_ERR_COMM, std::string("ncclCommInitRank: ") + ncclGetErrorString(e));
  }
  const size_t n = (size_t)count;
  if (hipMalloc(&a, sizeof(double) * n) != hipSuccess || hipMalloc(&b, sizeof(double) * n) != hipSuccess)
    return set_error(nullptr, MLFF_ERR_NOMEM, "device allocation failed");
  std::vector<double> h(n);
  double worst = 0.0;
  // every collective sits between a producing kernel and a consuming copy on the same stream
  // (no host synchronisation in between), so a transport that ran off-stream would read the
  // input before it is written or leave the poisoned output in place
  auto check = [&](const double *src, double scale) -> int {
    MLFF_HIP(ctx, hipMemcpyAsync(h.data(), src, sizeof(double) * n, hipMemcpyDeviceToHost, ctx->stream));
    MLFF_HIP(ctx, hipStreamSynchronize(ctx->stream));
    for (size_t i = 0; i < n; ++i) {
      const double d = std::fabs(h[i] - scale * (1.0 + 0.5 * (double)i));
      worst = std::isfinite(d) ? std::max(worst, d) : INFINITY;
    }
    return MLFF_OK;
  };
  auto fill = [&](double *p, double scale) {
    hipLaunchKernelGGL(k_selftest_fill, dim3(256), dim3(256), 0, ctx->stream, p, n, scale);
  };
  auto poison = [&](double *p) { return hipMemsetAsync(p, 0xff, sizeof(double) * n, ctx->stream); };
  // allreduce in place
  fill(a, 1.0);
  if (int rc = rccl_allreduce(ctx, a, n)) return rc;
  if (int rc = check(a, 1.0)) return rc;
  // allgather out of place, then in place (send == recv + rank * count)
  fill(a, 2.0);
  MLFF_HIP(ctx, poison(b));
  if (int rc = rccl_allgather(ctx, a, b, n)) return rc;
  if (int rc = check(b, 2.0)) return rc;
  fill(b, 3.0);
  if (int rc = rccl_allgather(ctx, b, b, n)) return rc;
  if (int rc = check(b, 3.0)) return rc;
  // reduce-scatter out of place
  fill(b, 4.0);
  MLFF_HIP(ctx, poison(a));
  if (int rc = rccl_reduce_scatter(ctx, b, a, n)) return rc;
  if (int rc = check(a, 4.0)) return rc;
  *max_err_out = worst;
  return MLFF_OK;
  MLFF_API_END(nullptr)
}

const char *mlff_last_error(mlff_ctx *ctx) {
  if (ctx != nullptr) return ctx->err.c_str();
  return g_last_error.c_str();
}

int mlff_ctx_create(int device, int rank, int world, const unsigned char *comm_id,
                    int64_t n_global, mlff_ctx **ctx_out) {
  MLFF_API_BEGIN
  if (ctx_out == nullptr) return set_error(nullptr, MLFF_ERR_ARG, "null ctx_out");
  *ctx_out = nullptr;
  if (world < 1 || rank < 0 || rank >= world) return set_error(nullptr, MLFF_ERR_ARG, "bad rank/world");
  if (n_global < 1) return set_error(nullptr, MLFF_ERR_ARG, "N must be >= 1");
  if (world > 1 && comm_id == nullptr) return set_error(nullptr, MLFF_ERR_ARG, "comm_id required for world > 1");
  int ndev = 0;
  if (hipGetDeviceCount(&ndev) != hipSuccess || ndev < 1)
    return set_error(nullptr, MLFF_ERR_HIP, "no HIP device available");
  if (device < 0 || device >= ndev) return set_error(nullptr, MLFF_ERR_ARG, "bad device id");
  if (world > 1 && std::getenv("MLFF_EXACT_SUMS") != nullptr && std::atoi(std::getenv("MLFF_EXACT_SUMS")) != 0)
    return set_error(nullptr, MLFF_ERR_ARG, "MLFF_EXACT_SUMS runs on one rank");
  mlff_ctx *ctx = new mlff_ctx();
  ctx->device = device;
  for (auto [name, flag] : {std::pair<const char *, bool *>{"MLFF_FUSE_P", &ctx->fuse_p},
                            std::pair<const char *, bool *>{"MLFF_FUSE_XR", &ctx->fuse_xr},
                            std::pair<const char *, bool *>{"MLFF_CHO_FAST", &ctx->cho_fast}}) {
    const char *e = std::getenv(name);
    *flag = e == nullptr || std::atoi(e) != 0;
  }
  if (const char *e = std::getenv("MLFF_FUSE_XR_RANKS")) ctx->fuse_xr_ranks = std::atoi(e) != 0;
  if (const char *e = std::getenv("MLFF_PQ_PUBLISH")) ctx->pq_publish = std::atoi(e) != 0;
  if (const char *e = std::getenv("MLFF_WB_REFINE")) ctx->wb_refine = std::max(0, std::atoi(e));
  if (const char *e = std::getenv("MLFF_NYS_REFINE")) ctx->nys_refine = std::atoi(e) != 0;
  if (const char *e = std::getenv("MLFF_WB_GRAM")) ctx->wb_gram_dd = std::max(0, std::min(2, std::atoi(e)));
  if (const char *e = std::getenv("MLFF_EXACT_SUMS")) ctx->exact_sums = std::atoi(e) != 0;
  ctx->rank = rank;
  ctx->world = world;
  ctx->N = n_global;
  ctx->rows_per = (n_global + world - 1) / world;
  ctx->row0 = std::min<int64_t>((int64_t)rank * ctx->rows_per, n_global);
  ctx->nrows = std::max<int64_t>(0, std::min<int64_t>(ctx->rows_per, n_global - ctx->row0));
  // world > 1: rank blocks hold whole tiles of the symmetric operator
  ctx->blk = round_up(ctx->rows_per, world > 1 ? kSymTile : kPad);
  ctx->ld = (int64_t)world * ctx->blk;
  auto fail = [&](int rc) {
    mlff_ctx_destroy(ctx);
    return rc;
  };
  if (hipSetDevice(device) != hipSuccess) return fail(set_error(nullptr, MLFF_ERR_HIP, "hipSetDevice failed"));
  if (hipStreamCreateWithFlags(&ctx->stream, hipStreamNonBlocking) != hipSuccess)
    return fail(set_error(nullptr, MLFF_ERR_HIP, "hipStreamCreate failed"));
  if (world > 1 && std::memcmp(comm_id, "SOLO:", 5) == 0) {
    ctx->solo = true;
  } else if (world > 1 && std::memcmp(comm_id, "LOCAL:", 6) == 0) {
    const std::string key((const char *)comm_id, strnlen((const char *)comm_id, 128));
    ctx->local = join_local_group(key, world);
    if (ctx->local->world != world) return fail(set_error(nullptr, MLFF_ERR_ARG, "LOCAL group size mismatch"));
  } else if (world > 1) {
    ncclUniqueId id;
    std::memcpy(&id, comm_id, 128);
    const ncclResult_t e = ncclCommInitRank(&ctx->comm, world, id, rank);
    if (e != ncclSuccess) {
      ctx->comm = nullptr;
      return fail(set_error(nullptr, MLFF_ERR_COMM, std::string("ncclCommInitRank: ") + ncclGetErrorString(e)));
    }
  }
  double **vecs[] = {&ctx->x, &ctx->r, &ctx->z, &ctx->q, &ctx->b};
  for (double **v : vecs) {
    if (hipMalloc(v, sizeof(double) * ctx->blk) != hipSuccess) return fail(set_error(nullptr, MLFF_ERR_NOMEM, "alloc"));
    hipMemset(*v, 0, sizeof(double) * ctx->blk);
  }
  // full-length operands are padded to whole tiles (entries >= ld stay zero)
  const int64_t ldp = round_up(ctx->ld, kSymTile);
  if (hipMalloc(&ctx->p_full, sizeof(double) * ldp) != hipSuccess ||
      hipMalloc(&ctx->xg, sizeof(double) * ldp) != hipSuccess ||
      hipMalloc(&ctx->part, sizeof(double) * 4 * kMaxPart) != hipSuccess ||
      hipMalloc(&ctx->st, sizeof(DevState)) != hipSuccess ||
      hipHostMalloc(&ctx->h_st, sizeof(DevState)) != hipSuccess ||
      hipMalloc(&ctx->dwork, sizeof(double) * ctx->blk) != hipSuccess ||
      hipMalloc(&ctx->pivflag, sizeof(int) * ctx->blk) != hipSuccess ||
      hipMalloc(&ctx->perm, sizeof(int64_t) * n_global) != hipSuccess)
    return fail(set_error(nullptr, MLFF_ERR_NOMEM, "device allocation failed"));
  {
    // the gather buffer: z | rho partials per rank (one rank: the fused tile iteration's operand)
    ctx->gstride = ctx->blk + kVecGrid;
    if (hipMalloc(&ctx->gb, sizeof(double) * world * ctx->gstride) != hipSuccess)
      return fail(set_error(nullptr, MLFF_ERR_NOMEM, "device allocation failed"));
    hipMemset(ctx->gb, 0, sizeof(double) * world * ctx->gstride);
  }
  hipMemset(ctx->p_full, 0, sizeof(double) * ldp);
  hipMemset(ctx->xg, 0, sizeof(double) * ldp);
  hipMemset(ctx->part, 0, sizeof(double) * 4 * kMaxPart);
  hipMemset(ctx->st, 0, sizeof(DevState));
  std::memset(ctx->h_st, 0, sizeof(DevState));
  if (hipDeviceSynchronize() != hipSuccess) return fail(set_error(nullptr, MLFF_ERR_HIP, "init sync failed"));
  *ctx_out = ctx;
  return MLFF_OK;
  MLFF_API_END(nullptr)
}

int mlff_ctx_destroy(mlff_ctx *ctx) {
  MLFF_API_BEGIN
  if (ctx == nullptr) return MLFF_OK;
  hipSetDevice(ctx->device);
  if (ctx->stream) hipStreamSynchronize(ctx->stream);
  for (void *p : {(void *)ctx->K, (void *)ctx->x, (void *)ctx->r, (void *)ctx->z, (void *)ctx->q,
                  (void *)ctx->b, (void *)ctx->p_full, (void *)ctx->xg, (void *)ctx->part,
                  (void *)ctx->st, (void *)ctx->trace, (void *)ctx->T, (void *)ctx->tpart_base,
                  (void *)ctx->perm, (void *)ctx->dwork, (void *)ctx->pivflag, (void *)ctx->prow, (void *)ctx->zpart, (void *)ctx->lr_zpart, (void *)ctx->lr_slots, (void *)ctx->lr_fault, (void *)ctx->gb})
    dev_free(p);
  for (const auto &c : ctx->scratch_chunks) dev_free(c.p);
  ctx->scratch_chunks.clear();
  sym_free(ctx->sym);
  mf_free(ctx->mf);
  rbf_free(ctx);
  if (ctx->h_st) hipHostFree(ctx->h_st);
  for (hipEvent_t e : ctx->timing.ev) hipEventDestroy(e);
  if (ctx->comm) ncclCommDestroy(ctx->comm);
  ctx->local.reset();
  if (ctx->stream) hipStreamDestroy(ctx->stream);
  delete ctx;
  return MLFF_OK;
  MLFF_API_END(ctx)
}

int mlff_comm_abort(mlff_ctx *ctx) {
  MLFF_API_BEGIN
  if (ctx == nullptr) return set_error(nullptr, MLFF_ERR_ARG, "null ctx");
  ctx->aborted = true;
  if (ctx->local) ctx->local->abort();
  if (ctx->comm != nullptr) {
    (void)hipSetDevice(ctx->device);
    ncclCommAbort(ctx->comm);
    ctx->comm = nullptr;
  }
  return MLFF_OK;
  MLFF_API_END(ctx)
}

int mlff_shard_range(mlff_ctx *ctx, int64_t *row0_out, int64_t *nrows_out) {
  MLFF_API_BEGIN
  MLFF_ENTER(ctx);
  if (row0_out) *row0_out = ctx->row0;
  if (nrows_out) *nrows_out = ctx->nrows;
  return MLFF_OK;
  MLFF_API_END(ctx)
}

int mlff_matrix_ld(mlff_ctx *ctx, int64_t *ld_out) {
  MLFF_API_BEGIN
  if (ctx == nullptr || ld_out == nullptr) return set_error(ctx, MLFF_ERR_ARG, "null pointer");
  *ld_out = ctx->ld;
  return MLFF_OK;
  MLFF_API_END(ctx)
}

int mlff_synchronize(mlff_ctx *ctx) {
  MLFF_API_BEGIN
  MLFF_ENTER(ctx);
  MLFF_HIP(ctx, hipStreamSynchronize(ctx->stream));
  return MLFF_OK;
  MLFF_API_END(ctx)
}

int mlff_stream(mlff_ctx *ctx, void **stream_out) {
  MLFF_API_BEGIN
  if (ctx == nullptr || stream_out == nullptr) return set_error(ctx, MLFF_ERR_ARG, "null pointer");
  *stream_out = (void *)ctx->stream;
  return MLFF_OK;
  MLFF_API_END(ctx)
}

int mlff_set_matrix_host(mlff_ctx *ctx, const double *K_local, int64_t ld_host) {
  MLFF_API_BEGIN
  MLFF_ENTER(ctx);
  if (K_local == nullptr && ctx->nrows > 0) return set_error(ctx, MLFF_ERR_ARG, "null K");
  if (ld_host < ctx->N) return set_error(ctx, MLFF_ERR_ARG, "ld_host < N");
  MLFF_TRY(ensure_matrix(ctx));
  MLFF_HIP(ctx, hipMemsetAsync(ctx->K, 0, sizeof(double) * ctx->blk * ctx->ld, ctx->stream));
  for (int r = 0; r < ctx->world && ctx->nrows > 0; ++r) {
    const int64_t g0 = (int64_t)r * ctx->rows_per;
    if (g0 >= ctx->N) break;
    const int64_t cnt = std::min<int64_t>(ctx->rows_per, ctx->N - g0);
    MLFF_HIP(ctx, hipMemcpy2DAsync(ctx->K + (int64_t)r * ctx->blk, sizeof(double) * ctx->ld,
                                   K_local + g0, sizeof(double) * ld_host, sizeof(double) * cnt,
                                   ctx->nrows, hipMemcpyHostToDevice, ctx->stream));
  }
  MLFF_HIP(ctx, hipStreamSynchronize(ctx->stream));
  ctx->has_matrix = true;
  ctx->K_symmetric = false;
  ctx->sym.ready = false;
  mf_free(ctx->mf);
  rbf_free(ctx);
  return MLFF_OK;
  MLFF_API_END(ctx)
}

int mlff_get_matrix_rows(mlff_ctx *ctx, int64_t r0, int64_t nr, double *out, int64_t ld_out) {
  MLFF_API_BEGIN
  MLFF_ENTER(ctx);
  if (out == nullptr) return set_error(ctx, MLFF_ERR_ARG, "null pointer");
  if (!ctx->has_matrix && !ctx->rbf.ready) return set_error(ctx, MLFF_ERR_STATE, "no kernel matrix set");
  if (r0 < 0 || nr < 0 || r0 + nr > ctx->nrows || ld_out < ctx->N)
    return set_error(ctx, MLFF_ERR_ARG, "row range / ld_out");
  // rows of the dense K, or of the RBF source generated chunk-wise into scratch
  ScratchScope scope(ctx);
  const int64_t chunk = ctx->has_matrix ? nr : std::max<int64_t>(1, std::min<int64_t>(nr, (int64_t)(256e6 / (8.0 * ctx->ld))));
  double *tmp = nullptr;
  if (!ctx->has_matrix) MLFF_TRY(scratch_alloc(ctx, &tmp, (size_t)chunk * ctx->ld));
  for (int64_t c0 = 0; c0 < nr; c0 += chunk) {
    const int64_t cn = std::min<int64_t>(chunk, nr - c0);
    const double *src = ctx->K + (r0 + c0) * ctx->ld;
    if (!ctx->has_matrix) {
      launch_gen_rbf(tmp, ctx->ld, cn, ctx->row0 + r0 + c0, ctx->rows_per, ctx->blk, ctx->N,
                     ctx->rbf.Xs, ctx->rbf.d, ctx->rbf.jitter, ctx->stream);
      MLFF_HIP(ctx, hipGetLastError());
      src = tmp;
    }
    for (int r = 0; r < ctx->world; ++r) {
      const int64_t g0 = (int64_t)r * ctx->rows_per;
      if (g0 >= ctx->N) break;
      const int64_t cnt = std::min<int64_t>(ctx->rows_per, ctx->N - g0);
      MLFF_HIP(ctx, hipMemcpy2DAsync(out + c0 * ld_out + g0, sizeof(double) * ld_out,
                                     src + (int64_t)r * ctx->blk, sizeof(double) * ctx->ld,
                                     sizeof(double) * cnt, cn, hipMemcpyDeviceToHost, ctx->stream));
    }
    MLFF_HIP(ctx, hipStreamSynchronize(ctx->stream));
  }
  return MLFF_OK;
  MLFF_API_END(ctx)
}

int mlff_gen_rbf(mlff_ctx *ctx, const double *X, int d, double length_scale, double jitter) {
  MLFF_API_BEGIN
  MLFF_ENTER(ctx);
  if (X == nullptr || d < 1 || d > 8 || !(length_scale > 0.0))
    return set_error(ctx, MLFF_ERR_ARG, "gen_rbf: need X, 1 <= d <= 8, length_scale > 0");
  // the points (scaled as sklearn does, X / length_scale) are the kernel: tiles, columns,
  // diagonal and (for the DENSE storage only) the rows are evaluated from them on device
  std::vector<double> Xs((size_t)ctx->N * d);
  for (size_t i = 0; i < Xs.size(); ++i) Xs[i] = X[i] / length_scale;
  sym_free(ctx->sym);
  mf_free(ctx->mf);
  rbf_free(ctx);
  if (ctx->K != nullptr) {  // a dense matrix set earlier is not this kernel
    (void)hipFree(ctx->K);
    ctx->K = nullptr;
  }
  ctx->has_matrix = false;
  MLFF_HIP(ctx, hipMalloc(&ctx->rbf.Xs, sizeof(double) * Xs.size()));
  MLFF_HIP(ctx, hipMemcpy(ctx->rbf.Xs, Xs.data(), sizeof(double) * Xs.size(), hipMemcpyHostToDevice));
  ctx->rbf.d = d;
  ctx->rbf.jitter = jitter;
  ctx->rbf.ready = true;
  ctx->K_symmetric = true;
  return MLFF_OK;
  MLFF_API_END(ctx)
}

int mlff_assemble_sgdml(mlff_ctx *ctx, const double *R_desc, const double *R_d_desc, int64_t M,
                        int n_atoms, const int32_t *perms, int n_perms, double sig) {
  MLFF_API_BEGIN
  MLFF_ENTER(ctx);
  if (R_desc == nullptr || R_d_desc == nullptr || perms == nullptr || !(sig > 0.0))
    return set_error(ctx, MLFF_ERR_ARG, "assemble_sgdml: null input or sig <= 0");
  rbf_free(ctx);
  MLFF_TRY(ensure_matrix(ctx));
  MLFF_TRY(assemble_sgdml(ctx, R_desc, R_d_desc, M, n_atoms, perms, n_perms, sig));
  // the matrix-free form of the same operator (chosen by MLFF_STORAGE_AUTO when cheaper)
  MLFF_TRY(mf_setup(ctx, R_desc, R_d_desc, M, n_atoms, perms, n_perms, sig));
  ctx->has_matrix = true;
  ctx->K_symmetric = true;  // the assembly mirrors the lower block triangle
  ctx->sym.ready = false;
  return MLFF_OK;
  MLFF_API_END(ctx)
}

int mlff_sgdml_operator(mlff_ctx *ctx, const double *R_desc, const double *R_d_desc, int64_t M,
                        int n_atoms, const int32_t *perms, int n_perms, double sig) {
  MLFF_API_BEGIN
  MLFF_ENTER(ctx);
  if (R_desc == nullptr || R_d_desc == nullptr || perms == nullptr || !(sig > 0.0))
    return set_error(ctx, MLFF_ERR_ARG, "sgdml_operator: null input or sig <= 0");
  rbf_free(ctx);
  MLFF_TRY(mf_setup(ctx, R_desc, R_d_desc, M, n_atoms, perms, n_perms, sig));
  ctx->use_mf = false;
  ctx->has_matrix = false;  // a dense K set earlier is not this operator
  ctx->sym.ready = false;
  return MLFF_OK;
  MLFF_API_END(ctx)
}

int mlff_test_gemm(mlff_ctx *ctx, int ta, int tb, int64_t M, int64_t N, int64_t K, double alpha,
                   const double *A, int64_t lda, const double *B, int64_t ldb, double beta,
                   double *C, int64_t ldc, int splits) {
  MLFF_API_BEGIN
  MLFF_ENTER(ctx);
  if (A == nullptr || B == nullptr || C == nullptr || M < 0 || N < 0 || K < 0 || splits < 1 ||
      lda < (ta ? M : K) || ldb < (tb ? K : N) || ldc < N)
    return set_error(ctx, MLFF_ERR_ARG, "test_gemm: bad arguments");
  return test_gemm(ctx, ta, tb, M, N, K, alpha, A, lda, B, ldb, beta, C, ldc, splits);
  MLFF_API_END(ctx)
}

int mlff_test_gram(mlff_ctx *ctx, const double *W, int64_t k, int64_t ncols, int mode,
                   double *G_out) {
  MLFF_API_BEGIN
  MLFF_ENTER(ctx);
  if (W == nullptr || G_out == nullptr || k < 1 || ncols < 1 || mode < 0 || mode > 2)
    return set_error(ctx, MLFF_ERR_ARG, "test_gram: bad arguments");
  ScratchScope scope(ctx);
  double *dW = nullptr, *dG = nullptr;
  MLFF_TRY(scratch_alloc(ctx, &dW, (size_t)(k * ncols)));
  MLFF_TRY(scratch_alloc(ctx, &dG, (size_t)(k * k)));
  MLFF_HIP(ctx, hipMemcpyAsync(dW, W, sizeof(double) * k * ncols, hipMemcpyHostToDevice, ctx->stream));
  if (mode == 0)
    MLFF_TRY(syrk_wide(ctx, dW, k, ncols, ncols, dG));
  else
    MLFF_TRY(gram_wide_dd(ctx, dW, k, ncols, ncols, dG, mode == 2));
  MLFF_HIP(ctx, hipMemcpyAsync(G_out, dG, sizeof(double) * k * k, hipMemcpyDeviceToHost, ctx->stream));
  MLFF_HIP(ctx, hipStreamSynchronize(ctx->stream));
  return MLFF_OK;
  MLFF_API_END(ctx)
}

int mlff_sym_min_eig(mlff_ctx *ctx, const double *M, int64_t m, double *lo_eig_out,
                     double *d_out, double *e_out) {
  MLFF_API_BEGIN
  MLFF_ENTER(ctx);
  if (M == nullptr || m < 1 || lo_eig_out == nullptr)
    return set_error(ctx, MLFF_ERR_ARG, "sym_min_eig: bad arguments");
  ScratchScope scope(ctx);
  double *dM = nullptr;
  MLFF_TRY(scratch_alloc(ctx, &dM, (size_t)(m * m)));
  MLFF_HIP(ctx, hipMemcpyAsync(dM, M, sizeof(double) * m * m, hipMemcpyHostToDevice, ctx->stream));
  return sym_min_eig(ctx, dM, m, lo_eig_out, d_out, e_out);
  MLFF_API_END(ctx)
}

int mlff_cho_factor_stable(mlff_ctx *ctx, const double *M, int64_t m, double *L_out,
                           double *lo_eig_out) {
  MLFF_API_BEGIN
  MLFF_ENTER(ctx);
  if (M == nullptr || m < 1 || L_out == nullptr)
    return set_error(ctx, MLFF_ERR_ARG, "cho_factor_stable: bad arguments");
  ScratchScope scope(ctx);
  double *dM = nullptr;
  MLFF_TRY(scratch_alloc(ctx, &dM, (size_t)(m * m)));
  MLFF_HIP(ctx, hipMemcpyAsync(dM, M, sizeof(double) * m * m, hipMemcpyHostToDevice, ctx->stream));
  MLFF_TRY(cho_factor_stable(ctx, dM, m, lo_eig_out));
  MLFF_HIP(ctx, hipMemcpyAsync(L_out, dM, sizeof(double) * m * m, hipMemcpyDeviceToHost, ctx->stream));
  MLFF_HIP(ctx, hipStreamSynchronize(ctx->stream));
  return MLFF_OK;
  MLFF_API_END(ctx)
}

int mlff_spectrum(mlff_ctx *ctx, int preconditioned, double *eig_out) {
  MLFF_API_BEGIN
  MLFF_ENTER(ctx);
  if (eig_out == nullptr) return set_error(ctx, MLFF_ERR_ARG, "null pointer");
  MLFF_TRY(require_operator(ctx));
  return spectrum(ctx, preconditioned != 0, eig_out);
  MLFF_API_END(ctx)
}

int mlff_set_energy_constraints(mlff_ctx *ctx, int use_E_cstr) {
  MLFF_API_BEGIN
  MLFF_ENTER(ctx);
  if (use_E_cstr && ctx->world > 1)
    return set_error(ctx, MLFF_ERR_ARG, "use_E_cstr: energy constraints run on one rank");
  ctx->use_E_cstr = use_E_cstr != 0;
  return MLFF_OK;
  MLFF_API_END(ctx)
}

int mlff_sgdml_descriptors(const double *R, int64_t M, int n_atoms, double *R_desc_out,
                           double *R_d_desc_out) {
  MLFF_API_BEGIN
  if (R == nullptr || R_desc_out == nullptr || R_d_desc_out == nullptr || M < 1 || n_atoms < 2)
    return set_error(nullptr, MLFF_ERR_ARG, "sgdml_descriptors: bad arguments");
  const int rc = sgdml_descriptors(R, M, n_atoms, R_desc_out, R_d_desc_out);
  if (rc != MLFF_OK) return set_error(nullptr, rc, "sgdml_descriptors: HIP failure");
  return MLFF_OK;
  MLFF_API_END(nullptr)
}

int mlff_sgdml_energies(mlff_ctx *ctx, const double *alphas, double *E_out, int64_t *i0_out,
                        int64_t *ni_out) {
  MLFF_API_BEGIN
  MLFF_ENTER(ctx);
  if (alphas == nullptr || E_out == nullptr) return set_error(ctx, MLFF_ERR_ARG, "null pointer");
  if (!ctx->mf.ready) return set_error(ctx, MLFF_ERR_STATE, "no sGDML operator set");
  const MfData &mf = ctx->mf;
  const int64_t MP = mf.M * mf.n_perms;
  std::vector<double> pairs((size_t)std::max<int64_t>(mf.ni, 1) * MP);
  MLFF_TRY(mf_energies(ctx, alphas, pairs.data()));
  for (int64_t i = 0; i < mf.ni; ++i) {
    double e = 0.0;
    for (int64_t jp = 0; jp < MP; ++jp) e += pairs[(size_t)i * MP + jp];
    E_out[i] = e;
  }
  if (i0_out) *i0_out = mf.i0;
  if (ni_out) *ni_out = mf.ni;
  return MLFF_OK;
  MLFF_API_END(ctx)
}

int mlff_set_operator(mlff_ctx *ctx, double sigma_K, double lam) {
  MLFF_API_BEGIN
  MLFF_ENTER(ctx);
  if (!(lam > 0.0)) return set_error(ctx, MLFF_ERR_ARG, "lam must be > 0");
  if (sigma_K != 1.0 && sigma_K != -1.0) return set_error(ctx, MLFF_ERR_ARG, "sigma_K must be +-1");
  ctx->sigma_K = sigma_K;
  ctx->lam = lam;
  ctx->has_operator = true;
  return MLFF_OK;
  MLFF_API_END(ctx)
}

int mlff_set_storage(mlff_ctx *ctx, int mode) {
  MLFF_API_BEGIN
  MLFF_ENTER(ctx);
  if (mode != MLFF_STORAGE_DENSE && mode != MLFF_STORAGE_SYMTILE && mode != MLFF_STORAGE_AUTO &&
      mode != MLFF_STORAGE_MATFREE)
    return set_error(ctx, MLFF_ERR_ARG, "bad storage mode");
  if (mode != ctx->storage) {
    ctx->storage = mode;
    ctx->use_sym = false;
    ctx->use_mf = false;
    if (mode == MLFF_STORAGE_DENSE || mode == MLFF_STORAGE_MATFREE) sym_free(ctx->sym);
  }
  return MLFF_OK;
  MLFF_API_END(ctx)
}

int mlff_operator_form(mlff_ctx *ctx, int *form_out) {
  MLFF_API_BEGIN
  MLFF_ENTER(ctx);
  if (form_out == nullptr) return set_error(ctx, MLFF_ERR_ARG, "null form_out");
  *form_out = ctx->mf.ready ? mf_form(ctx) : -1;
  return MLFF_OK;
  MLFF_API_END(ctx)
}

int mlff_storage_info(mlff_ctx *ctx, int *mode_out, double *bytes_per_matvec_out) {
  MLFF_API_BEGIN
  MLFF_ENTER(ctx);
  MLFF_TRY(require_operator(ctx));
  MLFF_TRY(resolve_storage(ctx));
  if (mode_out)
    *mode_out = ctx->use_mf ? MLFF_STORAGE_MATFREE
                            : (ctx->use_sym ? MLFF_STORAGE_SYMTILE : MLFF_STORAGE_DENSE);
  if (bytes_per_matvec_out) *bytes_per_matvec_out = operator_bytes(ctx);
  return MLFF_OK;
  MLFF_API_END(ctx)
}

int mlff_matvec(mlff_ctx *ctx, const double *v_global, double *y_local) {
  MLFF_API_BEGIN
  MLFF_ENTER(ctx);
  MLFF_TRY(require_operator(ctx));
  if (v_global == nullptr || (y_local == nullptr && ctx->nrows > 0)) return set_error(ctx, MLFF_ERR_ARG, "null vector");
  MLFF_TRY(resolve_storage(ctx));
  MLFF_TRY(scatter_global(ctx, v_global, ctx->xg));
  MLFF_TRY(launch_operator(ctx, ctx->xg, ctx->q, ctx->xg + (int64_t)ctx->rank * ctx->blk, nullptr));
  MLFF_HIP(ctx, hipGetLastError());
  if (ctx->nrows > 0)
    MLFF_HIP(ctx, hipMemcpyAsync(y_local, ctx->q, sizeof(double) * ctx->nrows, hipMemcpyDeviceToHost, ctx->stream));
  MLFF_HIP(ctx, hipStreamSynchronize(ctx->stream));
  return MLFF_OK;
  MLFF_API_END(ctx)
}

int mlff_get_diag(mlff_ctx *ctx, double *diag_local) {
  MLFF_API_BEGIN
  MLFF_ENTER(ctx);
  if (!ctx->has_matrix && !ctx->mf.ready && !ctx->rbf.ready)
    return set_error(ctx, MLFF_ERR_STATE, "no kernel matrix set");
  MLFF_TRY(operator_diag(ctx, ctx->dwork));
  if (ctx->nrows > 0)
    MLFF_HIP(ctx, hipMemcpyAsync(diag_local, ctx->dwork, sizeof(double) * ctx->nrows, hipMemcpyDeviceToHost, ctx->stream));
  MLFF_HIP(ctx, hipStreamSynchronize(ctx->stream));
  return MLFF_OK;
  MLFF_API_END(ctx)
}

int mlff_precon_none(mlff_ctx *ctx) {
  MLFF_API_BEGIN
  MLFF_ENTER(ctx);
  ctx->precon_kind = MLFF_PRECON_NONE;
  ctx->k = 0;
  return MLFF_OK;
  MLFF_API_END(ctx)
}

int mlff_precon_pivchol(mlff_ctx *ctx, int64_t k, int build_woodbury, int64_t *index_columns_out,
                        double *seconds_out) {
  MLFF_API_BEGIN
  MLFF_ENTER(ctx);
  MLFF_TRY(require_operator(ctx));
  if (k < 1 || k > ctx->N || k > 65536)
    return set_error(ctx, MLFF_ERR_ARG, "pivoted Cholesky rank k must satisfy 1 <= k <= min(N, 65536)");
  const auto t0 = std::chrono::steady_clock::now();
  ctx->precon_kind = MLFF_PRECON_NONE;
  MLFF_TRY(alloc_panel(ctx, k));
  if (ctx->prow) hipFree(ctx->prow);
  ctx->prow = nullptr;
  MLFF_HIP(ctx, hipMalloc(&ctx->prow, sizeof(double) * (k + 1)));
  MLFF_TRY(pivoted_cholesky(ctx, k, index_columns_out));
  ctx->k = k;  // without Woodbury the panel holds L^T (mlff_precon_get_panel), unused by PCG
  ctx->piv_woodbury_s = 0.0;
  if (build_woodbury) {
    const auto tw = std::chrono::steady_clock::now();
    MLFF_TRY(woodbury_inplace(ctx, ctx->T, k));
    ctx->piv_woodbury_s = std::chrono::duration<double>(std::chrono::steady_clock::now() - tw).count();
    ctx->precon_kind = MLFF_PRECON_PIVCHOL;
    ctx->sigma_p = 1.0;
  }
  MLFF_HIP(ctx, hipStreamSynchronize(ctx->stream));
  if (seconds_out)
    *seconds_out = std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count();
  return MLFF_OK;
  MLFF_API_END(ctx)
}

int mlff_pivchol_times(mlff_ctx *ctx, double *col_seconds_out, int64_t k,
                       double *woodbury_seconds_out) {
  MLFF_API_BEGIN
  MLFF_ENTER(ctx);
  if (k < 0 || (k > 0 && col_seconds_out == nullptr)) return set_error(ctx, MLFF_ERR_ARG, "bad output");
  const int64_t n = std::min<int64_t>(k, (int64_t)ctx->piv_col_s.size());
  for (int64_t c = 0; c < n; ++c) col_seconds_out[c] = ctx->piv_col_s[c];
  for (int64_t c = n; c < k; ++c) col_seconds_out[c] = 0.0;
  if (woodbury_seconds_out) *woodbury_seconds_out = ctx->piv_woodbury_s;
  return MLFF_OK;
  MLFF_API_END(ctx)
}

int mlff_precon_nystrom(mlff_ctx *ctx, const int64_t *idx, int64_t k, int variant,
                        double *seconds_out) {
  MLFF_API_BEGIN
  MLFF_ENTER(ctx);
  MLFF_TRY(require_operator(ctx));
  if (variant != 0 && variant != 1) return set_error(ctx, MLFF_ERR_ARG, "variant must be 0 or 1");
  MLFF_TRY(check_idx(ctx, idx, k));
  const auto t0 = std::chrono::steady_clock::now();
  ctx->precon_kind = MLFF_PRECON_NONE;
  MLFF_TRY(alloc_panel(ctx, k));
  MLFF_TRY(nystrom_panel(ctx, idx, k, variant, ctx->lam, ctx->T));
  ctx->precon_kind = variant == 0 ? MLFF_PRECON_NYSTROM : MLFF_PRECON_NYSTROM_SB;
  ctx->k = k;
  ctx->sigma_p = -1.0;  // _P_vec returns (B^T B v - v)/lam; _sb returns -(v - P^T P v)/lam
  if (seconds_out)
    *seconds_out = std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count();
  return MLFF_OK;
  MLFF_API_END(ctx)
}

int mlff_precon_lowrank(mlff_ctx *ctx, const double *Lt_local, int64_t k) {
  MLFF_API_BEGIN
  MLFF_ENTER(ctx);
  MLFF_TRY(require_operator(ctx));
  if (k < 1 || k > ctx->N || (Lt_local == nullptr && ctx->nrows > 0))
    return set_error(ctx, MLFF_ERR_ARG, "lowrank: bad factor");
  ctx->precon_kind = MLFF_PRECON_NONE;
  MLFF_TRY(alloc_panel(ctx, k));
  if (ctx->nrows > 0)
    MLFF_HIP(ctx, hipMemcpy2DAsync(ctx->T, sizeof(double) * ctx->blk, Lt_local,
                                   sizeof(double) * ctx->nrows, sizeof(double) * ctx->nrows, k,
                                   hipMemcpyHostToDevice, ctx->stream));
  MLFF_TRY(woodbury_inplace(ctx, ctx->T, k));
  ctx->precon_kind = MLFF_PRECON_LOWRANK;
  ctx->k = k;
  ctx->sigma_p = 1.0;
  return MLFF_OK;
  MLFF_API_END(ctx)
}

int mlff_precon_eig(mlff_ctx *ctx, int64_t k, int mask_mode, int64_t dim_i, int build_woodbury,
                    double *evals_out, double *rowlev_out) {
  MLFF_API_BEGIN
  MLFF_ENTER(ctx);
  if (mask_mode < 0 || mask_mode > 2 || (mask_mode == 2 && (dim_i < 3 || dim_i % 3 != 0)))
    return set_error(ctx, MLFF_ERR_ARG, "eig: bad mask_mode / dim_i");
  if (mask_mode == 2) {  // the masked matrix is formed from this rank's rows of the dense K
    MLFF_TRY(require_matrix(ctx));
  } else {
    MLFF_TRY(require_operator(ctx));
  }
  if (k < 1 || k > ctx->N) return set_error(ctx, MLFF_ERR_ARG, "eig: need 1 <= k <= N");
  ctx->precon_kind = MLFF_PRECON_NONE;
  MLFF_TRY(alloc_panel(ctx, k));
  MLFF_TRY(eig_lowrank(ctx, k, mask_mode, dim_i, ctx->T, evals_out, rowlev_out));
  if (build_woodbury) {
    MLFF_TRY(woodbury_inplace(ctx, ctx->T, k));
    ctx->precon_kind = MLFF_PRECON_EIG;
    ctx->k = k;
    ctx->sigma_p = 1.0;
  }
  return MLFF_OK;
  MLFF_API_END(ctx)
}

int mlff_eig_info(mlff_ctx *ctx, int *converged_out, double *rel_resid_out) {
  MLFF_API_BEGIN
  MLFF_ENTER(ctx);
  if (converged_out) *converged_out = ctx->eig_converged ? 1 : 0;
  if (rel_resid_out) *rel_resid_out = ctx->eig_rel_resid;
  return MLFF_OK;
  MLFF_API_END(ctx)
}

int mlff_precon_info(mlff_ctx *ctx, int *kind_out, int64_t *k_out) {
  MLFF_API_BEGIN
  MLFF_ENTER(ctx);
  if (kind_out) *kind_out = ctx->precon_kind;
  if (k_out) *k_out = ctx->k;
  return MLFF_OK;
  MLFF_API_END(ctx)
}

int mlff_precon_apply_traffic(mlff_ctx *ctx, int *one_pass_out, double *bytes_out) {
  MLFF_API_BEGIN
  MLFF_ENTER(ctx);
  const double N = (double)ctx->blk, n = (double)ctx->nrows, k = (double)ctx->k;
  const bool one = ctx->precon_kind != MLFF_PRECON_NONE && (ctx->lr_rows || ctx->lr_cluster);
  if (one_pass_out) *one_pass_out = one ? (ctx->lr_cluster ? 2 : 1) : 0;
  if (bytes_out) {
    if (ctx->precon_kind == MLFF_PRECON_NONE)
      *bytes_out = 0.0;
    else if (one)
      *bytes_out = 8.0 * k * N +
                   16.0 * (double)(ctx->lr_cluster ? ctx->lr_q : lr_rows_groups(ctx->k)) * N +
                   24.0 * n;
    else
      *bytes_out = 16.0 * k * N + 24.0 * n;
  }
  return MLFF_OK;
  MLFF_API_END(ctx)
}

int mlff_precon_apply(mlff_ctx *ctx, const double *r_local, double *z_local) {
  MLFF_API_BEGIN
  MLFF_ENTER(ctx);
  MLFF_TRY(require_operator(ctx));
  hipStream_t s = ctx->stream;
  ScratchScope scope(ctx);
  double *rd = nullptr, *zd = nullptr;
  MLFF_TRY(scratch_alloc(ctx, &rd, ctx->blk));
  MLFF_TRY(scratch_alloc(ctx, &zd, ctx->blk));
  MLFF_HIP(ctx, hipMemsetAsync(rd, 0, sizeof(double) * ctx->blk, s));
  if (ctx->nrows > 0)
    MLFF_HIP(ctx, hipMemcpyAsync(rd, r_local, sizeof(double) * ctx->nrows, hipMemcpyHostToDevice, s));
  if (ctx->precon_kind == MLFF_PRECON_NONE) {
    MLFF_HIP(ctx, hipMemcpyAsync(zd, rd, sizeof(double) * ctx->blk, hipMemcpyDeviceToDevice, s));
  } else {
    ctx->spec_t = false;  // tpart is reused below
    if (ctx->exact_sums) {  // the measurement anchor's apply (kernels_dd.hip)
      launch_dd_lowrank(ctx->T, ctx->blk, ctx->k, rd, zd, ctx->nrows, ctx->sigma_p, 1.0 / ctx->lam,
                        ctx->tpart, nullptr, s);
      MLFF_HIP(ctx, hipGetLastError());
      if (ctx->nrows > 0)
        MLFF_HIP(ctx, hipMemcpyAsync(z_local, zd, sizeof(double) * ctx->nrows, hipMemcpyDeviceToHost, s));
      MLFF_HIP(ctx, hipStreamSynchronize(s));
      return MLFF_OK;
    }
    if (ctx->lr_rows || ctx->lr_cluster) {
      if (ctx->lr_rows) {
        launch_lr_apply_rows(ctx->T, ctx->blk, ctx->k, rd, zd, ctx->nrows, ctx->sigma_p,
                             1.0 / ctx->lam, nullptr, nullptr, s, ctx->lr_zpart);
      } else {
        MLFF_HIP(ctx, hipMemsetAsync(ctx->lr_fault, 0, sizeof(int), s));
        launch_lr_apply_cluster(ctx->T, ctx->blk, ctx->k, ctx->lr_q, rd, zd, ctx->nrows,
                                ctx->sigma_p, 1.0 / ctx->lam, nullptr, nullptr, s, ctx->lr_zpart,
                                ctx->lr_slots, next_lr_epoch(ctx), ctx->lr_fault);
      }
      MLFF_HIP(ctx, hipGetLastError());
      if (ctx->lr_cluster) {
        int fault = 0;
        MLFF_HIP(ctx, hipMemcpyAsync(&fault, ctx->lr_fault, sizeof(int), hipMemcpyDeviceToHost, s));
        MLFF_HIP(ctx, hipStreamSynchronize(s));
        if (fault != 0) {  // hand-offs timed out (members not all resident): two passes
          ctx->lr_cluster = false;
          ctx->lr_fallbacks += 1;
          launch_gemv_split(ctx->T, ctx->blk, ctx->k, ctx->blk, ctx->tsplit, rd, ctx->tpart, nullptr, s);
          launch_precon_z(ctx->T, ctx->blk, ctx->k, ctx->tsplit, ctx->tpart, rd, zd, ctx->nrows,
                          ctx->sigma_p, 1.0 / ctx->lam, nullptr, nullptr, s, ctx->zpart, ctx->zsplit);
          MLFF_HIP(ctx, hipGetLastError());
        }
      }
      if (ctx->nrows > 0)
        MLFF_HIP(ctx, hipMemcpyAsync(z_local, zd, sizeof(double) * ctx->nrows, hipMemcpyDeviceToHost, s));
      MLFF_HIP(ctx, hipStreamSynchronize(s));
      return MLFF_OK;
    }
    launch_gemv_split(ctx->T, ctx->blk, ctx->k, ctx->blk, ctx->tsplit, rd, ctx->tpart, nullptr, s);
    MLFF_TRY(allreduce(ctx, ctx->tpart, (size_t)(ctx->k * ctx->tsplit)));
    launch_precon_z(ctx->T, ctx->blk, ctx->k, ctx->tsplit, ctx->tpart, rd, zd, ctx->nrows,
                    ctx->sigma_p, 1.0 / ctx->lam, nullptr, nullptr, s, ctx->zpart, ctx->zsplit);
  }
  MLFF_HIP(ctx, hipGetLastError());
  if (ctx->nrows > 0)
    MLFF_HIP(ctx, hipMemcpyAsync(z_local, zd, sizeof(double) * ctx->nrows, hipMemcpyDeviceToHost, s));
  MLFF_HIP(ctx, hipStreamSynchronize(s));
  return MLFF_OK;
  MLFF_API_END(ctx)
}

int mlff_precon_get_panel(mlff_ctx *ctx, double *T_local, int64_t ld_out) {
  MLFF_API_BEGIN
  MLFF_ENTER(ctx);
  if (ctx->T == nullptr || ctx->k < 1) return set_error(ctx, MLFF_ERR_STATE, "no low-rank panel");
  if (T_local == nullptr || ld_out < ctx->nrows) return set_error(ctx, MLFF_ERR_ARG, "bad output");
  if (ctx->nrows > 0)
    MLFF_HIP(ctx, hipMemcpy2DAsync(T_local, sizeof(double) * ld_out, ctx->T, sizeof(double) * ctx->blk,
                                   sizeof(double) * ctx->nrows, ctx->k, hipMemcpyDeviceToHost, ctx->stream));
  MLFF_HIP(ctx, hipStreamSynchronize(ctx->stream));
  return MLFF_OK;
  MLFF_API_END(ctx)
}

int mlff_lev_scores(mlff_ctx *ctx, const int64_t *idx, int64_t k, double lam, double *scores_out) {
  MLFF_API_BEGIN
  MLFF_ENTER(ctx);
  if (!ctx->has_matrix && !ctx->mf.ready && !ctx->rbf.ready)
    return set_error(ctx, MLFF_ERR_STATE, "no kernel matrix set");
  if (!(lam > 0.0) || scores_out == nullptr) return set_error(ctx, MLFF_ERR_ARG, "lev_scores: bad args");
  MLFF_TRY(check_idx(ctx, idx, k));
  hipStream_t s = ctx->stream;
  double *W = nullptr;
  MLFF_HIP(ctx, hipMalloc(&W, sizeof(double) * round_up(k, 8) * ctx->blk));
  MLFF_HIP(ctx, hipMemsetAsync(W, 0, sizeof(double) * round_up(k, 8) * ctx->blk, s));
  int rc = nystrom_panel(ctx, idx, k, 0, lam, W);
  if (rc != MLFF_OK) {
    hipFree(W);
    return rc;
  }
  MLFF_HIP(ctx, hipMemsetAsync(ctx->xg, 0, sizeof(double) * ctx->ld, s));
  launch_colsumsq(W, k, ctx->nrows, ctx->blk, ctx->xg + (int64_t)ctx->rank * ctx->blk, s);
  MLFF_TRY(allgather_blocks(ctx, ctx->xg));
  for (int r = 0; r < ctx->world; ++r) {
    const int64_t g0 = (int64_t)r * ctx->rows_per;
    if (g0 >= ctx->N) break;
    const int64_t cnt = std::min<int64_t>(ctx->rows_per, ctx->N - g0);
    MLFF_HIP(ctx, hipMemcpyAsync(scores_out + g0, ctx->xg + (int64_t)r * ctx->blk,
                                 sizeof(double) * cnt, hipMemcpyDeviceToHost, s));
  }
  MLFF_HIP(ctx, hipStreamSynchronize(s));
  hipFree(W);
  return MLFF_OK;
  MLFF_API_END(ctx)
}

int mlff_pcg_start(mlff_ctx *ctx, const double *b_local, const double *x0_local, double tol,
                   int64_t maxiter, int *early_exit_out) {
  MLFF_API_BEGIN
  MLFF_ENTER(ctx);
  MLFF_TRY(require_operator(ctx));
  if ((b_local == nullptr && ctx->nrows > 0) || maxiter < 1 || !(tol >= 0.0))
    return set_error(ctx, MLFF_ERR_ARG, "pcg_start: need b, maxiter >= 1, tol >= 0");
  MLFF_TRY(resolve_storage(ctx));
  hipStream_t s = ctx->stream;
  if (ctx->trace_cap < maxiter + 1) {
    if (ctx->trace) hipFree(ctx->trace);
    ctx->trace = nullptr;
    MLFF_HIP(ctx, hipMalloc(&ctx->trace, sizeof(double) * (maxiter + 1)));
    ctx->trace_cap = maxiter + 1;
  }
  for (double *v : {ctx->b, ctx->x, ctx->r, ctx->z, ctx->q})
    MLFF_HIP(ctx, hipMemsetAsync(v, 0, sizeof(double) * ctx->blk, s));
  MLFF_HIP(ctx, hipMemsetAsync(ctx->p_full, 0, sizeof(double) * ctx->ld, s));
  if (ctx->gb != nullptr)
    MLFF_HIP(ctx, hipMemsetAsync(ctx->gb, 0, sizeof(double) * ctx->world * ctx->gstride, s));
  if (ctx->nrows > 0) {
    MLFF_HIP(ctx, hipMemcpyAsync(ctx->b, b_local, sizeof(double) * ctx->nrows, hipMemcpyHostToDevice, s));
    if (x0_local)
      MLFF_HIP(ctx, hipMemcpyAsync(ctx->x, x0_local, sizeof(double) * ctx->nrows, hipMemcpyHostToDevice, s));
  }
  double bb = 0.0, xx = 0.0;
  MLFF_TRY(dot_sync(ctx, ctx->b, ctx->b, &bb));
  MLFF_TRY(dot_sync(ctx, ctx->x, ctx->x, &xx));
  const double bnorm = std::sqrt(bb);
  double r0 = bnorm;
  if (xx != 0.0) {
    // r = b - A x0
    MLFF_HIP(ctx, hipMemcpyAsync(ctx->xg + (int64_t)ctx->rank * ctx->blk, ctx->x,
                                 sizeof(double) * ctx->blk, hipMemcpyDeviceToDevice, s));
    MLFF_TRY(allgather_blocks(ctx, ctx->xg));
    MLFF_TRY(launch_operator(ctx, ctx->xg, ctx->q, ctx->x, nullptr));
    launch_residual(ctx->b, ctx->q, ctx->r, ctx->nrows, rr_part(ctx), s);
    MLFF_TRY(allreduce(ctx, rr_part(ctx), kVecGrid));
    launch_reduce_to(rr_part(ctx), kVecGrid, &ctx->st->pad0, s);
    double rr = 0.0;
    MLFF_HIP(ctx, hipMemcpyAsync(&rr, &ctx->st->pad0, sizeof(double), hipMemcpyDeviceToHost, s));
    MLFF_HIP(ctx, hipStreamSynchronize(s));
    r0 = std::sqrt(rr);
  } else {
    MLFF_HIP(ctx, hipMemcpyAsync(ctx->r, ctx->b, sizeof(double) * ctx->blk, hipMemcpyDeviceToDevice, s));
  }
  DevState h{};
  h.maxiter = maxiter;
  h.atol = (bnorm == 0.0) ? tol : tol * bnorm;
  h.status = ST_RUNNING;
  h.resid = r0;
  int early = 0;
  if (r0 <= tol) {          // _get_atol legacy: ||A x0 - b|| <= tol -> return x0
    h.status = ST_CONVERGED;
    early = 1;
  } else if (r0 < h.atol) {  // CGREVCOM: ||r0|| < TOL -> converged before the first iteration
    h.status = ST_CONVERGED;
  }
  MLFF_HIP(ctx, hipMemcpyAsync(ctx->st, &h, sizeof(DevState), hipMemcpyHostToDevice, s));
  MLFF_HIP(ctx, hipMemcpyAsync(ctx->trace, &r0, sizeof(double), hipMemcpyHostToDevice, s));
  MLFF_HIP(ctx, hipStreamSynchronize(s));
  *ctx->h_st = h;
  ctx->spec_t = false;
  ctx->tol = tol;
  ctx->bnorm = bnorm;
  ctx->pcg_done = 0;
  ctx->pcg_active = true;
  if (early_exit_out) *early_exit_out = early;
  return MLFF_OK;
  MLFF_API_END(ctx)
}

int mlff_pcg_run(mlff_ctx *ctx, int64_t n_iter, int64_t chunk, int *status_out) {
  MLFF_API_BEGIN
  MLFF_ENTER(ctx);
  if (!ctx->pcg_active) return set_error(ctx, MLFF_ERR_STATE, "mlff_pcg_start not called");
  if (n_iter < 0) return set_error(ctx, MLFF_ERR_ARG, "n_iter < 0");
  if (chunk <= 0) chunk = 32;
  hipStream_t s = ctx->stream;
  const long long maxiter = ctx->h_st->maxiter;
  const int64_t target = std::min<int64_t>(ctx->pcg_done + n_iter, maxiter);
  std::vector<GemvMark> marks;
  while (ctx->h_st->status == ST_RUNNING && ctx->pcg_done < target) {
    const int64_t first = ctx->pcg_done + 1;
    const int64_t last = std::min<int64_t>(first + chunk - 1, target);
    ctx->timing.used = 0;
    marks.clear();
    hipEvent_t c0 = nullptr, c1 = nullptr;
    if (ctx->timing.on) {
      c0 = timing_event(ctx);
      if (c0) hipEventRecord(c0, s);
    }
    for (int64_t it = first; it <= last; ++it)
      MLFF_TRY(launch_iteration(ctx, it, &marks, it > first, it == last));
    if (ctx->timing.on) {
      c1 = timing_event(ctx);
      if (c1) hipEventRecord(c1, s);
    }
    MLFF_HIP(ctx, hipGetLastError());
    MLFF_TRY(poll_state(ctx));
    if (ctx->h_st->status == ST_FAULT && ctx->lr_cluster) {
      // the cluster apply could not complete its hand-offs (its workgroups were not all
      // resident, e.g. another process's kernels held CUs): nothing of iteration iters + 1
      // was written past its (idempotent) stop test, so the solve continues from there on
      // the two-pass apply
      ctx->lr_cluster = false;
      ctx->lr_fallbacks += 1;
      ctx->h_st->status = ST_RUNNING;
      MLFF_HIP(ctx, hipMemsetAsync(&ctx->st->status, 0, sizeof(int), s));  // ST_RUNNING
    }
    const int64_t done_now = ctx->h_st->iters;
    if (ctx->timing.on && c0 && c1) {
      for (const GemvMark &mk : marks) {
        if (mk.it > done_now) continue;  // gated launches after convergence
        float ms = 0.f;
        if (hipEventElapsedTime(&ms, ctx->timing.ev[mk.ev0], ctx->timing.ev[mk.ev1]) == hipSuccess) {
          if (mk.kind == 0) {
            ctx->timing.gemv_ms += ms;
            ctx->timing.gemv_count += 1;
          } else if (mk.kind == 1 || mk.kind == 3) {  // 3: second part of one apply
            ctx->timing.pre_ms += ms;
            if (mk.kind == 1) ctx->timing.pre_count += 1;
          } else {
            ctx->timing.comm_ms += ms;
            ctx->timing.comm_count += 1;
          }
        }
      }
      float ms = 0.f;
      if (hipEventElapsedTime(&ms, c0, c1) == hipSuccess) {
        ctx->timing.iter_ms += ms;
        ctx->timing.iter_count += done_now - ctx->pcg_done;
      }
    }
    while (ctx->h_st->status == ST_RECHECK) {
      MLFF_TRY(do_recheck(ctx));
      MLFF_TRY(poll_state(ctx));
      ctx->spec_t = false;  // r was recomputed: the speculative T r is stale
    }
    ctx->pcg_done = ctx->h_st->iters;
  }
  if (ctx->h_st->status == ST_FAULT)
    return set_error(ctx, MLFF_ERR_HIP, "PCG: a cluster hand-off of the one-pass apply timed out");
  if (status_out) *status_out = ctx->h_st->status;
  return MLFF_OK;
  MLFF_API_END(ctx)
}

int mlff_pcg_result(mlff_ctx *ctx, int64_t *iters_out, int *status_out, double *resid_out,
                    int *info_out) {
  MLFF_API_BEGIN
  MLFF_ENTER(ctx);
  if (!ctx->pcg_active) return set_error(ctx, MLFF_ERR_STATE, "mlff_pcg_start not called");
  MLFF_TRY(poll_state(ctx));
  const DevState &h = *ctx->h_st;
  if (iters_out) *iters_out = h.iters;
  if (status_out) *status_out = h.status;
  if (resid_out) *resid_out = h.resid;
  if (info_out) *info_out = (h.status == ST_CONVERGED) ? 0 : (int)h.iters;
  return MLFF_OK;
  MLFF_API_END(ctx)
}

int mlff_pcg_get_x(mlff_ctx *ctx, double *x_local) {
  MLFF_API_BEGIN
  MLFF_ENTER(ctx);
  if (ctx->nrows > 0) {
    if (x_local == nullptr) return set_error(ctx, MLFF_ERR_ARG, "null x");
    MLFF_HIP(ctx, hipMemcpyAsync(x_local, ctx->x, sizeof(double) * ctx->nrows, hipMemcpyDeviceToHost, ctx->stream));
  }
  MLFF_HIP(ctx, hipStreamSynchronize(ctx->stream));
  return MLFF_OK;
  MLFF_API_END(ctx)
}

int mlff_pcg_get_trace(mlff_ctx *ctx, double *trace_out, int64_t n) {
  MLFF_API_BEGIN
  MLFF_ENTER(ctx);
  if (!ctx->pcg_active || ctx->trace == nullptr) return set_error(ctx, MLFF_ERR_STATE, "no solve");
  if (trace_out == nullptr || n < 0) return set_error(ctx, MLFF_ERR_ARG, "bad output");
  MLFF_TRY(poll_state(ctx));
  const int64_t avail = ctx->h_st->iters + 1;
  const int64_t cnt = std::min<int64_t>(n, avail);
  if (cnt > 0)
    MLFF_HIP(ctx, hipMemcpy(trace_out, ctx->trace, sizeof(double) * cnt, hipMemcpyDeviceToHost));
  return MLFF_OK;
  MLFF_API_END(ctx)
}

int mlff_timing_enable(mlff_ctx *ctx, int on) {
  MLFF_API_BEGIN
  MLFF_ENTER(ctx);
  ctx->timing.on = on != 0;
  ctx->timing.every = on > 1 ? on : 1;
  if (ctx->timing.on && ctx->timing.ev.size() < kTimingPool) ctx->timing.ev.reserve(kTimingPool);
  return MLFF_OK;
  MLFF_API_END(ctx)
}

int mlff_timing_read(mlff_ctx *ctx, double *gemv_ms, int64_t *gemv_count, double *iter_ms,
                     int64_t *iter_count) {
  MLFF_API_BEGIN
  MLFF_ENTER(ctx);
  if (gemv_ms) *gemv_ms = ctx->timing.gemv_ms;
  if (gemv_count) *gemv_count = ctx->timing.gemv_count;
  if (iter_ms) *iter_ms = ctx->timing.iter_ms;
  if (iter_count) *iter_count = ctx->timing.iter_count;
  return MLFF_OK;
  MLFF_API_END(ctx)
}

int mlff_timing_read_precon(mlff_ctx *ctx, double *ms, int64_t *count) {
  MLFF_API_BEGIN
  MLFF_ENTER(ctx);
  if (ms) *ms = ctx->timing.pre_ms;
  if (count) *count = ctx->timing.pre_count;
  return MLFF_OK;
  MLFF_API_END(ctx)
}

int mlff_timing_read_comm(mlff_ctx *ctx, double *ms, int64_t *count) {
  MLFF_API_BEGIN
  MLFF_ENTER(ctx);
  if (ms) *ms = ctx->timing.comm_ms;
  if (count) *count = ctx->timing.comm_count;
  return MLFF_OK;
  MLFF_API_END(ctx)
}

int mlff_device_memory(mlff_ctx *ctx, int64_t *free_out, int64_t *total_out) {
  MLFF_API_BEGIN
  MLFF_ENTER(ctx);
  size_t fr = 0, tot = 0;
  MLFF_HIP(ctx, hipMemGetInfo(&fr, &tot));
  if (free_out) *free_out = (int64_t)fr;
  if (total_out) *total_out = (int64_t)tot;
  return MLFF_OK;
  MLFF_API_END(ctx)
}

int mlff_timing_reset(mlff_ctx *ctx) {
  MLFF_API_BEGIN
  MLFF_ENTER(ctx);
  ctx->timing.gemv_ms = 0.0;
  ctx->timing.gemv_count = 0;
  ctx->timing.pre_ms = 0.0;
  ctx->timing.pre_count = 0;
  ctx->timing.iter_ms = 0.0;
  ctx->timing.iter_count = 0;
  ctx->timing.comm_ms = 0.0;
  ctx->timing.comm_count = 0;
  return MLFF_OK;
  MLFF_API_END(ctx)
}

}  // extern "C"
