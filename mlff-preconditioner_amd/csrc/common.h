// Shared definitions of the gfx950 PCG library: context layout, device scalar
// block, launcher prototypes.  Everything here is private to libmlffpcg.so; the
// public surface is include/mlffpcg.h.
#pragma once

#include <hip/hip_runtime.h>
#include <rccl/rccl.h>

#include <cstdint>
#include <memory>
#include <string>
#include <cstdlib>
#include <vector>

#include "../../include/mlffpcg.h"

namespace mlff {

constexpr int kWave = 64;
constexpr int kBlock = 256;       // threads per workgroup for streaming kernels
constexpr int kPad = 64;          // row / vector padding (doubles) = 512 B
constexpr int kMaxPart = 1024;    // partial-sum slots per reduction
constexpr int kVecGrid = 512;     // workgroups of the grid-stride vector kernels
constexpr int kSymTile = 512;     // tile edge of the symmetric tiled operator

__host__ __device__ inline int64_t round_up(int64_t a, int64_t b) { return (a + b - 1) / b * b; }

// PCG status values kept on the device (status gating: every kernel of an
// iteration returns immediately unless status == RUNNING).
enum : int { ST_RUNNING = 0, ST_RECHECK = 1, ST_CONVERGED = 2, ST_MAXITER = 3, ST_FAULT = 4 };

// Device-resident scalars of the solver.  One instance per context.
struct DevState {
  double rho, rho1, alpha, pq, rr, resid, atol, pad0;
  long long iters;     // completed CG iterations (scipy ITER)
  long long maxiter;
  int status;
  int linalg_err;      // set by the Cholesky kernels on a non-positive pivot
  int pivot_err;       // set by the pivoted-Cholesky finaliser (pivot <= 0)
  int pad1;
  long long m_pi;      // current pivot (global index) of the pivoted Cholesky
  double sqrt_piv;     // its sqrt(pivot)
  double best_val;     // argmax of this rank
  long long best_pos;
  double rho_new;      // fused p update: rho of the iteration, published by k_rec_g for k_rec_fin
};

// Lower-block-triangle tiles of K owned by this rank (kernels_sym.hip).
struct SymPack {
  bool ready = false;
  double *tiles = nullptr;   // ntiles x B x B
  int2 *list = nullptr;      // (I, J) of each stored tile, I >= J
  int64_t ntiles = 0;
  int64_t Np = 0;            // padded global length (multiple of B)
  int64_t nb = 0;            // Np / B
  int64_t tiles_per_rank = 0;
  double *P = nullptr;       // slot buffer nb x Np
  // the last (ntiles - nwhole) tiles of `list` run as 2^lsub sub-unit workgroups each;
  // their column partials of sub-units 1.. go to Pq (2^lsub - 1 planes of nb x Np)
  int64_t nwhole = 0;
  int lsub = 2;              // split tiles run as 2^lsub sub-units (row slices) each
  int64_t pq_planes = 0;     // planes allocated in Pq (2^lsub - 1 needed)
  double *Pq = nullptr;
  unsigned char *split = nullptr;  // nb x nb: tile (I, J) is split
  int *own = nullptr;              // nb x nb owned slots per row block + nb counts (W > 1)
  // the same slots as a flat load list per row block (W > 1, k_sym_reduce_wl): entry
  // t | plane << 16 (plane 0 = P, h >= 1 = Pq plane h - 1; a split slot's planes follow it),
  // pstride entries per row block, then nb counts; pmax = the largest count
  int *plist = nullptr;
  int64_t pstride = 0;
  int pmax = 0;
  int64_t t_split = 0;             // smallest I of a split tile (nb if none)
  int64_t dyn = 0;                 // > 0: k_symv_dyn with this many workgroups
  unsigned long long *ticket = nullptr;  // its work counter (reset by the slot reduction)
  double *yg = nullptr;      // world > 1: this rank's partial y, rank blocks of ystride
  double *yr = nullptr;      // world > 1: reduce-scatter result (ystride)
  int64_t ystride = 0;       // blk + tail (p.q shares of every rank)
};

// Matrix-free sGDML operator data (kernels_mf.hip).
struct MfData {
  bool ready = false;
  int64_t M = 0, D = 0;
  int n = 0, n_perms = 0;
  double sig = 0.0;
  int64_t i0 = 0, ni = 0;            // training points touched by this rank's rows
  double *Rd = nullptr, *Rdd = nullptr;   // M x D, M x D x 3
  double *Rt = nullptr, *Zt = nullptr;    // (M n_perms) x D
  int32_t *Pt = nullptr, *ps = nullptr, *pt = nullptr;
  bool ident = false;                     // one identity permutation: Rt == Rd, Pt unused
  double *m5 = nullptr, *w = nullptr;     // ni x (M n_perms), x independent
  double *c = nullptr, *F = nullptr;      // ni x (M n_perms), ni x D scratch
  double *part = nullptr;                 // nz x ni x (M n_perms) pair partial sums
  double *ypart = nullptr;                // J^T partial rows (slices x nrows)
  double *xc = nullptr;                   // contiguous operand (world > 1)
  int nz = 1;                             // descriptor slices of the pair sums
  int64_t dslice = 0;
  std::vector<int32_t> perms, piinv;      // host copies (diagonal blocks)
  // single-column path (kernels_gen.hip k_sgdml_col): (r = i, s = j) records of every
  // (local point, point, permutation), ni x M x n_perms x (6 n + 2), and device atom maps;
  // null when the table would exceed kMfColTableBytes (columns then go through the
  // whole operator)
  double *uvk = nullptr;
  int32_t *pi_d = nullptr, *piinv_d = nullptr;
  // record-factored operator (kernels_mf.hip k_rec_g / k_rec_fin), used when uvk exists:
  // wt = w transposed ((M n_perms) x ni), sv = the per-application pair scalars
  // 5 m (v . x_j) (ni x M n_perms), rpart = J^T G partial rows of every pair block
  // (rblk slots x ni x 3n)
  bool rec = false;
  int rec_rg = 8;         // k_rec_g query points per workgroup, identity permutation (MLFF_REC_RG)
  bool rec_wc16 = true;   // k_rec_g w / x staged as one 16-slot chunk when MP <= 16 (MLFF_REC_WC16)
  int rblk = 0;
  int64_t ldw = 0;
  double *wt = nullptr, *sv = nullptr, *rpart = nullptr;
  // pair-tile form (kernels_pt.hip k_pt_pair / k_pt_fin; few atoms, D <= 288): in use when
  // ptile is set (the default where it exists; MLFF_MF_FORM=rec|pair|pt overrides); pt_S chunks
  // of the (j, p) range, ptpart = pt_S x ni x (padded D) partial F
  bool ptile = false;
  int pt_S = 1;
  double *ptpart = nullptr;
  // energy constraints (use_E_cstr, train.py:212-236; iterative_solver.py:423-440): the
  // operand and result carry M energy entries after the nF = 3 n M force entries (one rank)
  bool E = false;
  int64_t nF = 0;
  double *kee = nullptr;    // ni x M: sum_p (1 + nrm/sig (1 + nrm/(3 sig))) exp(-nrm/sig)
  double *eterm = nullptr;  // ni x (M n_perms): a_ijp w_ijp of the last application
};

// Synthetic RBF kernel source (tools/utils.py:173-187): the points, scaled by 1 / length
// scale, stay on the device and every consumer evaluates K from them -- the symmetric
// tiles are generated directly, columns / the diagonal / requested rows on demand -- so no
// dense N x N copy exists unless the DENSE storage asks for it (mlff_gen_rbf).
struct RbfData {
  bool ready = false;
  double *Xs = nullptr;  // N x d
  int d = 0;
  double jitter = 0.0;
};

// K[i, g] (i != g) of the sklearn RBF kernel: exp(-0.5 * sum_t (xs_i - xs_g)^2), the
// squared distance formed without FMA contraction (scipy pdist 'sqeuclidean' order).
// (xs_i - xs_g)^2 == (xs_g - xs_i)^2 exactly, so the generated kernel is exactly symmetric.
__device__ __forceinline__ double rbf_value(const double (&xi)[8], const double *__restrict__ Xs,
                                            int64_t g, int d) {
  double s = 0.0;
#pragma unroll
  for (int t = 0; t < 8; ++t)
    if (t < d) {
      const double df = __dsub_rn(xi[t], Xs[g * d + t]);
      s = __dadd_rn(s, __dmul_rn(df, df));
    }
  return exp(-0.5 * s);
}

// The scipy stop test of iteration `it` (k_stoptest), done by every workgroup of the
// next iteration's first kernel instead of a launch of its own (rr_part == nullptr: none).
struct StopFold {
  const double *rr_part = nullptr;
  DevState *st = nullptr;
  double *trace = nullptr;
  long long it = 0;
};

// The CG update of the previous iteration (k_update_xr: alpha = rho / (p.q); x += alpha p;
// r -= alpha q; rr partials) folded into this iteration's one-pass low-rank apply: k_lr_rows
// forms r - alpha q on the fly, k_lr_fin writes x, r and the rr partials (x == nullptr: none)
struct XrFold {
  double *x = nullptr;
  double *r = nullptr;
  const double *p = nullptr;
  const double *q = nullptr;
  const double *pq_part = nullptr;
  double *rr_part = nullptr;
  DevState *st = nullptr;
};

// flags of the timing-only events (stamps read after a stream synchronisation): no
// system-scope fence, so recording one does not write back and invalidate the caches
// between the kernels it brackets (MLFF_EVENT_FENCE=1 restores the default, for A/B)
inline unsigned timing_event_flags() {
  static const unsigned f = std::getenv("MLFF_EVENT_FENCE") ? hipEventDefault
                                                            : hipEventDisableSystemFence;
  return f;
}

struct Timing {
  bool on = false;
  int every = 1;        // bracket every `every`-th PCG iteration only (mlff_timing_enable)
  bool sample = true;   // the iteration being launched is bracketed
  std::vector<hipEvent_t> ev;  // pool, pairs (start, stop)
  size_t used = 0;             // events used in the current chunk
  double gemv_ms = 0.0;
  int64_t gemv_count = 0;
  double pre_ms = 0.0;     // low-rank preconditioner apply (one rank)
  int64_t pre_count = 0;
  double iter_ms = 0.0;
  int64_t iter_count = 0;
  double comm_ms = 0.0;    // collectives of the sharded iteration (one rank's stream)
  int64_t comm_count = 0;
};


// the search direction of the fused forms: p = z at ITER 1, else fma(beta, p_old, z)
// (k_update_p's arithmetic)
__device__ __forceinline__ double fused_p(double pold, double z, double beta, bool first) {
  return first ? z : fma(beta, pold, z);
}

__device__ __forceinline__ double wave_sum(double v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v += __shfl_down(v, o, 64);
  return v;
}

// Sum over a 256-thread block; result valid in thread 0.  Fixed order, so every
// workgroup that reduces the same values obtains the same bits.
__device__ __forceinline__ double block_sum256(double v, double *sh) {
  v = wave_sum(v);
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  __syncthreads();
  if (lane == 0) sh[w] = v;
  __syncthreads();
  double t = 0.0;
  if (threadIdx.x == 0) t = (sh[0] + sh[1]) + (sh[2] + sh[3]);
  return t;
}

// Deterministic sum of np partials, broadcast to every thread of the block.
__device__ __forceinline__ double reduce_parts_bcast(const double *__restrict__ part, int np,
                                                     double *sh) {
  double v = 0.0;
  for (int i = threadIdx.x; i < np; i += 256) v += part[i];
  v = block_sum256(v, sh);
  __syncthreads();
  if (threadIdx.x == 0) sh[4] = v;
  __syncthreads();
  return sh[4];
}

// scipy's stop test of iteration f.it on the summed rr partials (k_stoptest); block (0, 0)
// writes the state.  True: the solver continues.
__device__ __forceinline__ bool stop_decide(const StopFold &f, double rr) {
  const double resid = sqrt(rr);
  DevState *st = f.st;
  int dec = ST_RUNNING;
  if (resid <= st->atol)
    dec = f.it > 1 ? ST_RECHECK : ST_CONVERGED;
  else if (f.it >= st->maxiter)
    dec = ST_MAXITER;
  if (blockIdx.x == 0 && blockIdx.y == 0 && threadIdx.x == 0) {
    st->rr = rr;
    st->resid = resid;
    st->iters = f.it;
    f.trace[f.it] = resid;
    if (dec != ST_RUNNING)
      st->status = dec;
    else
      st->rho1 = st->rho;
  }
  return dec == ST_RUNNING;
}

// reduce_parts_bcast for a workgroup of any multiple of 256 threads: the first 256 threads
// reduce the partials exactly as reduce_parts_bcast does (same bits), every thread gets it
__device__ __forceinline__ double reduce_parts_bcast_wide(const double *__restrict__ part, int np,
                                                          double *sh) {
  double v = 0.0;
  if (threadIdx.x < 256)
    for (int i = threadIdx.x; i < np; i += 256) v += part[i];
  v = wave_sum(v);
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  __syncthreads();
  if (lane == 0 && w < 4) sh[w] = v;
  __syncthreads();
  const double t = (sh[0] + sh[1]) + (sh[2] + sh[3]);
  __syncthreads();  // sh is reused by the caller
  return t;
}

// The same sum in two halves, so the loads can be issued long before the reduction:
// parts_thread_sum is the thread's share (the loop of reduce_parts_bcast), parts_bcast the
// block reduction of those shares (same bits as reduce_parts_bcast)
__device__ __forceinline__ double parts_thread_sum(const double *__restrict__ part, int np) {
  double v = 0.0;
  for (int i = threadIdx.x; i < np; i += 256) v += part[i];
  return v;
}
__device__ __forceinline__ double parts_bcast(double v, double *sh) {
  v = block_sum256(v, sh);
  __syncthreads();
  if (threadIdx.x == 0) sh[4] = v;
  __syncthreads();
  return sh[4];
}

}  // namespace mlff

namespace mlff {
struct LocalGroup;  // in-process transport (api.hip), see comm_allreduce
}

struct mlff_ctx {
  int device = 0, rank = 0, world = 1;
  int64_t N = 0;        // kernel size
  int64_t rows_per = 0; // ceil(N / world)
  int64_t row0 = 0, nrows = 0;
  int64_t blk = 0;      // padded local length (multiple of 64) = column block per rank
  int64_t ld = 0;       // world * blk: padded global length / K leading dimension
  hipStream_t stream = nullptr;
  ncclComm_t comm = nullptr;                   // RCCL (one process per GPU)
  std::shared_ptr<mlff::LocalGroup> local;     // or: ranks as threads of one process
  bool solo = false;                           // or: one rank alone (profiling, api.hip)

  // kernel matrix, blk rows x ld columns (padding rows/cols are zero)
  double *K = nullptr;
  bool has_matrix = false;
  double sigma_K = 1.0, lam = 0.0;
  bool has_operator = false;
  bool K_symmetric = false;
  bool use_E_cstr = false;   // mlff_set_energy_constraints: sGDML systems of size 3 n M + M  // known symmetric by construction (generated / assembled)
  int storage = MLFF_STORAGE_AUTO;  // requested operator storage
  bool use_sym = false;             // resolved: symmetric tiles in use
  bool use_mf = false;              // resolved: matrix-free sGDML operator in use
  mlff::SymPack sym;
  mlff::MfData mf;                  // matrix-free sGDML operator (optional)
  mlff::RbfData rbf;                // synthetic RBF kernel from its points (optional)

  // CG vectors.  local: blk entries; p_full / xg: ld entries (rank blocks)
  double *x = nullptr, *r = nullptr, *z = nullptr, *q = nullptr, *b = nullptr;
  double *p_full = nullptr, *xg = nullptr;
  double *gb = nullptr;    // world > 1: allgather buffer, world blocks of gstride
  int64_t gstride = 0;     // blk + kVecGrid (z block + its rho partials)
  double *part = nullptr;  // partial sums: 3 * kMaxPart + tpart (k * S)
  mlff::DevState *st = nullptr;
  mlff::DevState *h_st = nullptr;  // pinned mirror
  double *trace = nullptr;
  int64_t trace_cap = 0;
  bool pcg_active = false;
  int64_t pcg_done = 0;   // iterations known complete on the host side
  double tol = 0.0, bnorm = 0.0;

  // preconditioner
  int precon_kind = MLFF_PRECON_NONE;
  int64_t k = 0;
  double *T = nullptr;    // k x blk (row stride blk)
  double sigma_p = 1.0;   // z = sigma_p * (r - T^T T r) / lam
  int tsplit = 1;         // column splits of the T GEMV
  int zsplit = 1;         // row splits of the T^T t GEMV
  double *zpart = nullptr;  // zsplit x blk partials
  bool lr_rows = false;        // one-pass low-rank apply (launch_lr_apply_rows), one rank
  // CG vector updates folded into the matrix-free nanotube iteration; read from
  // MLFF_FUSE_P / MLFF_FUSE_XR (=0: separate launches) when the context is created
  bool fuse_p = true, fuse_xr = true;
  bool cho_fast = true;  // cho_factor_stable: shifted Cholesky first inside builds (MLFF_CHO_FAST)
  // sharded tiled iteration: k_update_xr_shares folded into the next T r pass (MLFF_FUSE_XR_RANKS=1;
  // off by default: SOLO floors 4.5 us slower at W = 4, equal at W = 8)
  bool fuse_xr_ranks = false;
  bool pq_publish = false;
  bool piv_persist_off = false;  // the persistent pivoted Cholesky timed out once (kernels_pivchol.hip)  // MLFF_PQ_PUBLISH=1: the separate k_pq_publish launch (A/B)
  // Woodbury panel re-orthogonalised by a second CholeskyQR step (MLFF_WB_REFINE, woodbury_inplace;
  // configs[1] at full size: 571 -> 366 iterations, the oracle's 367) and the same for the
  // Nystrom panel (MLFF_NYS_REFINE)
  int wb_refine = 0;  // re-orthogonalisation steps (MLFF_WB_REFINE=1 / 2 ...; 0: the reference's one-step panel)
  // the Woodbury Gram matrices L^T L (and the refinement's T T^T): 0 the fp64 matrix-core GEMM,
  // 1 chunked double-double on the matrix cores, 2 exact products in double-double
  // (MLFF_WB_GRAM; kernels_dd.hip gram_wide_dd)
  int wb_gram_dd = 1;
  bool nys_refine = false;
  // exact-sum anchor (MLFF_EXACT_SUMS=1, kernels_dd.hip): dense-row operator and two-pass low-rank
  // apply with double-double dot products rounded once per entry; one rank; measurement only
  bool exact_sums = false;
  bool lr_cluster = false;     // the same for long rows (launch_lr_apply_cluster)
  int lr_q = 0;                // its clusters
  double *lr_zpart = nullptr;  // lr_rows_groups(k) (or lr_q) x blk partials
  unsigned long long *lr_slots = nullptr;  // cluster hand-off granules (k x C x 2)
  unsigned lr_epoch = 0;       // per cluster launch, never 0 in a launch
  int *lr_fault = nullptr;     // ST_FAULT when a cluster hand-off timed out (precon_apply)
  int lr_fallbacks = 0;        // cluster applies that timed out and fell back to two passes
  double last_lo_eig = 0.0;
  bool cho_flipped = false;  // a cho_factor_stable retried upward after a noisy lo > 0
  bool eig_converged = true;   // last truncated eigensolve met kEigTol (kernels_eig.hip)
  double eig_rel_resid = 0.0;  // its worst Ritz residual / |theta_0|    // lo_eig of the last _cho_factor_stable (cho_factor_stable)
  double *tpart = nullptr;       // = tpart_base + kVecGrid
  double *tpart_base = nullptr;
  bool spec_t = false;           // tpart already holds T r of the current r (merged collective)

  // pivoted Cholesky scratch
  int64_t *perm = nullptr;   // global permutation (replicated)
  double *dwork = nullptr;   // residual diagonal (local)
  int *pivflag = nullptr;    // local rows already pivoted
  double *prow = nullptr;    // L[m_pi, :m]
  std::vector<double> piv_col_s;  // device seconds per column of the last build
  double piv_woodbury_s = 0.0;    // its Woodbury build (G, chol, T)

  mlff::Timing timing;
  std::string err;
  bool aborted = false;  // mlff_comm_abort was called: every entry point fails

  // device scratch arena (ScratchScope / scratch_get): chunks, current chunk and offset
  struct ScratchChunk {
    char *p;
    size_t size;
  };
  std::vector<ScratchChunk> scratch_chunks;
  size_t scratch_cur = 0, scratch_off = 0;
  int scratch_depth = 0;  // open ScratchScopes
};

namespace mlff {

// ---- error helpers (api.hip) ------------------------------------------------
int set_error(mlff_ctx *ctx, int code, const std::string &msg);
int hip_check(mlff_ctx *ctx, hipError_t e, const char *what);
int nccl_check(mlff_ctx *ctx, ncclResult_t e, const char *what);

#define MLFF_HIP(ctx, call)                                   \
  do {                                                        \
    hipError_t e__ = (call);                                  \
    if (e__ != hipSuccess) return mlff::hip_check(ctx, e__, #call); \
  } while (0)
#define MLFF_NCCL(ctx, call)                                  \
  do {                                                        \
    ncclResult_t e__ = (call);                                \
    if (e__ != ncclSuccess) return mlff::nccl_check(ctx, e__, #call); \
  } while (0)
// every ABI entry point with a context: null check, then make the context's device
// current on the calling thread (one thread may drive contexts on several devices)
#define MLFF_ENTER(ctx)                                                        \
  do {                                                                         \
    if ((ctx) == nullptr) return mlff::set_error(nullptr, MLFF_ERR_ARG, "null ctx"); \
    if ((ctx)->aborted)                                                        \
      return mlff::set_error((ctx), MLFF_ERR_COMM, "communicator aborted (mlff_comm_abort)"); \
    (void)hipSetDevice((ctx)->device);                                         \
  } while (0)
#define MLFF_TRY(x)             \
  do {                          \
    int rc__ = (x);             \
    if (rc__ != MLFF_OK) return rc__; \
  } while (0)

// No C++ exception may cross the C ABI (ctypes would see std::terminate): every
// extern "C" body runs inside MLFF_API_BEGIN / MLFF_API_END(ctx), which maps
// std::bad_alloc to MLFF_ERR_NOMEM and anything else to MLFF_ERR_HIP, aborting the
// rank's in-process group so that its peers leave their collectives.
int api_exception(mlff_ctx *ctx, int code, const char *what);
#define MLFF_API_BEGIN try {
#define MLFF_API_END(ctx)                                                             \
  }                                                                                   \
  catch (const std::bad_alloc &) {                                                    \
    return mlff::api_exception((ctx), MLFF_ERR_NOMEM, "host allocation failed");      \
  }                                                                                   \
  catch (const std::exception &e__) {                                                 \
    return mlff::api_exception((ctx), MLFF_ERR_HIP, e__.what());                      \
  }                                                                                   \
  catch (...) {                                                                       \
    return mlff::api_exception((ctx), MLFF_ERR_HIP, "unknown C++ exception");         \
  }

// Device scratch of a build function, from the context's arena (mlff_ctx::scratch):
// a bump allocator over chunks obtained once with hipMalloc and kept until
// mlff_ctx_destroy.  Every user runs on ctx->stream, so memory handed out again after a
// ScratchScope has closed is only touched by kernels ordered after the previous user's.
// (No stream-ordered allocator: hipMallocAsync pools outlive the contexts' streams.)
struct ScratchScope {
  mlff_ctx *ctx;
  size_t chunk, off;
  explicit ScratchScope(mlff_ctx *c);
  ~ScratchScope();
  ScratchScope(const ScratchScope &) = delete;
  ScratchScope &operator=(const ScratchScope &) = delete;
};
// bytes (rounded up to 256) of scratch valid until the innermost open ScratchScope closes
int scratch_get(mlff_ctx *ctx, size_t bytes, void **out);
template <typename T>
int scratch_alloc(mlff_ctx *ctx, T **out, size_t count) {
  return scratch_get(ctx, sizeof(T) * (count > 0 ? count : 1), reinterpret_cast<void **>(out));
}

// ---- collectives (api.hip): RCCL, or the in-process transport ---------------
// sum-allreduce of n doubles in place (no-op on one rank)
int comm_allreduce(mlff_ctx *ctx, double *buf, size_t n);
// allgather: recv[r * count ...] = send of rank r; send may alias recv + rank * count
int comm_allgather(mlff_ctx *ctx, const double *send, double *recv, size_t count);

// ---- vector / GEMV kernels (kernels_vec.hip) ---------------------------------
// y = sigma * M v + lam * vloc  over `rows` rows of M (ld columns).
void launch_gemv_rows(const double *M, int64_t ld, int64_t rows, const double *v, double *y,
                      double sigma, double lam, const double *vloc, const int *status,
                      hipStream_t s);
// partial T GEMV: tpart[sp * k + j] = sum_{c in split sp} T[j, c] * r[c]
void launch_gemv_split(const double *T, int64_t ldt, int64_t k, int64_t ncols, int splits,
                       const double *r, double *tpart, const int *status, hipStream_t s,
                       StopFold fold = StopFold{});
int choose_tsplit(int64_t k, int64_t ncols);
// split factor of the apply's T^T t pass (choose_ksplit adjusted to fill whole waves)
int choose_zsplit(int64_t k, int64_t ncols);
// z = sigma_p/lam * (r - T^T t), t = sum_sp tpart; rho partials (r . z)
// (split-K over the k rows of T: zpart holds zsplit x ldt partial sums)
void launch_precon_z(const double *T, int64_t ldt, int64_t k, int splits, const double *tpart,
                     const double *r, double *z, int64_t n, double sigma_p, double lam_inv,
                     double *rho_part, const int *status, hipStream_t s, double *zpart,
                     int zsplit, StopFold fold = StopFold{});
// one-pass apply z = sigma_p/lam (r - T^T T r) with rho partials, one rank, for panels whose
// rows fit a workgroup's registers (lr_rows_fits); zpart: lr_rows_groups(k) x ldt scratch
bool lr_rows_fits(int64_t ldt);
int lr_rows_groups(int64_t k);
void launch_lr_apply_rows(const double *T, int64_t ldt, int64_t k, const double *r, double *z,
                          int64_t n, double sigma_p, double lam_inv, double *rho_part,
                          const int *status, hipStream_t s, double *zpart,
                          StopFold fold = StopFold{}, XrFold xf = XrFold{});
// the one-pass apply for long rows (clusters of lr_cluster_members(ldt) workgroups, one per
// CU, hand-offs of the per-row partial dots); lr_cluster_count = clusters resident at once
bool lr_cluster_fits(int64_t ldt);
int lr_cluster_members(int64_t ldt);
int lr_cluster_count(int64_t ldt, int device);
void launch_lr_apply_cluster(const double *T, int64_t ldt, int64_t k, int Q, const double *r,
                             double *z, int64_t n, double sigma_p, double lam_inv,
                             double *rho_part, const int *status, hipStream_t s, double *zpart,
                             unsigned long long *slots, unsigned epoch, int *fault,
                             StopFold fold = StopFold{});
// part[ks * ldw + c] = sum_{j in slice ks} W[j, c] * (sum_sp tsrc[sp * tstride + j])
void launch_colgemv_part(const double *W, int64_t ldw, int64_t k, const double *tsrc,
                         int tsplits, int64_t tstride, int ksplit, double *part,
                         const int *status, hipStream_t s, StopFold fold = StopFold{},
                         int64_t cached_rows = 0, const long long *tcol = nullptr,
                         const int *spec_hit = nullptr, int64_t spec_m0 = 0);
// C (M x N) = op(A) op(B) with K split over enough workgroups to fill the chip, the slices
// summed in a fixed order (deterministic); scratch from the context's arena
int gemm_splitk(mlff_ctx *ctx, bool ta, bool tb, int64_t M, int64_t N, int64_t K, const double *A,
                int64_t lda, const double *B, int64_t ldb, double *C, int64_t ldc);
int choose_ksplit(int64_t k, int64_t ncols);
// leading rows of a k x ldt panel read with default-policy (MALL-resident) loads
int64_t panel_cached_rows(int64_t k, int64_t ldt);
// rho partials of r . r (no preconditioner)
void launch_dot_part(const double *a, const double *b, int64_t n, double *part,
                     const int *status, hipStream_t s, StopFold fold = StopFold{});
// p = z + (rho/rho1) p   (p = z at iteration 1); rho = sum(rho_part)
void launch_update_p(const double *z, double *p, int64_t n, const double *rho_part,
                     DevState *st, long long it, const int *status, hipStream_t s);
// several ranks (gather buffer gb: rank blocks of gstride = blk + kVecGrid holding z_g
// and its rho partials): dst = r with r.r partials (no preconditioner);
// p_full = z_full + (rho/rho1) p_full with rho summed from all ranks' partials
void launch_copy_dot(const double *r, int64_t n, double *dst, double *part, const int *status,
                     hipStream_t s, StopFold fold = StopFold{});
void launch_update_p_gathered(const double *gb, int64_t gstride, int64_t blk, int world,
                              double *p_full, DevState *st, long long it, const int *status,
                              hipStream_t s);
// several ranks, symmetric tiles: pq = sum of the world shares; q = sigma y + lam p;
// alpha = rho/pq; x += alpha p; r -= alpha q; rr partials
void launch_update_xr_shares(double *x, double *r, const double *p, const double *y,
                             const double *shares, int world, int64_t n, double sigma, double lam,
                             double *rr_part, DevState *st, const int *status, hipStream_t s);
// launch_update_xr_shares folded into the T r pass of the next apply (launch_gemv_split's
// tpart): r_new = r - alpha q into r_out (the caller swaps r and r_out), x, the rr partials
// and T r_new, the bits of the two launches; xr_fold_fits: the split / row-count shapes it
// covers
bool xr_fold_fits(int64_t ncols, int splits, int64_t n);
// kernels_dd.hip (MLFF_EXACT_SUMS): y = sigma fl(M v) + lam vloc with double-double row sums;
// z = sigma_p lam_inv (r - fl(T^T fl(T r))) with double-double dot products (t: k doubles)
void launch_dd_gemv_rows(const double *M, int64_t ld, int64_t rows, int64_t ncols, const double *v,
                         double *y, double sigma, double lam, const double *vloc, const int *status,
                         hipStream_t s);
void launch_dd_lowrank(const double *T, int64_t ldt, int64_t k, const double *r, double *z, int64_t n,
                       double sigma_p, double lam_inv, double *t, const int *status, hipStream_t s);
// G = W W^T (k x k, symmetric) of a wide k x ncols panel, each entry rounded once from a
// double-double sum: exact_products -- every product exact (correctly rounded but for ties);
// else 64-column chunks summed in fp64 on the matrix cores and the chunk partials added in
// double-double.  The Woodbury panel's Gram matrices (MLFF_WB_GRAM)
int gram_wide_dd(mlff_ctx *ctx, const double *W, int64_t k, int64_t ncols, int64_t ldw, double *G,
                 bool exact_products);
void launch_gemv_xr(const double *T, int64_t ldt, int64_t k, int64_t ncols, int splits,
                    const double *r, double *r_out, double *x, const double *p, const double *y,
                    const double *shares, int world, int64_t n, double sigma, double lam,
                    double *rr_part, DevState *st, double *tpart, const int *status,
                    hipStream_t s);
// pq = sum(pq_part); alpha = rho/pq; x += alpha p; r -= alpha q; rr partials
void launch_update_xr(double *x, double *r, const double *p, const double *q, int64_t n,
                      const double *pq_part, double *rr_part, DevState *st, const int *status,
                      hipStream_t s);
// rr -> resid, trace, status (scipy stop test)
void launch_stoptest(const double *rr_part, DevState *st, double *trace, long long it,
                     hipStream_t s);
// recheck: r = b - q, rr partials
void launch_residual(const double *b, const double *q, double *r, int64_t n, double *rr_part,
                     hipStream_t s);
void launch_recheck_finish(const double *rr_part, DevState *st, double *trace, hipStream_t s);
// sum of partials into a device double (1 workgroup)
void launch_reduce_to(const double *part, int np, double *out, hipStream_t s);
void launch_scale_copy(const double *a, double *y, int64_t n, double alpha, hipStream_t s);

// ---- dense linear algebra (kernels_dense.hip) -------------------------------
// C = alpha * op(A) op(B) + beta * C ; row-major; op(A): M x Kd, op(B): Kd x Nc
void launch_gemm(bool ta, bool tb, int64_t M, int64_t Nc, int64_t Kd, double alpha,
                 const double *A, int64_t lda, const double *B, int64_t ldb, double beta,
                 double *C, int64_t ldc, hipStream_t s);
// G = W W^T (k x k) over ncols columns of W (k x ncols, row stride ldw); split-K
// with a deterministic slab reduction; work: >= splits * k * k doubles
int syrk_wide(mlff_ctx *ctx, const double *W, int64_t k, int64_t ncols, int64_t ldw, double *G);
// G = A B^T (k x k) over ncols columns of the wide panels A, B (row stride ldw); split-K
// with a deterministic slab reduction (syrk_wide is gram_wide(W, W))
int gram_wide(mlff_ctx *ctx, const double *A, const double *B, int64_t k, int64_t ncols,
              int64_t ldw, double *G);
// in-place lower Cholesky of the k x k matrix A (row-major, ld = k)
// ok_out: report a matrix that is not positive definite there (MLFF_OK returned) instead of
// as MLFF_ERR_LINALG
int potrf_lower(mlff_ctx *ctx, double *A, int64_t k, bool *ok_out = nullptr);
// smallest eigenvalue of the lower triangle of a device m x m matrix (kernels_syev.hip:
// Householder tridiagonalisation + Sturm bisection, the eigh of _cho_factor_stable);
// d_host / e_host (optional): the tridiagonal
int sym_min_eig(mlff_ctx *ctx, const double *M, int64_t m, double *lo_eig, double *d_host,
                double *e_host);
// W <- L^-1 W, L k x k lower (ld = k), W k x ncols (row stride ldw)
int trsm_lower_wide(mlff_ctx *ctx, const double *L, int64_t k, double *W, int64_t ncols,
                    int64_t ldw);
void launch_add_diag(double *A, int64_t k, double v, hipStream_t s);
void launch_zero_upper(double *A, int64_t k, hipStream_t s);
// column sums of squares: out[c] = sum_j W[j, c]^2
void launch_colsumsq(const double *W, int64_t k, int64_t ncols, int64_t ldw, double *out,
                     hipStream_t s);

// ---- generators (kernels_gen.hip) -------------------------------------------
void launch_gen_rbf(double *K, int64_t ld, int64_t nrows, int64_t row0, int64_t rows_per,
                    int64_t blk, int64_t N, const double *Xs, int d, double jitter,
                    hipStream_t s);
void launch_diag_of(const double *K, int64_t ld, int64_t nrows, int64_t row0, int64_t rows_per,
                    int64_t blk, double sigma, double *out, hipStream_t s);
// gather columns idx (global) of the local rows: W[j, i] = sigma * K[i, pos(idx_j)]
void launch_gather_cols(const double *K, int64_t ld, int64_t nrows, const int64_t *idx,
                        int64_t k, int64_t rows_per, int64_t blk, double sigma, double *W,
                        int64_t ldw, hipStream_t s);
// Smm[j, j'] = W[j, idx_j' - row0] if idx_j' is local else 0
void launch_gather_mm(const double *W, int64_t ldw, const int64_t *idx, int64_t k,
                      int64_t row0, int64_t nrows, double *Smm, hipStream_t s);
// out[jc * ldo + r] = sigma K[row0 + r, col_jc] of the RBF source for the local rows;
// col_jc = cols[jc] (device, ncols) or, with cols == nullptr, st->m_pi
void launch_rbf_cols(const RbfData &rbf, int64_t N, int64_t row0, int64_t nrows,
                     const int64_t *cols, int64_t ncols, const DevState *st, double sigma,
                     double *out, int64_t ldo, hipStream_t s);
void launch_fill(double *y, int64_t n, double v, hipStream_t s);
int assemble_sgdml(mlff_ctx *ctx, const double *R_desc, const double *R_d_desc, int64_t M,
                   int n_atoms, const int32_t *perms, int n_perms, double sig);
int sgdml_descriptors(const double *R, int64_t M, int n_atoms, double *R_desc,
                      double *R_d_desc);
// kee[il * M + j] = sum_p Kee(sqrt5 |Rd_{i0+il} - Rd_j[P_p]|) (use_E_cstr, train.py:232-234)
void launch_sgdml_kee(const double *Rd, int64_t M, int64_t D, int64_t i0, int64_t ni,
                      const int32_t *Pt, int n_perms, double sig, double *kee, hipStream_t s);
// (r = i, s = j) point-pair records of the local points [i0, i0 + ni) (k_sgdml_uv, no mirror)
void launch_sgdml_records(const double *Rd, const double *Rdd, int64_t M, int n, int64_t D,
                          int64_t i0, int64_t ni, const int32_t *Pt, const int32_t *piinv,
                          int n_perms, double sig, double *uvk, hipStream_t s);
// out[jc * ldo + r] = sigma K_op[row0 + r, col_jc] for the local rows; col_jc = cols[jc]
// (device array, ncols entries) or, with cols == nullptr and ncols == 1, st->m_pi
void launch_sgdml_columns(const double *Rdd, int64_t M, int n, int64_t D, int64_t i0,
                          const int32_t *pi, const int32_t *piinv, int n_perms,
                          const double *uvk, int64_t row0, int64_t nrows, const int64_t *cols,
                          int64_t ncols, const DevState *st, double sigma, double *out,
                          int64_t ldo, hipStream_t s);

// ---- symmetric tiled operator (kernels_sym.hip) -----------------------------
// build the tiles this rank owns from the dense rows; check_symmetry compares
// every tile with its mirror (one rank only)
int sym_build(mlff_ctx *ctx, bool check_symmetry, bool *symmetric_out);
void sym_free(SymPack &sp);
// The search-direction update of the sharded iteration (k_update_p_gathered: p = z + beta p,
// z and every rank's rho partials in the gather buffer gb) folded into the tile mat-vec: the
// tile workgroups form the operand entries they read, the slot reduction writes p (gb null:
// not fused)
struct PGather {
  const double *gb = nullptr;
  int64_t gstride = 0, blk = 0;
  int world = 1;
  DevState *st = nullptr;
  long long it = 0;
};
// P <- slot partials of K v_full over the stored tiles
void launch_symv(const SymPack &sp, const double *v_full, double *P, const int *status,
                 hipStream_t s, PGather pg = PGather{});
// one rank: y[i] = sum of the slots of row i (i < n_out); epilogue y = sigma y + lam vloc
void launch_sym_reduce(const SymPack &sp, int64_t n_out, double *y, bool epilogue, double sigma,
                       double lam, const double *vloc, const int *status, hipStream_t s);
// one rank, PCG: q = sigma (slot sums) + lam p over n_out rows, and the p.q partial sums
// of the kVecGrid workgroups into pq_part
void launch_sym_reduce_pq(const SymPack &sp, int64_t n_out, double *y, double sigma, double lam,
                          const double *p, double *pq_part, const int *status, hipStream_t s,
                          PGather pg = PGather{});
// several ranks: sp.yg = this rank's slot sums of every row (rank blocks of sp.ystride);
// with p_full: also this rank's share sigma p.y_g + lam ||p_loc||^2 published into the
// tail slot `rank` of every block (pq_part / pp_part: kVecGrid scratch each)
void launch_sym_reduce_ranks(const SymPack &sp, int rank, int world, int64_t blk,
                             const double *p_full, double *pq_part, double *pp_part,
                             double sigma, double lam, const int *status, hipStream_t s,
                             PGather pg = PGather{}, bool separate_publish = false);
// y = sigma * src + lam * vloc over n entries (src may alias y)
void launch_axpby_loc(const double *src, double *y, int64_t n, double sigma, double lam,
                      const double *vloc, const int *status, hipStream_t s);
// reduce-scatter (sum) of ld doubles into blk doubles per rank
int comm_reduce_scatter(mlff_ctx *ctx, const double *send, double *recv, size_t count);

// ---- matrix-free sGDML operator (kernels_mf.hip) ---------------------------
int mf_setup(mlff_ctx *ctx, const double *R_desc, const double *R_d_desc, int64_t M, int n_atoms,
             const int32_t *perms, int n_perms, double sig);
// pq_part != nullptr: also the x_loc . y_loc partials (kVecGrid, as launch_dot_part)
// the search-direction update p = z + (rho / rho1) p (k_update_p) fused into the
// matrix-free operator of a PCG iteration (x_full = x_loc = p_old on one rank)
struct PFuse {
  const double *z;
  const double *rho_part;
  DevState *st;
  long long it;
  StopFold sf;  // the previous iteration's stop test (after a folded k_update_xr), or none
};
bool mf_can_fuse_p(const mlff_ctx *ctx);
void launch_mf_operator(const mlff_ctx *ctx, const double *x_full, double *y_loc,
                        const double *x_loc, const int *status, double sigma, double lam,
                        double *pq_part = nullptr, const PFuse *pf = nullptr);
int mf_diag(mlff_ctx *ctx, double *out);
// Zt = (J_j x_j)[P_p] of every (j, p) (k_mf_z), status gated.  pf: the operand is the search
// direction p = z + beta p_old formed on the fly from xc = p_old (k_update_p's arithmetic, the
// same bits), and the previous iteration's stop test runs in its first workgroup (pf->sf)
void launch_mf_zt(const MfData &mf, const double *xc, const int *status, hipStream_t s,
                  const PFuse *pf = nullptr);
// pair-tile form (kernels_pt.hip): available for D <= 288; its (j, p) chunks, padded D and the
// operator y_loc = sigma K x + lam x_loc (+ the x_loc . y_loc partials when pq_part is set)
bool pt_supported(int64_t D);
int pt_chunks(int64_t D, int64_t ni, int64_t MP);
int64_t pt_padded_d(int64_t D);
// pf (one rank, every row here): the search-direction update fused (k_mf_z forms p on the fly,
// k_pt_fin writes it) and the previous iteration's stop test folded into k_mf_z
void launch_pt_operator(const MfData &mf, const double *Rt, const double *xc, int64_t row0,
                        int64_t nrows, const double *x_loc, double *y_loc, const int *status,
                        double sigma, double lam, double *pq_part, hipStream_t s,
                        const PFuse *pf = nullptr);
// operator form in use: 0 pair sums (k_mf_pair ...), 1 record-factored, 2 pair-tile
int mf_form(const mlff_ctx *ctx);
// sigma K_op columns through the single-column path (mf.uvk); false when it is not set up
bool mf_columns(const mlff_ctx *ctx, const int64_t *cols, int64_t ncols, double sigma,
                double *out, int64_t ldo);
// training-set energy pair terms for coefficients alphas (N, contiguous): ni x M n_perms
int mf_energies(mlff_ctx *ctx, const double *alphas, double *E_pairs_host);
// diag(sigma K) of this rank's rows: dense rows or the matrix-free sGDML data
int operator_diag(mlff_ctx *ctx, double *out);
int sgdml_diag(mlff_ctx *ctx, const double *dRd, const double *dRdd, int64_t M, int n,
               const int32_t *dP, const int32_t *perms_host, const int32_t *piinv_host,
               int n_perms, double sig, double *diag_out);
double mf_bytes(const mlff_ctx *ctx);
// modelled seconds of one application of the matrix-free operator in its form on this rank,
// from the rates measured on MI355X: the storage choice of MLFF_STORAGE_AUTO
double mf_seconds(const mlff_ctx *ctx);
void mf_free(MfData &mf);
int desc_perm_tables(mlff_ctx *ctx, const int32_t *perms, int n, int n_perms,
                     std::vector<int32_t> &Pt, std::vector<int32_t> &piinv);

// ---- operator access for the builds (api.hip) --------------------------------
// require the operator and resolve its storage (builds the tiles if they are to be used)
int operator_prepare(mlff_ctx *ctx);
// y_loc = sigma_K K x over this rank's rows; x_loc = this rank's block (blk entries)
int operator_apply_local(mlff_ctx *ctx, const double *x_loc, double *y_loc);

// ---- eigen preconditioner (kernels_eig.hip) ----------------------------------
int eig_lowrank(mlff_ctx *ctx, int64_t k, int mask_mode, int64_t dim_i, double *Lt_out,
                double *evals_out, double *rowlev_out);
// eigenvalues (descending) of P_op A (preconditioned, the set low-rank preconditioner) or of
// A = sigma K + lam I: Iterative.solve(flag_eigvals=True) diagnostics, one rank
int spectrum(mlff_ctx *ctx, bool preconditioned, double *eig_out);
// test hook: C = alpha op(A) op(B) + beta C on the device from host arrays (splits > 1: the
// split-K slab path, returning C - alpha op(A) op(B) with beta = 1)
int test_gemm(mlff_ctx *ctx, int ta, int tb, int64_t M, int64_t Nc, int64_t Kd, double alpha,
              const double *A, int64_t lda, const double *B, int64_t ldb, double beta, double *C,
              int64_t ldc, int splits);

// ---- pivoted Cholesky (kernels_pivchol.hip) ---------------------------------
int pivoted_cholesky(mlff_ctx *ctx, int64_t k, int64_t *index_columns_out);

}  // namespace mlff
