// Truncated eigen preconditioner and rank-k leverage scores on the device.
//
// Reference (src/sGDML/sgdml/solvers/iterative_solver.py):
//   _init_precon_operator_eigvals :1177-1329   U, s, V = svd(K) (masked K for the
//       *_block_diagonal / *_atomic_interactions variants, :1238-1268);
//       L = U sqrt(s)[:, :k]; Woodbury (svd_preconditioner :1313-1329)
//   _rank_k_leverage_scores       :1110-1175   ||U[:, :k] row|| (not squared)
// S = sigma_K K is symmetric PSD, so its SVD is its eigen-decomposition ordered by
// |eigenvalue|.  The O(N^3) symmetric eigensolve is a build-time LAPACK call (as
// scipy's svd is in the reference): rocSOLVER dsyevd, loaded with dlopen so the
// library has no link-time dependency on it.  Everything around it (copy/scale,
// masking, the k x N factor gather, Woodbury) is this library's own kernels.
#include <dlfcn.h>

#include <algorithm>
#include <cmath>
#include <numeric>

#include "common.h"

namespace mlff {

namespace {

typedef int (*fn_create_t)(void **);
typedef int (*fn_destroy_t)(void *);
typedef int (*fn_set_stream_t)(void *, hipStream_t);
typedef int (*fn_dsyevd_t)(void *, int, int, int, double *, int, double *, double *, int *);
constexpr int kEvectOriginal = 211;  // rocblas_evect_original
constexpr int kFillLower = 122;      // rocblas_fill_lower

struct RocSolver {
  bool ok = false;
  std::string why;
  fn_create_t create = nullptr;
  fn_destroy_t destroy = nullptr;
  fn_set_stream_t set_stream = nullptr;
  fn_dsyevd_t dsyevd = nullptr;
};

RocSolver &rocsolver() {
  static RocSolver r = [] {
    RocSolver s;
    void *hb = dlopen("librocblas.so.5", RTLD_NOW | RTLD_GLOBAL);
    if (!hb) hb = dlopen("/opt/rocm/lib/librocblas.so.5", RTLD_NOW | RTLD_GLOBAL);
    void *hs = dlopen("librocsolver.so.0", RTLD_NOW | RTLD_GLOBAL);
    if (!hs) hs = dlopen("/opt/rocm/lib/librocsolver.so.0", RTLD_NOW | RTLD_GLOBAL);
    if (!hb || !hs) {
      s.why = std::string("cannot load rocBLAS/rocSOLVER: ") + (dlerror() ? dlerror() : "");
      return s;
    }
    s.create = (fn_create_t)dlsym(hb, "rocblas_create_handle");
    s.destroy = (fn_destroy_t)dlsym(hb, "rocblas_destroy_handle");
    s.set_stream = (fn_set_stream_t)dlsym(hb, "rocblas_set_stream");
    s.dsyevd = (fn_dsyevd_t)dlsym(hs, "rocsolver_dsyevd");
    s.ok = s.create && s.destroy && s.set_stream && s.dsyevd;
    if (!s.ok) s.why = "rocBLAS/rocSOLVER symbols missing";
    return s;
  }();
  return r;
}

__global__ void k_absmax_part(const double *__restrict__ A, int64_t n_elem,
                              double *__restrict__ part) {
  __shared__ double sh[256];
  double m = 0.0;
  for (int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x; i < n_elem;
       i += (int64_t)gridDim.x * 256)
    m = fmax(m, fabs(A[i]));
  sh[threadIdx.x] = m;
  __syncthreads();
  for (int o = 128; o > 0; o >>= 1) {
    if (threadIdx.x < o) sh[threadIdx.x] = fmax(sh[threadIdx.x], sh[threadIdx.x + o]);
    __syncthreads();
  }
  if (threadIdx.x == 0) part[blockIdx.x] = sh[0];
}

// iterative_solver.py:1238-1253: zero every entry except the same-atom 3x3 blocks
// (row and column atom equal modulo the molecule) and the entries equal to max|K|.
__global__ void k_mask_atomic(double *__restrict__ A, int64_t n, int64_t lda, int64_t dim_i,
                              const double *__restrict__ part, int np) {
  double mx = 0.0;
  for (int t = 0; t < np; ++t) mx = fmax(mx, part[t]);
  for (int64_t e = (int64_t)blockIdx.x * 256 + threadIdx.x; e < n * n;
       e += (int64_t)gridDim.x * 256) {
    const int64_t a = e / n, b = e % n;
    const bool same_atom = ((a % dim_i) / 3) == ((b % dim_i) / 3);
    double &v = A[a * lda + b];
    if (!same_atom && fabs(v) < mx) v = 0.0;
  }
}

// Lt[j, i] = scale_j * V[sel_j, i]  (eigenvector sel_j is row sel_j of the row-major
// view of the column-major dsyevd output)
__global__ void k_gather_eigvecs(const double *__restrict__ V, int64_t ldv, int64_t n,
                                 const int64_t *__restrict__ sel,
                                 const double *__restrict__ scale, double *__restrict__ Lt,
                                 int64_t ldl) {
  const int64_t j = blockIdx.y;
  const double sc = scale[j];
  const double *src = V + sel[j] * ldv;
  for (int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x; i < n;
       i += (int64_t)gridDim.x * 256)
    Lt[j * ldl + i] = sc * src[i];
}

}  // namespace

int eig_lowrank(mlff_ctx *ctx, int64_t k, int mask_mode, int64_t dim_i, double *Lt_out,
                double *evals_out, double *rowlev_out) {
  hipStream_t s = ctx->stream;
  const int64_t n = ctx->N, ld = ctx->ld;
  MLFF_HIP(ctx, hipMemsetAsync(Lt_out, 0, sizeof(double) * round_up(k, 8) * ctx->blk, s));
  if (mask_mode == 1) {
    // eigvec_precon_block_diagonal zeroes the whole matrix (:1261): s = 0, L = 0
    if (evals_out) std::fill(evals_out, evals_out + k, 0.0);
    if (rowlev_out) {
      for (int64_t i = 0; i < n; ++i) rowlev_out[i] = (i < k) ? 1.0 : 0.0;
    }
    MLFF_HIP(ctx, hipStreamSynchronize(s));
    return MLFF_OK;
  }
  RocSolver &rs = rocsolver();
  if (!rs.ok) return set_error(ctx, MLFF_ERR_HIP, rs.why);
  double *A = nullptr, *D = nullptr, *E = nullptr, *part = nullptr, *dscale = nullptr;
  int64_t *dsel = nullptr;
  int *dinfo = nullptr;
  MLFF_HIP(ctx, hipMalloc(&A, sizeof(double) * n * ld));
  MLFF_HIP(ctx, hipMalloc(&D, sizeof(double) * n));
  MLFF_HIP(ctx, hipMalloc(&E, sizeof(double) * n));
  MLFF_HIP(ctx, hipMalloc(&part, sizeof(double) * 1024));
  MLFF_HIP(ctx, hipMalloc(&dinfo, sizeof(int)));
  launch_scale_copy(ctx->K, A, n * ld, ctx->sigma_K, s);  // S = sigma_K K
  if (mask_mode == 2) {
    hipLaunchKernelGGL(k_absmax_part, dim3(1024), dim3(256), 0, s, A, n * ld, part);
    hipLaunchKernelGGL(k_mask_atomic, dim3(4096), dim3(256), 0, s, A, n, ld, dim_i, part, 1024);
  }
  MLFF_HIP(ctx, hipGetLastError());
  void *handle = nullptr;
  if (rs.create(&handle) != 0) return set_error(ctx, MLFF_ERR_HIP, "rocblas_create_handle failed");
  rs.set_stream(handle, s);
  const int st = rs.dsyevd(handle, kEvectOriginal, kFillLower, (int)n, A, (int)ld, D, E, dinfo);
  int hinfo = 0;
  MLFF_HIP(ctx, hipMemcpyAsync(&hinfo, dinfo, sizeof(int), hipMemcpyDeviceToHost, s));
  MLFF_HIP(ctx, hipStreamSynchronize(s));
  rs.destroy(handle);
  if (st != 0 || hinfo != 0) {
    hipFree(A);
    return set_error(ctx, MLFF_ERR_LINALG, "rocsolver_dsyevd failed (status " + std::to_string(st) +
                                               ", info " + std::to_string(hinfo) + ")");
  }
  // order by |eigenvalue| descending (= singular values of svd)
  std::vector<double> w(n);
  MLFF_HIP(ctx, hipMemcpy(w.data(), D, sizeof(double) * n, hipMemcpyDeviceToHost));
  std::vector<int64_t> order(n);
  std::iota(order.begin(), order.end(), 0);
  std::stable_sort(order.begin(), order.end(),
                   [&](int64_t a, int64_t b) { return std::fabs(w[a]) > std::fabs(w[b]); });
  std::vector<int64_t> sel(order.begin(), order.begin() + k);
  std::vector<double> scale(k), ones(k, 1.0);
  for (int64_t j = 0; j < k; ++j) {
    scale[j] = std::sqrt(std::fabs(w[sel[j]]));
    if (evals_out) evals_out[j] = std::fabs(w[sel[j]]);
  }
  MLFF_HIP(ctx, hipMalloc(&dsel, sizeof(int64_t) * k));
  MLFF_HIP(ctx, hipMalloc(&dscale, sizeof(double) * k));
  MLFF_HIP(ctx, hipMemcpy(dsel, sel.data(), sizeof(int64_t) * k, hipMemcpyHostToDevice));
  const unsigned gx = (unsigned)std::min<int64_t>((n + 255) / 256, 64);
  if (rowlev_out) {
    // ||U[i, :k]||: column norms of the unscaled k x N panel
    MLFF_HIP(ctx, hipMemcpy(dscale, ones.data(), sizeof(double) * k, hipMemcpyHostToDevice));
    hipLaunchKernelGGL(k_gather_eigvecs, dim3(gx, (unsigned)k), dim3(256), 0, s, A, ld, n, dsel,
                       dscale, Lt_out, ctx->blk);
    launch_colsumsq(Lt_out, k, n, ctx->blk, D, s);
    MLFF_HIP(ctx, hipMemcpyAsync(rowlev_out, D, sizeof(double) * n, hipMemcpyDeviceToHost, s));
    MLFF_HIP(ctx, hipStreamSynchronize(s));
    for (int64_t i = 0; i < n; ++i) rowlev_out[i] = std::sqrt(rowlev_out[i]);
  }
  MLFF_HIP(ctx, hipMemcpy(dscale, scale.data(), sizeof(double) * k, hipMemcpyHostToDevice));
  hipLaunchKernelGGL(k_gather_eigvecs, dim3(gx, (unsigned)k), dim3(256), 0, s, A, ld, n, dsel,
                     dscale, Lt_out, ctx->blk);
  MLFF_HIP(ctx, hipGetLastError());
  MLFF_HIP(ctx, hipStreamSynchronize(s));
  hipFree(A);
  hipFree(D);
  hipFree(E);
  hipFree(part);
  hipFree(dinfo);
  hipFree(dsel);
  hipFree(dscale);
  return MLFF_OK;
}

}  // namespace mlff
