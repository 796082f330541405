// Truncated eigen preconditioner and rank-k leverage scores on the device, without LAPACK.
//
// Reference (src/sGDML/sgdml/solvers/iterative_solver.py):
//   _init_precon_operator_eigvals :1177-1329   U, s, V = svd(K) (masked K for the
//       *_block_diagonal / *_atomic_interactions variants, :1238-1268);
//       L = U sqrt(s)[:, :k]; Woodbury (svd_preconditioner :1313-1329)
//   _rank_k_leverage_scores       :1110-1175   ||U[:, :k] row|| (not squared)
// S = sigma_K K is symmetric, so its SVD is its eigen-decomposition ordered by |eigenvalue|
// (U = eigenvectors, s = |eigenvalues|).  Only the top k pairs are used, so instead of
// the reference's O(N^3) full decomposition this is a truncated one:
//
//   block subspace iteration on the operator itself (any storage: matrix-free sGDML,
//   symmetric tiles, dense rows; sharded over the ranks like the PCG operator)
//     Q (b x N "wide" panel, b = k + max(16, k/2) rows) <- orth(S Q)
//   orth: shifted CholeskyQR3 (G = W W^T + shift, POTRF, TRSM; syrk/potrf/trsm kernels of
//         kernels_dense.hip; G all-reduced over the ranks, factored replicated)
//   every 4 iterations Rayleigh-Ritz: H = Q (S Q)^T (b x b), H = V diag(theta) V^T by a
//         cyclic parallel Jacobi on the device, Q <- V^T Q, stop when every one of the k
//         leading Ritz pairs has ||S u - theta u|| <= 1e-11 |theta_0|.
//   When b >= N / 2 the subspace is the whole space (Q = I, one Rayleigh-Ritz = the full
//   eigen-decomposition of S by Jacobi).
//
// The span after t iterations is span(S^t Q0) whatever happens in between, so the Ritz
// pairs converge at the subspace-iteration rate |lambda_{b+1} / lambda_i|^t; the
// Woodbury panel L L^T = U_k diag(s_k) U_k^T and the row norms ||U_k[i, :]|| only depend
// on the converged k-dimensional invariant subspace (not on a basis within it).  Q0 is a
// hash-seeded Gaussian panel indexed by GLOBAL row, so every row split starts from the
// same subspace.
#include <algorithm>
#include <cmath>
#include <numeric>

#include "common.h"

namespace mlff {

namespace {

__device__ __forceinline__ uint64_t splitmix64(uint64_t x) {
  x += 0x9E3779B97F4A7C15ull;
  x = (x ^ (x >> 30)) * 0xBF58476D1CE4E5B9ull;
  x = (x ^ (x >> 27)) * 0x94D049BB133111EBull;
  return x ^ (x >> 31);
}

// Q[j, i] ~ N(0, 1), a function of (seed, j, global row) only
__global__ __launch_bounds__(256) void k_eig_rand(double *__restrict__ Q, int64_t ldq,
                                                  int64_t nrows, int64_t row0, uint64_t seed) {
  const int64_t j = blockIdx.y;
  for (int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x; i < nrows;
       i += (int64_t)gridDim.x * 256) {
    const uint64_t h1 = splitmix64(seed ^ splitmix64((uint64_t)j * 0x100000001B3ull + (uint64_t)(row0 + i)));
    const uint64_t h2 = splitmix64(h1);
    const double u1 = ((double)(h1 >> 11) + 1.0) * (1.0 / 9007199254740993.0);  // (0, 1]
    const double u2 = (double)(h2 >> 11) * (1.0 / 9007199254740992.0);
    Q[j * ldq + i] = sqrt(-2.0 * log(u1)) * cos(6.283185307179586 * u2);
  }
}

// Q = the rows [g0, g0 + b) of the identity (global index g -> local column g - row0)
__global__ void k_eig_identity(double *__restrict__ Q, int64_t ldq, int64_t b, int64_t row0,
                               int64_t nrows) {
  const int64_t j = (int64_t)blockIdx.x * 256 + threadIdx.x;
  if (j >= b) return;
  const int64_t i = j - row0;
  if (i >= 0 && i < nrows) Q[j * ldq + i] = 1.0;
}

// ---- cyclic parallel Jacobi for a symmetric b x b matrix (row-major) ---------------
// Round r of a sweep pairs all m = b + (b odd) indices (circle method: index 0 fixed,
// 1..m-1 rotating; the index b of an odd b is a dummy), so the m/2 rotations of a round
// touch disjoint rows / columns: H <- G^T H G, V <- V G with G = I except
// G[p,p] = G[q,q] = c, G[p,q] = s, G[q,p] = -s, (c, s) zeroing H[p, q].
__device__ __forceinline__ void jac_pair(int m, int r, int i, int &p, int &q) {
  const int a = i == 0 ? 0 : 1 + (r + i - 1) % (m - 1);
  const int c = 1 + (r + m - 2 - i) % (m - 1);
  p = a < c ? a : c;
  q = a < c ? c : a;
}

// one workgroup per pair: rotation from (H_pp, H_qq, H_pq), then rows p, q
__global__ __launch_bounds__(256) void k_jac_rows(double *__restrict__ H, int b, int m, int r,
                                                  double *__restrict__ cs) {
  int p, q;
  jac_pair(m, r, blockIdx.x, p, q);
  __shared__ double sc[2];
  if (q >= b) {  // the dummy partner of an odd b
    if (threadIdx.x == 0) {
      cs[2 * blockIdx.x] = 1.0;
      cs[2 * blockIdx.x + 1] = 0.0;
    }
    return;
  }
  if (threadIdx.x == 0) {
    const double app = H[(int64_t)p * b + p], aqq = H[(int64_t)q * b + q];
    const double apq = H[(int64_t)p * b + q];
    double c = 1.0, s = 0.0;
    if (apq != 0.0) {
      const double th = (aqq - app) / (2.0 * apq);
      const double t = fabs(th) > 1e150 ? 0.5 / th
                                        : (th >= 0.0 ? 1.0 : -1.0) / (fabs(th) + sqrt(th * th + 1.0));
      c = 1.0 / sqrt(t * t + 1.0);
      s = t * c;
    }
    sc[0] = c;
    sc[1] = s;
    cs[2 * blockIdx.x] = c;
    cs[2 * blockIdx.x + 1] = s;
  }
  __syncthreads();
  const double c = sc[0], s = sc[1];
  if (s == 0.0) return;
  double *hp = H + (int64_t)p * b, *hq = H + (int64_t)q * b;
  for (int j = threadIdx.x; j < b; j += 256) {
    const double x = hp[j], y = hq[j];
    hp[j] = c * x - s * y;
    hq[j] = s * x + c * y;
  }
}

// columns p, q of H and V, rows split over blockIdx.y
__global__ __launch_bounds__(256) void k_jac_cols(double *__restrict__ H, double *__restrict__ V,
                                                  int b, int m, int r,
                                                  const double *__restrict__ cs) {
  int p, q;
  jac_pair(m, r, blockIdx.x, p, q);
  if (q >= b) return;
  const double c = cs[2 * blockIdx.x], s = cs[2 * blockIdx.x + 1];
  if (s == 0.0) return;
  const int i = blockIdx.y * 256 + threadIdx.x;
  if (i >= b) return;
  double *h = H + (int64_t)i * b, *v = V + (int64_t)i * b;
  const double x = h[p], y = h[q];
  h[p] = c * x - s * y;
  h[q] = s * x + c * y;
  const double vx = v[p], vy = v[q];
  v[p] = c * vx - s * vy;
  v[q] = s * vx + c * vy;
}

// partial sums of the squared off-diagonal and diagonal entries
__global__ __launch_bounds__(256) void k_jac_norms(const double *__restrict__ H, int b,
                                                   double *__restrict__ part) {
  __shared__ double sh[8];
  double off = 0.0, dia = 0.0;
  const int64_t nn = (int64_t)b * b;
  for (int64_t e = (int64_t)blockIdx.x * 256 + threadIdx.x; e < nn; e += (int64_t)gridDim.x * 256) {
    const double v = H[e];
    if (e / b == e % b)
      dia = fma(v, v, dia);
    else
      off = fma(v, v, off);
  }
  off = block_sum256(off, sh);
  __syncthreads();
  dia = block_sum256(dia, sh);
  if (threadIdx.x == 0) {
    part[2 * blockIdx.x] = off;  // block_sum256 leaves thread 0's result in its register
    part[2 * blockIdx.x + 1] = dia;
  }
}

__global__ void k_symmetrize(double *__restrict__ H, int b) {
  const int64_t e = (int64_t)blockIdx.x * 256 + threadIdx.x;
  if (e >= (int64_t)b * b) return;
  const int i = (int)(e / b), j = (int)(e % b);
  if (j <= i) return;
  const double v = 0.5 * (H[(int64_t)i * b + j] + H[(int64_t)j * b + i]);
  H[(int64_t)i * b + j] = v;
  H[(int64_t)j * b + i] = v;
}

__global__ void k_set_identity(double *__restrict__ V, int b) {
  const int64_t e = (int64_t)blockIdx.x * 256 + threadIdx.x;
  if (e >= (int64_t)b * b) return;
  V[e] = (e / b == e % b) ? 1.0 : 0.0;
}

// Vs[:, j] = V[:, ord[j]] (b x b)
__global__ void k_permute_cols(const double *__restrict__ V, const int *__restrict__ ord, int b,
                               double *__restrict__ Vs) {
  const int64_t e = (int64_t)blockIdx.x * 256 + threadIdx.x;
  if (e >= (int64_t)b * b) return;
  const int i = (int)(e / b), j = (int)(e % b);
  Vs[e] = V[(int64_t)i * b + ord[j]];
}

// res[j] = || Y[j] - theta_j Q[j] ||^2 over the local columns (one workgroup per row)
__global__ __launch_bounds__(256) void k_ritz_resid(const double *__restrict__ Y,
                                                    const double *__restrict__ Q, int64_t ld,
                                                    int64_t ncols, const double *__restrict__ theta,
                                                    double *__restrict__ res) {
  __shared__ double sh[8];
  const int64_t j = blockIdx.x;
  const double t = theta[j];
  double a = 0.0;
  for (int64_t i = threadIdx.x; i < ncols; i += 256) {
    const double d = Y[j * ld + i] - t * Q[j * ld + i];
    a = fma(d, d, a);
  }
  a = block_sum256(a, sh);
  if (threadIdx.x == 0) res[j] = a;
}

// Lt[j, i] = scale_j * Q[j, i]
__global__ void k_scale_rows(const double *__restrict__ Q, int64_t ld, int64_t ncols,
                             const double *__restrict__ scale, double *__restrict__ Lt) {
  const int64_t j = blockIdx.y;
  for (int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x; i < ncols;
       i += (int64_t)gridDim.x * 256)
    Lt[j * ld + i] = scale[j] * Q[j * ld + i];
}

// mask of iterative_solver.py:1238-1253 (atomic_interactions): zero every entry except the
// same-atom 3x3 blocks and the entries equal to max|K|
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

// rows of this rank (global row = row0 + a), columns in the padded layout (position c -> global
// column (c / blk) rows_per + c % blk; padding positions hold zeros); the global max|K| is the
// max of the W per-rank maxima in rmax
__global__ void k_mask_atomic(double *__restrict__ A, int64_t nrows, int64_t lda, int64_t dim_i,
                              int64_t row0, int64_t rows_per, int64_t blk,
                              const double *__restrict__ rmax, int world) {
  double mx = 0.0;
  for (int t = 0; t < world; ++t) mx = fmax(mx, rmax[t]);
  for (int64_t e = (int64_t)blockIdx.x * 256 + threadIdx.x; e < nrows * lda;
       e += (int64_t)gridDim.x * 256) {
    const int64_t a = row0 + e / lda, c = e % lda;
    const int64_t b = (c / blk) * rows_per + c % blk;
    const bool same_atom = ((a % dim_i) / 3) == ((b % dim_i) / 3);
    double &v = A[e];
    if (!same_atom && fabs(v) < mx) v = 0.0;
  }
}

__global__ void k_max_of(const double *__restrict__ part, int np, double *__restrict__ out) {
  if (threadIdx.x == 0) {
    double m = 0.0;
    for (int t = 0; t < np; ++t) m = fmax(m, part[t]);
    out[0] = m;
  }
}

constexpr double kEigTol = 1e-11;   // Ritz residual / |theta_0| of the k leading pairs
// accepted after kEigMaxIter iterations (slowly decaying spectrum around k): the pairs still
// span a good preconditioner subspace; the solve reports it (mlff_eig_info -> a warning)
constexpr double kEigAcceptTol = 1e-6;
constexpr int kEigMaxIter = 600;    // subspace iterations
constexpr int kEigRREvery = 4;      // Rayleigh-Ritz every this many iterations
constexpr int kJacMaxSweeps = 60;

unsigned grid1(int64_t n) { return (unsigned)std::max<int64_t>(1, std::min<int64_t>((n + 255) / 256, 65535)); }

}  // namespace

// symmetric eigen-decomposition H = V diag(theta) V^T of a b x b matrix in device memory
// (H is overwritten by diag(theta) to rounding, V by the eigenvectors as columns)
int jacobi_eigh(mlff_ctx *ctx, double *H, int b, double *V) {
  hipStream_t s = ctx->stream;
  ScratchScope scope(ctx);
  const int m = b + (b & 1);
  const int np = m / 2;
  double *cs = nullptr, *part = nullptr;
  MLFF_TRY(scratch_alloc(ctx, &cs, 2 * (size_t)np));
  constexpr int kNormBlocks = 128;
  MLFF_TRY(scratch_alloc(ctx, &part, 2 * kNormBlocks));
  hipLaunchKernelGGL(k_set_identity, dim3(grid1((int64_t)b * b)), dim3(256), 0, s, V, b);
  if (b < 2) return MLFF_OK;
  std::vector<double> h(2 * kNormBlocks);
  const dim3 gcols((unsigned)np, (unsigned)((b + 255) / 256));
  for (int sweep = 0; sweep < kJacMaxSweeps; ++sweep) {
    hipLaunchKernelGGL(k_jac_norms, dim3(kNormBlocks), dim3(256), 0, s, H, b, part);
    MLFF_HIP(ctx, hipMemcpyAsync(h.data(), part, sizeof(double) * h.size(), hipMemcpyDeviceToHost, s));
    MLFF_HIP(ctx, hipStreamSynchronize(s));
    double off = 0.0, dia = 0.0;
    for (int t = 0; t < kNormBlocks; ++t) {
      off += h[2 * t];
      dia += h[2 * t + 1];
    }
    if (!(off > 1e-30 * (off + dia))) break;  // ||offdiag||_F <= 1e-15 ||H||_F (or zero)
    for (int r = 0; r < m - 1; ++r) {
      hipLaunchKernelGGL(k_jac_rows, dim3((unsigned)np), dim3(256), 0, s, H, b, m, r, cs);
      hipLaunchKernelGGL(k_jac_cols, gcols, dim3(256), 0, s, H, V, b, m, r, (const double *)cs);
    }
    MLFF_HIP(ctx, hipGetLastError());
  }
  return MLFF_OK;
}

namespace {

// W (b x ncols wide, row stride ldw) <- C^-1 W with C C^T = W W^T (+ shift): orthonormal
// rows, nested spans.  Shifted CholeskyQR3 (Fukaya et al.): the first pass shifts the Gram
// matrix by 11 (N b + b (b + 1)) u ||W||_F^2 so the Cholesky exists for any conditioning.
int chol_qr3(mlff_ctx *ctx, double *W, int64_t b, int64_t ldw, double *G) {
  hipStream_t s = ctx->stream;
  for (int pass = 0; pass < 3; ++pass) {
    MLFF_TRY(syrk_wide(ctx, W, b, ctx->blk, ldw, G));
    MLFF_TRY(comm_allreduce(ctx, G, (size_t)(b * b)));
    bool shift = pass == 0;
    for (int attempt = 0; attempt < 2; ++attempt) {
      double *Gf = G + b * b;  // the factor is formed in a copy (G kept for a retry)
      MLFF_HIP(ctx, hipMemcpyAsync(Gf, G, sizeof(double) * b * b, hipMemcpyDeviceToDevice, s));
      if (shift) {
        std::vector<double> d(b);
        MLFF_HIP(ctx, hipMemcpy2DAsync(d.data(), sizeof(double), G, sizeof(double) * (b + 1),
                                       sizeof(double), b, hipMemcpyDeviceToHost, s));
        MLFF_HIP(ctx, hipStreamSynchronize(s));
        double tr = 0.0;
        for (double v : d) tr += v;
        const double shift_v =
            11.0 * ((double)ctx->N * b + (double)b * (b + 1)) * 1.1102230246251565e-16 * tr;
        launch_add_diag(Gf, b, shift_v, s);
      }
      const int rc = potrf_lower(ctx, Gf, b);
      if (rc == MLFF_OK) {
        MLFF_TRY(trsm_lower_wide(ctx, Gf, b, W, ctx->blk, ldw));
        break;
      }
      if (rc != MLFF_ERR_LINALG || shift) return rc;
      ctx->err.clear();
      shift = true;  // plain pass lost definiteness: repeat it shifted
    }
  }
  return MLFF_OK;
}

}  // namespace

int eig_lowrank(mlff_ctx *ctx, int64_t k, int mask_mode, int64_t dim_i, double *Lt_out,
                double *evals_out, double *rowlev_out) {
  hipStream_t s = ctx->stream;
  const int64_t n = ctx->N, blk = ctx->blk, nrows = ctx->nrows;
  MLFF_HIP(ctx, hipMemsetAsync(Lt_out, 0, sizeof(double) * round_up(k, 8) * blk, s));
  if (mask_mode == 1) {
    // eigvec_precon_block_diagonal zeroes the whole matrix (:1261): s = 0, L = 0
    if (evals_out) std::fill(evals_out, evals_out + k, 0.0);
    if (rowlev_out)
      for (int64_t i = 0; i < n; ++i) rowlev_out[i] = (i < k) ? 1.0 : 0.0;
    MLFF_HIP(ctx, hipStreamSynchronize(s));
    return MLFF_OK;
  }
  ScratchScope scope(ctx);
  // operator: S = sigma_K K in its resolved storage, or the masked dense copy (mask 2)
  double *A = nullptr;
  if (mask_mode == 2) {
    // this rank's rows of the masked S; the mask's threshold max|K| over all ranks (the
    // per-rank maxima all-gathered)
    double *part = nullptr, *rmax = nullptr;
    MLFF_TRY(scratch_alloc(ctx, &A, (size_t)blk * ctx->ld));
    MLFF_TRY(scratch_alloc(ctx, &part, 1024));
    MLFF_TRY(scratch_alloc(ctx, &rmax, (size_t)ctx->world));
    launch_scale_copy(ctx->K, A, blk * ctx->ld, ctx->sigma_K, s);
    hipLaunchKernelGGL(k_absmax_part, dim3(1024), dim3(256), 0, s, A, nrows * ctx->ld, part);
    hipLaunchKernelGGL(k_max_of, dim3(1), dim3(64), 0, s, part, 1024, rmax + ctx->rank);
    MLFF_TRY(comm_allgather(ctx, rmax + ctx->rank, rmax, 1));
    hipLaunchKernelGGL(k_mask_atomic, dim3(4096), dim3(256), 0, s, A, nrows, ctx->ld, dim_i,
                       ctx->row0, ctx->rows_per, blk, rmax, ctx->world);
    MLFF_HIP(ctx, hipGetLastError());
  } else {
    MLFF_TRY(operator_prepare(ctx));
  }
  auto apply = [&](const double *x_loc, double *y_loc) -> int {
    if (A == nullptr) return operator_apply_local(ctx, x_loc, y_loc);
    MLFF_HIP(ctx, hipMemcpyAsync(ctx->xg + (int64_t)ctx->rank * blk, x_loc, sizeof(double) * blk,
                                 hipMemcpyDeviceToDevice, s));
    if (ctx->world > 1)
      MLFF_TRY(comm_allgather(ctx, ctx->xg + (int64_t)ctx->rank * blk, ctx->xg, (size_t)blk));
    launch_gemv_rows(A, ctx->ld, nrows, ctx->xg, y_loc, 1.0, 0.0, nullptr, nullptr, s);
    return MLFF_OK;
  };

  const bool full = 2 * (k + std::max<int64_t>(16, k / 2)) >= n;
  const int64_t b = full ? n : std::min<int64_t>(n, k + std::max<int64_t>(16, k / 2));
  double *Q = nullptr, *Y = nullptr, *T = nullptr, *G = nullptr, *V = nullptr, *Vs = nullptr;
  double *theta_d = nullptr, *res_d = nullptr;
  int *ord_d = nullptr;
  const size_t panel = (size_t)round_up(b, 8) * blk;
  MLFF_TRY(scratch_alloc(ctx, &Q, panel));
  MLFF_TRY(scratch_alloc(ctx, &Y, panel));
  MLFF_TRY(scratch_alloc(ctx, &T, panel));
  MLFF_TRY(scratch_alloc(ctx, &G, 2 * (size_t)b * b));
  MLFF_TRY(scratch_alloc(ctx, &V, (size_t)b * b));
  MLFF_TRY(scratch_alloc(ctx, &Vs, (size_t)b * b));
  MLFF_TRY(scratch_alloc(ctx, &theta_d, b));
  MLFF_TRY(scratch_alloc(ctx, &res_d, b));
  MLFF_TRY(scratch_alloc(ctx, &ord_d, b));
  MLFF_HIP(ctx, hipMemsetAsync(Q, 0, sizeof(double) * panel, s));
  MLFF_HIP(ctx, hipMemsetAsync(Y, 0, sizeof(double) * panel, s));
  if (full) {
    hipLaunchKernelGGL(k_eig_identity, dim3(grid1(b)), dim3(256), 0, s, Q, blk, b, ctx->row0, nrows);
  } else {
    if (nrows > 0)
      hipLaunchKernelGGL(k_eig_rand, dim3((unsigned)std::min<int64_t>((nrows + 255) / 256, 64), (unsigned)b),
                         dim3(256), 0, s, Q, blk, nrows, ctx->row0, (uint64_t)0x5EEDull);
    MLFF_TRY(chol_qr3(ctx, Q, b, blk, G));
  }
  std::vector<double> theta(b), res(b);
  std::vector<int> ord(b);
  bool converged = false;
  for (int it = 1; it <= (full ? 1 : kEigMaxIter) && !converged; ++it) {
    for (int64_t j = 0; j < b; ++j) MLFF_TRY(apply(Q + j * blk, Y + j * blk));
    if (full || it % kEigRREvery == 0 || it == kEigMaxIter) {
      // Rayleigh-Ritz: H = Q Y^T, H = V diag(theta) V^T, Q <- V^T Q, Y <- V^T Y
      MLFF_TRY(gram_wide(ctx, Q, Y, b, blk, blk, G));
      MLFF_TRY(comm_allreduce(ctx, G, (size_t)(b * b)));
      hipLaunchKernelGGL(k_symmetrize, dim3(grid1(b * b)), dim3(256), 0, s, G, (int)b);
      MLFF_TRY(jacobi_eigh(ctx, G, (int)b, V));
      std::vector<double> hd(b);
      MLFF_HIP(ctx, hipMemcpy2DAsync(hd.data(), sizeof(double), G, sizeof(double) * (b + 1),
                                     sizeof(double), b, hipMemcpyDeviceToHost, s));
      MLFF_HIP(ctx, hipStreamSynchronize(s));
      std::iota(ord.begin(), ord.end(), 0);
      std::stable_sort(ord.begin(), ord.end(),
                       [&](int x, int y) { return std::fabs(hd[x]) > std::fabs(hd[y]); });
      for (int64_t j = 0; j < b; ++j) theta[j] = hd[ord[j]];
      MLFF_HIP(ctx, hipMemcpyAsync(ord_d, ord.data(), sizeof(int) * b, hipMemcpyHostToDevice, s));
      MLFF_HIP(ctx, hipMemcpyAsync(theta_d, theta.data(), sizeof(double) * b, hipMemcpyHostToDevice, s));
      hipLaunchKernelGGL(k_permute_cols, dim3(grid1(b * b)), dim3(256), 0, s, V, ord_d, (int)b, Vs);
      launch_gemm(true, false, b, blk, b, 1.0, Vs, b, Q, blk, 0.0, T, blk, s);
      std::swap(Q, T);
      launch_gemm(true, false, b, blk, b, 1.0, Vs, b, Y, blk, 0.0, T, blk, s);
      std::swap(Y, T);
      hipLaunchKernelGGL(k_ritz_resid, dim3((unsigned)b), dim3(256), 0, s, Y, Q, blk, blk, theta_d, res_d);
      MLFF_TRY(comm_allreduce(ctx, res_d, (size_t)b));
      MLFF_HIP(ctx, hipMemcpyAsync(res.data(), res_d, sizeof(double) * b, hipMemcpyDeviceToHost, s));
      MLFF_HIP(ctx, hipStreamSynchronize(s));
      double worst = 0.0;
      for (int64_t j = 0; j < k; ++j) worst = std::max(worst, std::sqrt(std::max(res[j], 0.0)));
      converged = worst <= kEigTol * std::fabs(theta[0]) || full;
    }
    if (!converged) {  // Q <- orth(S Q)
      MLFF_HIP(ctx, hipMemcpyAsync(Q, Y, sizeof(double) * panel, hipMemcpyDeviceToDevice, s));
      MLFF_TRY(chol_qr3(ctx, Q, b, blk, G));
    }
  }
  {
    double worst = 0.0;
    for (int64_t j = 0; j < k; ++j) worst = std::max(worst, std::sqrt(std::max(res[j], 0.0)));
    ctx->eig_rel_resid = theta[0] != 0.0 ? worst / std::fabs(theta[0]) : 0.0;
    ctx->eig_converged = converged;
  }
  if (!converged && !(ctx->eig_rel_resid <= kEigAcceptTol))
    return set_error(ctx, MLFF_ERR_LINALG, "truncated eigensolver: no convergence in " +
                                               std::to_string(kEigMaxIter) + " subspace iterations");
  // outputs: s_j = |theta_j|, L rows = sqrt(s_j) u_j, ||U_k[i, :]||
  std::vector<double> scale(k);
  for (int64_t j = 0; j < k; ++j) {
    scale[j] = std::sqrt(std::fabs(theta[j]));
    if (evals_out) evals_out[j] = std::fabs(theta[j]);
  }
  if (rowlev_out) {
    MLFF_HIP(ctx, hipMemsetAsync(ctx->xg, 0, sizeof(double) * ctx->ld, s));
    launch_colsumsq(Q, k, nrows, blk, ctx->xg + (int64_t)ctx->rank * blk, s);
    if (ctx->world > 1)
      MLFF_TRY(comm_allgather(ctx, ctx->xg + (int64_t)ctx->rank * blk, ctx->xg, (size_t)blk));
    for (int r = 0; r < ctx->world; ++r) {
      const int64_t g0 = (int64_t)r * ctx->rows_per;
      if (g0 >= n) break;
      const int64_t cnt = std::min<int64_t>(ctx->rows_per, n - g0);
      MLFF_HIP(ctx, hipMemcpyAsync(rowlev_out + g0, ctx->xg + (int64_t)r * blk,
                                   sizeof(double) * cnt, hipMemcpyDeviceToHost, s));
    }
    MLFF_HIP(ctx, hipStreamSynchronize(s));
    for (int64_t i = 0; i < n; ++i) rowlev_out[i] = std::sqrt(rowlev_out[i]);
  }
  MLFF_HIP(ctx, hipMemcpyAsync(theta_d, scale.data(), sizeof(double) * k, hipMemcpyHostToDevice, s));
  if (nrows > 0)
    hipLaunchKernelGGL(k_scale_rows, dim3((unsigned)std::min<int64_t>((nrows + 255) / 256, 64), (unsigned)k),
                       dim3(256), 0, s, Q, blk, nrows, theta_d, Lt_out);
  MLFF_HIP(ctx, hipGetLastError());
  MLFF_HIP(ctx, hipStreamSynchronize(s));
  return MLFF_OK;
}

// ---------------------------------------------------------------------------
// Spectrum diagnostics of Iterative.solve(flag_eigvals=True) (iterative_solver.py:978-989,
// dev_utils.py:8-25): the reference forms K = -K_op column by column, P_K = P_op @ K and
// takes scipy.linalg.eigvals(P_K) (and of K alone for eigvals_K).  Here, with A = sigma K +
// lam I the PCG operator (= -K_op for the sGDML sign) and P_op = sigma_p (I - T^T T) / lam
// the low-rank preconditioner: A = R R^T (Cholesky), eig(P_op A) = sigma_p eig(R^T W R) with
// the symmetric R^T W R = (R^T R - (T R)^T (T R)) / lam, W = (I - T^T T) / lam; without a
// preconditioner eig(A).  Symmetric eigenvalues by the device Jacobi, sorted descending.
// One rank; O(N^3) like the reference's dense eigvals.
namespace {
__global__ void k_copy_block_diag(const double *__restrict__ Y, int64_t ldy, int64_t n, double lam,
                                  double *__restrict__ A) {
  for (int64_t e = (int64_t)blockIdx.x * 256 + threadIdx.x; e < n * n;
       e += (int64_t)gridDim.x * 256) {
    const int64_t i = e / n, j = e % n;
    A[e] = Y[i * ldy + j] + (i == j ? lam : 0.0);
  }
}
}  // namespace

int spectrum(mlff_ctx *ctx, bool preconditioned, double *eig_out) {
  hipStream_t s = ctx->stream;
  const int64_t n = ctx->N, blk = ctx->blk;
  if (ctx->world > 1) return set_error(ctx, MLFF_ERR_ARG, "spectrum: one rank only");
  if (n > 46340) return set_error(ctx, MLFF_ERR_ARG, "spectrum: N too large for a dense N x N");
  if (preconditioned && ctx->precon_kind == MLFF_PRECON_NONE) preconditioned = false;
  MLFF_TRY(operator_prepare(ctx));
  ScratchScope scope(ctx);
  double *Y = nullptr, *A = nullptr, *V = nullptr, *x = nullptr;
  MLFF_TRY(scratch_alloc(ctx, &Y, (size_t)round_up(n, 8) * blk));
  MLFF_TRY(scratch_alloc(ctx, &A, (size_t)n * n));
  MLFF_TRY(scratch_alloc(ctx, &V, (size_t)n * n));
  MLFF_TRY(scratch_alloc(ctx, &x, (size_t)round_up(n, 8) * blk));
  // A = sigma K + lam I, row j = the operator applied to e_j (K symmetric)
  MLFF_HIP(ctx, hipMemsetAsync(x, 0, sizeof(double) * round_up(n, 8) * blk, s));
  hipLaunchKernelGGL(k_eig_identity, dim3(grid1(n)), dim3(256), 0, s, x, blk, n, (int64_t)0, ctx->nrows);
  for (int64_t j = 0; j < n; ++j) MLFF_TRY(operator_apply_local(ctx, x + j * blk, Y + j * blk));
  hipLaunchKernelGGL(k_copy_block_diag, dim3(grid1(n * n)), dim3(256), 0, s, Y, blk, n, ctx->lam, A);
  hipLaunchKernelGGL(k_symmetrize, dim3(grid1(n * n)), dim3(256), 0, s, A, (int)n);
  double *H = A;
  if (preconditioned) {
    // R = chol(A) (lower, in place in a copy); H = (R^T R - X^T X) / lam, X = T R (k x n)
    double *R = Y;  // Y is free now (n x n fits in its n x blk)
    MLFF_HIP(ctx, hipMemcpyAsync(R, A, sizeof(double) * n * n, hipMemcpyDeviceToDevice, s));
    MLFF_TRY(potrf_lower(ctx, R, n));
    const int64_t k = ctx->k;
    double *X = x;  // k x n
    launch_gemm(false, false, k, n, n, 1.0, ctx->T, blk, R, n, 0.0, X, n, s);
    launch_gemm(true, false, n, n, n, 1.0 / ctx->lam, R, n, R, n, 0.0, A, n, s);
    launch_gemm(true, false, n, n, k, -1.0 / ctx->lam, X, n, X, n, 1.0, A, n, s);
    hipLaunchKernelGGL(k_symmetrize, dim3(grid1(n * n)), dim3(256), 0, s, A, (int)n);
    MLFF_HIP(ctx, hipGetLastError());
  }
  MLFF_TRY(jacobi_eigh(ctx, H, (int)n, V));
  std::vector<double> d(n);
  MLFF_HIP(ctx, hipMemcpy2DAsync(d.data(), sizeof(double), H, sizeof(double) * (n + 1), sizeof(double),
                                 n, hipMemcpyDeviceToHost, s));
  MLFF_HIP(ctx, hipStreamSynchronize(s));
  const double sg = preconditioned ? ctx->sigma_p : 1.0;
  for (int64_t i = 0; i < n; ++i) d[i] *= sg;
  std::sort(d.begin(), d.end(), [](double a, double b) { return a > b; });
  std::copy(d.begin(), d.end(), eig_out);
  return MLFF_OK;
}

}  // namespace mlff
