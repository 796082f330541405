// Smallest eigenvalue of a symmetric m x m matrix on the device: the eigenvalue test of the
// reference's _cho_factor_stable (src/sGDML/sgdml/solvers/iterative_solver.py:576-579,
// `lo_eig = scipy.linalg.eigh(M, eigvals_only=True, eigvals=(0, 0))`, lower triangle).  For
// one eigenvalue scipy's eigh runs LAPACK dsyevr with RANGE='I', IL = IU = 1, which reduces M
// to tridiagonal form (dsytrd, Householder reflectors on the lower triangle) and bisects the
// tridiagonal matrix with Sturm counts (dstebz).  The same two steps here:
//
//  1. Householder tridiagonalisation (dsytd2's algorithm, UPLO = 'L'), two launches per
//     column j: k_trd_reflect (one workgroup) forms w_{j-1} = p - tau/2 (p.v) v from the
//     previous column's p = tau A v, applies that column's pending rank-2 update to row j
//     (= column j: the working copy is kept fully symmetric) and builds reflector j (dlarfg);
//     k_trd_update_symv (one wave per row of the trailing block) applies the pending update
//     A -= v w^T + w v^T to its row and forms p = tau A v of reflector j in the same pass,
//     so the trailing block is read and written once per column.
//  2. Multisection with Sturm counts (dstebz's count with its pivmin guard) in one wave:
//     64 shifts per round, the interval shrinks 65x per round, from the Gershgorin interval
//     down to a few ulps.
//
// The computed value carries the backward error of the reduction (~ m eps ||M||), as LAPACK's
// does; its sign is therefore the reference's decision wherever |lo_eig| is above that
// rounding level.
#include "common.h"

#include <algorithm>
#include <cstdlib>

namespace mlff {

namespace {

constexpr int kRefThreads = 1024;

__device__ inline double block_sum_1024(double v, double *red) {
  // wave sums, then the 16 wave sums in a fixed order (same bits in every thread)
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o);
  const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63;
  __syncthreads();
  if (lane == 0) red[wave] = v;
  __syncthreads();
  double s = 0.0;
#pragma unroll
  for (int w = 0; w < kRefThreads / 64; ++w) s += red[w];
  return s;
}

// Symmetrise the lower triangle of M into the working copy A (eigh reads UPLO = 'L').
__global__ __launch_bounds__(256) void k_trd_copy_lower(const double *__restrict__ M,
                                                        double *__restrict__ A, int64_t m) {
  for (int64_t e = (int64_t)blockIdx.x * 256 + threadIdx.x; e < m * m;
       e += (int64_t)gridDim.x * 256) {
    const int64_t i = e / m, j = e % m;
    A[e] = (j <= i) ? M[e] : M[j * m + i];
  }
}

// Column j: (1) w_{j-1} from p and v_{j-1} (j >= 1), (2) row j with the pending update of
// step j-1, d[j], (3) the reflector of x = A[j+1:, j] (dlarfg): v_j (v_j[j+1] = 1), tau[j],
// e[j].  One workgroup.
__global__ __launch_bounds__(kRefThreads) void k_trd_reflect(
    const double *__restrict__ A, int64_t m, int64_t j, const double *__restrict__ p,
    const double *__restrict__ vprev, double *__restrict__ wprev, double *__restrict__ vnew,
    double *__restrict__ tau, double *__restrict__ d, double *__restrict__ e) {
  __shared__ double red[kRefThreads / 64];
  const int tid = threadIdx.x;
  const double *row = A + j * m;
  if (j >= 1) {
    // w = p - (tau/2) (p . v) v over the trailing block of step j-1 (indices >= j)
    double s = 0.0;
    for (int64_t i = j + tid; i < m; i += kRefThreads) s += p[i] * vprev[i];
    const double pv = block_sum_1024(s, red);
    const double alpha = -0.5 * tau[j - 1] * pv;
    for (int64_t i = j + tid; i < m; i += kRefThreads) wprev[i] = p[i] + alpha * vprev[i];
    __syncthreads();  // wprev[j] is read by every thread below
  }
  const double vj = (j >= 1) ? vprev[j] : 0.0, wj = (j >= 1) ? wprev[j] : 0.0;
  auto a_at = [&](int64_t i) {
    double a = row[i];
    if (j >= 1) a = a - vj * wprev[i] - wj * vprev[i];
    return a;
  };
  if (tid == 0) d[j] = a_at(j);
  if (j == m - 1) return;
  // xnorm of A[j+2:, j] (dnrm2 up to rounding: a plain sum of squares)
  double s = 0.0;
  for (int64_t i = j + 2 + tid; i < m; i += kRefThreads) {
    const double a = a_at(i);
    s += a * a;
  }
  const double xnorm = sqrt(block_sum_1024(s, red));
  const double alpha = a_at(j + 1);
  double t = 0.0, beta = alpha, scal = 0.0;
  if (xnorm != 0.0) {
    beta = -copysign(hypot(alpha, xnorm), alpha);
    t = (beta - alpha) / beta;
    scal = 1.0 / (alpha - beta);
  }
  if (tid == 0) {
    tau[j] = t;
    e[j] = beta;
    vnew[j + 1] = 1.0;
  }
  for (int64_t i = j + 2 + tid; i < m; i += kRefThreads) vnew[i] = a_at(i) * scal;
}

// Trailing block of column j (rows / columns > j): A -= vprev wprev^T + wprev vprev^T (the
// pending update of step j-1, j >= 1) written back, and p = tau_j A v_j.  One wave per row.
__global__ __launch_bounds__(256) void k_trd_update_symv(
    double *__restrict__ A, int64_t m, int64_t j, const double *__restrict__ vprev,
    const double *__restrict__ wprev, const double *__restrict__ v, const double *__restrict__ tau,
    double *__restrict__ p) {
  const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63;
  const int64_t r = j + 1 + (int64_t)blockIdx.x * 4 + wave;
  if (r >= m) return;
  double *row = A + r * m;
  double s = 0.0;
  if (j >= 1) {
    const double vr = vprev[r], wr = wprev[r];
    for (int64_t c = j + 1 + lane; c < m; c += 64) {
      const double a = row[c] - vr * wprev[c] - wr * vprev[c];
      row[c] = a;
      s += a * v[c];
    }
  } else {
    for (int64_t c = j + 1 + lane; c < m; c += 64) s += row[c] * v[c];
  }
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) s += __shfl_xor(s, o);
  if (lane == 0) p[r] = tau[j] * s;
}

// ---------------------------------------------------------------------------
// Blocked reduction (dsytrd / dlatrd, UPLO = 'L'): panels of NB columns.  Inside a panel the
// trailing block is only READ (y = A v with the block as the last SYR2K left it, the panel's
// pending updates applied as corrections V t + W s); after the panel one GEMM applies them all,
// A -= [V W] [W V]^T.  Per column: the symv reads the trailing block once (8 bytes per entry
// instead of the unblocked update's read + write, 16), the rank-2 NB updates run on the matrix
// cores.  VW / WV: m x 2 NB row-major, row i = [V(i, 0:NB) | W(i, 0:NB)] and [W | V].
constexpr int kNB = 16;

__device__ inline void block_sum_many_1024(double (&v)[2 * kNB], int cnt, double *red, double *out) {
  // the 16 wave sums of each of the cnt values, then the waves added in order by thread q
  const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63;
  __syncthreads();
#pragma unroll
  for (int q = 0; q < 2 * kNB; ++q) {
    if (q >= cnt) break;
    double x = v[q];
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) x += __shfl_xor(x, o);
    if (lane == 0) red[wave * 2 * kNB + q] = x;
  }
  __syncthreads();
  if (threadIdx.x < cnt) {
    double sum = 0.0;
    for (int w = 0; w < kRefThreads / 64; ++w) sum += red[w * 2 * kNB + threadIdx.x];
    out[threadIdx.x] = sum;
  }
  __syncthreads();
}

// Column j of its panel (c = j - j0): (1) c > 0: W(:, c - 1) from the symv y of reflector
// v_{j-1} (t = W^T v, s = V^T v over the panel's earlier columns; w = tau (y - V t - W s);
// w += -tau/2 (w . v) v), (2) column j of A with the panel's updates applied, d[j], (3) the
// reflector of column j (dlarfg) -> V(:, c), tau[j], e[j].  last: only step (1) (the panel's
// final w; c = the panel width).  One workgroup.
__global__ __launch_bounds__(kRefThreads) void k_trd_panel_col(
    const double *__restrict__ A, int64_t m, int64_t j0, int64_t j, int c, bool last,
    const double *__restrict__ y, double *__restrict__ VW, double *__restrict__ WV,
    double *__restrict__ col, double *__restrict__ tau, double *__restrict__ d,
    double *__restrict__ e) {
  __shared__ double red[(kRefThreads / 64) * 2 * kNB];
  __shared__ double ts[2 * kNB];
  const int tid = threadIdx.x;
  const int64_t ld = 2 * kNB;
  if (c > 0) {
    // reflector c - 1 lives in rows >= j (v[j] = 1); its symv y over rows >= j
    const int q = c - 1;
    double acc[2 * kNB];
#pragma unroll
    for (int u = 0; u < 2 * kNB; ++u) acc[u] = 0.0;
    for (int64_t i = j + tid; i < m; i += kRefThreads) {
      const double vi = VW[i * ld + q];
      const double *row = VW + i * ld;
#pragma unroll
      for (int u = 0; u < kNB; ++u) {
        if (u >= q) break;
        acc[u] = fma(row[kNB + u], vi, acc[u]);   // t_u = W(:, u) . v
        acc[kNB + u] = fma(row[u], vi, acc[kNB + u]);  // s_u = V(:, u) . v
      }
    }
    // compact: [t_0 .. t_{q-1}, s_0 .. s_{q-1}]
    double pk[2 * kNB];
#pragma unroll
    for (int u = 0; u < 2 * kNB; ++u) pk[u] = 0.0;
#pragma unroll
    for (int u = 0; u < kNB; ++u)
      if (u < q) {
        pk[u] = acc[u];
        pk[q + u] = acc[kNB + u];
      }
    block_sum_many_1024(pk, 2 * q, red, ts);
    const double tq = tau[j - 1];
    double dot = 0.0;
    for (int64_t i = j + tid; i < m; i += kRefThreads) {
      const double *row = VW + i * ld;
      double w = y[i];
      for (int u = 0; u < q; ++u) w -= row[u] * ts[u] + row[kNB + u] * ts[q + u];
      w *= tq;
      col[i] = w;  // staged
      dot += w * row[q];
    }
    const double alpha = -0.5 * tq * block_sum_1024(dot, red);
    for (int64_t i = j + tid; i < m; i += kRefThreads) {
      const double w = fma(alpha, VW[i * ld + q], col[i]);
      VW[i * ld + kNB + q] = w;
      WV[i * ld + q] = w;
    }
    __syncthreads();
  }
  if (last || j >= m) return;
  // column j (= row j: A symmetric) with the panel's c updates, rows >= j
  const double *arow = A + j * m;
  const double *vj = VW + j * ld;
  for (int64_t i = j + tid; i < m; i += kRefThreads) {
    const double *row = VW + i * ld;
    double a = arow[i];
    for (int u = 0; u < c; ++u) a -= row[u] * vj[kNB + u] + row[kNB + u] * vj[u];
    col[i] = a;
  }
  __syncthreads();
  if (tid == 0) d[j] = col[j];
  if (j == m - 1) return;
  double sq = 0.0;
  for (int64_t i = j + 2 + tid; i < m; i += kRefThreads) sq += col[i] * col[i];
  const double xnorm = sqrt(block_sum_1024(sq, red));
  const double alpha = col[j + 1];
  double t = 0.0, beta = alpha, scal = 0.0;
  if (xnorm != 0.0) {
    beta = -copysign(hypot(alpha, xnorm), alpha);
    t = (beta - alpha) / beta;
    scal = 1.0 / (alpha - beta);
  }
  if (tid == 0) {
    tau[j] = t;
    e[j] = beta;
    VW[(j + 1) * ld + c] = 1.0;
    WV[(j + 1) * ld + kNB + c] = 1.0;
  }
  for (int64_t i = j + 2 + tid; i < m; i += kRefThreads) {
    const double v = col[i] * scal;
    VW[i * ld + c] = v;
    WV[i * ld + kNB + c] = v;
  }
}

// y[r] = sum_{k > j} A[r, k] v[k] for rows r > j (v = VW(:, c), zero at rows <= j): the trailing
// block read once, one wave per row, 16-byte loads
__global__ __launch_bounds__(256) void k_trd_symv_ro(const double *__restrict__ A, int64_t m,
                                                     int64_t j, const double *__restrict__ VW,
                                                     int c, double *__restrict__ y) {
  const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63;
  const int64_t r = j + 1 + (int64_t)blockIdx.x * 4 + wave;
  if (r >= m) return;
  const double *row = A + r * m;
  const int64_t ld = 2 * kNB;
  double s = 0.0;
  for (int64_t k = j + 1 + lane; k < m; k += 64) s = fma(row[k], VW[k * ld + c], s);
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) s += __shfl_xor(s, o);
  if (lane == 0) y[r] = s;
}

// dstebz's Sturm count: number of eigenvalues of the tridiagonal (d, e) below x
__device__ inline int sturm_count(const double *__restrict__ d, const double *__restrict__ e,
                                  int64_t m, double x, double pivmin) {
  int cnt = 0;
  double q = d[0] - x;
  if (fabs(q) < pivmin) q = -pivmin;
  if (q <= 0.0) ++cnt;
  for (int64_t i = 1; i < m; ++i) {
    q = d[i] - x - e[i - 1] * e[i - 1] / q;
    if (fabs(q) < pivmin) q = -pivmin;
    if (q <= 0.0) ++cnt;
  }
  return cnt;
}

// Smallest eigenvalue of the tridiagonal (d, e) by multisection; one wave.
__global__ __launch_bounds__(64) void k_trd_min_eig(const double *__restrict__ d,
                                                    const double *__restrict__ e, int64_t m,
                                                    double *__restrict__ out) {
  const int lane = threadIdx.x;
  double lo = 1e308, hi = -1e308, emax2 = 0.0;
  for (int64_t i = lane; i < m; i += 64) {
    const double el = (i > 0) ? fabs(e[i - 1]) : 0.0, er = (i + 1 < m) ? fabs(e[i]) : 0.0;
    lo = fmin(lo, d[i] - el - er);
    hi = fmax(hi, d[i] + el + er);
    if (i + 1 < m) emax2 = fmax(emax2, e[i] * e[i]);
  }
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) {
    lo = fmin(lo, __shfl_xor(lo, o));
    hi = fmax(hi, __shfl_xor(hi, o));
    emax2 = fmax(emax2, __shfl_xor(emax2, o));
  }
  const double safmin = 2.2250738585072014e-308, eps = 1.1102230246251565e-16;
  const double pivmin = safmin * fmax(1.0, emax2);
  const double tnorm = fmax(fabs(lo), fabs(hi));
  // widen by a few ulps of the norm, as dstebz does, so count(lo) = 0 and count(hi) = m
  const double fudge = 2.1 * eps * tnorm + 2.1 * 2.0 * pivmin;
  lo -= fudge;
  hi += fudge;
  for (int round = 0; round < 40; ++round) {
    if (!(hi - lo > 2.0 * eps * fmax(fabs(lo), fabs(hi)) + pivmin)) break;
    const double x = lo + (hi - lo) * (double)(lane + 1) / 65.0;
    const bool hit = sturm_count(d, e, m, x, pivmin) >= 1;
    const unsigned long long mask = __ballot(hit);
    if (mask == 0ull) {
      lo = __shfl(x, 63);
    } else {
      const int first = __ffsll((long long)mask) - 1;
      const double xf = __shfl(x, first);
      const double xb = (first > 0) ? __shfl(x, first - 1) : lo;
      lo = xb;
      hi = xf;
    }
  }
  if (lane == 0) out[0] = 0.5 * (lo + hi);
}

}  // namespace

// the blocked reduction only on request (MLFF_SYEV_BLOCKED=1; =0 / unset: the unblocked one).
// Measured (scripts/bench_syev.py, profiles/r04/syev/): m = 2701 0.250 s blocked vs 0.053 s
// unblocked, m = 14670 10.3 s vs 5.3 s -- its one-workgroup panel column (269 us per column at
// m = 14670) and the symv's 256-byte-strided reads of v (298 us per column) cost more than the
// halved trailing-block traffic saves
bool syev_blocked(int64_t m) {
  (void)m;
  if (const char *e = std::getenv("MLFF_SYEV_BLOCKED")) return std::atoi(e) != 0;
  return false;
}

// lo_eig of the lower triangle of the device matrix M (m x m, row-major), on ctx->stream;
// the value is returned to the host (and the tridiagonal (d, e) when d_host / e_host are
// given: m and m - 1 entries).  M itself is not modified.
int sym_min_eig(mlff_ctx *ctx, const double *M, int64_t m, double *lo_eig, double *d_host,
                double *e_host) {
  if (m < 1) return set_error(ctx, MLFF_ERR_ARG, "sym_min_eig: empty matrix");
  hipStream_t s = ctx->stream;
  ScratchScope scope(ctx);
  double *A = nullptr, *buf = nullptr;
  MLFF_TRY(scratch_alloc(ctx, &A, (size_t)(m * m)));
  // V[2], W[2], p, tau, d, e (m each), out
  MLFF_TRY(scratch_alloc(ctx, &buf, (size_t)(8 * m + 8)));
  double *V[2] = {buf, buf + m}, *W[2] = {buf + 2 * m, buf + 3 * m};
  double *p = buf + 4 * m, *tau = buf + 5 * m, *d = buf + 6 * m, *e = buf + 7 * m;
  double *out = buf + 8 * m;
  MLFF_HIP(ctx, hipMemsetAsync(buf, 0, sizeof(double) * (8 * m + 8), s));
  const unsigned gc = (unsigned)std::min<int64_t>((m * m + 255) / 256, 8192);
  hipLaunchKernelGGL(k_trd_copy_lower, dim3(gc), dim3(256), 0, s, M, A, m);
  if (syev_blocked(m)) {
    // blocked reduction: panels of kNB columns, trailing block read-only inside a panel
    double *VW = nullptr, *WV = nullptr;
    MLFF_TRY(scratch_alloc(ctx, &VW, (size_t)(m * 2 * kNB)));
    MLFF_TRY(scratch_alloc(ctx, &WV, (size_t)(m * 2 * kNB)));
    for (int64_t j0 = 0; j0 < m; j0 += kNB) {
      const int nbp = (int)std::min<int64_t>(kNB, m - j0);
      MLFF_HIP(ctx, hipMemsetAsync(VW, 0, sizeof(double) * m * 2 * kNB, s));
      MLFF_HIP(ctx, hipMemsetAsync(WV, 0, sizeof(double) * m * 2 * kNB, s));
      for (int c = 0; c < nbp; ++c) {
        const int64_t j = j0 + c;
        hipLaunchKernelGGL(k_trd_panel_col, dim3(1), dim3(kRefThreads), 0, s, (const double *)A, m,
                           j0, j, c, false, (const double *)p, VW, WV, W[0], tau, d, e);
        if (j + 1 < m)
          hipLaunchKernelGGL(k_trd_symv_ro, dim3((unsigned)((m - j - 1 + 3) / 4)), dim3(256), 0, s,
                             (const double *)A, m, j, (const double *)VW, c, p);
      }
      const int64_t T0 = j0 + nbp;  // the trailing block after the panel
      if (T0 < m) {
        // the panel's last w, then A[T0:, T0:] -= [V W] [W V]^T (K = 2 kNB)
        hipLaunchKernelGGL(k_trd_panel_col, dim3(1), dim3(kRefThreads), 0, s, (const double *)A, m,
                           j0, T0, nbp, true, (const double *)p, VW, WV, W[0], tau, d, e);
        launch_gemm(false, true, m - T0, m - T0, 2 * kNB, -1.0, VW + T0 * 2 * kNB, 2 * kNB,
                    WV + T0 * 2 * kNB, 2 * kNB, 1.0, A + T0 * m + T0, m, s);
      }
      MLFF_HIP(ctx, hipGetLastError());
    }
    hipLaunchKernelGGL(k_trd_min_eig, dim3(1), dim3(64), 0, s, (const double *)d,
                       (const double *)e, m, out);
    MLFF_HIP(ctx, hipGetLastError());
    MLFF_HIP(ctx, hipMemcpyAsync(lo_eig, out, sizeof(double), hipMemcpyDeviceToHost, s));
    if (d_host) MLFF_HIP(ctx, hipMemcpyAsync(d_host, d, sizeof(double) * m, hipMemcpyDeviceToHost, s));
    if (e_host && m > 1)
      MLFF_HIP(ctx, hipMemcpyAsync(e_host, e, sizeof(double) * (m - 1), hipMemcpyDeviceToHost, s));
    MLFF_HIP(ctx, hipStreamSynchronize(s));
    return MLFF_OK;
  }
  // R(0); then per column j: S(j), R(j + 1)
  hipLaunchKernelGGL(k_trd_reflect, dim3(1), dim3(kRefThreads), 0, s, (const double *)A, m,
                     (int64_t)0, (const double *)p, (const double *)V[1], W[1], V[0], tau, d, e);
  for (int64_t j = 0; j + 1 < m; ++j) {
    const int64_t rows = m - j - 1;
    hipLaunchKernelGGL(k_trd_update_symv, dim3((unsigned)((rows + 3) / 4)), dim3(256), 0, s, A,
                       m, j, (const double *)V[(j + 1) & 1], (const double *)W[(j + 1) & 1],
                       (const double *)V[j & 1], (const double *)tau, p);
    hipLaunchKernelGGL(k_trd_reflect, dim3(1), dim3(kRefThreads), 0, s, (const double *)A, m,
                       j + 1, (const double *)p, (const double *)V[j & 1], W[j & 1],
                       V[(j + 1) & 1], tau, d, e);
    if ((j & 255) == 255) MLFF_HIP(ctx, hipGetLastError());
  }
  hipLaunchKernelGGL(k_trd_min_eig, dim3(1), dim3(64), 0, s, (const double *)d,
                     (const double *)e, m, out);
  MLFF_HIP(ctx, hipGetLastError());
  MLFF_HIP(ctx, hipMemcpyAsync(lo_eig, out, sizeof(double), hipMemcpyDeviceToHost, s));
  if (d_host) MLFF_HIP(ctx, hipMemcpyAsync(d_host, d, sizeof(double) * m, hipMemcpyDeviceToHost, s));
  if (e_host && m > 1)
    MLFF_HIP(ctx, hipMemcpyAsync(e_host, e, sizeof(double) * (m - 1), hipMemcpyDeviceToHost, s));
  MLFF_HIP(ctx, hipStreamSynchronize(s));
  return MLFF_OK;
}

}  // namespace mlff
