// Streaming kernels of one PCG iteration on gfx950: the dense fp64 kernel
// mat-vec (the hot path, HBM bound), the low-rank preconditioner apply and the
// fused CG vector updates with deterministic fixed-order reductions.
//
// Reference semantics: scipy 1.7.3 CGREVCOM + python wrapper as called from
// src/sGDML/sgdml/solvers/iterative_solver.py:995-1005; preconditioner applies
// iterative_cholesky.py:145-148, iterative_solver.py:315-318 and :376-379.
#include "common.h"

namespace mlff {

typedef double d2 __attribute__((ext_vector_type(2)));

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

// ---------------------------------------------------------------------------
// Dense row GEMV: y[row] = sigma * sum_c M[row, c] v[c] + lam * vloc[row]   (EPI=1)
//                 part[split * out_stride + row] = sum_{c in split} M[row,c] v[c] (EPI=0)
// R rows per workgroup share every 16-B load of v (v is L2 resident); M is
// streamed once with non-temporal 16-B loads, U loads in flight per row.
// `rows` of M must be allocated up to a multiple of R (padding rows are zero).
template <int R, int U, int EPI>
__global__ __launch_bounds__(256) void k_gemv(const double *__restrict__ M, int64_t ld,
                                              int64_t rows, int64_t n2, int64_t cs2,
                                              const double *__restrict__ v,
                                              double *__restrict__ out, int64_t out_stride,
                                              double sigma, double lam,
                                              const double *__restrict__ vloc,
                                              const int *__restrict__ status) {
  if (status != nullptr && *status != ST_RUNNING) return;
  __shared__ double sh[4 * R];
  const int64_t r0 = (int64_t)blockIdx.x * R;
  const int64_t c_begin = (int64_t)blockIdx.y * cs2;
  int64_t c_end = c_begin + cs2;
  if (c_end > n2) c_end = n2;
  const d2 *__restrict__ v2 = reinterpret_cast<const d2 *>(v);
  const d2 *rowp[R];
#pragma unroll
  for (int r = 0; r < R; ++r) rowp[r] = reinterpret_cast<const d2 *>(M + (r0 + r) * ld);
  double acc[R];
#pragma unroll
  for (int r = 0; r < R; ++r) acc[r] = 0.0;

  int64_t c = c_begin + threadIdx.x;
  // main body: U full strides without bounds checks
  for (; c + (int64_t)(U - 1) * 256 < c_end; c += (int64_t)256 * U) {
    d2 xv[U];
    d2 kv[R][U];
#pragma unroll
    for (int u = 0; u < U; ++u) xv[u] = v2[c + u * 256];
#pragma unroll
    for (int r = 0; r < R; ++r)
#pragma unroll
      for (int u = 0; u < U; ++u) kv[r][u] = __builtin_nontemporal_load(rowp[r] + c + u * 256);
#pragma unroll
    for (int r = 0; r < R; ++r)
#pragma unroll
      for (int u = 0; u < U; ++u) {
        acc[r] = fma(kv[r][u].x, xv[u].x, acc[r]);
        acc[r] = fma(kv[r][u].y, xv[u].y, acc[r]);
      }
  }
  for (; c < c_end; c += 256) {
    const d2 xv = v2[c];
#pragma unroll
    for (int r = 0; r < R; ++r) {
      const d2 kv = __builtin_nontemporal_load(rowp[r] + c);
      acc[r] = fma(kv.x, xv.x, acc[r]);
      acc[r] = fma(kv.y, xv.y, acc[r]);
    }
  }
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
#pragma unroll
  for (int r = 0; r < R; ++r) {
    const double s = wave_sum(acc[r]);
    if (lane == 0) sh[w * R + r] = s;
  }
  __syncthreads();
  if (threadIdx.x < R) {
    const int r = threadIdx.x;
    const int64_t row = r0 + r;
    if (row < rows) {
      const double s = (sh[r] + sh[R + r]) + (sh[2 * R + r] + sh[3 * R + r]);
      if (EPI == 1) {
        double yv = sigma * s;
        if (vloc != nullptr) yv += lam * vloc[row];
        out[row] = yv;
      } else {
        out[(int64_t)blockIdx.y * out_stride + row] = s;
      }
    }
  }
}

void launch_gemv_rows(const double *M, int64_t ld, int64_t rows, const double *v, double *y,
                      double sigma, double lam, const double *vloc, const int *status,
                      hipStream_t s) {
  constexpr int R = 4, U = 4;
  const int64_t n2 = ld / 2;
  dim3 grid((unsigned)((rows + R - 1) / R), 1);
  hipLaunchKernelGGL((k_gemv<R, U, 1>), grid, dim3(256), 0, s, M, ld, rows, n2, n2, v, y,
                     (int64_t)0, sigma, lam, vloc, status);
}

int choose_tsplit(int64_t k, int64_t ncols) {
  const int64_t row_groups = (k + 3) / 4;
  int64_t splits = (1024 + row_groups - 1) / row_groups;
  const int64_t max_by_cols = (ncols / 2 + 255) / 256;  // at least 256 double2 per split
  if (splits > max_by_cols) splits = max_by_cols;
  if (splits < 1) splits = 1;
  if (splits > 64) splits = 64;
  return (int)splits;
}

void launch_gemv_split(const double *T, int64_t ldt, int64_t k, int64_t ncols, int splits,
                       const double *r, double *tpart, const int *status, hipStream_t s) {
  constexpr int R = 4, U = 2;
  const int64_t n2 = ncols / 2;  // ncols is the padded local length (even)
  const int64_t cs2 = (n2 + splits - 1) / splits;
  dim3 grid((unsigned)((k + R - 1) / R), (unsigned)splits);
  hipLaunchKernelGGL((k_gemv<R, U, 0>), grid, dim3(256), 0, s, T, ldt, k, n2, cs2, r, tpart, k,
                     1.0, 0.0, (const double *)nullptr, status);
}

// ---------------------------------------------------------------------------
// z = sigma_p * (lam_inv * (r - T^T t)), t_j = sum_sp tpart[sp*k + j]; rho partials r.z
// A workgroup owns 128 columns per pass; wave w accumulates rows j = w (mod 4).
__global__ __launch_bounds__(256) void k_precon_z(const double *__restrict__ T, int64_t ldt,
                                                  int64_t k, int splits,
                                                  const double *__restrict__ tpart,
                                                  const double *__restrict__ r,
                                                  double *__restrict__ z, int64_t n,
                                                  double sigma_p, double lam_inv,
                                                  double *__restrict__ rho_part,
                                                  const int *__restrict__ status) {
  if (status != nullptr && *status != ST_RUNNING) return;
  extern __shared__ double smem[];
  double *t_sh = smem;                 // k
  d2 *red = reinterpret_cast<d2 *>(smem + round_up(k, 2));  // 256 d2
  double *sh = smem + round_up(k, 2) + 512;
  for (int64_t j = threadIdx.x; j < k; j += 256) {
    double a = 0.0;
    for (int sp = 0; sp < splits; ++sp) a += tpart[(int64_t)sp * k + j];
    t_sh[j] = a;
  }
  __syncthreads();
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  double rho_acc = 0.0;
  for (int64_t c0 = (int64_t)blockIdx.x * 128; c0 < n; c0 += (int64_t)gridDim.x * 128) {
    const int64_t c = c0 + 2 * lane;
    d2 acc = {0.0, 0.0};
    if (c < n) {
      const double *base = T + c;
      int64_t j = w;
      for (; j + 12 < k; j += 16) {
        const d2 a0 = *reinterpret_cast<const d2 *>(base + j * ldt);
        const d2 a1 = *reinterpret_cast<const d2 *>(base + (j + 4) * ldt);
        const d2 a2 = *reinterpret_cast<const d2 *>(base + (j + 8) * ldt);
        const d2 a3 = *reinterpret_cast<const d2 *>(base + (j + 12) * ldt);
        acc.x = fma(a0.x, t_sh[j], acc.x);
        acc.y = fma(a0.y, t_sh[j], acc.y);
        acc.x = fma(a1.x, t_sh[j + 4], acc.x);
        acc.y = fma(a1.y, t_sh[j + 4], acc.y);
        acc.x = fma(a2.x, t_sh[j + 8], acc.x);
        acc.y = fma(a2.y, t_sh[j + 8], acc.y);
        acc.x = fma(a3.x, t_sh[j + 12], acc.x);
        acc.y = fma(a3.y, t_sh[j + 12], acc.y);
      }
      for (; j < k; j += 4) {
        const d2 a0 = *reinterpret_cast<const d2 *>(base + j * ldt);
        acc.x = fma(a0.x, t_sh[j], acc.x);
        acc.y = fma(a0.y, t_sh[j], acc.y);
      }
    }
    red[w * 64 + lane] = acc;
    __syncthreads();
    if (w == 0 && c < n) {
      const d2 s = (red[lane] + red[64 + lane]) + (red[128 + lane] + red[192 + lane]);
      const d2 rv = *reinterpret_cast<const d2 *>(r + c);
      d2 zv;
      zv.x = sigma_p * (lam_inv * (rv.x - s.x));
      zv.y = sigma_p * (lam_inv * (rv.y - s.y));
      if (c + 1 >= n) zv.y = 0.0;  // padding stays zero
      *reinterpret_cast<d2 *>(z + c) = zv;
      rho_acc = fma(rv.x, zv.x, rho_acc);
      rho_acc = fma(rv.y, zv.y, rho_acc);
    }
    __syncthreads();
  }
  const double tot = block_sum256(rho_acc, sh);
  if (threadIdx.x == 0 && rho_part != nullptr) rho_part[blockIdx.x] = tot;
}

void launch_precon_z(const double *T, int64_t ldt, int64_t k, int splits, const double *tpart,
                     const double *r, double *z, int64_t n, double sigma_p, double lam_inv,
                     double *rho_part, const int *status, hipStream_t s) {
  const size_t shbytes = (size_t)(round_up(k, 2) + 512 + 8) * sizeof(double);
  hipLaunchKernelGGL(k_precon_z, dim3(kVecGrid), dim3(256), shbytes, s, T, ldt, k, splits,
                     tpart, r, z, n, sigma_p, lam_inv, rho_part, status);
}

// ---------------------------------------------------------------------------
__global__ __launch_bounds__(256) void k_dot_part(const double *__restrict__ a,
                                                  const double *__restrict__ b, int64_t n,
                                                  double *__restrict__ part,
                                                  const int *__restrict__ status) {
  if (status != nullptr && *status != ST_RUNNING) return;
  __shared__ double sh[8];
  double acc = 0.0;
  for (int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x; i < n;
       i += (int64_t)gridDim.x * 256)
    acc = fma(a[i], b[i], acc);
  const double t = block_sum256(acc, sh);
  if (threadIdx.x == 0) part[blockIdx.x] = t;
}

void launch_dot_part(const double *a, const double *b, int64_t n, double *part,
                     const int *status, hipStream_t s) {
  hipLaunchKernelGGL(k_dot_part, dim3(kVecGrid), dim3(256), 0, s, a, b, n, part, status);
}

// p = z + beta p  (Fortran: DAXPY(beta, P, Z); DCOPY(Z, P)); p = z at ITER == 1
__global__ __launch_bounds__(256) void k_update_p(const double *__restrict__ z,
                                                  double *__restrict__ p, int64_t n,
                                                  const double *__restrict__ rho_part,
                                                  DevState *st, long long it,
                                                  const int *__restrict__ status) {
  if (*status != ST_RUNNING) return;
  __shared__ double sh[8];
  const double rho = reduce_parts_bcast(rho_part, kVecGrid, sh);
  if (blockIdx.x == 0 && threadIdx.x == 0) st->rho = rho;
  if (it > 1) {
    const double beta = rho / st->rho1;
    for (int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x; i < n;
         i += (int64_t)gridDim.x * 256)
      p[i] = fma(beta, p[i], z[i]);
  } else {
    for (int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x; i < n;
         i += (int64_t)gridDim.x * 256)
      p[i] = z[i];
  }
}

void launch_update_p(const double *z, double *p, int64_t n, const double *rho_part,
                     DevState *st, long long it, const int *status, hipStream_t s) {
  hipLaunchKernelGGL(k_update_p, dim3(kVecGrid), dim3(256), 0, s, z, p, n, rho_part, st, it,
                     status);
}

// alpha = rho / (p.q); x += alpha p; r -= alpha q; rr partials
__global__ __launch_bounds__(256) void k_update_xr(double *__restrict__ x, double *__restrict__ r,
                                                   const double *__restrict__ p,
                                                   const double *__restrict__ q, int64_t n,
                                                   const double *__restrict__ pq_part,
                                                   double *__restrict__ rr_part, DevState *st,
                                                   const int *__restrict__ status) {
  if (*status != ST_RUNNING) return;
  __shared__ double sh[8];
  const double pq = reduce_parts_bcast(pq_part, kVecGrid, sh);
  const double alpha = st->rho / pq;
  if (blockIdx.x == 0 && threadIdx.x == 0) {
    st->pq = pq;
    st->alpha = alpha;
  }
  double acc = 0.0;
  for (int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x; i < n;
       i += (int64_t)gridDim.x * 256) {
    x[i] = fma(alpha, p[i], x[i]);
    const double ri = fma(-alpha, q[i], r[i]);
    r[i] = ri;
    acc = fma(ri, ri, acc);
  }
  const double t = block_sum256(acc, sh);
  if (threadIdx.x == 0) rr_part[blockIdx.x] = t;
}

void launch_update_xr(double *x, double *r, const double *p, const double *q, int64_t n,
                      const double *pq_part, double *rr_part, DevState *st, const int *status,
                      hipStream_t s) {
  hipLaunchKernelGGL(k_update_xr, dim3(kVecGrid), dim3(256), 0, s, x, r, p, q, n, pq_part,
                     rr_part, st, status);
}

// scipy stop test (iterative.py _stoptest): resid = ||r||; converged if resid <= atol;
// the python wrapper re-checks with the true residual when ITER > 1.
__global__ __launch_bounds__(256) void k_stoptest(const double *__restrict__ rr_part,
                                                  DevState *st, double *__restrict__ trace,
                                                  long long it) {
  if (st->status != ST_RUNNING) return;
  __shared__ double sh[8];
  const double rr = reduce_parts_bcast(rr_part, kVecGrid, sh);
  if (threadIdx.x != 0) return;
  const double resid = sqrt(rr);
  st->rr = rr;
  st->resid = resid;
  st->iters = it;
  trace[it] = resid;
  if (resid <= st->atol) {
    st->status = it > 1 ? ST_RECHECK : ST_CONVERGED;
  } else if (it >= st->maxiter) {
    st->status = ST_MAXITER;
  } else {
    st->rho1 = st->rho;
  }
}

void launch_stoptest(const double *rr_part, DevState *st, double *trace, long long it,
                     hipStream_t s) {
  hipLaunchKernelGGL(k_stoptest, dim3(1), dim3(256), 0, s, rr_part, st, trace, it);
}

__global__ __launch_bounds__(256) void k_residual(const double *__restrict__ b,
                                                  const double *__restrict__ q,
                                                  double *__restrict__ r, int64_t n,
                                                  double *__restrict__ rr_part) {
  __shared__ double sh[8];
  double acc = 0.0;
  for (int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x; i < n;
       i += (int64_t)gridDim.x * 256) {
    const double ri = b[i] - q[i];
    r[i] = ri;
    acc = fma(ri, ri, acc);
  }
  const double t = block_sum256(acc, sh);
  if (threadIdx.x == 0) rr_part[blockIdx.x] = t;
}

void launch_residual(const double *b, const double *q, double *r, int64_t n, double *rr_part,
                     hipStream_t s) {
  hipLaunchKernelGGL(k_residual, dim3(kVecGrid), dim3(256), 0, s, b, q, r, n, rr_part);
}

// After the true-residual recheck: converged, or continue (RHO1 = RHO), or maxiter.
__global__ __launch_bounds__(256) void k_recheck_finish(const double *__restrict__ rr_part,
                                                        DevState *st,
                                                        double *__restrict__ trace) {
  __shared__ double sh[8];
  const double rr = reduce_parts_bcast(rr_part, kVecGrid, sh);
  if (threadIdx.x != 0) return;
  const double resid = sqrt(rr);
  st->rr = rr;
  st->resid = resid;
  trace[st->iters] = resid;
  if (resid <= st->atol) {
    st->status = ST_CONVERGED;
  } else if (st->iters >= st->maxiter) {
    st->status = ST_MAXITER;
  } else {
    st->rho1 = st->rho;
    st->status = ST_RUNNING;
  }
}

void launch_recheck_finish(const double *rr_part, DevState *st, double *trace, hipStream_t s) {
  hipLaunchKernelGGL(k_recheck_finish, dim3(1), dim3(256), 0, s, rr_part, st, trace);
}

__global__ __launch_bounds__(256) void k_reduce_to(const double *__restrict__ part, int np,
                                                   double *__restrict__ out) {
  __shared__ double sh[8];
  const double v = reduce_parts_bcast(part, np, sh);
  if (threadIdx.x == 0) *out = v;
}

void launch_reduce_to(const double *part, int np, double *out, hipStream_t s) {
  hipLaunchKernelGGL(k_reduce_to, dim3(1), dim3(256), 0, s, part, np, out);
}

__global__ __launch_bounds__(256) void k_scale_copy(const double *__restrict__ a,
                                                    double *__restrict__ y, int64_t n,
                                                    double alpha) {
  for (int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x; i < n;
       i += (int64_t)gridDim.x * 256)
    y[i] = alpha * a[i];
}

void launch_scale_copy(const double *a, double *y, int64_t n, double alpha, hipStream_t s) {
  hipLaunchKernelGGL(k_scale_copy, dim3(kVecGrid), dim3(256), 0, s, a, y, n, alpha);
}

}  // namespace mlff
