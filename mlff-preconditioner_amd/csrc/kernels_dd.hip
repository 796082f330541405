// Exact-sum anchor: the dense-row operator and the low-rank apply with every product and sum of
// their dot products carried in double-double (TwoProd / TwoSum, ~106-bit significand) and rounded
// to fp64 ONCE per output entry -- the GPU counterpart of tests/golden/make_rbf_band.py --ld (the
// oracle's mat-vec and panel apply in np.longdouble, rounded once per application).  The CG
// recurrence around them stays the ordinary fp64 one.  Measurement only (MLFF_EXACT_SUMS=1 at
// context creation): it answers where the PCG iteration count of a chaotic system
// (configs[2], iterative_solver.py:995-1005) lands when the operator's summation-order error is
// removed, so that the fp64 count of every summation order -- the GPU's and the oracle's -- can be
// held to that anchor instead of to an extrapolated band.  Compute-bound by design (~12 fp64
// operations per matrix entry); never the default path.
#include "common.h"

// TwoSum / TwoProd are exact only if no a*b + c is contracted into an fma behind our back
#pragma clang fp contract(off)

namespace mlff {
namespace {

struct DD {
  double hi, lo;
};

__device__ __forceinline__ DD two_sum(double a, double b) {
  const double s = a + b;
  const double bb = s - a;
  return DD{s, (a - (s - bb)) + (b - bb)};
}

__device__ __forceinline__ DD fast_two_sum(double a, double b) {  // |a| >= |b|
  const double s = a + b;
  return DD{s, b - (s - a)};
}

// accurate double-double addition (relative error ~2^-104 of |a| + |b|)
__device__ __forceinline__ DD dd_add(DD a, DD b) {
  DD s = two_sum(a.hi, b.hi);
  const DD t = two_sum(a.lo, b.lo);
  s.lo += t.hi;
  s = fast_two_sum(s.hi, s.lo);
  s.lo += t.lo;
  return fast_two_sum(s.hi, s.lo);
}

// acc + x * y with the product exact (TwoProd by fma)
__device__ __forceinline__ DD dd_add_prod(DD acc, double x, double y) {
  const double p = x * y;
  return dd_add(acc, DD{p, fma(x, y, -p)});
}

// double-double sum of the 256 threads' partials (fixed tree order); the result in every thread
__device__ __forceinline__ DD block_sum_dd(DD v, double *sh_hi, double *sh_lo) {
  const int t = threadIdx.x;
  sh_hi[t] = v.hi;
  sh_lo[t] = v.lo;
  __syncthreads();
  for (int w = 128; w > 0; w >>= 1) {
    if (t < w) {
      const DD o = dd_add(DD{sh_hi[t], sh_lo[t]}, DD{sh_hi[t + w], sh_lo[t + w]});
      sh_hi[t] = o.hi;
      sh_lo[t] = o.lo;
    }
    __syncthreads();
  }
  return DD{sh_hi[0], sh_lo[0]};
}

// y[row] = sigma * fl(sum_c M[row, c] v[c]) + lam * vloc[row]: one workgroup per row
__global__ __launch_bounds__(256) void k_dd_gemv_rows(const double *__restrict__ M, int64_t ld,
                                                      int64_t ncols, const double *__restrict__ v,
                                                      double *__restrict__ y, double sigma,
                                                      double lam, const double *__restrict__ vloc,
                                                      const int *__restrict__ status) {
  if (status != nullptr && *status != ST_RUNNING) return;
  __shared__ double sh_hi[256], sh_lo[256];
  const int64_t row = blockIdx.x;
  const double *__restrict__ m = M + row * ld;
  DD acc{0.0, 0.0};
  for (int64_t c = threadIdx.x; c < ncols; c += 256) acc = dd_add_prod(acc, m[c], v[c]);
  const DD s = block_sum_dd(acc, sh_hi, sh_lo);
  if (threadIdx.x == 0) {
    const double sv = s.hi + s.lo;  // the one rounding to fp64
    double yv = sigma * sv;
    if (vloc != nullptr) yv = yv + lam * vloc[row];
    y[row] = yv;
  }
}

// t[j] = fl(sum_i T[j, i] r[i]), i < n: one workgroup per panel row
__global__ __launch_bounds__(256) void k_dd_tr(const double *__restrict__ T, int64_t ldt, int64_t n,
                                               const double *__restrict__ r, double *__restrict__ t,
                                               const int *__restrict__ status) {
  if (status != nullptr && *status != ST_RUNNING) return;
  __shared__ double sh_hi[256], sh_lo[256];
  const double *__restrict__ row = T + (int64_t)blockIdx.x * ldt;
  DD acc{0.0, 0.0};
  for (int64_t i = threadIdx.x; i < n; i += 256) acc = dd_add_prod(acc, row[i], r[i]);
  const DD s = block_sum_dd(acc, sh_hi, sh_lo);
  if (threadIdx.x == 0) t[blockIdx.x] = s.hi + s.lo;
}

// u_i = fl(sum_j T[j, i] t[j]) (j in increasing order, one thread per i: coalesced panel rows);
// z_i = sigma_p (lam_inv (r_i - u_i)) as k_precon_fin forms it
__global__ __launch_bounds__(256) void k_dd_ttz(const double *__restrict__ T, int64_t ldt, int64_t k,
                                                int64_t n, const double *__restrict__ t,
                                                const double *__restrict__ r, double *__restrict__ z,
                                                double sigma_p, double lam_inv,
                                                const int *__restrict__ status) {
  if (status != nullptr && *status != ST_RUNNING) return;
  const int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x;
  if (i >= n) return;
  DD acc{0.0, 0.0};
  for (int64_t j = 0; j < k; ++j) acc = dd_add_prod(acc, T[j * ldt + i], t[j]);
  const double u = acc.hi + acc.lo;
  z[i] = sigma_p * (lam_inv * (r[i] - u));
}

}  // namespace

void launch_dd_gemv_rows(const double *M, int64_t ld, int64_t rows, int64_t ncols, const double *v,
                         double *y, double sigma, double lam, const double *vloc, const int *status,
                         hipStream_t s) {
  if (rows <= 0) return;
  hipLaunchKernelGGL(k_dd_gemv_rows, dim3((unsigned)rows), dim3(256), 0, s, M, ld, ncols, v, y, sigma,
                     lam, vloc, status);
}

void launch_dd_lowrank(const double *T, int64_t ldt, int64_t k, const double *r, double *z, int64_t n,
                       double sigma_p, double lam_inv, double *t, const int *status, hipStream_t s) {
  if (n <= 0 || k <= 0) return;
  hipLaunchKernelGGL(k_dd_tr, dim3((unsigned)k), dim3(256), 0, s, T, ldt, n, r, t, status);
  hipLaunchKernelGGL(k_dd_ttz, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, s, T, ldt, k, n, t, r,
                     z, sigma_p, lam_inv, status);
}

}  // namespace mlff
