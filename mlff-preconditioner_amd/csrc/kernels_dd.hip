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

#include <algorithm>

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

// Gram matrix of a wide panel in double-double: slab z of G[i, j] (i >= j, the lower triangle)
// = sum over the columns of slab z of W[i, c] W[j, c], products exact, sums double-double; a
// 64 x 64 output tile per 256-thread workgroup (4 x 4 per thread, columns staged 16 at a time
// through LDS as k_gemm stages them).  hi / lo slabs: splits x k x k each.
__global__ __launch_bounds__(256) void k_gram_dd(const double *__restrict__ W, int64_t ldw, int64_t k,
                                                 int64_t ncols, int64_t kchunk,
                                                 double *__restrict__ hi, double *__restrict__ lo) {
  constexpr int BM = 64, BK = 16;
  if ((int64_t)blockIdx.x > (int64_t)blockIdx.y) return;  // upper tiles: mirrored later
  __shared__ double As[BK][BM + 1];
  __shared__ double Bs[BK][BM + 1];
  const int tid = threadIdx.x, tx = tid & 15, ty = tid >> 4;
  const int64_t m0 = (int64_t)blockIdx.y * BM, n0 = (int64_t)blockIdx.x * BM;
  const int64_t kb = (int64_t)blockIdx.z * kchunk;
  const int64_t ke = kb + kchunk < ncols ? kb + kchunk : ncols;
  DD acc[4][4];
#pragma unroll
  for (int i = 0; i < 4; ++i)
#pragma unroll
    for (int j = 0; j < 4; ++j) acc[i][j] = DD{0.0, 0.0};
  for (int64_t k0 = kb; k0 < ke; k0 += BK) {
#pragma unroll
    for (int l = 0; l < 4; ++l) {
      const int e = tid + 256 * l;
      const int rr = e >> 4, kk = e & 15;
      const int64_t gk = k0 + kk;
      const int64_t ga = m0 + rr, gb = n0 + rr;
      As[kk][rr] = (ga < k && gk < ke) ? W[ga * ldw + gk] : 0.0;
      Bs[kk][rr] = (gb < k && gk < ke) ? W[gb * ldw + gk] : 0.0;
    }
    __syncthreads();
#pragma unroll 4
    for (int kk = 0; kk < BK; ++kk) {
      double a[4], b[4];
#pragma unroll
      for (int i = 0; i < 4; ++i) a[i] = As[kk][ty + 16 * i];
#pragma unroll
      for (int j = 0; j < 4; ++j) b[j] = Bs[kk][tx + 16 * j];
#pragma unroll
      for (int i = 0; i < 4; ++i)
#pragma unroll
        for (int j = 0; j < 4; ++j) acc[i][j] = dd_add_prod(acc[i][j], a[i], b[j]);
    }
    __syncthreads();
  }
  const int64_t off = (int64_t)blockIdx.z * k * k;
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    const int64_t gm = m0 + ty + 16 * i;
    if (gm >= k) continue;
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      const int64_t gn = n0 + tx + 16 * j;
      if (gn >= k || gn > gm) continue;
      hi[off + gm * k + gn] = acc[i][j].hi;
      lo[off + gm * k + gn] = acc[i][j].lo;
    }
  }
}

// The same Gram on the matrix cores with blocked double-double accumulation: each 16 x 16 block
// accumulates kDDChunk columns in fp64 (v_mfma_f64_16x16x4f64, 4 products per step), and every
// chunk partial is added to a double-double accumulator -- the fp64 error is that of a short
// chunk's partial sums, the chunks add exactly (a BLAS-like blocked sum with an exact outer sum),
// at matrix-core speed.  64 x 64 output tile per 256-thread workgroup, waves 2 x 2 over it,
// columns staged 16 at a time through LDS.  hi / lo slabs as k_gram_dd.
typedef double v4d __attribute__((ext_vector_type(4)));
constexpr int kDDChunk = 64;
__global__ __launch_bounds__(256) void k_gram_mfma_dd(const double *__restrict__ W, int64_t ldw,
                                                      int64_t k, int64_t ncols, int64_t kchunk,
                                                      double *__restrict__ hi,
                                                      double *__restrict__ lo) {
  // BK = 32 columns per staged step (round 6: half the barriers of 16; the MFMA k-steps and the
  // 64-column double-double folds are the same, so the same bits)
  constexpr int BM = 64, BK = 32, LP = 80, PL = BM * BK / 256;
  if ((int64_t)blockIdx.x > (int64_t)blockIdx.y) return;
  __shared__ double As[BK][LP];
  __shared__ double Bs[BK][LP];
  const int tid = threadIdx.x, lane = tid & 63, wv = tid >> 6;
  const int wm = (wv >> 1) * 32, wn = (wv & 1) * 32;
  const int64_t m0 = (int64_t)blockIdx.y * BM, n0 = (int64_t)blockIdx.x * BM;
  const int64_t kb = (int64_t)blockIdx.z * kchunk;
  const int64_t ke = kb + kchunk < ncols ? kb + kchunk : ncols;
  v4d acc[2][2];
  DD dacc[2][2][4];
#pragma unroll
  for (int i = 0; i < 2; ++i)
#pragma unroll
    for (int j = 0; j < 2; ++j) {
      acc[i][j] = v4d{0.0, 0.0, 0.0, 0.0};
#pragma unroll
      for (int r = 0; r < 4; ++r) dacc[i][j][r] = DD{0.0, 0.0};
    }
  int stage = 0;
  // software pipeline (round 6): the next 16 columns' loads are in flight while the matrix cores
  // work on the current ones -- the same operands in the same order, so the same bits
  double va[PL], vb[PL];
  auto load_stage = [&](int64_t k0) {
#pragma unroll
    for (int l = 0; l < PL; ++l) {
      const int e = tid + 256 * l;
      const int rr = e / BK, kk = e % BK;
      const int64_t gk = k0 + kk, ga = m0 + rr, gb = n0 + rr;
      va[l] = (ga < k && gk < ke) ? W[ga * ldw + gk] : 0.0;
      vb[l] = (gb < k && gk < ke) ? W[gb * ldw + gk] : 0.0;
    }
  };
  if (kb < ke) load_stage(kb);
  for (int64_t k0 = kb; k0 < ke; k0 += BK) {
    __syncthreads();  // the previous stage's fragment reads are done
#pragma unroll
    for (int l = 0; l < PL; ++l) {
      const int e = tid + 256 * l;
      const int rr = e / BK, kk = e % BK;
      As[kk][rr] = va[l];
      Bs[kk][rr] = vb[l];
    }
    __syncthreads();
    if (k0 + BK < ke) load_stage(k0 + BK);
#pragma unroll
    for (int ks = 0; ks < BK / 4; ++ks) {
      const int kr = 4 * ks + (lane >> 4);
      double a[2], b[2];
#pragma unroll
      for (int i = 0; i < 2; ++i) a[i] = As[kr][wm + 16 * i + (lane & 15)];
#pragma unroll
      for (int j = 0; j < 2; ++j) b[j] = Bs[kr][wn + 16 * j + (lane & 15)];
#pragma unroll
      for (int i = 0; i < 2; ++i)
#pragma unroll
        for (int j = 0; j < 2; ++j)
          acc[i][j] = __builtin_amdgcn_mfma_f64_16x16x4f64(a[i], b[j], acc[i][j], 0, 0, 0);
    }
    if (++stage == kDDChunk / BK || k0 + BK >= ke) {  // fold the chunk's fp64 partials
      stage = 0;
#pragma unroll
      for (int i = 0; i < 2; ++i)
#pragma unroll
        for (int j = 0; j < 2; ++j) {
#pragma unroll
          for (int r = 0; r < 4; ++r) dacc[i][j][r] = dd_add(dacc[i][j][r], DD{acc[i][j][r], 0.0});
          acc[i][j] = v4d{0.0, 0.0, 0.0, 0.0};
        }
    }
  }
  const int64_t off = (int64_t)blockIdx.z * k * k;
#pragma unroll
  for (int i = 0; i < 2; ++i)
#pragma unroll
    for (int j = 0; j < 2; ++j)
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int64_t gm = m0 + wm + 16 * i + (lane >> 4) + 4 * r;
        const int64_t gn = n0 + wn + 16 * j + (lane & 15);
        if (gm >= k || gn >= k || gn > gm) continue;
        hi[off + gm * k + gn] = dacc[i][j][r].hi;
        lo[off + gm * k + gn] = dacc[i][j][r].lo;
      }
}

// G[i, j] = fl(sum_z slab_z) (double-double, slab order) for i >= j, mirrored to j > i
__global__ __launch_bounds__(256) void k_gram_dd_fin(const double *__restrict__ hi,
                                                     const double *__restrict__ lo, int splits,
                                                     int64_t k, double *__restrict__ G) {
  for (int64_t e = (int64_t)blockIdx.x * 256 + threadIdx.x; e < k * k; e += (int64_t)gridDim.x * 256) {
    const int64_t i = e / k, j = e % k;
    const int64_t src = j > i ? j * k + i : e;
    DD a{0.0, 0.0};
    for (int z = 0; z < splits; ++z) a = dd_add(a, DD{hi[z * k * k + src], lo[z * k * k + src]});
    G[e] = a.hi + a.lo;
  }
}

}  // namespace

int gram_wide_dd(mlff_ctx *ctx, const double *W, int64_t k, int64_t ncols, int64_t ldw, double *G,
                 bool exact_products) {
  if (k <= 0) return MLFF_OK;
  ScratchScope scope(ctx);
  const int64_t nt = (k + 63) / 64, tiles = nt * (nt + 1) / 2;
  int64_t splits = (512 + tiles - 1) / tiles;
  const int64_t max_splits = (ncols + 511) / 512;
  if (splits > max_splits) splits = max_splits;
  if (splits < 1) splits = 1;
  if (splits > 64) splits = 64;
  const int64_t kchunk = round_up((ncols + splits - 1) / splits, 16);
  double *hi = nullptr, *lo = nullptr;
  MLFF_TRY(scratch_alloc(ctx, &hi, (size_t)(splits * k * k)));
  MLFF_TRY(scratch_alloc(ctx, &lo, (size_t)(splits * k * k)));
  if (exact_products)
    hipLaunchKernelGGL(k_gram_dd, dim3((unsigned)nt, (unsigned)nt, (unsigned)splits), dim3(256), 0,
                       ctx->stream, W, ldw, k, ncols, kchunk, hi, lo);
  else
    hipLaunchKernelGGL(k_gram_mfma_dd, dim3((unsigned)nt, (unsigned)nt, (unsigned)splits), dim3(256), 0,
                       ctx->stream, W, ldw, k, ncols, kchunk, hi, lo);
  hipLaunchKernelGGL(k_gram_dd_fin, dim3((unsigned)std::min<int64_t>((k * k + 255) / 256, 4096)),
                     dim3(256), 0, ctx->stream, hi, lo, (int)splits, k, G);
  MLFF_HIP(ctx, hipGetLastError());
  return MLFF_OK;
}

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
