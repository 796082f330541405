// Streaming kernels of one PCG iteration on gfx950: the dense fp64 kernel
// mat-vec (the hot path, HBM bound), the low-rank preconditioner apply and the
// fused CG vector updates with deterministic fixed-order reductions.
//
// Reference semantics: scipy 1.7.3 CGREVCOM + python wrapper as called from
// src/sGDML/sgdml/solvers/iterative_solver.py:995-1005; preconditioner applies
// iterative_cholesky.py:145-148, iterative_solver.py:315-318 and :376-379.
#include <cstdio>
#include <cstring>

#include "common.h"

#include <algorithm>
#include <cstdlib>

namespace mlff {

typedef double d2 __attribute__((ext_vector_type(2)));

// Stop test of iteration f.it (as k_stoptest) at the start of the next iteration's first
// kernel: every workgroup reduces the same partials in the same order and reaches the
// same decision; workgroup (0, 0) writes the state.  All threads of the block call it.
// Returns false when the solver stops (the caller returns).
__device__ __forceinline__ bool stop_prologue(const StopFold &f, double *sh) {
  if (f.rr_part == nullptr) return true;
  const double rr = reduce_parts_bcast(f.rr_part, kVecGrid, sh);
  __syncthreads();  // sh is reused by the caller
  return stop_decide(f, rr);
}

// The same for a workgroup of any multiple of 256 threads: the first 256 threads reduce
// the partials exactly as reduce_parts_bcast does (same bits), the rest wait.
__device__ __forceinline__ bool stop_prologue_wide(const StopFold &f, double *sh) {
  if (f.rr_part == nullptr) return true;
  double v = 0.0;
  if (threadIdx.x < 256)
    for (int i = threadIdx.x; i < kVecGrid; i += 256) v += f.rr_part[i];
  v = wave_sum(v);
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  __syncthreads();
  if (lane == 0 && w < 4) sh[w] = v;
  __syncthreads();
  const double rr = (sh[0] + sh[1]) + (sh[2] + sh[3]);
  __syncthreads();  // sh is reused by the caller
  return stop_decide(f, rr);
}

// ---------------------------------------------------------------------------
// the column range [c_begin, c_end) of R rows, dot v; NT: non-temporal loads of M.
// Operand entry c is v2[c - voff] (voff = c_begin: v staged for the range only, k_gemv_xr)
template <int R, int U, bool NT>
__device__ __forceinline__ void gemv_rows_body(const d2 *const (&rowp)[R], const d2 *__restrict__ v2,
                                               int64_t c_begin, int64_t c_end, double (&acc)[R],
                                               int64_t voff = 0) {
  int64_t c = c_begin + threadIdx.x;
  // main body: U full strides without bounds checks
  for (; c + (int64_t)(U - 1) * 256 < c_end; c += (int64_t)256 * U) {
    d2 xv[U];
    d2 kv[R][U];
#pragma unroll
    for (int u = 0; u < U; ++u) xv[u] = v2[c - voff + u * 256];
#pragma unroll
    for (int r = 0; r < R; ++r)
#pragma unroll
      for (int u = 0; u < U; ++u)
        kv[r][u] = NT ? __builtin_nontemporal_load(rowp[r] + c + u * 256) : rowp[r][c + u * 256];
#pragma unroll
    for (int r = 0; r < R; ++r)
#pragma unroll
      for (int u = 0; u < U; ++u) {
        acc[r] = fma(kv[r][u].x, xv[u].x, acc[r]);
        acc[r] = fma(kv[r][u].y, xv[u].y, acc[r]);
      }
  }
  for (; c < c_end; c += 256) {
    const d2 xv = v2[c - voff];
#pragma unroll
    for (int r = 0; r < R; ++r) {
      const d2 kv = NT ? __builtin_nontemporal_load(rowp[r] + c) : rowp[r][c];
      acc[r] = fma(kv.x, xv.x, acc[r]);
      acc[r] = fma(kv.y, xv.y, acc[r]);
    }
  }
}

// Dense row GEMV: y[row] = sigma * sum_c M[row, c] v[c] + lam * vloc[row]   (EPI=1)
//                 part[split * out_stride + row] = sum_{c in split} M[row,c] v[c] (EPI=0)
// R rows per workgroup share every 16-B load of v (v is L2 resident); M is
// streamed once with non-temporal 16-B loads, U loads in flight per row; rows below
// `cached_rows` are read with default-policy loads even when NT (a panel's leading rows
// stay in the MALL for the next pass, panel_cached_rows).
// `rows` of M must be allocated up to a multiple of R (padding rows are zero).
template <int R, int U, int EPI, bool NT = true>
__global__ __launch_bounds__(256) void k_gemv(const double *__restrict__ M, int64_t ld,
                                              int64_t rows, int64_t n2, int64_t cs2,
                                              const double *__restrict__ v,
                                              double *__restrict__ out, int64_t out_stride,
                                              double sigma, double lam,
                                              const double *__restrict__ vloc,
                                              const int *__restrict__ status, StopFold fold,
                                              int64_t cached_rows = 0) {
  if (status != nullptr && *status != ST_RUNNING) return;
  __shared__ double sh[4 * R > 8 ? 4 * R : 8];
  if (!stop_prologue(fold, sh)) return;
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
  if (NT && r0 + R > cached_rows)
    gemv_rows_body<R, U, true>(rowp, v2, c_begin, c_end, acc);
  else
    gemv_rows_body<R, U, false>(rowp, v2, c_begin, c_end, acc);
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
  if (rows <= 0) return;
  const int64_t n2 = ld / 2;
  dim3 grid((unsigned)((rows + R - 1) / R), 1);
  hipLaunchKernelGGL((k_gemv<R, U, 1>), grid, dim3(256), 0, s, M, ld, rows, n2, n2, v, y,
                     (int64_t)0, sigma, lam, vloc, status, StopFold{});
}

// Split factors of the two panel passes, from split-factor sweeps on MI355X (round 1;
// per-kernel times on one box): T r with ~512 workgroups or more (RBF k = 256: ts 16 -> 8,
// same 24 us); T^T t with ~96 panel rows per workgroup (RBF: 32 rows 24.8 us, 128 rows
// 21.5 us; nanotube: 80 rows 57.8 us, 300 rows 66.7 us).  Both passes are resident all
// at once, so a grid that leaves some CUs one workgroup more than others runs at the
// pace of the busier ones: among splits a little above the minimum, take the one whose
// grid best fills whole multiples of 256 workgroups (nanotube k = 2701: T r 676 -> 2028
// workgroups, T^T t 899 -> 1023; apply 5.73 -> 5.93 TB/s, same box).
static double wave_fill(int64_t wgs) {
  const int64_t full = (wgs + 255) / 256 * 256;
  return (double)wgs / (double)full;
}

int choose_tsplit(int64_t k, int64_t ncols) {
  const int64_t row_groups = (k + 3) / 4;
  int64_t lo = (512 + row_groups - 1) / row_groups;
  int64_t hi = 2 * lo + 1;
  const int64_t max_by_cols = (ncols / 2 + 255) / 256;  // at least 256 double2 per split
  if (hi > max_by_cols) hi = max_by_cols;
  if (hi > 64) hi = 64;
  if (lo > hi) lo = hi;
  if (lo < 1) lo = 1;
  int64_t best = lo;
  for (int64_t sp = lo; sp <= hi; ++sp)
    if (wave_fill(row_groups * sp) > wave_fill(row_groups * best) + 1e-9) best = sp;
  return (int)best;
}

int choose_zsplit(int64_t k, int64_t ncols) {
  const int64_t slabs = (ncols / 2 + 255) / 256;  // 512-column workgroups
  const int64_t lo = choose_ksplit(k, ncols);
  int64_t hi = lo + (lo + 3) / 4 + 1;
  const int64_t cap = std::min<int64_t>((k + 15) / 16, 256);
  if (hi > cap) hi = cap;
  int64_t best = lo;
  for (int64_t zs = lo; zs <= hi; ++zs)
    if (wave_fill(slabs * zs) > wave_fill(slabs * best) + 1e-9) best = zs;
  return (int)best;
}

// panels above this size do not share the 256 MB MALL with the operator's tables
constexpr double kPanelMallBytes = 192.0e6;
bool panel_streams(int64_t k, int64_t ldt) { return 8.0 * (double)k * (double)ldt > kPanelMallBytes; }

// A streamed panel's leading rows, up to kPanelCachedBytes, are still read with
// default-policy loads by both passes (T r, T^T t): they stay in the MALL from one pass to
// the next and from one iteration to the next, the rest streams (MLFF_PANEL_CACHE_MB
// overrides the budget for sweeps).  Nanotube k = 2701 (336 MB), same box, interleaved:
// 0 / 64 / 128 / 176 / 224 MB -> apply 5.93 / 6.03 / 6.11 / 6.11 / 6.17 TB/s, operator
// unchanged up to 176 MB and 9 % slower at 224 MB (its tables lose the MALL)
constexpr double kPanelCachedBytes = 128.0e6;
int64_t panel_cached_rows(int64_t k, int64_t ldt) {
  if (!panel_streams(k, ldt)) return k;
  static const double budget = [] {
    const char *e = std::getenv("MLFF_PANEL_CACHE_MB");
    return e ? 1.0e6 * std::atof(e) : kPanelCachedBytes;
  }();
  const int64_t rows = (int64_t)(budget / (8.0 * (double)ldt));
  return rows < k ? rows : k;
}

void launch_gemv_split(const double *T, int64_t ldt, int64_t k, int64_t ncols, int splits,
                       const double *r, double *tpart, const int *status, hipStream_t s,
                       StopFold fold) {
  constexpr int R = 4, U = 2;
  const int64_t n2 = ncols / 2;  // ncols is the padded local length (even)
  const int64_t cs2 = (n2 + splits - 1) / splits;
  dim3 grid((unsigned)((k + R - 1) / R), (unsigned)splits);
  // A panel that fits the 256 MB MALL with room to spare (134 MB at k = 256, N = 65536)
  // is read with default-policy loads, so the T^T t pass finds it there; a larger one
  // (the nanotube's 336 MB at k = 2701) is streamed non-temporally so it does not evict
  // the operator's tables (panel_streams)
  if (panel_streams(k, ldt))
    hipLaunchKernelGGL((k_gemv<R, U, 0, true>), grid, dim3(256), 0, s, T, ldt, k, n2, cs2, r, tpart,
                       k, 1.0, 0.0, (const double *)nullptr, status, fold,
                       panel_cached_rows(k, ldt));
  else
    hipLaunchKernelGGL((k_gemv<R, U, 0, false>), grid, dim3(256), 0, s, T, ldt, k, n2, cs2, r, tpart,
                       k, 1.0, 0.0, (const double *)nullptr, status, fold);
}

// ---------------------------------------------------------------------------
// Split-K column GEMV  part[ks, c] = sum_{j in slice ks} W[j, c] t_j,
// t_j = sum_{sp < tsplits} tsrc[sp * tstride + j].  Workgroup = 512 columns (one
// double2 per thread, the 4 waves read 4 KB of every row) x one slice of rows, so
// a k x N panel is spread over ~1024 workgroups whatever its shape.
template <bool NT>
__device__ __forceinline__ d2 colgemv_slice(const d2 *__restrict__ w2, int64_t ld2, int64_t j0,
                                            int64_t j1, const double *t_sh) {
  d2 acc0 = {0.0, 0.0}, acc1 = {0.0, 0.0};
  int64_t j = j0;
  for (; j + 7 < j1; j += 8) {  // 8 rows (128 B per lane) in flight
    d2 a[8];
#pragma unroll
    for (int u = 0; u < 8; ++u)
      a[u] = NT ? __builtin_nontemporal_load(w2 + (j + u) * ld2) : w2[(j + u) * ld2];
#pragma unroll
    for (int u = 0; u < 8; u += 2) {
      const double t0 = t_sh[j + u - j0], t1 = t_sh[j + u + 1 - j0];
      acc0.x = fma(a[u].x, t0, acc0.x);
      acc0.y = fma(a[u].y, t0, acc0.y);
      acc1.x = fma(a[u + 1].x, t1, acc1.x);
      acc1.y = fma(a[u + 1].y, t1, acc1.y);
    }
  }
  for (; j < j1; ++j) {
    const d2 a0 = w2[j * ld2];
    const double t0 = t_sh[j - j0];
    acc0.x = fma(a0.x, t0, acc0.x);
    acc0.y = fma(a0.y, t0, acc0.y);
  }
  return acc0 + acc1;
}

template <bool NT>
__global__ __launch_bounds__(256) void k_colgemv_part(const double *__restrict__ W, int64_t ldw,
                                                      int64_t k, const double *__restrict__ tsrc,
                                                      int tsplits, int64_t tstride,
                                                      int64_t kslice, double *__restrict__ part,
                                                      const int *__restrict__ status,
                                                      StopFold fold, int64_t cached_rows,
                                                      const long long *__restrict__ tcol,
                                                      const int *__restrict__ spec_hit,
                                                      int64_t spec_m0) {
  if (status != nullptr && *status != ST_RUNNING) return;
  extern __shared__ double t_sh[];
  if (!stop_prologue(fold, t_sh)) return;
  int64_t j0 = (int64_t)blockIdx.y * kslice;
  const int64_t j1 = (j0 + kslice) < k ? (j0 + kslice) : k;
  // pivoted-Cholesky speculation hit: the rows below spec_m0 are already summed (a GEMM at
  // the block start); this slice keeps only its rows from spec_m0 on (zeros if none)
  if (spec_hit != nullptr && *spec_hit >= 0 && j0 < spec_m0) j0 = spec_m0 < j1 ? spec_m0 : j1;
  if (tcol != nullptr) {  // t = column *tcol of W itself (the pivot row of L, one rank)
    const int64_t gc = *tcol < 0 ? 0 : (int64_t)*tcol;  // no pivot: the result is unused
    for (int64_t j = j0 + threadIdx.x; j < j1; j += 256) t_sh[j - j0] = W[j * ldw + gc];
  } else {
    for (int64_t j = j0 + threadIdx.x; j < j1; j += 256) {
      double a = 0.0;
      for (int sp = 0; sp < tsplits; ++sp) a += tsrc[(int64_t)sp * tstride + j];
      t_sh[j - j0] = a;
    }
  }
  __syncthreads();
  const int64_t c2 = (int64_t)blockIdx.x * 256 + threadIdx.x;
  if (2 * c2 >= ldw) return;
  const d2 *w2 = reinterpret_cast<const d2 *>(W) + c2;
  const int64_t ld2 = ldw / 2;
  const d2 acc = (NT && j1 > cached_rows) ? colgemv_slice<true>(w2, ld2, j0, j1, t_sh)
                                           : colgemv_slice<false>(w2, ld2, j0, j1, t_sh);
  reinterpret_cast<d2 *>(part + (int64_t)blockIdx.y * ldw)[c2] = acc;
}

int choose_ksplit(int64_t k, int64_t ncols) {
  const int64_t slabs = (ncols + 511) / 512;
  // ~96 panel rows per workgroup (32 or 300 were slower), and at least ~256 workgroups
  int64_t sk = std::max<int64_t>((k + 95) / 96, (256 + slabs - 1) / slabs);
  const int64_t cap = (k + 15) / 16;  // at least 16 rows per slice
  if (sk > cap) sk = cap;
  if (sk < 1) sk = 1;
  if (sk > 256) sk = 256;
  return (int)sk;
}

void launch_colgemv_part(const double *W, int64_t ldw, int64_t k, const double *tsrc,
                         int tsplits, int64_t tstride, int ksplit, double *part,
                         const int *status, hipStream_t s, StopFold fold, int64_t cached_rows,
                         const long long *tcol, const int *spec_hit, int64_t spec_m0) {
  const int64_t kslice = (k + ksplit - 1) / ksplit;
  const dim3 grid((unsigned)((ldw / 2 + 255) / 256), (unsigned)ksplit);
  const size_t shm = sizeof(double) * (kslice + 1 > 8 ? kslice + 1 : 8);
  if (panel_streams(k, ldw))
    hipLaunchKernelGGL(k_colgemv_part<true>, grid, dim3(256), shm, s, W, ldw, k, tsrc, tsplits,
                       tstride, kslice, part, status, fold, cached_rows, tcol, spec_hit, spec_m0);
  else
    hipLaunchKernelGGL(k_colgemv_part<false>, grid, dim3(256), shm, s, W, ldw, k, tsrc, tsplits,
                       tstride, kslice, part, status, fold, cached_rows, tcol, spec_hit, spec_m0);
}

// z = sigma_p * (lam_inv * (r - sum_ks part[ks])) over n local entries; rho partials r.z
__global__ __launch_bounds__(256) void k_precon_fin(const double *__restrict__ part, int ksplit,
                                                    int64_t ldp,
                                                    const double *r,  // = xf.r when fused: no restrict
                                                    double *__restrict__ z, int64_t n,
                                                    double sigma_p, double lam_inv,
                                                    double *__restrict__ rho_part,
                                                    const int *__restrict__ status) {
  if (status != nullptr && *status != ST_RUNNING) return;
  __shared__ double sh[8];
  double rho_acc = 0.0;
  for (int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x; i < n;
       i += (int64_t)gridDim.x * 256) {
    // the ksplit slice partials in slice order, 8 loads in flight
    double sv = 0.0;
    int ks = 0;
    for (; ks + 7 < ksplit; ks += 8) {
      double t[8];
#pragma unroll
      for (int u = 0; u < 8; ++u) t[u] = part[(int64_t)(ks + u) * ldp + i];
#pragma unroll
      for (int u = 0; u < 8; ++u) sv += t[u];
    }
    for (; ks < ksplit; ++ks) sv += part[(int64_t)ks * ldp + i];
    const double rv = r[i];
    const double zv = sigma_p * (lam_inv * (rv - sv));
    z[i] = zv;
    rho_acc = fma(rv, zv, rho_acc);
  }
  const double tot = block_sum256(rho_acc, sh);
  if (threadIdx.x == 0 && rho_part != nullptr) rho_part[blockIdx.x] = tot;
}

void launch_precon_z(const double *T, int64_t ldt, int64_t k, int splits, const double *tpart,
                     const double *r, double *z, int64_t n, double sigma_p, double lam_inv,
                     double *rho_part, const int *status, hipStream_t s, double *zpart,
                     int zsplit, StopFold fold) {
  launch_colgemv_part(T, ldt, k, tpart, splits, k, zsplit, zpart, status, s, fold,
                      panel_cached_rows(k, ldt));
  hipLaunchKernelGGL(k_precon_fin, dim3(kVecGrid), dim3(256), 0, s, zpart, zsplit, ldt, r, z, n,
                     sigma_p, lam_inv, rho_part, status);
}

// ---------------------------------------------------------------------------
// One-pass low-rank apply (one rank; panel rows short enough to sit in registers):
//   z = sigma_p * lam_inv * (r - T^T (T r))          (iterative_cholesky.py:145-148)
// Workgroup w owns the panel rows [w rpw, (w + 1) rpw).  Row i is loaded into registers
// once (512 threads, M double2 each, 16-B loads), t_i = T[i, :] . r is formed against r
// staged in LDS (thread partial -> wave sum -> the 8 wave sums in a fixed order, the same
// bits in every thread), and zacc += T[i, :] t_i from the same registers.  t_i never
// leaves the workgroup, so the panel is read ONCE per apply where the two-pass apply
// (T r, then T^T t) reads it twice; the price is one partial vector per workgroup
// (G x ldt doubles, 32 MB at the nanotube's k = 2701, N = 15540 instead of 336 MB of
// panel), summed in a fixed order by k_lr_fin.  Row i + 1 is in flight while row i is
// reduced (two register buffers, one LDS barrier per row).
constexpr int kLrThreads = 512;
constexpr int64_t kLrMaxCols = 16 * 2 * kLrThreads;  // M <= 16 double2 per thread

bool lr_rows_fits(int64_t ldt) { return ldt > 0 && ldt % 2 == 0 && ldt <= kLrMaxCols; }
// at least 7 rows per workgroup: fewer partial z vectors (16 N bytes each) for small k
// (ethanol N = 15741, k = 1264: 5 -> 7 rows, 253 -> 181 workgroups, apply 39.3 -> 38.1 us; 10 rows:
// 39.0 us; nanotube k = 2701 keeps its 11 (14: 69.3-70.5 vs 68.4-69.0 us), profiles/r04/rpw_ab/;
// round 4 kept 5 only because the golden nanotube drop-in moved 322 -> 321, which the
// double-double Woodbury Gram of round 5 gives either way).  MLFF_LR_MIN_RPW overrides (A/B)
int lr_rows_per_wg(int64_t k) {
  static const int min_rpw = [] {
    const char *e = std::getenv("MLFF_LR_MIN_RPW");
    return e != nullptr ? std::max(1, std::atoi(e)) : 7;
  }();
  return std::max((int)((k + 255) / 256), min_rpw);
}
int lr_rows_groups(int64_t k) {
  const int rpw = lr_rows_per_wg(k);
  return (int)((k + rpw - 1) / rpw);
}

// row loads through a buffer descriptor of the row: one VGPR offset for all M loads (the
// m-th at soffset m * 8 KB), and the descriptor's range check returns zeros beyond the row
// (no bounds test, no 64-bit address per load).  aux 2 = non-temporal.
typedef unsigned int u4 __attribute__((ext_vector_type(4)));

template <int M, int AUX>
__device__ __forceinline__ void lr_load_row(d2 (&buf)[M], const double *row, int bytes) {
  const __amdgpu_buffer_rsrc_t rs =
      __builtin_amdgcn_make_buffer_rsrc(const_cast<double *>(row), 0, bytes, 0x00020000);
  const int voff = (int)threadIdx.x * 16;
#pragma unroll
  for (int m = 0; m < M; ++m)
    buf[m] = __builtin_bit_cast(d2, __builtin_amdgcn_raw_buffer_load_b128(rs, voff, m * kLrThreads * 16, AUX));
}

// Registers per lane: the row being reduced (cur), the next row in flight (nxt) and r, M
// double2 each; the partial z of the workgroup's rows lives in LDS slots private to the
// thread (z_sh[m * kLrThreads + tid]), so no barrier guards them.
// Row i (in cur): t_i, z_sh += cur t_i; row i + 1 loaded into nxt first (a descriptor of
// zero bytes past the last row: the loads return zeros and move nothing).
template <int M, int AUX>
__device__ __forceinline__ void lr_row_step(d2 (&cur)[M], d2 (&nxt)[M], const d2 (&rv)[M],
                                            d2 *z_sh, const double *__restrict__ T, int64_t ldt,
                                            int64_t i, int64_t i0, int64_t i1, double *red) {
  lr_load_row<M, AUX>(nxt, T + (i + 1 < i1 ? i + 1 : i) * ldt, i + 1 < i1 ? (int)(ldt * 8) : 0);
  double a0 = 0.0, a1 = 0.0;
#pragma unroll
  for (int m = 0; m < M; ++m) {
    a0 = fma(cur[m].x, rv[m].x, a0);
    a1 = fma(cur[m].y, rv[m].y, a1);
  }
  const double s = wave_sum(a0 + a1);
  const int p = (int)((i - i0) & 1);  // two slot sets: one barrier per row suffices
  if ((threadIdx.x & 63) == 0) red[p * 8 + (threadIdx.x >> 6)] = s;
  __builtin_amdgcn_fence(__ATOMIC_RELEASE, "workgroup");
  __builtin_amdgcn_s_barrier();
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "workgroup");
  static_assert(kLrThreads == 512, "eight wave sums per row");
  const double *q = red + p * 8;
  const double t = ((q[0] + q[1]) + (q[2] + q[3])) + ((q[4] + q[5]) + (q[6] + q[7]));
#pragma unroll
  for (int m = 0; m < M; m += 4) {
#pragma unroll
    for (int u = 0; u < 4 && m + u < M; ++u) {
      d2 zv = z_sh[threadIdx.x + kLrThreads * (m + u)];
      zv.x = fma(cur[m + u].x, t, zv.x);
      zv.y = fma(cur[m + u].y, t, zv.y);
      z_sh[threadIdx.x + kLrThreads * (m + u)] = zv;
    }
    __builtin_amdgcn_sched_barrier(0);
  }
}

// the workgroup's rows [i0, i1), all read with one load policy (AUX)
template <int M, int AUX>
__device__ __forceinline__ bool lr_rows_loop(const d2 (&rv)[M], d2 *z_sh,
                                             const double *__restrict__ T, int64_t ldt,
                                             int64_t i0, int64_t i1, double *red,
                                             const StopFold &fold) {
  d2 A[M], B[M];
  lr_load_row<M, AUX>(A, T + i0 * ldt, i0 < i1 ? (int)(ldt * 8) : 0);
  // the stop test of the previous iteration while the first row is in flight (every
  // thread reaches the same decision; false: the solver stopped)
  if (!stop_prologue_wide(fold, red)) return false;
#pragma unroll
  for (int m = 0; m < M; ++m) z_sh[threadIdx.x + kLrThreads * m] = d2{0.0, 0.0};
  int64_t i = i0;
  for (; i + 1 < i1; i += 2) {
    lr_row_step<M, AUX>(A, B, rv, z_sh, T, ldt, i, i0, i1, red);
    lr_row_step<M, AUX>(B, A, rv, z_sh, T, ldt, i + 1, i0, i1, red);
  }
  if (i < i1) lr_row_step<M, AUX>(A, B, rv, z_sh, T, ldt, i, i0, i1, red);
  return true;
}

template <int M>
__global__ __launch_bounds__(kLrThreads) void k_lr_rows(const double *__restrict__ T, int64_t ldt,
                                                        int64_t k, int rpw,
                                                        const double *__restrict__ r,
                                                        double *__restrict__ zpart,
                                                        int cached_wgs,
                                                        const int *__restrict__ status,
                                                        StopFold fold, XrFold xf) {
  // the status word is read here and tested once r (and q) are requested: a stopped solver
  // drops them unused, a running one does not wait a round trip for the gate first
  const int st0 = status != nullptr ? *status : ST_RUNNING;
  __shared__ d2 z_sh[M * kLrThreads];
  __shared__ double red[16];
  const int bytes = (int)(ldt * 8);
  const int64_t i0 = (int64_t)blockIdx.x * rpw;
  const int64_t i1 = i0 + rpw < k ? i0 + rpw : k;
  // r and the first row are requested before the stop test of the previous iteration
  // (its partials' round trip then overlaps them; a stopped solver drops them unused)
  d2 rv[M];
  lr_load_row<M, 0>(rv, r, bytes);  // zeros beyond ldt
  if (xf.x == nullptr && st0 != ST_RUNNING) return;  // uniform
  if (xf.x != nullptr) {
    // the residual of the previous iteration, r - alpha q (k_update_xr's arithmetic), before
    // the first row is requested (q, r and a row in registers at once would spill)
    d2 qv[M];
    lr_load_row<M, 0>(qv, xf.q, bytes);
    if (st0 != ST_RUNNING) return;  // uniform: before the first barrier
    const double rho = xf.st->rho;
    const double pq = reduce_parts_bcast_wide(xf.pq_part, kVecGrid, red);
    const double alpha = rho / pq;
    if (blockIdx.x == 0 && threadIdx.x == 0) {  // k_update_xr's state; k_lr_fin reads alpha
      xf.st->pq = pq;
      xf.st->alpha = alpha;
    }
#pragma unroll
    for (int m = 0; m < M; ++m) {
      rv[m].x = fma(-alpha, qv[m].x, rv[m].x);
      rv[m].y = fma(-alpha, qv[m].y, rv[m].y);
    }
  }
  const bool go = blockIdx.x < cached_wgs ? lr_rows_loop<M, 0>(rv, z_sh, T, ldt, i0, i1, red, fold)
                                           : lr_rows_loop<M, 2>(rv, z_sh, T, ldt, i0, i1, red, fold);
  if (!go) return;
  const __amdgpu_buffer_rsrc_t out = __builtin_amdgcn_make_buffer_rsrc(
      zpart + (int64_t)blockIdx.x * ldt, 0, bytes, 0x00020000);
  const int voff = (int)threadIdx.x * 16;
#pragma unroll
  for (int m = 0; m < M; ++m)
    __builtin_amdgcn_raw_buffer_store_b128(__builtin_bit_cast(u4, z_sh[threadIdx.x + kLrThreads * m]),
                                           out, voff, m * kLrThreads * 16, 0);
}

// z[j] = sigma_p lam_inv (r[j] - sum_{g < G} zpart[g, j]) for j < n, the G partials in
// order (wave w sums its quarter, the quarters in order); rho partials r . z in kVecGrid
// slots: a workgroup takes the 64-column blocks blockIdx.x + i gridDim.x (grid <= kVecGrid)
// and writes one slot, the slots past the grid are zero
template <int NW>  // waves per workgroup, each summing 1/NW of the partials
__global__ __launch_bounds__(64 * NW) void k_lr_fin(const double *__restrict__ zpart, int G,
                                                    int64_t ldp,
                                                    const double *r,  // = xf.r when fused: no restrict
                                                    double *__restrict__ z, int64_t n,
                                                    double sigma_p, double lam_inv,
                                                    double *__restrict__ rho_part,
                                                    const int *__restrict__ status, XrFold xf) {
  // the status word gates the stores only: tested once the first block's loads are issued
  const int st0 = status != nullptr ? *status : ST_RUNNING;
  __shared__ double sh[NW][64];
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  const int g0 = (G * w) / NW, g1 = (G * (w + 1)) / NW;
  double rho = 0.0, rr = 0.0;
  const bool fx = xf.x != nullptr;
  // k_update_xr of the previous iteration: alpha = rho / (p.q) as k_lr_rows formed it
  const double alpha = fx ? xf.st->alpha : 0.0;
  for (int64_t jb = blockIdx.x; jb * 64 < n; jb += gridDim.x) {
    const int64_t j = jb * 64 + lane;
    double s = 0.0;
    // wave 0's row operands, requested before the partials
    double rv = 0.0, qj = 0.0, pj = 0.0, xj = 0.0;
    if (w == 0 && j < n) {
      rv = r[j];
      if (fx) {
        qj = xf.q[j];
        pj = xf.p[j];
        xj = xf.x[j];
      }
    }
    if (j < n) {
      // batches of 16 partials in flight, the last one predicated (no serial tail)
      const double *zp = zpart + j;
      for (int g = g0; g < g1; g += 16) {
        double t[16];
#pragma unroll
        for (int u = 0; u < 16; ++u) t[u] = g + u < g1 ? zp[(int64_t)(g + u) * ldp] : 0.0;
#pragma unroll
        for (int u = 0; u < 16; ++u) s += t[u];
      }
    }
    if (st0 != ST_RUNNING) return;  // uniform: before the first barrier and any store
    __syncthreads();  // sh of the previous block
    sh[w][lane] = s;
    __syncthreads();
    if (w == 0 && j < n) {
      double sv = sh[0][lane];  // the wave sums in wave order
#pragma unroll
      for (int q = 1; q < NW; ++q) sv += sh[q][lane];
      if (fx) {  // x += alpha p; r -= alpha q (k_update_xr), rr partials of that residual
        xf.x[j] = fma(alpha, pj, xj);
        rv = fma(-alpha, qj, rv);
        xf.r[j] = rv;
        rr = fma(rv, rv, rr);
      }
      const double zv = sigma_p * (lam_inv * (rv - sv));
      z[j] = zv;
      rho = fma(rv, zv, rho);
    }
  }
  if (st0 != ST_RUNNING) return;  // uniform (a block without columns)
  if (w == 0) {
    const double tot = wave_sum(rho);
    if (lane == 0 && rho_part != nullptr) rho_part[blockIdx.x] = tot;
    if (fx) {
      const double tr = wave_sum(rr);
      if (lane == 0) xf.rr_part[blockIdx.x] = tr;
    }
  }
  if (blockIdx.x == 0 && rho_part != nullptr)
    for (int64_t i = gridDim.x + threadIdx.x; i < kVecGrid; i += 64 * NW) rho_part[i] = 0.0;
  if (blockIdx.x == 0 && fx)
    for (int64_t i = gridDim.x + threadIdx.x; i < kVecGrid; i += 64 * NW) xf.rr_part[i] = 0.0;
}

// waves of k_lr_fin: 16 for the rows form's G = 256 partials (nanotube, 2 interleaved rounds:
// apply 66.3-66.6 us with 4, 65.8-65.9 with 16; k_lr_fin 8.1 -> 7.1 us), 4 for the cluster
// form's few (configs[2], Q = 25: apply 38.2-38.3 us with 4, 38.4-38.5 with 8, 42.2-42.3 with 16,
// profiles/r04/lc_fin_ab/).  MLFF_LR_FIN_WAVES = 4 / 8 / 16 overrides (A/B)
static int lr_fin_waves(int G) {
  static const int forced = [] {
    const char *e = std::getenv("MLFF_LR_FIN_WAVES");
    const int v = e ? std::atoi(e) : 0;
    return v == 4 || v == 8 || v == 16 ? v : 0;
  }();
  return forced != 0 ? forced : (G >= 128 ? 16 : 4);
}

static void launch_lr_fin(const double *zpart, int G, int64_t ldp, const double *r, double *z,
                          int64_t n, double sigma_p, double lam_inv, double *rho_part,
                          const int *status, hipStream_t s, unsigned grid, XrFold xf = XrFold{}) {
  const int nw = lr_fin_waves(G);
  if (nw == 16)
    hipLaunchKernelGGL(k_lr_fin<16>, dim3(grid), dim3(1024), 0, s, zpart, G, ldp, r, z, n, sigma_p,
                       lam_inv, rho_part, status, xf);
  else if (nw == 8)
    hipLaunchKernelGGL(k_lr_fin<8>, dim3(grid), dim3(512), 0, s, zpart, G, ldp, r, z, n, sigma_p,
                       lam_inv, rho_part, status, xf);
  else
    hipLaunchKernelGGL(k_lr_fin<4>, dim3(grid), dim3(256), 0, s, zpart, G, ldp, r, z, n, sigma_p,
                       lam_inv, rho_part, status, xf);
}

static unsigned lr_fin_grid(int64_t n) {
  const int64_t b = (n + 63) / 64;
  return (unsigned)(b < kVecGrid ? b : kVecGrid);
}

// ---------------------------------------------------------------------------
// One-pass low-rank apply for rows longer than one workgroup's registers (one rank,
// N_loc up to kLcMaxC x 7168 columns, e.g. the N = 156510 nanotube system).  A row
// is split over a CLUSTER of C workgroups (column segments of kLcSeg = 7168 columns, 56 KB:
// 448 row threads x 8 double2 in registers, plus one sync wave; r's and the partial z's
// segments in LDS), and the Q = floor(CUs / C) clusters own contiguous row ranges.  Per row
// each member forms its segment's partial dot (fixed-order block sum) and publishes it as two
// 8-byte {epoch, 32 bits} granules (relaxed agent-scope atomic stores, MI355X "R2" hand-off:
// the data is the flag); D row-steps later every member's sync wave reads the C granule pairs
// of that row until every tag equals the launch's epoch, sums the C partials in member order
// (the same bits in every member) and the members accumulate z_seg += T[i, seg] t_i from the
// row still held in registers.  D + L + 1 register buffers: row j (consumed), rows j + 1 …
// j + D - 1 (waiting for their partials), j + D (partial formed and published; loaded L steps
// earlier), rows in flight up to j + D + L (loading): D row-steps of slack for the hand-off,
// L steps between a row's load and its use.  A member that waits for more than ~0.1 s writes
// ST_FAULT to `fault` and leaves (the host reports an error; a cluster can only stall if its
// members are not all resident, which the host checks with the occupancy query before it
// chooses this path).
//
// Why 7 row waves and D = 4 (round 4, profiles/r04/lc_*_ab/): the step time is the hand-off
// round trip / D.  With 8 row waves + the sync wave a workgroup is 9 waves, 3 on some SIMD, so
// every wave gets <= 168 registers: 4 row buffers (D = 2, L = 1).  At D = 2 the apply took
// ~3.2 us per row-step whatever the bytes per step (segments of 4096 / 6144 / 8192 columns:
// nanotube N = 156510 8.4 / 5.1 / 4.0 ms).  7 row waves + the sync wave are 8 waves, 2 per
// SIMD, 256 registers each: 6 buffers, D = 4: 2.73 ms (frac 0.84; D = 3: 2.92, D = 2: 4.25).
constexpr int kLcThreads = 448;  // row threads (7 waves); the workgroup is kLcThreads + 64
constexpr int kLcM = 8;          // double2 per thread per row
constexpr int kLcSeg = kLcM * 2 * kLcThreads;
constexpr int kLcMaxC = 44;  // members per cluster.  Apply time against two passes (round 3,
                             // 8192-column segments, D = 2; nanotube, rule-of-thumb k):
                             // C = 3..14 -21..-41 %, C = 20 -31 %, C = 28 -27 %, C = 41 -8 %,
                             // C = 62 (N = 505050) +14 %
constexpr int kLcD = 4, kLcL = 1;

template <int M, int RT, int AUX>
__device__ __forceinline__ void lc_load(d2 (&buf)[M], const double *T, int64_t ldt,
                                        int64_t row, int64_t i1, int64_t c0, int segbytes) {
  const bool ok = row < i1;
  const __amdgpu_buffer_rsrc_t rs = __builtin_amdgcn_make_buffer_rsrc(
      const_cast<double *>(T + (ok ? row : 0) * ldt + c0), 0, ok ? segbytes : 0, 0x00020000);
  const int voff = (int)threadIdx.x * 16;
#pragma unroll
  for (int m = 0; m < M; ++m)
    buf[m] = __builtin_bit_cast(d2, __builtin_amdgcn_raw_buffer_load_b128(rs, voff, m * RT * 16, AUX));
}

// the RT / 64 row waves' partial sums in a fixed tree (8 waves: ((q0 + q1) + (q2 + q3)) +
// ((q4 + q5) + (q6 + q7)))
template <int NW>
__device__ __forceinline__ double lc_wave_tree(const double *q) {
  if constexpr (NW == 1) {
    return q[0];
  } else {
    return lc_wave_tree<NW / 2>(q) + lc_wave_tree<NW - NW / 2>(q + NW / 2);
  }
}

struct LcArgs {
  const double *T;
  int64_t ldt, c0;
  int i0, i1;  // the cluster's rows (32-bit: scalar compares in the row loop)
  int segbytes, C, c;
  unsigned long long *slots;  // k x C x 2 granules
  unsigned epoch;
  int mute;  // test hook: this member never publishes (its cluster times out)
};

// wave 0: the C partials of row `row` (granule pairs), summed in member order; false on
// timeout.  x0 / x1: this lane's granules as loaded at the start of the step (before the
// step's row loads, so the first look does not queue behind them); re-polled until every
// tag equals the epoch.  Every lane returns the same t.
__device__ __forceinline__ unsigned long long *lc_granule(const LcArgs &a, int row) {
  const int lane = threadIdx.x & 63;
  return a.slots + ((size_t)row * a.C + (lane < a.C ? lane : 0)) * 2;
}

__device__ __forceinline__ bool lc_consume(const LcArgs &a, int row, unsigned long long x0,
                                           unsigned long long x1, double &t) {
  const int lane = threadIdx.x & 63;
  unsigned long long *g = lc_granule(a, row);
  const unsigned long long t0 = wall_clock64();
  for (;;) {
    const bool ok = lane >= a.C ||
                    ((unsigned)(x0 >> 32) == a.epoch && (unsigned)(x1 >> 32) == a.epoch);
    if (__all(ok)) break;
    // ~0.1 s at 100 MHz: far above any hand-off of a resident cluster (the whole apply takes
    // <= 50 ms at N = 505050), short enough that a cluster starved by another process's
    // kernels falls back to two passes quickly (the next preconditioner build re-checks)
    if (wall_clock64() - t0 > 10000000ull) return false;
    __builtin_amdgcn_s_sleep(1);
    if (lane < a.C) {
      x0 = __hip_atomic_load(g, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      x1 = __hip_atomic_load(g + 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    }
  }
  const double v = __builtin_bit_cast(double, (x1 << 32) | (x0 & 0xffffffffull));
  double s = 0.0;
  for (int m = 0; m < a.C; ++m) s += __shfl(v, m, 64);
  t = s;
  return true;
}

// One row-step at row j with NB register buffers, split between the two kinds of wave (a
// wave-uniform branch: both execute one barrier per step).  Row waves (0-7) hold the row
// segment: b0 = row j (consumed), bp = row j + D (its partial formed), bl = row j + D + L
// (loading); the rows between wait for their partials or are in flight.  The sync
// wave (8) polls, sums and publishes: its hand-off loads never queue behind row loads, and
// the row waves' code holds no hand-off load a counter wait could be charged for.
template <int D, int L, int M, int RT, int AUX>
__device__ __forceinline__ bool lc_row_step(const LcArgs &a, int j, d2 (&b0)[M],
                                            d2 (&b2)[M], d2 (&b3)[M], const d2 *r_sh,
                                            d2 *z_sh, double *red, const double *tsh,
                                            const int *bail) {
  const int w = threadIdx.x >> 6;
  const int jp = j + D;
  lc_load<M, RT, AUX>(b3, a.T, a.ldt, j + D + L, a.i1, a.c0, a.segbytes);
  if (jp >= a.i0 && jp < a.i1) {
    double a0 = 0.0, a1 = 0.0;
#pragma unroll
    for (int m = 0; m < M; ++m) {
      const d2 rv = r_sh[threadIdx.x + RT * m];
      a0 = fma(b2[m].x, rv.x, a0);
      a1 = fma(b2[m].y, rv.y, a1);
    }
    const double sw = wave_sum(a0 + a1);
    if ((threadIdx.x & 63) == 0) red[(jp & 1) * 8 + w] = sw;
  }
  __syncthreads();
  if (*bail) return false;
  if (j >= a.i0 && j < a.i1) {
    const double t = tsh[j & 1];
#pragma unroll
    for (int m = 0; m < M; ++m) {
      d2 zv = z_sh[threadIdx.x + RT * m];
      zv.x = fma(b0[m].x, t, zv.x);
      zv.y = fma(b0[m].y, t, zv.y);
      z_sh[threadIdx.x + RT * m] = zv;
    }
  }
  return true;
}

// n0 / n1: row j's granules as loaded one step earlier (MLFF_LC_PREFETCH, default on): they were
// published D steps before j, so the look usually finds them complete and the step does not wait
// a memory round trip of its own; row j + 1's look is issued here for the next step.  Off: the
// look is issued at the start of the step and waited for (one round trip per step under the row
// stream's load: ~3.2 us at every D, L and segment width, profiles/r04/lc_cfg_ab/)
template <int D, int RT>
__device__ __forceinline__ bool lc_sync_step(const LcArgs &a, int j, const double *red,
                                             double *tsh, int *bail, unsigned long long &n0,
                                             unsigned long long &n1, bool prefetch) {
  const int lane = threadIdx.x & 63;
  const int jp = j + D;
  if (j >= a.i0 && j < a.i1) {
    unsigned long long x0 = 0, x1 = 0;
    if (prefetch) {
      x0 = n0;
      x1 = n1;
      if (lane < a.C && j + 1 < a.i1) {
        unsigned long long *g = lc_granule(a, j + 1);
        n0 = __hip_atomic_load(g, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        n1 = __hip_atomic_load(g + 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      }
    } else if (lane < a.C) {
      unsigned long long *g = lc_granule(a, j);
      x0 = __hip_atomic_load(g, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      x1 = __hip_atomic_load(g + 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    }
    double t;
    const bool ok = lc_consume(a, j, x0, x1, t);
    if (lane == 0) {
      tsh[j & 1] = t;
      *bail = ok ? 0 : 1;
    }
  }
  __syncthreads();
  if (*bail) return false;
  if (jp >= a.i0 && jp < a.i1 && lane == 0 && !a.mute) {
    const double *q = red + (jp & 1) * 8;
    const double ps = lc_wave_tree<RT / 64>(q);
    const unsigned long long bits = __builtin_bit_cast(unsigned long long, ps);
    unsigned long long *g = a.slots + ((size_t)jp * a.C + a.c) * 2;
    __hip_atomic_store(g, ((unsigned long long)a.epoch << 32) | (bits & 0xffffffffull),
                       __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    __hip_atomic_store(g + 1, ((unsigned long long)a.epoch << 32) | (bits >> 32), __ATOMIC_RELAXED,
                       __HIP_MEMORY_SCOPE_AGENT);
  }
  return true;
}

template <int D, int L, int M, int RT, int AUX, int U>
__device__ __forceinline__ bool lc_row_steps(const LcArgs &a, int j, d2 (&B)[D + L + 1][M],
                                             const d2 *r_sh, d2 *z_sh, double *red,
                                             const double *tsh, const int *bail) {
  constexpr int NB = D + L + 1;
  if constexpr (U == NB) {
    return true;
  } else {
    if (!lc_row_step<D, L, M, RT, AUX>(a, j + U, B[U], B[(U + D) % NB], B[(U + D + L) % NB], r_sh, z_sh,
                              red, tsh, bail))
      return false;
    return lc_row_steps<D, L, M, RT, AUX, U + 1>(a, j, B, r_sh, z_sh, red, tsh, bail);
  }
}

// AUX: the row loads' cache policy (2: non-temporal, the panel streams; 0: default, a panel that
// fits the MALL beside the operator stays there from one iteration to the next, panel_streams)
template <int D, int L, int M, int RT = kLcThreads, int AUX = 2>
__global__ __launch_bounds__(RT + 64) void k_lr_cluster(const double *__restrict__ T, int64_t ldt,
                                                           int64_t k, int C, int rpc,
                                                           const double *__restrict__ r,
                                                           double *__restrict__ zpart,
                                                           unsigned long long *slots,
                                                           unsigned epoch, int *fault,
                                                           int mute_block, int prefetch,
                                                           const int *__restrict__ status,
                                                           StopFold fold) {
  if (status != nullptr && *status != ST_RUNNING) return;
  constexpr int SEG = M * 2 * RT;
  __shared__ d2 r_sh[M * RT];
  __shared__ d2 z_sh[M * RT];
  __shared__ double red[16];
  __shared__ double tsh[2];
  __shared__ int bail;
  LcArgs a;
  a.T = T;
  a.ldt = ldt;
  a.C = C;
  const int q = blockIdx.x / C;
  a.c = blockIdx.x % C;
  a.c0 = (int64_t)a.c * SEG;
  const int64_t segcols = ldt - a.c0 < SEG ? ldt - a.c0 : SEG;
  a.segbytes = (int)(segcols * 8);
  a.i0 = q * rpc;
  a.i1 = a.i0 + rpc < (int)k ? a.i0 + rpc : (int)k;
  a.slots = slots;
  a.epoch = epoch;
  a.mute = (int)blockIdx.x == mute_block;
  const bool row_wave = threadIdx.x < RT;
  constexpr int NB = D + L + 1;
  if (row_wave) {
    d2 B[NB][M];
    d2 rv[M];
    const __amdgpu_buffer_rsrc_t rs = __builtin_amdgcn_make_buffer_rsrc(
        const_cast<double *>(r + a.c0), 0, a.segbytes, 0x00020000);
#pragma unroll
    for (int m = 0; m < M; ++m)
      rv[m] = __builtin_bit_cast(d2, __builtin_amdgcn_raw_buffer_load_b128(
                                         rs, (int)threadIdx.x * 16, m * RT * 16, 0));
#pragma unroll
    for (int t = 0; t < L; ++t)  // rows i0 .. i0 + L - 1 (the steps start at j = i0 - D)
      lc_load<M, RT, AUX>(B[(D + t) % NB], T, ldt, a.i0 + t, a.i1, a.c0, a.segbytes);
    if (!stop_prologue_wide(fold, red)) return;
#pragma unroll
    for (int m = 0; m < M; ++m) {
      r_sh[threadIdx.x + RT * m] = rv[m];
      z_sh[threadIdx.x + RT * m] = d2{0.0, 0.0};
    }
    __syncthreads();  // bail = 0 (sync wave)
    bool ok = true;
    for (int j = a.i0 - D; j < a.i1 && ok; j += NB)
      ok = lc_row_steps<D, L, M, RT, AUX, 0>(a, j, B, r_sh, z_sh, red, tsh, &bail);
    if (!ok) return;
    const __amdgpu_buffer_rsrc_t out = __builtin_amdgcn_make_buffer_rsrc(
        zpart + (int64_t)q * ldt + a.c0, 0, a.segbytes, 0x00020000);
#pragma unroll
    for (int m = 0; m < M; ++m)
      __builtin_amdgcn_raw_buffer_store_b128(__builtin_bit_cast(u4, z_sh[threadIdx.x + RT * m]),
                                             out, (int)threadIdx.x * 16, m * RT * 16, 0);
  } else {
    if (!stop_prologue_wide(fold, red)) return;
    if (threadIdx.x == RT) bail = 0;
    __syncthreads();
    bool ok = true;
    unsigned long long n0 = 0, n1 = 0;  // epoch 0 is never a launch's: the first look polls
    for (int j = a.i0 - D; j < a.i1 && ok; j += NB)
      for (int u = 0; u < NB && ok; ++u)
        ok = lc_sync_step<D, RT>(a, j + u, red, tsh, &bail, n0, n1, prefetch != 0);
    if (!ok && threadIdx.x == RT)
      __hip_atomic_store(fault, ST_FAULT, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  }
}

// MLFF_LC_CFG="D,L,M,RT" (A/B of the hand-off slack D, load distance L, double2 per thread M and
// row threads RT; segment 2 M RT columns): one of the instantiations below, else the default
// (4, 1, 8, 448)
struct LcCfg {
  int D, L, M, RT;
};
static LcCfg lc_cfg() {
  static const LcCfg cfg = [] {
    LcCfg c{kLcD, kLcL, kLcM, kLcThreads};
    if (const char *e = std::getenv("MLFF_LC_CFG")) {
      LcCfg w{0, 0, 0, kLcThreads};
      if (std::sscanf(e, "%d,%d,%d,%d", &w.D, &w.L, &w.M, &w.RT) >= 3) {
        const LcCfg ok[] = {{4, 1, 8, 448}, {3, 2, 8, 448}, {4, 2, 8, 448}, {5, 1, 8, 448},
                            {2, 1, 8, 512}, {3, 1, 6, 512}};
        for (const LcCfg &o : ok)
          if (o.D == w.D && o.L == w.L && o.M == w.M && o.RT == w.RT) c = w;
      }
    }
    return c;
  }();
  return cfg;
}
static int64_t lc_seg() { return (int64_t)lc_cfg().M * 2 * lc_cfg().RT; }
static int lc_threads() { return lc_cfg().RT + 64; }

// MLFF_LC_CACHED=0 / 1 (A/B): the row loads' policy regardless of the panel's size
static bool lc_cached(int64_t k, int64_t ldt) {
  static const int force = [] {
    const char *e = std::getenv("MLFF_LC_CACHED");
    return e != nullptr ? std::atoi(e) : -1;
  }();
  return force >= 0 ? force != 0 : !panel_streams(k, ldt);
}

template <typename F>
static auto lc_dispatch(F &&f, bool cached = false) {
  const LcCfg c = lc_cfg();
  if (cached && c.D == kLcD && c.L == kLcL && c.M == kLcM && c.RT == kLcThreads)
    return f(k_lr_cluster<kLcD, kLcL, kLcM, kLcThreads, 0>);
  if (c.RT == 448 && c.D == 3) return f(k_lr_cluster<3, 2, 8, 448>);
  if (c.RT == 448 && c.D == 4 && c.L == 2) return f(k_lr_cluster<4, 2, 8, 448>);
  if (c.RT == 448 && c.D == 5) return f(k_lr_cluster<5, 1, 8, 448>);
  if (c.RT == 512 && c.M == 8) return f(k_lr_cluster<2, 1, 8, 512>);  // round 3's form
  if (c.RT == 512 && c.M == 6) return f(k_lr_cluster<3, 1, 6, 512>);
  return f(k_lr_cluster<kLcD, kLcL, kLcM>);
}

int lr_cluster_members(int64_t ldt) { return (int)((ldt + lc_seg() - 1) / lc_seg()); }
bool lr_cluster_fits(int64_t ldt) {
  static const int maxc = [] {  // MLFF_LC_MAXC: sweeps of the member cap (at most 64: one wave polls)
    const char *e = std::getenv("MLFF_LC_MAXC");
    return e ? std::min(64, std::max(1, std::atoi(e))) : kLcMaxC;
  }();
  return ldt > 0 && ldt % 2 == 0 && lr_cluster_members(ldt) <= maxc;
}

// clusters of C members that the device keeps resident all at once (0: none)
int lr_cluster_count(int64_t ldt, int device) {
  const int C = lr_cluster_members(ldt);
  int cus = 0, per_cu = 0;
  if (hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, device) != hipSuccess)
    return 0;
  if (lc_dispatch([&](auto kern) {
        return hipOccupancyMaxActiveBlocksPerMultiprocessor(&per_cu, kern, lc_threads(), 0);
      }) != hipSuccess)
    return 0;
  const int resident = cus * std::min(per_cu, 1);  // one member per CU
  return resident / C;
}

void launch_lr_apply_cluster(const double *T, int64_t ldt, int64_t k, int Q, const double *r,
                             double *z, int64_t n, double sigma_p, double lam_inv,
                             double *rho_part, const int *status, hipStream_t s, double *zpart,
                             unsigned long long *slots, unsigned epoch, int *fault,
                             StopFold fold) {
  const int C = lr_cluster_members(ldt);
  const int rpc = (int)((k + Q - 1) / Q);
  // hand-off slack D = 2 steps, load distance L = 1 (D = 1, L = 2: apply 3.95 -> 4.22 ms at
  // N = 156510; the hand-off, not the load latency, sets the pace)
  // MLFF_LC_TEST_MUTE=<b>[@<e>]: workgroup b never publishes (from the launch with epoch e
  // on, default every launch), so its cluster's hand-offs time out (tests of the ~0.1 s fault
  // bail-out, also in the middle of a chunk of PCG iterations; never set in production)
  static const int prefetch = [] {
    const char *e = std::getenv("MLFF_LC_PREFETCH");
    return e != nullptr && std::atoi(e) == 0 ? 0 : 1;
  }();
  int mute = -1;
  if (const char *mute_env = std::getenv("MLFF_LC_TEST_MUTE")) {
    const char *at = std::strchr(mute_env, '@');
    const unsigned from = at ? (unsigned)std::atoi(at + 1) : 0u;
    if (epoch >= from) mute = std::atoi(mute_env);
  }
  lc_dispatch(
      [&](auto kern) {
        hipLaunchKernelGGL(kern, dim3((unsigned)(Q * C)), dim3(lc_threads()), 0, s, T, ldt, k, C,
                           rpc, r, zpart, slots, epoch, fault, mute, prefetch, status, fold);
        return 0;
      },
      lc_cached(k, ldt));
  if (n > 0)
    launch_lr_fin(zpart, Q, ldt, r, z, n, sigma_p, lam_inv, rho_part, status, s, lr_fin_grid(n));
}

void launch_lr_apply_rows(const double *T, int64_t ldt, int64_t k, const double *r, double *z,
                          int64_t n, double sigma_p, double lam_inv, double *rho_part,
                          const int *status, hipStream_t s, double *zpart, StopFold fold,
                          XrFold xf) {
  const int64_t n2 = ldt / 2;
  const int rpw = lr_rows_per_wg(k), G = lr_rows_groups(k);
  // rows read with default-policy loads stay in the MALL from one iteration to the next:
  // the panel_cached_rows budget as whole workgroups' rows (one load policy per workgroup);
  // MLFF_LR_CACHE_WGS overrides (A/B)
  int cached = panel_streams(k, ldt) ? (int)(panel_cached_rows(k, ldt) / rpw) : G;
  if (const char *e = std::getenv("MLFF_LR_CACHE_WGS")) cached = std::atoi(e);
  const dim3 grid((unsigned)G);
  if (n2 <= 4 * kLrThreads)
    hipLaunchKernelGGL(k_lr_rows<4>, grid, dim3(kLrThreads), 0, s, T, ldt, k, rpw, r, zpart, cached, status, fold, xf);
  else if (n2 <= 8 * kLrThreads)
    hipLaunchKernelGGL(k_lr_rows<8>, grid, dim3(kLrThreads), 0, s, T, ldt, k, rpw, r, zpart, cached, status, fold, xf);
  else if (n2 <= 12 * kLrThreads)
    hipLaunchKernelGGL(k_lr_rows<12>, grid, dim3(kLrThreads), 0, s, T, ldt, k, rpw, r, zpart, cached, status, fold, xf);
  else
    hipLaunchKernelGGL(k_lr_rows<16>, grid, dim3(kLrThreads), 0, s, T, ldt, k, rpw, r, zpart, cached, status, fold, xf);
  if (n > 0)
    launch_lr_fin(zpart, G, ldt, r, z, n, sigma_p, lam_inv, rho_part, status, s, lr_fin_grid(n), xf);
}

// ---------------------------------------------------------------------------
__global__ __launch_bounds__(256) void k_dot_part(const double *__restrict__ a,
                                                  const double *__restrict__ b, int64_t n,
                                                  double *__restrict__ part,
                                                  const int *__restrict__ status,
                                                  StopFold fold) {
  if (status != nullptr && *status != ST_RUNNING) return;
  __shared__ double sh[8];
  if (!stop_prologue(fold, sh)) return;
  double acc = 0.0;
  for (int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x; i < n;
       i += (int64_t)gridDim.x * 256)
    acc = fma(a[i], b[i], acc);
  const double t = block_sum256(acc, sh);
  if (threadIdx.x == 0) part[blockIdx.x] = t;
}

void launch_dot_part(const double *a, const double *b, int64_t n, double *part,
                     const int *status, hipStream_t s, StopFold fold) {
  hipLaunchKernelGGL(k_dot_part, dim3(kVecGrid), dim3(256), 0, s, a, b, n, part, status, fold);
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

// ---------------------------------------------------------------------------
// Several ranks: the search direction is formed from the all-gathered z instead of
// all-gathering p.  Rank g's block of the gather buffer gb (stride gstride) holds
// z_g (blk entries, zero padded) followed by its kVecGrid rho partials (r_g . z_g),
// so one allgather replaces allreduce(rho) + allgather(p).  Every rank then sums the
// world x kVecGrid rho partials in the same fixed order (bitwise identical rho on all
// ranks) and updates the whole p_full = z_full + beta p_full, whose rank blocks are
// exactly what the local update would produce.

// no preconditioner: z = r, copied into the gather block with its rho partials
__global__ __launch_bounds__(256) void k_copy_dot(const double *__restrict__ r, int64_t n,
                                                  double *__restrict__ dst,
                                                  double *__restrict__ part,
                                                  const int *__restrict__ status,
                                                  StopFold fold) {
  if (status != nullptr && *status != ST_RUNNING) return;
  __shared__ double sh[8];
  if (!stop_prologue(fold, sh)) return;
  double acc = 0.0;
  for (int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x; i < n;
       i += (int64_t)gridDim.x * 256) {
    const double v = r[i];
    dst[i] = v;
    acc = fma(v, v, acc);
  }
  const double t = block_sum256(acc, sh);
  if (threadIdx.x == 0) part[blockIdx.x] = t;
}

void launch_copy_dot(const double *r, int64_t n, double *dst, double *part, const int *status,
                     hipStream_t s, StopFold fold) {
  hipLaunchKernelGGL(k_copy_dot, dim3(kVecGrid), dim3(256), 0, s, r, n, dst, part, status, fold);
}

__global__ __launch_bounds__(256) void k_update_p_gathered(const double *__restrict__ gb,
                                                           int64_t gstride, int64_t blk,
                                                           int world, double *__restrict__ p,
                                                           DevState *st, long long it,
                                                           const int *__restrict__ status) {
  if (*status != ST_RUNNING) return;
  __shared__ double sh[8];
  double v = 0.0;
  // the thread's partials (world * kVecGrid / 256 of them) in order, 8 loads in flight
  const int np = world * kVecGrid;
  int f = threadIdx.x;
  for (; f + 7 * 256 < np; f += 8 * 256) {
    double t[8];
#pragma unroll
    for (int u = 0; u < 8; ++u) {
      const int g = f + u * 256;
      t[u] = gb[(int64_t)(g / kVecGrid) * gstride + blk + (g % kVecGrid)];
    }
#pragma unroll
    for (int u = 0; u < 8; ++u) v += t[u];
  }
  for (; f < np; f += 256) v += gb[(int64_t)(f / kVecGrid) * gstride + blk + (f % kVecGrid)];
  v = block_sum256(v, sh);
  __syncthreads();
  if (threadIdx.x == 0) sh[4] = v;
  __syncthreads();
  const double rho = sh[4];
  if (blockIdx.x == 0 && threadIdx.x == 0) st->rho = rho;
  const int64_t ld = (int64_t)world * blk;
  if (it > 1) {
    const double beta = rho / st->rho1;
    for (int64_t j = (int64_t)blockIdx.x * 256 + threadIdx.x; j < ld;
         j += (int64_t)gridDim.x * 256)
      p[j] = fma(beta, p[j], gb[(j / blk) * gstride + j % blk]);
  } else {
    for (int64_t j = (int64_t)blockIdx.x * 256 + threadIdx.x; j < ld;
         j += (int64_t)gridDim.x * 256)
      p[j] = gb[(j / blk) * gstride + j % blk];
  }
}

void launch_update_p_gathered(const double *gb, int64_t gstride, int64_t blk, int world,
                              double *p_full, DevState *st, long long it, const int *status,
                              hipStream_t s) {
  hipLaunchKernelGGL(k_update_p_gathered, dim3(256), dim3(256), 0, s, gb, gstride, blk, world,
                     p_full, st, it, status);
}

// the r update of the sharded symmetric-tile iteration for one entry: q = sigma y + lam p,
// r - alpha q (k_update_xr_shares and k_gemv_xr share it: the same bits)
__device__ __forceinline__ double xr_shares_r(double ri, double yi, double pi, double alpha,
                                              double sigma, double lam) {
  const double qi = sigma * yi + lam * pi;
  return fma(-alpha, qi, ri);
}

// Several ranks, symmetric tiles: y = this rank's reduce-scattered rows of K p,
// shares[0..world) = every rank's share of p.q (k_pq_publish).  pq = the shares
// summed in rank order; q = sigma y + lam p (as k_axpby_loc); then as k_update_xr.
__global__ __launch_bounds__(256) void k_update_xr_shares(double *__restrict__ x,
                                                          double *__restrict__ r,
                                                          const double *__restrict__ p,
                                                          const double *__restrict__ y,
                                                          const double *__restrict__ shares,
                                                          int world, int64_t n, double sigma,
                                                          double lam,
                                                          double *__restrict__ rr_part,
                                                          DevState *st,
                                                          const int *__restrict__ status) {
  if (*status != ST_RUNNING) return;
  __shared__ double sh[8];
  double pq = 0.0;
  for (int g = 0; g < world; ++g) pq += shares[g];
  const double alpha = st->rho / pq;
  if (blockIdx.x == 0 && threadIdx.x == 0) {
    st->pq = pq;
    st->alpha = alpha;
  }
  double acc = 0.0;
  for (int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x; i < n;
       i += (int64_t)gridDim.x * 256) {
    const double pi = p[i];
    x[i] = fma(alpha, pi, x[i]);
    const double ri = xr_shares_r(r[i], y[i], pi, alpha, sigma, lam);
    r[i] = ri;
    acc = fma(ri, ri, acc);
  }
  const double t = block_sum256(acc, sh);
  if (threadIdx.x == 0) rr_part[blockIdx.x] = t;
}

void launch_update_xr_shares(double *x, double *r, const double *p, const double *y,
                             const double *shares, int world, int64_t n, double sigma, double lam,
                             double *rr_part, DevState *st, const int *status, hipStream_t s) {
  hipLaunchKernelGGL(k_update_xr_shares, dim3(kVecGrid), dim3(256), 0, s, x, r, p, y, shares, world,
                     n, sigma, lam, rr_part, st, status);
}

// Several ranks, symmetric tiles, low-rank preconditioner: k_update_xr_shares folded into
// the T r pass of the next apply (k_gemv<4, 2, 0>).  Every workgroup forms r_new = r - alpha q
// for the columns of its split and stages it in LDS as the GEMV operand; the workgroups of row
// group 0 also write r_new into r_out (another buffer: the other row groups still read r),
// x += alpha p, and the rr partials of the 256-row blocks of their columns, each summed as
// k_update_xr_shares sums it (one 256-thread block_sum256 per 256 rows), the blocks past the
// local rows zeroed.  x, r, the rr partials and the T r partials are the bits of the two
// separate launches.  Needs 2 cs2 % 256 == 0 and n <= kVecGrid * 256 (xr_fold_fits).  Gated
// (solver stopped): row group 0 copies r into r_out, so the caller's buffer swap keeps the
// state.
template <int R, int U, bool NT>
__global__ __launch_bounds__(256) void k_gemv_xr(const double *__restrict__ M, int64_t ld,
                                                 int64_t rows, int64_t n2, int64_t cs2,
                                                 const double *__restrict__ r,
                                                 double *__restrict__ r_out,
                                                 double *__restrict__ x,
                                                 const double *__restrict__ p,
                                                 const double *__restrict__ y,
                                                 const double *__restrict__ shares, int world,
                                                 int64_t n, double sigma, double lam,
                                                 double *__restrict__ rr_part, DevState *st,
                                                 double *__restrict__ out, int64_t out_stride,
                                                 const int *__restrict__ status,
                                                 int64_t cached_rows) {
  extern __shared__ d2 vs[];  // r_new of this split's columns (cs2 entries)
  __shared__ double sh[4 * R > 8 ? 4 * R : 8];
  const int64_t c_begin = (int64_t)blockIdx.y * cs2;
  int64_t c_end = c_begin + cs2;
  if (c_end > n2) c_end = n2;
  const bool owner = blockIdx.x == 0;
  const d2 *__restrict__ r2 = reinterpret_cast<const d2 *>(r);
  d2 *__restrict__ ro2 = reinterpret_cast<d2 *>(r_out);
  if (*status != ST_RUNNING) {
    if (owner)
      for (int64_t c = c_begin + threadIdx.x; c < c_end; c += 256) ro2[c] = r2[c];
    return;
  }
  double pq = 0.0;
  for (int g = 0; g < world; ++g) pq += shares[g];
  const double alpha = st->rho / pq;
  if (owner && blockIdx.y == 0 && threadIdx.x == 0) {
    st->pq = pq;
    st->alpha = alpha;
  }
  for (int64_t c = c_begin + threadIdx.x; c < c_end; c += 256) {
    d2 rv = r2[c];
    const int64_t i = 2 * c;
    if (i < n) {
      const double pi = p[i];
      rv.x = xr_shares_r(rv.x, y[i], pi, alpha, sigma, lam);
      if (owner) x[i] = fma(alpha, pi, x[i]);
    }
    if (i + 1 < n) {
      const double pi = p[i + 1];
      rv.y = xr_shares_r(rv.y, y[i + 1], pi, alpha, sigma, lam);
      if (owner) x[i + 1] = fma(alpha, pi, x[i + 1]);
    }
    vs[c - c_begin] = rv;
    if (owner) ro2[c] = rv;
  }
  __syncthreads();
  if (owner) {
    const double *vd = reinterpret_cast<const double *>(vs);
    for (int64_t b0 = 2 * c_begin; b0 < 2 * c_end; b0 += 256) {
      const int64_t i = b0 + threadIdx.x;
      double acc = 0.0;
      if (i < n) {
        const double ri = vd[i - 2 * c_begin];
        acc = fma(ri, ri, acc);
      }
      const double t = block_sum256(acc, sh);
      if (threadIdx.x == 0) rr_part[b0 / 256] = t;
    }
    if (blockIdx.y == 0)
      for (int64_t b = (2 * n2 + 255) / 256 + threadIdx.x; b < kVecGrid; b += 256) rr_part[b] = 0.0;
    __syncthreads();  // sh is reused below
  }
  const int64_t r0 = (int64_t)blockIdx.x * R;
  const d2 *rowp[R];
#pragma unroll
  for (int q = 0; q < R; ++q) rowp[q] = reinterpret_cast<const d2 *>(M + (r0 + q) * ld);
  double acc[R];
#pragma unroll
  for (int q = 0; q < R; ++q) acc[q] = 0.0;
  if (NT && r0 + R > cached_rows)
    gemv_rows_body<R, U, true>(rowp, vs, c_begin, c_end, acc, c_begin);
  else
    gemv_rows_body<R, U, false>(rowp, vs, c_begin, c_end, acc, c_begin);
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
#pragma unroll
  for (int q = 0; q < R; ++q) {
    const double s = wave_sum(acc[q]);
    if (lane == 0) sh[w * R + q] = s;
  }
  __syncthreads();
  if (threadIdx.x < R) {
    const int q = threadIdx.x;
    const int64_t row = r0 + q;
    if (row < rows)
      out[(int64_t)blockIdx.y * out_stride + row] =
          (sh[q] + sh[R + q]) + (sh[2 * R + q] + sh[3 * R + q]);
  }
}

bool xr_fold_fits(int64_t ncols, int splits, int64_t n) {
  const int64_t n2 = ncols / 2, cs2 = (n2 + splits - 1) / splits;
  // the owner loop writes rr_part[b0 / 256] for every b0 < ncols (the padded block, which can
  // exceed the last rank's row count n): both must fit the kVecGrid partial slots
  return ncols % 2 == 0 && (2 * cs2) % 256 == 0 && cs2 * 16 <= 64 * 1024 &&
         n <= (int64_t)kVecGrid * 256 && ncols <= (int64_t)kVecGrid * 256;
}

void launch_gemv_xr(const double *T, int64_t ldt, int64_t k, int64_t ncols, int splits,
                    const double *r, double *r_out, double *x, const double *p, const double *y,
                    const double *shares, int world, int64_t n, double sigma, double lam,
                    double *rr_part, DevState *st, double *tpart, const int *status,
                    hipStream_t s) {
  constexpr int R = 4, U = 2;
  const int64_t n2 = ncols / 2;
  const int64_t cs2 = (n2 + splits - 1) / splits;
  const dim3 grid((unsigned)((k + R - 1) / R), (unsigned)splits);
  const size_t shm = sizeof(d2) * (size_t)cs2;
  if (panel_streams(k, ldt))
    hipLaunchKernelGGL((k_gemv_xr<R, U, true>), grid, dim3(256), shm, s, T, ldt, k, n2, cs2, r, r_out,
                       x, p, y, shares, world, n, sigma, lam, rr_part, st, tpart, k, status,
                       panel_cached_rows(k, ldt));
  else
    hipLaunchKernelGGL((k_gemv_xr<R, U, false>), grid, dim3(256), shm, s, T, ldt, k, n2, cs2, r, r_out,
                       x, p, y, shares, world, n, sigma, lam, rr_part, st, tpart, k, status,
                       (int64_t)0);
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
