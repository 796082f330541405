// Greedy diagonal-pivoted partial Cholesky of S = sigma_K * K on the device.
// Restates src/sGDML/sgdml/solvers/incomplete_cholesky.py:24-93:
//   i_argmax = argmax(diag[index_columns][m:]) + m        (first max in permuted order, :53)
//   swap index_columns[m], index_columns[i_argmax]          (:55)
//   L[m_pi, m] = sqrt(diag[m_pi]); assert pivot > 0        (:61-63)
//   L[i_pi, m] = (col[i_pi] - L[i_pi, :m] . L[m_pi, :m]) / L[m_pi, m]   (:66-75)
//   diag[i_pi] -= L[i_pi, m]^2                              (:78)
// where col = get_col(m_pi) = column m_pi of the operator (iterative_cholesky.py:152-156).
// L is kept transposed (Lt: k x blk, rows = pivot steps, columns = original row
// index), which is exactly the "wide" panel the Woodbury build consumes.
// Multi-rank: the argmax is an allgather of per-rank (value, position) winners,
// the pivot row L[m_pi, :m] an allreduce of a vector only its owner fills.
#include "common.h"
#include "sgdml_col.h"

#include <cstdio>
#include <cstdlib>
#include <algorithm>
#include <vector>

namespace mlff {

// speculative blocks of the Schur GEMV (see k_spec_top_part)
constexpr int kSpecB = 16;        // steps per speculative block
constexpr int kSpecC = 64;        // candidates per block
constexpr int kSpecGroups = 128;  // first-level groups of the candidate selection
constexpr int kSpecPer = 4;       // candidates kept per group (512 to merge)
constexpr int64_t kSpecMin = 64;  // no speculation before this many columns

struct ArgMax {
  double v;
  long long pos;
};

__device__ __forceinline__ bool better(double v, long long pos, double bv, long long bpos) {
  // larger value wins; ties (and NaN-free equality) go to the smaller position
  if (v > bv) return true;
  if (v == bv && pos < bpos) return true;
  return false;
}

// partial argmax over positions [m, N) of dwork[perm[pos] - row0] (local entries only)
__global__ __launch_bounds__(256) void k_piv_argmax(const double *__restrict__ dwork,
                                                    const int64_t *__restrict__ perm, int64_t N,
                                                    int64_t m, int64_t row0, int64_t nrows,
                                                    double *__restrict__ pv,
                                                    long long *__restrict__ pp) {
  __shared__ double sv[256];
  __shared__ long long sp[256];
  double bv = -INFINITY;
  long long bp = (long long)N;
  for (int64_t pos = m + (int64_t)blockIdx.x * 256 + threadIdx.x; pos < N;
       pos += (int64_t)gridDim.x * 256) {
    const int64_t g = perm[pos] - row0;
    if (g >= 0 && g < nrows) {
      const double v = dwork[g];
      if (better(v, pos, bv, bp)) {
        bv = v;
        bp = pos;
      }
    }
  }
  sv[threadIdx.x] = bv;
  sp[threadIdx.x] = bp;
  __syncthreads();
  for (int o = 128; o > 0; o >>= 1) {
    if (threadIdx.x < o) {
      if (better(sv[threadIdx.x + o], sp[threadIdx.x + o], sv[threadIdx.x], sp[threadIdx.x])) {
        sv[threadIdx.x] = sv[threadIdx.x + o];
        sp[threadIdx.x] = sp[threadIdx.x + o];
      }
    }
    __syncthreads();
  }
  if (threadIdx.x == 0) {
    pv[blockIdx.x] = sv[0];
    pp[blockIdx.x] = sp[0];
  }
}

// reduce the per-workgroup winners of this rank into rank_win[0..1] (value, pos as double)
__global__ __launch_bounds__(256) void k_piv_rank_winner(const double *__restrict__ pv,
                                                         const long long *__restrict__ pp, int np,
                                                         double *__restrict__ rank_win) {
  __shared__ double sv[256];
  __shared__ long long sp[256];
  double bv = -INFINITY;
  long long bp = LLONG_MAX;
  for (int t = threadIdx.x; t < np; t += 256)
    if (better(pv[t], pp[t], bv, bp)) {
      bv = pv[t];
      bp = pp[t];
    }
  sv[threadIdx.x] = bv;
  sp[threadIdx.x] = bp;
  __syncthreads();
  for (int o = 128; o > 0; o >>= 1) {
    if (threadIdx.x < o)
      if (better(sv[threadIdx.x + o], sp[threadIdx.x + o], sv[threadIdx.x], sp[threadIdx.x])) {
        sv[threadIdx.x] = sv[threadIdx.x + o];
        sp[threadIdx.x] = sp[threadIdx.x + o];
      }
    __syncthreads();
  }
  if (threadIdx.x == 0) {
    rank_win[0] = sv[0];
    rank_win[1] = (double)sp[0];  // exact for positions < 2^53
  }
}

// global winner over ranks; swap; pivot; owner writes Lt[m, m_pi] and the pivot row.
// Single rank (pv != nullptr): the per-workgroup winners pv/pp are reduced here, in the
// same total order as k_piv_rank_winner, so the pivot is the same without that launch.
// xunit != nullptr: sets e_{m_pi} in the padded global layout (matrix-free column fetch).
__global__ __launch_bounds__(256) void k_piv_finalize(const double *__restrict__ wins, int world,
                                                      const double *__restrict__ pv,
                                                      const long long *__restrict__ pp, int np,
                                                      int64_t *__restrict__ perm, int64_t m,
                                                      int64_t row0, int64_t nrows,
                                                      double *__restrict__ Lt, int64_t ldl,
                                                      int *__restrict__ pivflag,
                                                      double *__restrict__ prow,
                                                      double *__restrict__ xunit,
                                                      int64_t rows_per, int64_t blk,
                                                      DevState *st,
                                                      int64_t *__restrict__ iperm,
                                                      const int64_t *__restrict__ Cspec,
                                                      int *__restrict__ spec_hit) {
  __shared__ double sv[256];
  __shared__ long long sp[256];
  __shared__ long long s_mpi;
  __shared__ double s_sq;
  if (pv != nullptr) {  // block-uniform branch
    double bv = -INFINITY;
    long long bp = LLONG_MAX;
    for (int t = threadIdx.x; t < np; t += 256)
      if (better(pv[t], pp[t], bv, bp)) {
        bv = pv[t];
        bp = pp[t];
      }
    sv[threadIdx.x] = bv;
    sp[threadIdx.x] = bp;
    __syncthreads();
    for (int o = 128; o > 0; o >>= 1) {
      if (threadIdx.x < o)
        if (better(sv[threadIdx.x + o], sp[threadIdx.x + o], sv[threadIdx.x], sp[threadIdx.x])) {
          sv[threadIdx.x] = sv[threadIdx.x + o];
          sp[threadIdx.x] = sp[threadIdx.x + o];
        }
      __syncthreads();
    }
  }
  if (threadIdx.x == 0) {
    double bv = -INFINITY;
    long long bp = LLONG_MAX;
    if (pv != nullptr) {
      bv = sv[0];
      bp = sp[0];
    } else {
      for (int r = 0; r < world; ++r) {
        const double v = wins[2 * r];
        const long long p = (long long)wins[2 * r + 1];
        if (better(v, p, bv, bp)) {
          bv = v;
          bp = p;
        }
      }
    }
    long long mpi = -1;
    double sq = 0.0;
    if (bp >= m && bp < (long long)0x7fffffffffffffffLL && bv == bv && bv > -INFINITY) {
      const int64_t tmp = perm[m];
      perm[m] = perm[bp];
      perm[bp] = tmp;
      mpi = perm[m];
      iperm[mpi] = m;
      iperm[tmp] = bp;
      if (!(bv > 0.0)) st->pivot_err = 1;
      sq = sqrt(bv);
    } else {
      st->pivot_err = 1;
    }
    st->m_pi = mpi;
    st->sqrt_piv = sq;
    s_mpi = mpi;
    s_sq = sq;
    if (Cspec != nullptr) {  // speculation: is the pivot row one of the block's candidates?
      const long long gl = mpi - row0;
      int h = -1;
      for (int j = 0; j < kSpecC && mpi >= 0; ++j)
        if (Cspec[j] == gl) {
          h = j;
          break;
        }
      *spec_hit = h;
    }
    if (xunit != nullptr && mpi >= 0) xunit[(mpi / rows_per) * blk + mpi % rows_per] = 1.0;
  }
  __syncthreads();
  const long long mpi = s_mpi;
  const int64_t g = mpi - row0;
  const bool own = (mpi >= 0 && g >= 0 && g < nrows);
  // pivot row L[m_pi, :m] = Lt[:m, m_pi] (zeros on non-owner ranks: summed by allreduce);
  // on one rank (prow == nullptr) the Schur GEMV reads it from Lt itself
  if (prow != nullptr)
    for (int64_t c = threadIdx.x; c < m; c += 256) prow[c] = own ? Lt[c * ldl + g] : 0.0;
  if (threadIdx.x == 0 && own) {
    Lt[m * ldl + g] = s_sq;
    pivflag[g] = 1;
  }
}

// new column of L for every not-yet-pivoted local row i:
//   Lt[m, i] = (S[i, m_pi] - sum_{c<m} Lt[c, i] prow[c]) / sqrt_piv;  dwork[i] -= Lt[m,i]^2
// The sum comes from the split-K column GEMV (part, ksplit slices, row stride ldp);
// S[i, m_pi] from the dense rows (sigma * K[i, pos(m_pi)]) or, for the matrix-free
// operator, from colvec (= S e_{m_pi}, already scaled).
__global__ __launch_bounds__(256) void k_piv_fin(const double *__restrict__ K, int64_t ld,
                                                 double sigma, const double *__restrict__ colvec,
                                                 int64_t rows_per, int64_t blk, int64_t nrows,
                                                 int64_t m, const double *__restrict__ part,
                                                 int ksplit, int64_t ldp,
                                                 double *__restrict__ Lt, int64_t ldl,
                                                 const int *__restrict__ pivflag,
                                                 double *__restrict__ dwork,
                                                 const DevState *__restrict__ st,
                                                 double *__restrict__ xunit,
                                                 const int64_t *__restrict__ iperm,
                                                 int64_t row0, int64_t N,
                                                 double *__restrict__ pv,
                                                 long long *__restrict__ pp,
                                                 const double *__restrict__ Gspec,
                                                 const int *__restrict__ spec_hit) {
  __shared__ double sv[256];
  __shared__ long long sp[256];
  const long long mpi = st->m_pi;
  // speculation hit j: the Schur sum over the columns before the block is row j of Gspec
  const int hitj = spec_hit != nullptr ? *spec_hit : -1;
  const double *grow = hitj >= 0 ? Gspec + (int64_t)hitj * ldl : nullptr;
  if (mpi < 0) {  // no pivot (error already flagged): an empty candidate set
    if (threadIdx.x == 0) {
      pv[blockIdx.x] = -INFINITY;
      pp[blockIdx.x] = (long long)N;
    }
    return;
  }
  const double sq = st->sqrt_piv;
  const int64_t pos = (mpi / rows_per) * blk + (mpi % rows_per);
  // clears e_{m_pi} set by k_piv_finalize (the operator that read it ran before this kernel)
  if (xunit != nullptr && blockIdx.x == 0 && threadIdx.x == 0) xunit[pos] = 0.0;
  double bv = -INFINITY;
  long long bp = (long long)N;
  for (int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x; i < nrows;
       i += (int64_t)gridDim.x * 256) {
    if (pivflag[i]) continue;
    const double col = colvec != nullptr ? colvec[i] : sigma * K[i * ld + pos];
    double s0 = 0.0;  // slice partials in slice order, 8 loads in flight
    int ks = 0;
    for (; ks + 7 < ksplit; ks += 8) {
      double t[8];
#pragma unroll
      for (int u = 0; u < 8; ++u) t[u] = part[(int64_t)(ks + u) * ldp + i];
#pragma unroll
      for (int u = 0; u < 8; ++u) s0 += t[u];
    }
    for (; ks < ksplit; ++ks) s0 += part[(int64_t)ks * ldp + i];
    if (grow != nullptr) s0 += grow[i];
    const double v = (col - s0) / sq;
    Lt[m * ldl + i] = v;
    const double dn = dwork[i] - v * v;
    dwork[i] = dn;
    // the next step's argmax (k_piv_argmax's order: largest value, then smallest position)
    const long long pos_i = (long long)iperm[row0 + i];
    if (better(dn, pos_i, bv, bp)) {
      bv = dn;
      bp = pos_i;
    }
  }
  sv[threadIdx.x] = bv;
  sp[threadIdx.x] = bp;
  __syncthreads();
  for (int o = 128; o > 0; o >>= 1) {
    if (threadIdx.x < o)
      if (better(sv[threadIdx.x + o], sp[threadIdx.x + o], sv[threadIdx.x], sp[threadIdx.x])) {
        sv[threadIdx.x] = sv[threadIdx.x + o];
        sp[threadIdx.x] = sp[threadIdx.x + o];
      }
    __syncthreads();
  }
  if (threadIdx.x == 0) {
    pv[blockIdx.x] = sv[0];
    pp[blockIdx.x] = sp[0];
  }
}

// x[pos(m_pi)] = val: sets (1) and clears (0) the unit vector e_{m_pi} in the padded
// global layout, the operand of the matrix-free column fetch
__global__ void k_unit_pivot(double *__restrict__ x, int64_t rows_per, int64_t blk,
                             const DevState *__restrict__ st, double val) {
  if (threadIdx.x != 0) return;
  const long long mpi = st->m_pi;
  if (mpi >= 0) x[(mpi / rows_per) * blk + mpi % rows_per] = val;
}

// ---------------------------------------------------------------------------
// Speculative blocks (one rank).  The Schur GEMV of step m reads L[:, :m] (m N 8 bytes):
// summed over the build that is k^2 N 4 bytes (2.4 PB at the reference's N = 505050,
// k = 34609).  At the start of a block of kSpecB steps the kSpecC rows with the largest
// residual diagonal are the likely pivots of the block (measured on the golden systems:
// 83-93 % of the block's pivots are among the top 2-4 x block-size candidates); one GEMM
// G = L[C, :m0] L[:, :m0]^T reads L[:, :m0] once for all of them.  A step whose pivot is a
// candidate adds its G row and runs the GEMV over the block's own columns [m0, m) only; any
// other pivot runs the full GEMV.  Exact either way (a different summation order).

// (v, i) before (w, j) in the candidate order: value descending, then row ascending; an
// empty slot (i < 0) after everything
__device__ __forceinline__ bool cand_before(double v, long long i, double w, long long j) {
  if (i < 0) return false;
  if (j < 0) return true;
  return v > w || (v == w && i < j);
}

// best (value, row) over the 256 threads, broadcast to all of them
__device__ __forceinline__ void block_best(double &v, long long &i, double *sv, long long *si) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) {
    const double v2 = __shfl_xor(v, o, 64);
    const long long i2 = __shfl_xor(i, o, 64);
    if (cand_before(v2, i2, v, i)) {
      v = v2;
      i = i2;
    }
  }
  __syncthreads();
  if ((threadIdx.x & 63) == 0) {
    sv[threadIdx.x >> 6] = v;
    si[threadIdx.x >> 6] = i;
  }
  __syncthreads();
  v = sv[0];
  i = si[0];
#pragma unroll
  for (int w = 1; w < 4; ++w)
    if (cand_before(sv[w], si[w], v, i)) {
      v = sv[w];
      i = si[w];
    }
}

// top kSpecPer (value, row) of the non-pivoted rows of a chunk, in order (one workgroup per
// chunk): round r takes the best row after round r - 1's pick
__global__ __launch_bounds__(256) void k_spec_top_part(const double *__restrict__ dwork,
                                                       const int *__restrict__ pivflag,
                                                       int64_t nrows, double *__restrict__ cv,
                                                       long long *__restrict__ ci) {
  __shared__ double sv[4];
  __shared__ long long si[4];
  const int64_t cs = (nrows + gridDim.x - 1) / gridDim.x;
  const int64_t a = (int64_t)blockIdx.x * cs, b = a + cs < nrows ? a + cs : nrows;
  double pv = INFINITY;
  long long pi = -1;
  for (int r = 0; r < kSpecPer; ++r) {
    double bv = -INFINITY;
    long long bi = -1;
    for (int64_t i = a + threadIdx.x; i < b; i += 256) {
      if (pivflag[i]) continue;
      const double v = dwork[i];
      const bool later = pi < 0 || v < pv || (v == pv && i > pi);  // after the last pick
      if (later && cand_before(v, i, bv, bi)) {
        bv = v;
        bi = i;
      }
    }
    block_best(bv, bi, sv, si);
    if (threadIdx.x == 0) {
      cv[(int64_t)blockIdx.x * kSpecPer + r] = bv;
      ci[(int64_t)blockIdx.x * kSpecPer + r] = bi;
    }
    if (bi < 0) {  // chunk exhausted
      for (int r2 = r + 1 + threadIdx.x; r2 < kSpecPer; r2 += 256)
        ci[(int64_t)blockIdx.x * kSpecPer + r2] = -1;
      return;
    }
    pv = bv;
    pi = bi;
  }
}

// the block's candidates C[0..kSpecC): the best of the groups' kSpecGroups x kSpecPer picks in
// candidate order, by rank counting: the (value, row) pairs are distinct rows, so cand_before is
// a strict total order on them and a pair's rank -- how many pairs precede it -- is its position
// in the sorted list; a pair ranked below kSpecC writes C[rank], and workgroup 0 writes -1 to the
// slots past the non-empty count.  kSpecMergeWG workgroups of 64 pairs each (a wave per quarter
// of the pairs they are compared with): the same C as a full sort of the 512 pairs.  Round 5's
// one-workgroup bitonic network took 30 us per speculative block on the nanotube (5 ms of the
// k = 2701 build): 512 x 512 comparisons on one CU are its VALU time, whatever the network
constexpr int kSpecMergeWG = kSpecGroups * kSpecPer / 64;
__global__ __launch_bounds__(256) void k_spec_top_merge(const double *__restrict__ cv,
                                                        const long long *__restrict__ ci,
                                                        int64_t *__restrict__ C) {
  constexpr int n = kSpecGroups * kSpecPer;
  static_assert(n == 512 && n % 64 == 0, "two pairs per thread");
  __shared__ double sv[n];
  __shared__ long long si[n];
  __shared__ int part[4][64];
  __shared__ int s_ne;
  if (threadIdx.x == 0) s_ne = 0;
  // an empty slot (row < 0; its value was never written) as (-inf, max row): after every pair
  long long li[2];
  double lv[2];
#pragma unroll
  for (int h = 0; h < 2; ++h) {
    li[h] = ci[threadIdx.x + 256 * h];
    lv[h] = cv[threadIdx.x + 256 * h];
  }
  __syncthreads();  // s_ne
  int ne = 0;
#pragma unroll
  for (int h = 0; h < 2; ++h) {
    const bool ok = li[h] >= 0;
    sv[threadIdx.x + 256 * h] = ok ? lv[h] : -INFINITY;
    si[threadIdx.x + 256 * h] = ok ? li[h] : LLONG_MAX;
    ne += ok ? 1 : 0;
  }
  if (blockIdx.x == 0 && ne > 0) atomicAdd(&s_ne, ne);  // an integer count: any order
  __syncthreads();
  const int lane = threadIdx.x & 63, q = threadIdx.x >> 6;
  const int e = blockIdx.x * 64 + lane;
  const double v = sv[e];
  const long long i = si[e];
  int r = 0;
#pragma unroll 8
  for (int f = q * (n / 4); f < (q + 1) * (n / 4); ++f) {
    const double w = sv[f];
    const long long j = si[f];
    r += (w > v || (w == v && j < i)) ? 1 : 0;
  }
  part[q][lane] = r;
  __syncthreads();
  if (q == 0) {
    r = (part[0][lane] + part[1][lane]) + (part[2][lane] + part[3][lane]);
    if (i != LLONG_MAX && r < kSpecC) C[r] = i;
    if (blockIdx.x == 0 && lane < kSpecC && lane >= s_ne) C[lane] = -1;
  }
}

// A[c, j] = Lt[c, C_j] for c < m0 (m0 x kSpecC, zero for an empty candidate)
__global__ __launch_bounds__(256) void k_spec_gather(const double *__restrict__ Lt, int64_t ldl,
                                                     int64_t m0, const int64_t *__restrict__ C,
                                                     double *__restrict__ A) {
  const int64_t n = m0 * kSpecC;
  for (int64_t e = (int64_t)blockIdx.x * 256 + threadIdx.x; e < n; e += (int64_t)gridDim.x * 256) {
    const int64_t c = e / kSpecC, j = e % kSpecC;
    const int64_t g = C[j];
    A[e] = g >= 0 ? Lt[c * ldl + g] : 0.0;
  }
}

// ---------------------------------------------------------------------------
// Persistent steps (one rank; round 6).  The launch sequence above spends 4 dependent launches
// per pivot (finalise, column, Schur GEMV, finisher: ~21 us of kernels and ~13 us of launch gaps
// per step on the nanotube).  k_piv_persist runs a whole speculative block of steps
// in one launch: a grid of G resident workgroups (one per CU) synchronised by epoch-tagged
// per-workgroup granules (data as flag, no contended counter), one synchronisation per step on a
// speculation hit and two on a miss.  The arithmetic is the launch sequence's, operation for
// operation (the same column code, the same Schur slices and their summation order, the same
// finisher), so L, the pivots and the residual diagonal are bit-identical
// (tests/test_gpu_pivchol_persist.py).
//   step m: every workgroup reduces the G published (value, position, row) partials of step
//   m - 1 to the same winner; the pivot's row owner swaps perm / iperm, writes sqrt(pivot); on a
//   miss the whole grid runs k_colgemv_part's split-K slices (virtual workgroups) into `part`
//   and synchronises; then each row's thread evaluates its column entry (k_sgdml_col's body, or
//   the dense row), sums the Schur slices in k_piv_fin's order, writes L[m, i] and the residual
//   diagonal, and the workgroup publishes its partial argmax of step m.
struct PersistArgs {
  int64_t N, nrows, blk, rows_per;
  double *Lt;
  double *dwork;
  int *pivflag;
  int64_t *perm, *iperm;
  DevState *st;
  // column source: K != nullptr -> the dense rows; else the sGDML single-column path
  const double *K;
  int64_t ld;
  double sigma;
  const double *Rdd;
  int64_t M;
  int n;
  int64_t D, i0;
  const int32_t *pi, *piinv;
  int n_perms;
  const double *uvk;
  int chunks;   // sGDML: 64-row chunks per query point
  int nrw;      // row waves
  double *part;
  int kmax_split;
  const int64_t *Cspec;
  const double *Gspec;
  int64_t spec_m0;  // -1: no speculative block
  // partials of step m_begin - 1 (npc entries; rows == nullptr: row = position, step 0)
  const double *pv_in;
  const long long *pp_in, *pr_in;
  int npc;
  double *pv_out;  // this launch's last step: G entries
  long long *pp_out, *pr_out;
  unsigned long long *slots;  // G x 4 granules (tag << 32 | payload): value lo, hi, position, row
  unsigned long long *flags;  // G granules: the miss GEMV's arrival
  int64_t m_begin, m_end;
  int mute;  // test hook (MLFF_PIV_MUTE): this workgroup stops publishing after step m_begin
  unsigned long long *trace;  // MLFF_PIV_TRACE: 4 wall-clock stamps per (step, workgroup)
  unsigned long long *step_clock;  // 2 k: workgroup 0's wall clock at each step's start and end
  // the speculative block's candidates: each one's L value of every step (2 x kSpecC x 2
  // granules, by step parity), published by its row's owner; and their columns S e_c
  // (kSpecC x blk, k_sgdml_col before the launch; nullptr: evaluated in the step)
  unsigned long long *cands;
  const double *colbuf;
};

__host__ __device__ inline int ksplit_of(int64_t k, int64_t ncols) {  // choose_ksplit
  const int64_t slabs = (ncols + 511) / 512;
  int64_t sk = (k + 95) / 96;
  const int64_t fill = (256 + slabs - 1) / slabs;
  if (fill > sk) sk = fill;
  const int64_t cap = (k + 15) / 16;
  if (sk > cap) sk = cap;
  if (sk < 1) sk = 1;
  if (sk > 256) sk = 256;
  return (int)sk;
}

typedef double pd2 __attribute__((ext_vector_type(2)));

// colgemv_slice<false> (kernels_vec.hip) with t from LDS: the same fma chains
__device__ __forceinline__ pd2 persist_slice(const pd2 *__restrict__ w2, int64_t ld2, int64_t j0,
                                             int64_t j1, const double *t_sh) {
  pd2 acc0 = {0.0, 0.0}, acc1 = {0.0, 0.0};
  int64_t j = j0;
  for (; j + 7 < j1; j += 8) {
    pd2 a[8];
#pragma unroll
    for (int u = 0; u < 8; ++u) a[u] = w2[(j + u) * ld2];
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
    const pd2 a0 = w2[j * ld2];
    const double t0 = t_sh[j - j0];
    acc0.x = fma(a0.x, t0, acc0.x);
    acc0.y = fma(a0.y, t0, acc0.y);
  }
  return acc0 + acc1;
}

// one column's entry of colgemv_slice over rows [j0, j1) (the .x / .y lane of the same chains)
__device__ __forceinline__ double persist_slice1(const double *__restrict__ Lt, int64_t ldl,
                                                 int64_t i, int64_t j0, int64_t j1,
                                                 const double *t_sh) {
  double acc0 = 0.0, acc1 = 0.0;
  int64_t j = j0;
  for (; j + 7 < j1; j += 8) {
    double a[8];
#pragma unroll
    for (int u = 0; u < 8; ++u) a[u] = Lt[(j + u) * ldl + i];
#pragma unroll
    for (int u = 0; u < 8; u += 2) {
      acc0 = fma(a[u], t_sh[j + u - j0], acc0);
      acc1 = fma(a[u + 1], t_sh[j + u + 1 - j0], acc1);
    }
  }
  for (; j < j1; ++j) acc0 = fma(Lt[j * ldl + i], t_sh[j - j0], acc0);
  return acc0 + acc1;
}

constexpr unsigned long long kPersistTimeout = 100000000ull;  // 1 s of the 100 MHz clock

// thread t < count waits until granules g[t * per .. + per) all carry `tag`; false on timeout
// (every thread returns the same verdict through `bail`)
__device__ __forceinline__ bool persist_wait(unsigned long long *g, int count, int per, unsigned tag,
                                             unsigned long long *vals, int *bail) {
  const int t = threadIdx.x;
  if (t < count) {
    const unsigned long long t0 = wall_clock64();
    for (;;) {
      bool ok = true;
      for (int q = 0; q < per; ++q) {
        vals[q] = __hip_atomic_load(g + (int64_t)t * per + q, __ATOMIC_RELAXED,
                                    __HIP_MEMORY_SCOPE_AGENT);
        // tags only grow within a build: a workgroup already past this point may have
        // published a later one
        ok = ok && (unsigned)(vals[q] >> 32) >= tag;
      }
      if (ok) break;
      if ((unsigned long long)(wall_clock64() - t0) > kPersistTimeout) {
        *bail = 1;
        break;
      }
      __builtin_amdgcn_s_sleep(1);
    }
  }
  __syncthreads();
  const bool ok = *bail == 0;
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");
  return ok;
}

__device__ __forceinline__ void persist_publish(unsigned long long *g, int per, unsigned tag,
                                                const unsigned *payload) {
  for (int q = 0; q < per; ++q)
    __hip_atomic_store(g + q, ((unsigned long long)tag << 32) | payload[q], __ATOMIC_RELAXED,
                       __HIP_MEMORY_SCOPE_AGENT);
}

// argmax over the workgroup of (value, position, row, source) under better()'s strict total order
// (so every workgroup reducing the same candidates picks the same one); result in every thread
__device__ __forceinline__ void wg_argmax(double &v, long long &p, long long &r, int &src,
                                          double *sv, long long *sp, long long *sr, int *ss) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) {
    const double v2 = __shfl_xor(v, o, 64);
    const long long p2 = __shfl_xor(p, o, 64), r2 = __shfl_xor(r, o, 64);
    const int s2 = __shfl_xor(src, o, 64);
    if (better(v2, p2, v, p)) {
      v = v2;
      p = p2;
      r = r2;
      src = s2;
    }
  }
  const int w = threadIdx.x >> 6;
  __syncthreads();
  if ((threadIdx.x & 63) == 0) {
    sv[w] = v;
    sp[w] = p;
    sr[w] = r;
    ss[w] = src;
  }
  __syncthreads();
  v = sv[0];
  p = sp[0];
  r = sr[0];
  src = ss[0];
#pragma unroll
  for (int q = 1; q < 4; ++q)
    if (better(sv[q], sp[q], v, p)) {
      v = sv[q];
      p = sp[q];
      r = sr[q];
      src = ss[q];
    }
}

constexpr int kSlot = 4;  // granules per workgroup slot: value lo / hi, position, row

template <bool SG>
__global__ __launch_bounds__(256) void k_piv_persist(PersistArgs a) {
  extern __shared__ double t_sh[];  // the pivot row L[c, m_pi] over the step's Schur range
  __shared__ double sv[4];
  __shared__ long long sp[4], sr[4];
  __shared__ int ss[4];
  __shared__ long long s_C[kSpecC];
  __shared__ double s_ch[kSpecC][kSpecB];  // the candidates' L values over the block's steps
  __shared__ unsigned long long s_pg[4 * 256 + 2 * kSpecC];  // one poll round's granules
  __shared__ int s_bail;
  const int G = (int)gridDim.x, wg = (int)blockIdx.x, tid = threadIdx.x;
  const int lane = tid & 63, w = tid >> 6;
  if (tid == 0) s_bail = 0;
  if (a.st->pivot_err == 2) return;  // an earlier launch of this build timed out: host falls back
  const bool spec = a.spec_m0 >= 0;
  if (spec && tid < kSpecC) s_C[tid] = a.Cspec[tid];
  const int64_t ldl = a.blk;
  // ---- this thread's row (one row wave per wave: nrw <= 4 G) and its state in registers
  const int r = wg + G * w;
  int64_t i = -1;
  bool act = false;
  if (r < a.nrw) {
    if (SG) {
      const int n3 = 3 * a.n, t = (r % a.chunks) * kColRows + lane;
      i = (int64_t)(r / a.chunks) * n3 + t;
      act = t < n3 && i < a.nrows;
    } else {
      i = (int64_t)r * 64 + lane;
      act = i < a.nrows;
    }
  }
  bool piv = true;
  double dw = 0.0;
  long long ip = 0;
  if (act) {
    piv = a.pivflag[i] != 0;
    dw = a.dwork[i];
    ip = a.iperm[i];
  }
  double seg[kSpecB];  // L[spec_m0 + u, i] of this block's steps
#pragma unroll
  for (int u = 0; u < kSpecB; ++u) seg[u] = 0.0;
  __syncthreads();
  int cidx = -1;  // this row's index among the block's candidates
  if (spec && act)
    for (int c = 0; c < kSpecC; ++c)
      if (s_C[c] == i) cidx = c;
  long long mpi = -1;
  double sq = 0.0;
  for (int64_t m = a.m_begin; m < a.m_end; ++m) {
    const int S = spec ? (int)(m - a.spec_m0) : 0;  // segment length of the step-(m - 1) slots
    if (wg == 0 && tid == 0) a.step_clock[2 * m] = wall_clock64();
    // ---- the winner of step m from the partials of step m - 1
    double bv = -INFINITY;
    long long bp = LLONG_MAX, br = -1;
    int src = -1;
    if (m == a.m_begin) {
      for (int t = tid; t < a.npc; t += 256)
        if (better(a.pv_in[t], a.pp_in[t], bv, bp)) {
          bv = a.pv_in[t];
          bp = a.pp_in[t];
          br = a.pr_in != nullptr ? a.pr_in[t] : bp;
        }
    } else {
      // one round trip: the G slot headers of step m - 1 and the candidates' L values of that
      // step; thread t polls granules t, t + 256, ... (a workgroup one step ahead writes the
      // other buffer of each pair)
      const unsigned tag = (unsigned)m;
      const int nh = 4 * G, ne = nh + (spec ? 2 * kSpecC : 0);
      unsigned long long *gh = a.slots + (int64_t)(m & 1) * G * kSlot;
      unsigned long long *gc = a.cands + (int64_t)(m & 1) * 2 * kSpecC;
      const unsigned long long t0 = wall_clock64();
      for (int e = tid; e < ne; e += 256) {
        unsigned long long *ge = e < nh ? gh + e : gc + (e - nh);
        unsigned long long v = 0;
        if (e < nh || s_C[(e - nh) >> 1] >= 0)  // (an empty candidate publishes nothing)
          for (;;) {
            v = __hip_atomic_load(ge, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            if ((unsigned)(v >> 32) == tag) break;
            if ((unsigned long long)(wall_clock64() - t0) > kPersistTimeout) {
              s_bail = 1;
              break;
            }
            __builtin_amdgcn_s_sleep(2);
          }
        s_pg[e] = v;
      }
      __syncthreads();
      if (tid < G) {
        unsigned long long g[4];
#pragma unroll
        for (int q = 0; q < 4; ++q) g[q] = s_pg[4 * tid + q];
        bv = __builtin_bit_cast(double, (g[1] << 32) | (g[0] & 0xffffffffull));
        bp = (long long)(unsigned)(g[2] & 0xffffffffull);
        br = (long long)(int)(unsigned)(g[3] & 0xffffffffull);
        if (br < 0) bp = LLONG_MAX;  // an empty partial
        src = tid;
      }
      if (spec && tid < kSpecC && S > 0)
        s_ch[tid][S - 1] = __builtin_bit_cast(double, (s_pg[nh + 2 * tid + 1] << 32) |
                                                          (s_pg[nh + 2 * tid] & 0xffffffffull));
    }
    wg_argmax(bv, bp, br, src, sv, sp, sr, ss);
    if (s_bail) goto fault;
    const bool valid = bp >= m && bp < (long long)a.N && bv == bv && bv > -INFINITY && br >= 0;
    mpi = valid ? br : -1;
    sq = valid ? sqrt(bv) : 0.0;
    if (wg == 0 && tid == 0 && (!valid || !(bv > 0.0))) a.st->pivot_err = 1;
    int hit = -1;
    if (spec && mpi >= 0)
      for (int j = 0; j < kSpecC; ++j)
        if (s_C[j] == mpi) {
          hit = j;
          break;
        }
    const int ks = m > 0 ? min(a.kmax_split, ksplit_of(m, a.blk)) : 0;
    const int64_t kslice = ks > 0 ? (m + ks - 1) / ks : 1;
    if (hit >= 0) {
      // the pivot row over [spec_m0, m) is the winning candidate's history (s_ch)
    } else if (mpi >= 0 && ks > 0) {
      // a miss: every L row so far is written back and visible (fenced arrival), the whole
      // pivot row is staged, and the grid runs k_colgemv_part's split-K slices over [0, m)
      __builtin_amdgcn_fence(__ATOMIC_RELEASE, "agent");
      __syncthreads();
      if (tid == 0) {
        const unsigned zero = 0;
        persist_publish(a.flags + wg, 1, (unsigned)(2 * m + 1), &zero);
      }
      unsigned long long g1[1];
      if (!persist_wait(a.flags, G, 1, (unsigned)(2 * m + 1), g1, &s_bail)) goto fault;
      for (int64_t c = tid; c < m; c += 256) t_sh[c] = a.Lt[c * ldl + mpi];
      __syncthreads();
      const int64_t nbx = (a.blk / 2 + 255) / 256, nvb = nbx * ks, ld2 = a.blk / 2;
      for (int64_t vb = wg; vb < nvb; vb += G) {
        const int64_t bx = vb % nbx, by = vb / nbx;
        const int64_t j0 = by * kslice, j1 = j0 + kslice < m ? j0 + kslice : m;
        const int64_t c2 = bx * 256 + tid;
        if (2 * c2 < a.blk) {
          pd2 acc = {0.0, 0.0};
          if (j0 < j1)
            acc = persist_slice(reinterpret_cast<const pd2 *>(a.Lt) + c2, ld2, j0, j1, t_sh + j0);
          reinterpret_cast<pd2 *>(a.part + by * a.blk)[c2] = acc;
        }
      }
      __builtin_amdgcn_fence(__ATOMIC_RELEASE, "agent");
      __syncthreads();
      if (tid == 0) {
        const unsigned zero = 0;
        persist_publish(a.flags + wg, 1, (unsigned)(2 * m + 2), &zero);
      }
      if (!persist_wait(a.flags, G, 1, (unsigned)(2 * m + 2), g1, &s_bail)) goto fault;
    }
    if (a.trace != nullptr && tid == 0) a.trace[(m * G + wg) * 4 + 1] = wall_clock64();
    // ---- rows: column entry, Schur sum, L[m, i], residual diagonal, partial argmax
    {
      double col = 0.0;
      if (SG && hit >= 0 && a.colbuf != nullptr) {  // the candidate's column, evaluated before
        if (act) col = a.colbuf[(int64_t)hit * ldl + i];
      } else if (SG) {
        if (r < a.nrw && mpi >= 0) {  // wave-uniform: the column code is a wave sum
          bool a2;
          int64_t i2;
          col = a.sigma * sgdml_col_acc(a.Rdd, a.M, a.n, a.D, a.i0, a.pi, a.piinv, a.n_perms,
                                        a.uvk, 0, a.nrows, mpi, r / a.chunks,
                                        (r % a.chunks) * kColRows, lane, a2, i2);
        }
      } else if (act && mpi >= 0) {
        const int64_t pos = (mpi / a.rows_per) * a.blk + (mpi % a.rows_per);
        col = a.sigma * a.K[i * a.ld + pos];
      }
      double cbv = -INFINITY;
      long long cbp = (long long)a.N, cbr = -1;
      double lval = 0.0;  // this row's L[m, i] (0 for a row pivoted before: never written)
      if (act && mpi >= 0) {
        const int u_m = S;  // this step's index in the segment
        // (perm, the inverse of iperm, is written once after the build: two rows' owners on
        // different XCDs would write the same perm entry at different steps, and without a
        // fence on a hit step nothing orders the two write-backs)
        if (i == mpi) {  // k_piv_finalize's writes for the pivot row
          a.Lt[m * ldl + i] = sq;
          lval = sq;
          piv = true;
          ip = m;
        } else if (!piv) {
          if (ip == m) ip = bp;  // the row the swap moves from position m to bp
          double s0 = 0.0;
          if (hit >= 0) {  // the slices' sums from spec_m0 on (registers), in slice order
            const int64_t z0 = a.spec_m0 / kslice, z1 = (m - 1) / kslice;
            for (int64_t z = z0; z <= z1 && m > a.spec_m0; ++z) {
              const int64_t j0 = z * kslice > a.spec_m0 ? z * kslice : a.spec_m0;
              const int64_t j1 = (z + 1) * kslice < m ? (z + 1) * kslice : m;
              if (j0 >= j1) continue;
              const int64_t full = ((j1 - j0) / 8) * 8;
              double acc0 = 0.0, acc1 = 0.0;
#pragma unroll
              for (int u = 0; u < kSpecB; ++u) {
                const int64_t j = a.spec_m0 + u;
                if (j >= j0 && j < j1) {
                  const int64_t o = j - j0;
                  if (o < full && (o & 1))
                    acc1 = fma(seg[u], s_ch[hit][u], acc1);
                  else
                    acc0 = fma(seg[u], s_ch[hit][u], acc0);
                }
              }
              s0 += acc0 + acc1;
            }
            s0 += a.Gspec[(int64_t)hit * ldl + i];
          } else {
            int z = 0;
            for (; z + 7 < ks; z += 8) {
              double t[8];
#pragma unroll
              for (int u = 0; u < 8; ++u) t[u] = a.part[(int64_t)(z + u) * a.blk + i];
#pragma unroll
              for (int u = 0; u < 8; ++u) s0 += t[u];
            }
            for (; z < ks; ++z) s0 += a.part[(int64_t)z * a.blk + i];
          }
          const double v = (col - s0) / sq;
          a.Lt[m * ldl + i] = v;
          lval = v;
          dw = dw - v * v;
#pragma unroll
          for (int u = 0; u < kSpecB; ++u)
            if (u == u_m) seg[u] = v;
          if (better(dw, ip, cbv, cbp)) {
            cbv = dw;
            cbp = ip;
            cbr = i;
          }
        }
      }
      if (a.trace != nullptr && lane == 0)
        atomicMax(&a.trace[(m * G + wg) * 4 + 2], (unsigned long long)wall_clock64());
      int csrc = tid;
      wg_argmax(cbv, cbp, cbr, csrc, sv, sp, sr, ss);
      // the workgroup's partial of step m, and (candidate rows) their L[m, i]
      if (m + 1 < a.m_end) {
        const unsigned tag = (unsigned)m + 1;
        if (cidx >= 0) {
          const unsigned long long b = __builtin_bit_cast(unsigned long long, lval);
          const unsigned pl[2] = {(unsigned)(b & 0xffffffffull), (unsigned)(b >> 32)};
          persist_publish(a.cands + ((int64_t)((m + 1) & 1) * kSpecC + cidx) * 2, 2, tag, pl);
        }
        const bool mine = cbr >= 0 ? tid == csrc : tid == 0;
        if (mine && !(wg == a.mute && m > a.m_begin)) {
          unsigned long long *gs = a.slots + ((int64_t)((m + 1) & 1) * G + wg) * kSlot;
          const unsigned long long vb = __builtin_bit_cast(unsigned long long, cbv);
          const unsigned pl[4] = {(unsigned)(vb & 0xffffffffull), (unsigned)(vb >> 32),
                                  (unsigned)(cbr >= 0 ? cbp : 0), (unsigned)(int)cbr};
          persist_publish(gs, 4, tag, pl);
          if (a.trace != nullptr) a.trace[(m * G + wg) * 4 + 3] = wall_clock64();
        }
      } else if (tid == 0) {
        a.pv_out[wg] = cbv;
        a.pp_out[wg] = cbr >= 0 ? cbp : (long long)a.N;
        a.pr_out[wg] = cbr;
      }
    }
    if (a.trace != nullptr && tid == 0 && m + 1 < a.m_end)
      a.trace[((m + 1) * G + wg) * 4 + 0] = wall_clock64();
    if (wg == 0 && tid == 0) a.step_clock[2 * m + 1] = wall_clock64();
  }
  if (act) {  // the row state back for the next launch / the speculation kernels
    a.pivflag[i] = piv ? 1 : 0;
    a.dwork[i] = dw;
    a.iperm[i] = ip;
  }
  if (wg == 0 && tid == 0) {
    a.st->m_pi = mpi;
    a.st->sqrt_piv = sq;
  }
  return;
fault:
  if (tid == 0) a.st->pivot_err = 2;
}

// perm[iperm[i]] = i (the persistent form keeps only the row -> position map)
__global__ __launch_bounds__(256) void k_perm_from_iperm(const int64_t *__restrict__ iperm, int64_t n,
                                                         int64_t *__restrict__ perm) {
  for (int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x; i < n; i += (int64_t)gridDim.x * 256)
    perm[iperm[i]] = i;
}

// the persistent form applies: one rank, the dense rows or the sGDML single-column path, a panel
// short enough for its pivot row to sit in LDS, and MLFF_PIVCHOL_PERSIST not 0
static bool persist_grid(int64_t k, int64_t nrw, int *G_out) {
  const char *e0 = std::getenv("MLFF_PIVCHOL_PERSIST");  // read per build: 0 = launch sequence
  if ((e0 != nullptr && std::atoi(e0) == 0) || k > 12288) return false;
  int dev = 0, cus = 0;
  if (hipGetDevice(&dev) != hipSuccess) return false;
  hipDeviceProp_t prop;
  if (hipGetDeviceProperties(&prop, dev) != hipSuccess) return false;
  cus = prop.multiProcessorCount;
  int per = 0;
  const size_t shm = sizeof(double) * (size_t)std::max<int64_t>(k, 8);
  if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&per, reinterpret_cast<const void *>(k_piv_persist<true>),
                                                   256, shm) != hipSuccess || per < 1)
    return false;
  // every row wave is one wave of the grid (its rows' state lives in registers): G >= nrw / 4;
  // all of the grid resident at once (one workgroup per CU)
  const int64_t need = (nrw + 3) / 4, cap = std::min<int64_t>(256, cus);
  if (need > cap) return false;
  // fewer workgroups poll faster (configs[1], 63 needed: 64 / 128 / 256 -> 15.8 / 16.5 / 17.8 us
  // per step, profiles/r06/pivchol/)
  int64_t G = std::max<int64_t>(need, std::min<int64_t>(cap, 64));
  if (const char *e = std::getenv("MLFF_PIV_G")) G = std::max<int64_t>(need, std::min<int64_t>(cap, std::atoi(e)));
  *G_out = (int)G;
  return true;
}

int pivoted_cholesky(mlff_ctx *ctx, int64_t k, int64_t *index_columns_out) {
  hipStream_t s = ctx->stream;
  const int64_t N = ctx->N, nrows = ctx->nrows, blk = ctx->blk;
  const int np = (int)std::min<int64_t>(256, std::max<int64_t>(1, (N + 1023) / 1024));
  const unsigned gcol = (unsigned)std::min<int64_t>((nrows + 255) / 256, 1024);
  ScratchScope scope(ctx);
  double *pv = nullptr, *wins = nullptr;
  long long *pp = nullptr;
  int64_t *iperm = nullptr;
  const int npart = std::max<int>(np, (int)gcol);
  MLFF_TRY(scratch_alloc(ctx, &pv, npart));
  MLFF_TRY(scratch_alloc(ctx, &pp, npart));
  MLFF_TRY(scratch_alloc(ctx, &wins, 2 * ctx->world));
  MLFF_TRY(scratch_alloc(ctx, &iperm, N));
  // init: perm = iperm = arange(N), dwork = diag(S), pivflag = 0, Lt = 0
  std::vector<int64_t> hperm(N);
  for (int64_t i = 0; i < N; ++i) hperm[i] = i;
  MLFF_HIP(ctx, hipMemcpyAsync(ctx->perm, hperm.data(), sizeof(int64_t) * N, hipMemcpyHostToDevice, s));
  MLFF_HIP(ctx, hipMemcpyAsync(iperm, hperm.data(), sizeof(int64_t) * N, hipMemcpyHostToDevice, s));
  // column sources: the dense rows; the RBF points (k_rbf_cols); the matrix-free sGDML
  // operator -- its single-column path (one training point's pair records, k_sgdml_col)
  // when the table exists, else K_op e_{m_pi} through the whole operator
  const bool rbfcols = !ctx->has_matrix && ctx->rbf.ready;
  const bool mfcols = !ctx->has_matrix && !rbfcols;
  const bool colpath = rbfcols || (mfcols && (ctx->mf.uvk != nullptr || ctx->nrows == 0));
  double *colbuf = nullptr, *part = nullptr;
  if (!ctx->has_matrix) {
    MLFF_TRY(operator_diag(ctx, ctx->dwork));
    MLFF_TRY(scratch_alloc(ctx, &colbuf, blk));
    MLFF_HIP(ctx, hipMemsetAsync(ctx->xg, 0, sizeof(double) * ctx->ld, s));
  } else {
    launch_diag_of(ctx->K, ctx->ld, nrows, ctx->row0, ctx->rows_per, blk, ctx->sigma_K, ctx->dwork, s);
  }
  const int kmax_split = choose_ksplit(k, blk);
  MLFF_TRY(scratch_alloc(ctx, &part, kmax_split * blk));
  // speculative blocks (one rank; MLFF_PIVCHOL_SPEC=0 disables for A/B)
  static const bool spec_env = [] {
    const char *e = std::getenv("MLFF_PIVCHOL_SPEC");
    return e == nullptr || e[0] != '0';
  }();
  const bool spec = spec_env && ctx->world == 1 && k > kSpecMin + kSpecB &&
                    nrows > (int64_t)kSpecGroups * kSpecPer;
  double *Gspec = nullptr, *Aspec = nullptr, *cv = nullptr;
  long long *ci = nullptr;
  int64_t *Cspec = nullptr;
  int *hit = nullptr;
  if (spec) {
    MLFF_TRY(scratch_alloc(ctx, &Gspec, (size_t)kSpecC * blk));
    MLFF_TRY(scratch_alloc(ctx, &Aspec, (size_t)k * kSpecC));
    MLFF_TRY(scratch_alloc(ctx, &cv, (size_t)kSpecGroups * kSpecPer));
    MLFF_TRY(scratch_alloc(ctx, &ci, (size_t)kSpecGroups * kSpecPer));
    MLFF_TRY(scratch_alloc(ctx, &Cspec, (size_t)kSpecC));
    MLFF_TRY(scratch_alloc(ctx, &hit, 1));
  }
  int64_t spec_m0 = -1;  // start of the current speculative block (-1: none)
  MLFF_HIP(ctx, hipMemsetAsync(ctx->pivflag, 0, sizeof(int) * blk, s));
  MLFF_HIP(ctx, hipMemsetAsync(ctx->T, 0, sizeof(double) * round_up(k, 8) * blk, s));
  MLFF_HIP(ctx, hipMemsetAsync(&ctx->st->pivot_err, 0, sizeof(int), s));
  // per-column build times (incomplete_cholesky.py:48-80 records time_cholesky[m] for every
  // column; tools/create_data.py:117-148 compares the first 20 with the rest): a device
  // event every kStampEvery columns, the segment's time split evenly over its columns
  constexpr int64_t kStampEvery = 4;
  std::vector<hipEvent_t> stamps;
  stamps.reserve((size_t)(k / kStampEvery + 2));
  auto stamp = [&]() {
    hipEvent_t e = nullptr;
    if (hipEventCreateWithFlags(&e, timing_event_flags()) == hipSuccess) {
      hipEventRecord(e, s);
      stamps.push_back(e);
    }
  };
  std::vector<int64_t> stamp_col;  // the column each stamp precedes
  stamp_col.reserve(stamps.capacity());
  auto stamp_at = [&](int64_t m) {
    stamp();
    if (stamp_col.size() < stamps.size()) stamp_col.push_back(m);
  };
  // the persistent form (k_piv_persist): one launch per speculative block
  unsigned long long *step_clock = nullptr;  // its per-step clocks (split each launch's time)
  int Gp = 0;
  int64_t nrw = (nrows + 63) / 64;  // row waves: 64 dense rows, or 64 rows of a query point
  if (!ctx->has_matrix && mfcols && ctx->mf.uvk != nullptr) {
    const int64_t n3 = 3 * (int64_t)ctx->mf.n;
    nrw = ((nrows + n3 - 1) / n3) * ((n3 + kColRows - 1) / kColRows);  // one rank: row0 = 0
  }
  const bool persist = ctx->world == 1 && nrows > 0 && !rbfcols && !ctx->piv_persist_off &&
                       (ctx->has_matrix || (mfcols && ctx->mf.uvk != nullptr)) &&
                       persist_grid(k, nrw, &Gp);
  if (persist) {
    const bool sg = !ctx->has_matrix;
    const MfData &mf = ctx->mf;
    long long *pr = nullptr;
    double *pv2 = nullptr;
    long long *pp2 = nullptr, *pr2 = nullptr;
    unsigned long long *slots = nullptr, *flags = nullptr;
    MLFF_TRY(scratch_alloc(ctx, &pr, npart));
    MLFF_TRY(scratch_alloc(ctx, &pv2, std::max(npart, Gp)));
    MLFF_TRY(scratch_alloc(ctx, &pp2, std::max(npart, Gp)));
    MLFF_TRY(scratch_alloc(ctx, &pr2, std::max(npart, Gp)));
    MLFF_TRY(scratch_alloc(ctx, &slots, (size_t)2 * Gp * kSlot));
    MLFF_TRY(scratch_alloc(ctx, &flags, (size_t)Gp));
    unsigned long long *cands = nullptr;
    MLFF_TRY(scratch_alloc(ctx, &cands, (size_t)2 * 2 * kSpecC));
    MLFF_HIP(ctx, hipMemsetAsync(cands, 0, sizeof(unsigned long long) * 2 * 2 * kSpecC, s));
    double *colbuf = nullptr;  // the candidates' columns (sGDML path, speculative blocks)
    if (sg && spec) MLFF_TRY(scratch_alloc(ctx, &colbuf, (size_t)kSpecC * blk));
    MLFF_HIP(ctx, hipMemsetAsync(slots, 0, sizeof(unsigned long long) * 2 * Gp * kSlot, s));
    MLFF_HIP(ctx, hipMemsetAsync(flags, 0, sizeof(unsigned long long) * Gp, s));
    if (npart < Gp) {  // the partial buffers hold G entries
      MLFF_TRY(scratch_alloc(ctx, &pv, Gp));
      MLFF_TRY(scratch_alloc(ctx, &pp, Gp));
      MLFF_TRY(scratch_alloc(ctx, &pr, Gp));
    }
    PersistArgs pa{};
    pa.N = N;
    pa.nrows = nrows;
    pa.blk = blk;
    pa.rows_per = ctx->rows_per;
    pa.Lt = ctx->T;
    pa.dwork = ctx->dwork;
    pa.pivflag = ctx->pivflag;
    pa.perm = ctx->perm;
    pa.iperm = iperm;
    pa.st = ctx->st;
    pa.K = sg ? nullptr : ctx->K;
    pa.ld = ctx->ld;
    pa.sigma = ctx->sigma_K;
    if (sg) {
      pa.Rdd = mf.Rdd;
      pa.M = mf.M;
      pa.n = mf.n;
      pa.D = mf.D;
      pa.i0 = mf.i0;
      pa.pi = mf.pi_d;
      pa.piinv = mf.piinv_d;
      pa.n_perms = mf.n_perms;
      pa.uvk = mf.uvk;
      pa.chunks = (3 * mf.n + kColRows - 1) / kColRows;
    }
    pa.nrw = (int)nrw;
    pa.part = part;
    pa.kmax_split = kmax_split;
    pa.Cspec = Cspec;
    pa.Gspec = Gspec;
    pa.cands = cands;
    pa.colbuf = nullptr;
    pa.mute = -1;
    pa.trace = nullptr;
    MLFF_TRY(scratch_alloc(ctx, &pa.step_clock, (size_t)2 * k));
    MLFF_HIP(ctx, hipMemsetAsync(pa.step_clock, 0, sizeof(unsigned long long) * 2 * k, s));
    step_clock = pa.step_clock;
    const bool want_trace = std::getenv("MLFF_PIV_TRACE") != nullptr;
    if (want_trace) {
      MLFF_TRY(scratch_alloc(ctx, &pa.trace, (size_t)k * Gp * 4));
      MLFF_HIP(ctx, hipMemsetAsync(pa.trace, 0, sizeof(unsigned long long) * k * Gp * 4, s));
    }
    if (const char *e = std::getenv("MLFF_PIV_MUTE")) pa.mute = std::atoi(e);
    const size_t shm = sizeof(double) * (size_t)std::max<int64_t>(k, 8);
    hipLaunchKernelGGL(k_piv_argmax, dim3(np), dim3(256), 0, s, ctx->dwork, ctx->perm, N, (int64_t)0,
                       ctx->row0, nrows, pv, pp);
    const double *pin = pv;
    const long long *ppin = pp, *prin = nullptr;
    int npc = np;
    bool flip = false;
    stamp_at(0);
    for (int64_t m = 0; m < k;) {
      int64_t m_end = k;
      pa.spec_m0 = -1;
      if (spec) {
        if (m < kSpecMin) {
          m_end = std::min<int64_t>(k, kSpecMin);
          pa.colbuf = nullptr;
        } else {
          hipLaunchKernelGGL(k_spec_top_part, dim3(kSpecGroups), dim3(256), 0, s, ctx->dwork,
                             ctx->pivflag, nrows, cv, ci);
          hipLaunchKernelGGL(k_spec_top_merge, dim3(kSpecMergeWG), dim3(256), 0, s, (const double *)cv,
                             (const long long *)ci, Cspec);
          hipLaunchKernelGGL(k_spec_gather, dim3((unsigned)std::min<int64_t>((m * kSpecC + 255) / 256, 4096)),
                             dim3(256), 0, s, ctx->T, blk, m, Cspec, Aspec);
          MLFF_TRY(gemm_splitk(ctx, true, false, kSpecC, blk, m, Aspec, kSpecC, ctx->T, blk, Gspec, blk));
          if (colbuf != nullptr) {  // the candidates' columns, the steps' hits read them
            launch_sgdml_columns(mf.Rdd, mf.M, mf.n, mf.D, mf.i0, mf.pi_d, mf.piinv_d, mf.n_perms,
                                 mf.uvk, ctx->row0, nrows, Cspec, kSpecC, ctx->st, ctx->sigma_K,
                                 colbuf, blk, s);
            pa.colbuf = colbuf;
          }
          pa.spec_m0 = m;
          m_end = std::min<int64_t>(k, m + kSpecB);
        }
      }
      pa.pv_in = pin;
      pa.pp_in = ppin;
      pa.pr_in = prin;
      pa.npc = npc;
      pa.pv_out = flip ? pv : pv2;
      pa.pp_out = flip ? pp : pp2;
      pa.pr_out = flip ? pr : pr2;
      pa.slots = slots;
      pa.flags = flags;
      pa.m_begin = m;
      pa.m_end = m_end;
      if (sg)
        hipLaunchKernelGGL(k_piv_persist<true>, dim3((unsigned)Gp), dim3(256), shm, s, pa);
      else
        hipLaunchKernelGGL(k_piv_persist<false>, dim3((unsigned)Gp), dim3(256), shm, s, pa);
      MLFF_HIP(ctx, hipGetLastError());
      pin = pa.pv_out;
      ppin = pa.pp_out;
      prin = pa.pr_out;
      npc = Gp;
      flip = !flip;
      m = m_end;
      stamp_at(m);
    }
    hipLaunchKernelGGL(k_perm_from_iperm, dim3((unsigned)std::min<int64_t>((N + 255) / 256, 1024)),
                       dim3(256), 0, s, (const int64_t *)iperm, N, ctx->perm);
    if (want_trace) {  // per step: the medians over workgroups of each phase, and the step time
      std::vector<unsigned long long> tr((size_t)k * Gp * 4);
      MLFF_HIP(ctx, hipMemcpyAsync(tr.data(), pa.trace, sizeof(unsigned long long) * tr.size(),
                                   hipMemcpyDeviceToHost, s));
      MLFF_HIP(ctx, hipStreamSynchronize(s));
      double acc[4] = {0, 0, 0, 0};
      double slow_sum = 0.0, fast_sum = 0.0;  // steps with / without a grid-wide Schur GEMV
      int64_t cnt = 0, slow = 0;
      for (int64_t m = 1; m + 1 < k; ++m) {
        const unsigned long long *a0 = &tr[(size_t)m * Gp * 4], *a1 = &tr[(size_t)(m + 1) * Gp * 4];
        if (a0[0] == 0 || a1[0] == 0 || a0[3] == 0) continue;  // launch boundaries
        std::vector<double> ph[4];
        for (int g = 0; g < Gp; ++g) {
          const unsigned long long *e = a0 + 4 * g, *f = a1 + 4 * g;
          ph[0].push_back(10.0 * (double)(e[1] - e[0]));
          ph[1].push_back(e[2] > e[1] ? 10.0 * (double)(e[2] - e[1]) : 0.0);
          ph[2].push_back(10.0 * (double)(e[3] - (e[2] > e[1] ? e[2] : e[1])));
          ph[3].push_back(10.0 * (double)(f[0] - e[0]));
        }
        for (int q = 0; q < 4; ++q) {
          std::nth_element(ph[q].begin(), ph[q].begin() + Gp / 2, ph[q].end());
          acc[q] += ph[q][Gp / 2];
        }
        if (ph[0][Gp / 2] > 20000.0) {
          ++slow;
          slow_sum += ph[3][Gp / 2];
        } else {
          fast_sum += ph[3][Gp / 2];
        }
        ++cnt;
      }
      if (cnt > 0)
        std::fprintf(stderr, "[piv trace] G=%d steps=%lld median ns: winner+stage+miss %.0f, rows %.0f, "
                     "publish %.0f, step %.0f\n", Gp, (long long)cnt, acc[0] / cnt, acc[1] / cnt,
                     acc[2] / cnt, acc[3] / cnt);
      if (cnt > 0)
        std::fprintf(stderr, "[piv trace] %lld steps > 20 us before the rows (misses): %.2f ms; "
                     "the other %lld: %.2f ms\n", (long long)slow, 1e-6 * slow_sum,
                     (long long)(cnt - slow), 1e-6 * fast_sum);
    }
  } else {
  stamp_at(0);
  for (int64_t m = 0; m < k; ++m) {
    if (m > 0 && m % kStampEvery == 0) stamp_at(m);
    // candidates of step m: a scan of the positions [m, N) at m = 0 (and on a rank without
    // rows), afterwards the per-workgroup winners k_piv_fin left from step m - 1
    int npc = (int)gcol;
    if (m == 0 || gcol == 0) {
      hipLaunchKernelGGL(k_piv_argmax, dim3(np), dim3(256), 0, s, ctx->dwork, ctx->perm, N, m,
                         ctx->row0, nrows, pv, pp);
      npc = np;
    }
    if (spec && m >= kSpecMin && m % kSpecB == 0) {
      // a new block: candidates from the residual diagonal after step m - 1, and the
      // Schur sums of all of them over the columns [0, m) in one GEMM
      spec_m0 = m;
      hipLaunchKernelGGL(k_spec_top_part, dim3(kSpecGroups), dim3(256), 0, s, ctx->dwork,
                         ctx->pivflag, nrows, cv, ci);
      hipLaunchKernelGGL(k_spec_top_merge, dim3(kSpecMergeWG), dim3(256), 0, s, (const double *)cv,
                         (const long long *)ci, Cspec);
      hipLaunchKernelGGL(k_spec_gather, dim3((unsigned)std::min<int64_t>((m * kSpecC + 255) / 256, 4096)),
                         dim3(256), 0, s, ctx->T, blk, m, Cspec, Aspec);
      MLFF_TRY(gemm_splitk(ctx, true, false, kSpecC, blk, m, Aspec, kSpecC, ctx->T, blk, Gspec, blk));
    }
    const bool multi = ctx->world > 1;
    if (multi) {
      double *my = wins + 2 * ctx->rank;
      hipLaunchKernelGGL(k_piv_rank_winner, dim3(1), dim3(256), 0, s, pv, pp, npc, my);
      MLFF_TRY(comm_allgather(ctx, my, wins, 2));
    }
    double *xunit = (mfcols && !colpath) ? ctx->xg : nullptr;
    hipLaunchKernelGGL(k_piv_finalize, dim3(1), dim3(256), 0, s, wins, ctx->world,
                       multi ? nullptr : (const double *)pv,
                       multi ? nullptr : (const long long *)pp, npc, ctx->perm, m, ctx->row0,
                       nrows, ctx->T, blk, ctx->pivflag, multi ? ctx->prow : nullptr, xunit,
                       ctx->rows_per, blk, ctx->st, iperm, spec_m0 >= 0 ? Cspec : nullptr, hit);
    if (multi && m > 0) MLFF_TRY(comm_allreduce(ctx, ctx->prow, (size_t)m));
    if (rbfcols)
      launch_rbf_cols(ctx->rbf, N, ctx->row0, nrows, nullptr, 1, ctx->st, ctx->sigma_K, colbuf, blk, s);
    else if (colpath)
      mf_columns(ctx, nullptr, 1, ctx->sigma_K, colbuf, blk);  // column st->m_pi
    else if (mfcols)
      launch_mf_operator(ctx, ctx->xg, colbuf, nullptr, nullptr, ctx->sigma_K, 0.0);
    const int ks = m > 0 ? std::min(kmax_split, choose_ksplit(m, blk)) : 0;
    const bool in_spec = spec_m0 >= 0;
    // Schur column GEMV over L[:, :m] (on a speculation hit only over [spec_m0, m)); the
    // panel's leading rows (up to 128 MB) are read with default-policy loads so they stay in
    // the MALL from one step to the next
    if (ks > 0)
      launch_colgemv_part(ctx->T, blk, m, ctx->prow, 1, m, ks, part, nullptr, s, StopFold{},
                          panel_cached_rows(m, blk),
                          multi ? nullptr : (const long long *)&ctx->st->m_pi,
                          in_spec ? hit : nullptr, in_spec ? spec_m0 : 0);
    if (gcol > 0)
      hipLaunchKernelGGL(k_piv_fin, dim3(gcol), dim3(256), 0, s, ctx->K, ctx->ld, ctx->sigma_K,
                       (const double *)colbuf, ctx->rows_per, blk, nrows, m, part, ks, blk,
                       ctx->T, blk, ctx->pivflag, ctx->dwork, ctx->st, xunit, iperm, ctx->row0, N,
                       pv, pp, (const double *)Gspec, in_spec ? (const int *)hit : nullptr);
    else if (mfcols && !colpath)
      hipLaunchKernelGGL(k_unit_pivot, dim3(1), dim3(64), 0, s, ctx->xg, ctx->rows_per, blk,
                         ctx->st, 0.0);
    if ((m & 255) == 255) MLFF_HIP(ctx, hipGetLastError());
  }
  stamp_at(k);
  }
  MLFF_HIP(ctx, hipGetLastError());
  int perr = 0;
  MLFF_HIP(ctx, hipMemcpyAsync(&perr, &ctx->st->pivot_err, sizeof(int), hipMemcpyDeviceToHost, s));
  if (index_columns_out != nullptr)
    MLFF_HIP(ctx, hipMemcpyAsync(index_columns_out, ctx->perm, sizeof(int64_t) * N,
                                 hipMemcpyDeviceToHost, s));
  MLFF_HIP(ctx, hipStreamSynchronize(s));
  ctx->piv_col_s.assign((size_t)k, 0.0);
  std::vector<unsigned long long> clk;
  if (step_clock != nullptr && k > 0) {
    clk.resize((size_t)2 * k);
    MLFF_HIP(ctx, hipMemcpy(clk.data(), step_clock, sizeof(unsigned long long) * 2 * k,
                            hipMemcpyDeviceToHost));
  }
  if (stamp_col.size() == stamps.size()) {
    // each segment's event time over its columns: evenly, or (persistent form) in proportion to
    // the steps' own device clocks
    for (size_t g = 0; g + 1 < stamps.size(); ++g) {
      float ms = 0.f;
      (void)hipEventElapsedTime(&ms, stamps[g], stamps[g + 1]);
      const int64_t c0 = stamp_col[g], c1 = std::min<int64_t>(stamp_col[g + 1], k);
      double wsum = 0.0;
      for (int64_t c = c0; c < c1 && !clk.empty(); ++c)
        wsum += clk[2 * c + 1] > clk[2 * c] ? (double)(clk[2 * c + 1] - clk[2 * c]) : 0.0;
      for (int64_t c = c0; c < c1; ++c) {
        double w = 1.0 / (double)(c1 - c0);
        if (wsum > 0.0)
          w = (clk[2 * c + 1] > clk[2 * c] ? (double)(clk[2 * c + 1] - clk[2 * c]) : 0.0) / wsum;
        ctx->piv_col_s[c] = 1e-3 * ms * w;
      }
    }
  }
  for (hipEvent_t e : stamps) (void)hipEventDestroy(e);
  if (perr == 2 && persist) {
    // a workgroup of the persistent grid waited > 1 s for the others (not co-resident: another
    // process's kernels hold CUs): this context builds with the launch sequence from now on
    ctx->piv_persist_off = true;
    return pivoted_cholesky(ctx, k, index_columns_out);
  }
  if (perr)
    return set_error(ctx, MLFF_ERR_NOT_PSD,
                     "given matrix is not PSD (pivot <= 0 in pivoted Cholesky)");
  return MLFF_OK;
}

}  // namespace mlff
