// Matrix-free sGDML kernel operator: y = sigma * K x + lam * x without forming K.
//
// This is the operator the reference's CG actually applies: K_op / _K_vec
// (src/sGDML/sgdml/solvers/iterative_solver.py:383-445) runs a GDMLPredict force
// prediction at every training point with alphas = x (predict.py:72-234,
// set_alphas :400-445).  Per training point i (query) and training point j,
// permutation p (descriptor map P_p, desc.py:360-389):
//   z_j      = J_j x_j                       compact Jacobian (desc.py:464-508)
//   Zt[jp]   = z_j[P_p],  Rt[jp] = Rd_j[P_p]
//   diff     = Rd_i - Rt[jp],  norm = sqrt5 |diff|
//   m        = exp(-norm / sig) 5 / (3 sig^4),  w = (sig^2 + sig norm) m
//   F_i      = sum_jp 5 m (diff . Zt[jp]) diff - w Zt[jp]
//   y_i      = J_i^T F_i
// For a permutation group this is the assembled K (train.py:81-236); for other
// permutation sets it is the reference's K_op rather than its mirrored assembly.
//
// Work per mat-vec is O(M^2 n_perms D) flops over O(M n_perms D) data (the
// descriptor tables stay L2/MALL resident) instead of streaming 8 N^2 bytes of a
// dense K (N = 3 n M, D = n (n - 1) / 2): for the nanotube (M = 14, n = 370)
// ~60 MB of traffic instead of 1.9 GB.  The x-independent quantities (Rt, 5m, w)
// are computed once at setup.
//
// Kernels of one application (all status gated, fixed-order reductions):
//   k_mf_z     Zt[jp, d]            (M n_perms D)
//   k_mf_pair  c[i, jp] = 5m (diff . Zt[jp])   workgroup per (jp, 16 points)
//   k_mf_h     F[i, d]                          thread per (d, 16 points)
//   k_mf_jt    y rows of this rank = J_i^T F_i, epilogue sigma y + lam x
#include <cstdio>

#include "common.h"

#include <algorithm>
#include <cstdlib>
#include <string>

namespace mlff {

namespace {

constexpr int kIC = 16;  // training points per workgroup in the pair / F kernels
// largest pair-record table of the single-column path (beyond it, columns run through the
// whole operator as K_op e_i): 2 GB, or 5 % of the device's memory if that is more (the
// N = 505050 nanotube, M = 455, needs 3.7 GB)
constexpr double kMfColTableBytes = 2.0e9;
double col_table_cap() {
  size_t fr = 0, tot = 0;
  if (hipMemGetInfo(&fr, &tot) != hipSuccess) return kMfColTableBytes;
  return std::max(kMfColTableBytes, 0.05 * (double)tot);
}

__device__ __forceinline__ int64_t xpos(int64_t g, int64_t rows_per, int64_t blk) {
  return (g / rows_per) * blk + g % rows_per;
}

__global__ __launch_bounds__(256) void k_mf_rt(const double *__restrict__ Rd,
                                               const int32_t *__restrict__ Pt, int64_t M,
                                               int n_perms, int64_t D, double *__restrict__ Rt) {
  const int64_t jp = blockIdx.y;
  const int64_t j = jp / n_perms, p = jp % n_perms;
  for (int64_t d = (int64_t)blockIdx.x * 256 + threadIdx.x; d < D; d += (int64_t)gridDim.x * 256)
    Rt[jp * D + d] = Rd[j * D + Pt[p * D + d]];
}

// contiguous copy of the padded rank-block vector (several ranks only)
__global__ __launch_bounds__(256) void k_mf_contig(const double *__restrict__ x, int64_t N,
                                                   int64_t rows_per, int64_t blk,
                                                   double *__restrict__ xc,
                                                   const int *__restrict__ status) {
  if (status != nullptr && *status != ST_RUNNING) return;
  const int64_t g = (int64_t)blockIdx.x * 256 + threadIdx.x;
  if (g < N) xc[g] = x[xpos(g, rows_per, blk)];
}

// Zt[jp, d] = sum_c Rdd_j[e, c] (x_j[t_e, c] - x_j[s_e, c]),  e = P_p[d], pair e = (s_e > t_e)
// (x contiguous in the global index)
struct ZSrc {
  const double *Rdd;
  const int32_t *Pt, *ps, *pt;
  int n, n_perms;
  const double *x;
  double *Zt;  // written by the workgroups of the first point tile
};

__device__ __forceinline__ double z_entry(const ZSrc &zs, int64_t D, int64_t jp, int64_t d) {
  const int64_t j = jp / zs.n_perms, p = jp % zs.n_perms;
  const int64_t g0 = j * 3 * zs.n;
  const int64_t e = zs.Pt != nullptr ? (int64_t)zs.Pt[p * D + d] : d;  // Pt null: identity
  const int s = zs.ps[e], t = zs.pt[e];
  const double *r = zs.Rdd + (j * D + e) * 3;
  double z = 0.0;
#pragma unroll
  for (int c = 0; c < 3; ++c) {
    const double xt = zs.x[g0 + 3 * t + c];
    const double xs = zs.x[g0 + 3 * s + c];
    z = fma(r[c], xt - xs, z);
  }
  return z;
}

// FP: the operand is the search direction p = fused_p(x, pf.z) (beta = rho / rho1 with rho the
// fixed-order sum of the rho partials: k_update_p's bits), and block (0, 0) runs the previous
// iteration's stop test (pf.sf, as k_rec_g does) and publishes rho for k_pt_fin
template <bool FP = false>
__global__ __launch_bounds__(256) void k_mf_z(const double *__restrict__ Rdd,
                                              const int32_t *__restrict__ Pt,
                                              const int32_t *__restrict__ ps,
                                              const int32_t *__restrict__ pt, int64_t M,
                                              int n, int n_perms, int64_t D,
                                              const double *__restrict__ x,
                                              double *__restrict__ Zt,
                                              const int *__restrict__ status, PFuse pf = PFuse{},
                                              int rows = 1) {
  // the status word is read here and tested once the operand loads are in flight (it only
  // has to hold back the stores of an iteration past convergence)
  const int st0 = status != nullptr ? *status : ST_RUNNING;
  const ZSrc zs{Rdd, Pt, ps, pt, n, n_perms, x, Zt};
  if (rows > 1) {
    // short descriptors (D <= 128: few atoms): `rows` (j, p) rows per workgroup, one thread per
    // (row, entry) -- a full workgroup instead of D of 256 threads, and (fused) one rho sum per
    // `rows` rows; the operands are requested before the rho sum
    const int tid = threadIdx.x;
    const int64_t jp = (int64_t)blockIdx.x * rows + tid / D, d = tid % D;
    const bool ok = tid < rows * D && jp < M * n_perms;
    double r[3] = {0.0, 0.0, 0.0}, xt[3] = {0.0, 0.0, 0.0}, xs[3] = {0.0, 0.0, 0.0};
    double zt[3] = {0.0, 0.0, 0.0}, zsv[3] = {0.0, 0.0, 0.0};
    if (ok) {
      const int64_t j = jp / n_perms, p = jp % n_perms, g0 = j * 3 * n;
      const int64_t e = Pt != nullptr ? (int64_t)Pt[p * D + d] : d;
      const int sa = ps[e], ta = pt[e];
#pragma unroll
      for (int c = 0; c < 3; ++c) {
        r[c] = Rdd[(j * D + e) * 3 + c];
        xt[c] = x[g0 + 3 * ta + c];
        xs[c] = x[g0 + 3 * sa + c];
        if (FP) {
          zt[c] = pf.z[g0 + 3 * ta + c];
          zsv[c] = pf.z[g0 + 3 * sa + c];
        }
      }
    }
    double beta = 0.0;
    const bool first = FP && pf.it <= 1;
    const double rshare = FP ? parts_thread_sum(pf.rho_part, kVecGrid) : 0.0;
    if (st0 != ST_RUNNING) return;  // uniform: before the first barrier
    if (FP) {
      __shared__ double shq[8];
      const bool sfold = pf.sf.rr_part != nullptr;
      const double rho1 = sfold ? pf.st->rho : pf.st->rho1;
      const double rho = parts_bcast(rshare, shq);
      beta = rho / rho1;
      if (blockIdx.x == 0) {
        if (tid == 0) pf.st->rho_new = rho;
        if (sfold) stop_decide(pf.sf, reduce_parts_bcast(pf.sf.rr_part, kVecGrid, shq));
      }
    }
    if (!ok) return;
    double z = 0.0;
#pragma unroll
    for (int c = 0; c < 3; ++c) {
      const double a = FP ? fused_p(xt[c], zt[c], beta, first) : xt[c];
      const double b = FP ? fused_p(xs[c], zsv[c], beta, first) : xs[c];
      z = fma(r[c], a - b, z);
    }
    Zt[jp * D + d] = z;
    return;
  }
  if (st0 != ST_RUNNING) return;
  const int64_t jp = blockIdx.y;
  if (!FP) {
    for (int64_t d = (int64_t)blockIdx.x * 256 + threadIdx.x; d < D; d += (int64_t)gridDim.x * 256)
      Zt[jp * D + d] = z_entry(zs, D, jp, d);
    return;
  }
  __shared__ double shp[8];
  const bool first = pf.it <= 1, sfold = pf.sf.rr_part != nullptr;
  // rho1 as the (folded) stop test of the previous iteration leaves it
  const double rho1 = sfold ? pf.st->rho : pf.st->rho1;
  const double rho = parts_bcast(parts_thread_sum(pf.rho_part, kVecGrid), shp);
  const double beta = rho / rho1;
  if (blockIdx.x == 0 && blockIdx.y == 0) {
    if (threadIdx.x == 0) pf.st->rho_new = rho;
    if (sfold) stop_decide(pf.sf, reduce_parts_bcast(pf.sf.rr_part, kVecGrid, shp));
  }
  const int64_t j = jp / zs.n_perms, p = jp % zs.n_perms;
  const int64_t g0 = j * 3 * zs.n;
  for (int64_t d = (int64_t)blockIdx.x * 256 + threadIdx.x; d < D; d += (int64_t)gridDim.x * 256) {
    const int64_t e = zs.Pt != nullptr ? (int64_t)zs.Pt[p * D + d] : d;
    const int sa = zs.ps[e], ta = zs.pt[e];
    const double *r = zs.Rdd + (j * D + e) * 3;
    double z = 0.0;
#pragma unroll
    for (int c = 0; c < 3; ++c) {
      const int64_t it_ = g0 + 3 * ta + c, is_ = g0 + 3 * sa + c;
      const double xt = fused_p(x[it_], pf.z[it_], beta, first);
      const double xs = fused_p(x[is_], pf.z[is_], beta, first);
      z = fma(r[c], xt - xs, z);
    }
    Zt[jp * D + d] = z;
  }
}

// Partial pair sums over the descriptor slice z of this workgroup for a tile of
// 16 query points x 16 (training point, permutation) pairs, the slice staged through
// LDS in chunks of 64 entries; each wave sums a quarter of every chunk for 2 x 2 pairs
// per thread and the four wave partials of a pair are added in wave order:
//   MODE 0: |Rd_i - Rt[jp]|^2                (setup)
//   MODE 1: (Rd_i - Rt[jp]) . Zt[jp]
// part[(z * ni + il) * MP + jp]; k_mf_pair_fin sums the slices in a fixed order.
// FZ: the Zt entries of the tile are computed here (as k_mf_z, same bits) and stored by
// the workgroups of point tile 0, one launch less per mat-vec.
constexpr int kPT = 16;  // tile edge (points and pairs)
constexpr int kDC = 64;  // descriptor chunk staged in LDS
// waves_per_eu(5): 96 VGPRs (110 unconstrained), 5 resident workgroups per CU
template <int MODE, bool FZ = false>
__global__ __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(5, 8))) void k_mf_pair(const double *__restrict__ Rd,
                                                 const double *__restrict__ Rt,
                                                 const double *__restrict__ Zt, int64_t D,
                                                 int64_t dslice, int64_t i0, int64_t ni,
                                                 int64_t MP, double *__restrict__ part,
                                                 const int *__restrict__ status, ZSrc zs = {}) {
  if (MODE == 1 && status != nullptr && *status != ST_RUNNING) return;
  __shared__ double sR[kPT][kDC + 1];
  __shared__ double sT[kPT][kDC + 1];
  __shared__ double sZ[MODE == 1 ? kPT : 1][kDC + 1];
  const int64_t jp0 = (int64_t)blockIdx.x * kPT;
  const int64_t ic0 = (int64_t)blockIdx.y * kPT;
  const int64_t d0 = (int64_t)blockIdx.z * dslice;
  const int64_t d1 = (d0 + dslice) < D ? (d0 + dslice) : D;
  const int tj = threadIdx.x & (kPT - 1), ti = threadIdx.x / kPT;  // output pair
  const int wv = threadIdx.x >> 6, qi = (threadIdx.x & 63) >> 3, qj = threadIdx.x & 7;
  double acc[4] = {0.0, 0.0, 0.0, 0.0};
  constexpr int kPer = kPT * kDC / 256;  // staged entries per thread and array
  for (int64_t c0 = d0; c0 < d1; c0 += kDC) {
    // all loads of the chunk (and the Zt gathers) are issued before any LDS store, so
    // the thread's kPer dependent-load chains overlap instead of running one by one
    double vR[kPer], vT[kPer], vZ[kPer];
#pragma unroll
    for (int u = 0; u < kPer; ++u) {
      const int e = threadIdx.x + 256 * u;
      const int r = e / kDC, cc = e % kDC;
      const int64_t d = c0 + cc;
      const bool okd = d < d1;
      const int64_t il = ic0 + r, jp = jp0 + r;
      vR[u] = (okd && il < ni) ? Rd[(i0 + il) * D + d] : 0.0;
      vT[u] = (okd && jp < MP) ? Rt[jp * D + d] : 0.0;
      vZ[u] = 0.0;
      if (MODE == 1 && !FZ) vZ[u] = (okd && jp < MP) ? Zt[jp * D + d] : 0.0;
      if (MODE == 1 && FZ && okd && jp < MP) vZ[u] = z_entry(zs, D, jp, d);
    }
    if (MODE == 1 && FZ && blockIdx.y == 0) {
#pragma unroll
      for (int u = 0; u < kPer; ++u) {
        const int e = threadIdx.x + 256 * u;
        const int64_t d = c0 + e % kDC, jp = jp0 + e / kDC;
        if (d < d1 && jp < MP) zs.Zt[jp * D + d] = vZ[u];
      }
    }
    __syncthreads();
#pragma unroll
    for (int u = 0; u < kPer; ++u) {
      const int e = threadIdx.x + 256 * u;
      const int r = e / kDC, cc = e % kDC;
      sR[r][cc] = vR[u];
      sT[r][cc] = vT[u];
      if (MODE == 1) sZ[r][cc] = vZ[u];
    }
    __syncthreads();
    // wave w sums the chunk's entries [16 w, 16 w + 16) for a 2 x 2 block of pairs
    // (qi + 8 a, qj + 8 b): 6 LDS reads per 4 products instead of 3 per 1
#pragma unroll 4
    for (int c = 0; c < kDC / 4; ++c) {
      const int cc = wv * (kDC / 4) + c;
      const double r0 = sR[qi][cc], r1 = sR[qi + 8][cc];
      const double t0 = sT[qj][cc], t1 = sT[qj + 8][cc];
      const double z0 = MODE == 0 ? 0.0 : sZ[MODE == 1 ? qj : 0][cc];
      const double z1 = MODE == 0 ? 0.0 : sZ[MODE == 1 ? qj + 8 : 0][cc];
      const double d00 = r0 - t0, d01 = r0 - t1, d10 = r1 - t0, d11 = r1 - t1;
      acc[0] = fma(d00, MODE == 0 ? d00 : z0, acc[0]);
      acc[1] = fma(d01, MODE == 0 ? d01 : z1, acc[1]);
      acc[2] = fma(d10, MODE == 0 ? d10 : z0, acc[2]);
      acc[3] = fma(d11, MODE == 0 ? d11 : z1, acc[3]);
    }
  }
  // the 4 waves' partial sums of each pair, added in wave order
  __syncthreads();
  static_assert(kPT * (kDC + 1) >= 4 * 256, "wave partials fit in sR");
  double *red = &sR[0][0];  // 4 x 256 doubles
#pragma unroll
  for (int a = 0; a < 2; ++a)
#pragma unroll
    for (int b = 0; b < 2; ++b) red[wv * 256 + (qi + 8 * a) * kPT + qj + 8 * b] = acc[2 * a + b];
  __syncthreads();
  const double sum = ((red[threadIdx.x] + red[256 + threadIdx.x]) + red[512 + threadIdx.x]) +
                     red[768 + threadIdx.x];
  const int64_t il = ic0 + ti, jp = jp0 + tj;
  if (il < ni && jp < MP) part[((int64_t)blockIdx.z * ni + il) * MP + jp] = sum;
}

// MODE 0: m5 = 5 m, w from the squared norms; MODE 1: c = m5 * dot; MODE 2 (energies):
// w * dot.  One wave per output: lanes stride over the nz slices, fixed-order wave sum.
// Energy constraints (MODE 1, xE != nullptr): c += x_E[j] w (the energy coefficients' force
// term, predict.py:210-213) and eterm = dot * w (their energy term, predict.py:207).
struct EPair {
  const double *xE = nullptr;  // energy entries of the operand (M)
  const double *w = nullptr;   // ni x MP
  double *eterm = nullptr;     // ni x MP
  int64_t MP = 1;
  int n_perms = 1;
};
template <int MODE>
__global__ __launch_bounds__(256) void k_mf_pair_fin(const double *__restrict__ part, int nz,
                                                     int64_t nout, double sig,
                                                     const double *__restrict__ m5,
                                                     double *__restrict__ out0,
                                                     double *__restrict__ out1,
                                                     const int *__restrict__ status,
                                                     EPair ep = {}) {
  if (MODE >= 1 && status != nullptr && *status != ST_RUNNING) return;
  const int64_t o = (int64_t)blockIdx.x * 4 + (threadIdx.x >> 6);
  const int lane = threadIdx.x & 63;
  if (o >= nout) return;
  // the lane's slices in slice order, 8 loads in flight (same sum, same bits)
  double s = 0.0;
  int z = lane;
  for (; z + 7 * 64 < nz; z += 8 * 64) {
    double t[8];
#pragma unroll
    for (int u = 0; u < 8; ++u) t[u] = part[(int64_t)(z + u * 64) * nout + o];
#pragma unroll
    for (int u = 0; u < 8; ++u) s += t[u];
  }
  for (; z < nz; z += 64) s += part[(int64_t)z * nout + o];
#pragma unroll
  for (int off = 32; off > 0; off >>= 1) s += __shfl_down(s, off, 64);
  if (lane != 0) return;
  if (MODE == 0) {
    const double norm = sqrt(5.0) * sqrt(s);
    const double m = exp(-norm / sig) * 5.0 / (3.0 * sig * sig * sig * sig);
    out0[o] = 5.0 * m;
    out1[o] = (sig * sig + sig * norm) * m;
  } else if (MODE == 1 && ep.xE != nullptr) {
    const int64_t j = (o % ep.MP) / ep.n_perms;
    out0[o] = fma(ep.xE[j], ep.w[o], m5[o] * s);
    ep.eterm[o] = s * ep.w[o];
  } else {
    out0[o] = m5[o] * s;  // MODE 2: m5 holds w
  }
}

// F[il, d] = sum_jp c[il, jp] (Rd_i[d] - Rt[jp, d]) - w[il, jp] Zt[jp, d]   (fixed jp order)
// One wave per (64 descriptor entries, IC query points); the coefficients of the
// IC points are staged in LDS 64 pairs at a time.  IC = 4 when 16 would leave the
// chip with too few waves (few query points: latency bound).
// 1-D grid, XCD-aware: workgroups L and L + 8 share an XCD (round-robin dispatch), so the
// point groups of one descriptor block get consecutive slots of one XCD and read its
// Rt / Zt columns from that XCD's L2 instead of the fabric once per group.
template <int IC>
__global__ __launch_bounds__(64) void k_mf_h(const double *__restrict__ Rd,
                                             const double *__restrict__ Rt,
                                             const double *__restrict__ Zt, int64_t D,
                                             int64_t i0, int64_t ni, int64_t MP,
                                             const double *__restrict__ cf,
                                             const double *__restrict__ wf,
                                             double *__restrict__ F,
                                             const int *__restrict__ status) {
  if (status != nullptr && *status != ST_RUNNING) return;
  __shared__ double sc[IC][64];
  __shared__ double sw[IC][64];
  const int64_t gi = (ni + IC - 1) / IC;
  const int64_t slot = blockIdx.x / 8, grp = slot % gi;
  const int64_t dblock = (slot / gi) * 8 + blockIdx.x % 8;
  if (dblock * 64 >= D) return;
  const int64_t d = dblock * 64 + threadIdx.x;
  const int64_t ic0 = grp * IC;
  const int nk = (int)((ni - ic0) < IC ? (ni - ic0) : IC);
  const bool act = d < D;
  double rdi[IC], h[IC];
#pragma unroll
  for (int k = 0; k < IC; ++k) {
    rdi[k] = (act && k < nk) ? Rd[(i0 + ic0 + k) * D + d] : 0.0;
    h[k] = 0.0;
  }
  for (int64_t j0 = 0; j0 < MP; j0 += 64) {
    const int cnt = (int)((MP - j0) < 64 ? (MP - j0) : 64);
    __syncthreads();
    for (int k = 0; k < nk; ++k) {
      if (threadIdx.x < cnt) {
        sc[k][threadIdx.x] = cf[(ic0 + k) * MP + j0 + threadIdx.x];
        sw[k][threadIdx.x] = wf[(ic0 + k) * MP + j0 + threadIdx.x];
      }
    }
    __syncthreads();
    if (act) {
      int jj = 0;
      for (; jj + 7 < cnt; jj += 8) {  // 16 loads in flight per lane
        double r[8], z[8];
#pragma unroll
        for (int u = 0; u < 8; ++u) {
          r[u] = Rt[(j0 + jj + u) * D + d];
          z[u] = Zt[(j0 + jj + u) * D + d];
        }
#pragma unroll
        for (int u = 0; u < 8; ++u)
#pragma unroll
          for (int k = 0; k < IC; ++k)
            if (k < nk) h[k] = fma(sc[k][jj + u], rdi[k] - r[u], fma(-sw[k][jj + u], z[u], h[k]));
      }
      for (; jj < cnt; ++jj) {
        const double r = Rt[(j0 + jj) * D + d];
        const double z = Zt[(j0 + jj) * D + d];
#pragma unroll
        for (int k = 0; k < IC; ++k)
          if (k < nk) h[k] = fma(sc[k][jj], rdi[k] - r, fma(-sw[k][jj], z, h[k]));
      }
    }
  }
  if (act)
#pragma unroll
    for (int k = 0; k < IC; ++k)
      if (k < nk) F[(ic0 + k) * D + d] = h[k];
}

__device__ __forceinline__ int64_t pair_of(int a, int b) {
  return a > b ? (int64_t)a * (a - 1) / 2 + b : (int64_t)b * (b - 1) / 2 + a;
}

// rows of this rank: g = i 3n + 3a + c,  y = sum_{b != a} sgn * Rdd_i[pair(a,b), c] F_i[pair(a,b)]
// (J[pair, (t, c)] = +Rdd, J[pair, (s, c)] = -Rdd with s > t, desc.py:444-462).
// Workgroup = (point, block of 32 atoms a, slice of partner blocks); it walks the
// 32 x 32 blocks (A, B) of the pair triangle: for B < A the pairs of one atom a are
// 32 consecutive descriptor entries, for B > A those of one atom b are, so every
// block is read with coalesced loads into registers and parked in LDS (the next
// block's loads are issued before the current one is consumed).  8 threads per
// atom sum 4 partners each; slices are summed in order by k_mf_jt_fin.
constexpr int kAB = 32;
constexpr int kJSMax = 16;  // partner-block slices (gridDim.z of k_mf_jt, at most)

__device__ __forceinline__ void jt_load(const double *__restrict__ Fi,
                                        const double *__restrict__ Ri, int n, int A0, int B0,
                                        double (&f)[4], double (&r)[4][3], int (&la)[4],
                                        int (&lb)[4]) {
#pragma unroll
  for (int u = 0; u < 4; ++u) {
    const int e = threadIdx.x + 256 * u;
    const int rr = e / kAB, q = e % kAB;
    const int aa = B0 < A0 ? A0 + rr : A0 + q;
    const int bb = B0 < A0 ? B0 + q : B0 + rr;
    la[u] = aa - A0;
    lb[u] = bb - B0;
    f[u] = 0.0;
    r[u][0] = r[u][1] = r[u][2] = 0.0;
    if (aa < n && bb < n && aa != bb) {
      const int64_t d = pair_of(aa, bb);
      const double sg = aa > bb ? -1.0 : 1.0;
      f[u] = sg * Fi[d];
      r[u][0] = Ri[d * 3 + 0];
      r[u][1] = Ri[d * 3 + 1];
      r[u][2] = Ri[d * 3 + 2];
    }
  }
}

// partner-block slices of k_mf_jt (MLFF_MF_JS overrides, sweeps)
int mf_jt_slices(int n) {
  const int nblk = (n + kAB - 1) / kAB;
  int js = 4;
  if (const char *e = std::getenv("MLFF_MF_JS")) js = std::atoi(e);
  return std::max(1, std::min({js, nblk, kJSMax}));
}

// 1-D grid of nblk x ni x js workgroups in molecule-major order, dealt to the XCDs in
// contiguous eighths (workgroup L runs on XCD L mod 8): the 12 x js workgroups of one
// point, which read each of its (F, Rdd) pairs twice, mostly share one XCD's L2.
__global__ __launch_bounds__(256) void k_mf_jt(const double *__restrict__ Rdd,
                                               const double *__restrict__ F, int64_t D, int n,
                                               int64_t i0, int64_t ni, int js, int64_t row0,
                                               int64_t nrows, double *__restrict__ part,
                                               const int *__restrict__ status) {
  if (status != nullptr && *status != ST_RUNNING) return;
  __shared__ double sF[kAB][kAB + 1];
  __shared__ double sR[3][kAB][kAB + 1];
  const int nblk = (n + kAB - 1) / kAB;
  const int64_t total = (int64_t)nblk * ni * js, per = (total + 7) / 8;
  const int64_t v = (int64_t)(blockIdx.x % 8) * per + blockIdx.x / 8;
  if (v >= total) return;
  const int64_t il = v / ((int64_t)nblk * js);
  const int zz = (int)((v / nblk) % js);
  const int A0 = (int)(v % nblk) * kAB;
  const int64_t i = i0 + il;
  const int64_t n3 = 3 * (int64_t)n;
  const int64_t gfirst = i * n3 + 3 * (int64_t)A0;
  const int64_t glast = i * n3 + 3 * (int64_t)(A0 + kAB < n ? A0 + kAB : n) - 1;
  if (glast < row0 || gfirst >= row0 + nrows) return;
  const double *Fi = F + il * D;
  const double *Ri = Rdd + i * D * 3;
  const int al = threadIdx.x >> 3, pt = threadIdx.x & 7;
  const int a = A0 + al;
  const int bz0 = (int)(((int64_t)nblk * zz) / js);
  const int bz1 = (int)(((int64_t)nblk * (zz + 1)) / js);
  double acc[3] = {0.0, 0.0, 0.0};
  double f[4], r[4][3];
  int la[4], lb[4];
  if (bz0 < bz1) jt_load(Fi, Ri, n, A0, bz0 * kAB, f, r, la, lb);
  for (int bk = bz0; bk < bz1; ++bk) {
    __syncthreads();
#pragma unroll
    for (int u = 0; u < 4; ++u) {
      sF[la[u]][lb[u]] = f[u];
      sR[0][la[u]][lb[u]] = r[u][0];
      sR[1][la[u]][lb[u]] = r[u][1];
      sR[2][la[u]][lb[u]] = r[u][2];
    }
    __syncthreads();
    if (bk + 1 < bz1) jt_load(Fi, Ri, n, A0, (bk + 1) * kAB, f, r, la, lb);
#pragma unroll
    for (int k = 0; k < kAB / 8; ++k) {
      const int q = pt * (kAB / 8) + k;
      const double fv = sF[al][q];
      acc[0] = fma(sR[0][al][q], fv, acc[0]);
      acc[1] = fma(sR[1][al][q], fv, acc[1]);
      acc[2] = fma(sR[2][al][q], fv, acc[2]);
    }
  }
#pragma unroll
  for (int c = 0; c < 3; ++c) {
    double v = acc[c];
    v += __shfl_down(v, 4, 8);
    v += __shfl_down(v, 2, 8);
    v += __shfl_down(v, 1, 8);
    acc[c] = v;
  }
  if (pt == 0 && a < n) {
#pragma unroll
    for (int c = 0; c < 3; ++c) {
      const int64_t rr = i * n3 + 3 * (int64_t)a + c - row0;
      if (rr < 0 || rr >= nrows) continue;
      part[(int64_t)zz * nrows + rr] = acc[c];
    }
  }
}

// y = sigma * sum_z part[z] + lam * x (fixed slice order).  PQ: also the x . y partials
// of the CG step, on the kVecGrid grid-stride layout of k_dot_part (same terms, same
// order: the separate dot launch it replaces gives the same bits)
// Energy rows (one rank, use_E_cstr): row nF + i = -(sum_jp eterm[i, jp] + sum_j kee[i, j]
// x_E[j]) (the predicted energy with a flipped sign, iterative_solver.py:439-440).
struct ERows {
  int64_t nF = INT64_MAX;  // rows >= nF are energy rows
  const double *eterm = nullptr, *kee = nullptr, *xE = nullptr;
  int64_t M = 0, MP = 0;
};
template <bool PQ>
__global__ __launch_bounds__(256) void k_mf_jt_fin(const double *__restrict__ part, int js,
                                                   int64_t nrows,
                                                   double sigma, double lam,
                                                   const double *__restrict__ xloc,
                                                   double *__restrict__ y,
                                                   double *__restrict__ pq_part,
                                                   const int *__restrict__ status, ERows er = {}) {
  if (status != nullptr && *status != ST_RUNNING) return;
  __shared__ double sh[8];
  double acc = 0.0;
  for (int64_t r = (int64_t)blockIdx.x * 256 + threadIdx.x; r < nrows;
       r += (int64_t)gridDim.x * 256) {
    double s = 0.0;
    if (r >= er.nF) {
      const int64_t i = r - er.nF;
      double e = 0.0;
      for (int64_t jp = 0; jp < er.MP; ++jp) e += er.eterm[i * er.MP + jp];
      for (int64_t j = 0; j < er.M; ++j) e = fma(er.kee[i * er.M + j], er.xE[j], e);
      s = -e;
    } else {
      for (int z = 0; z < js; ++z) s += part[(int64_t)z * nrows + r];
    }
    double yv = sigma * s;
    if (xloc != nullptr) yv += lam * xloc[r];
    y[r] = yv;
    if (PQ) acc = fma(xloc[r], yv, acc);
  }
  if (PQ) {
    const double t = block_sum256(acc, sh);
    if (threadIdx.x == 0) pq_part[blockIdx.x] = t;
  }
}

__global__ void k_mf_ediag(const double *__restrict__ kee, int64_t M, double *__restrict__ out) {
  const int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x;
  if (i < M) out[i] = -kee[i * M + i];
}

// ---------------------------------------------------------------------------
// Record-factored operator.  With the x-independent pair records of the single-column
// path (k_sgdml_uv, mirror = 0: u = J_i^T diff, v = J_j^T P_p^T diff, m, w per (i, j, p))
// the reference's K_op (predict.py:172-220 with alphas = x) regroups exactly as
//   c_ijp = 5 m (diff . Zt_jp) = 5 m (v_ijp . x_j)
//   y_i   = J_i^T sum_jp (c diff - w Zt_jp) = sum_jp c_ijp u_ijp - J_i^T G_i,
//   G_i   = sum_jp w_ijp Zt_jp,   Zt_jp = (J_j x_j)[P_p]
// so the two full-descriptor (O(M^2 D)) reductions of the pair sums and the F pass
// become one: G, a w-weighted sum of Zt, which k_rec_g forms on the fly (Zt from Rdd
// and x, never stored) and contracts with J_i^T inside the same workgroup.  Two launches:
//   k_rec_g    workgroup per (16 x 16 atom pair block (A >= B), 16 query points): Zt of the
//              block's pairs for every (j, p), G of its points, J_i^T G partial rows into
//              slot B (atoms of A) and slot A (atoms of B); extra workgroups: the pair
//              scalars s_ijp = 5 m (v . x_j), one wave each
//   k_rec_fin  y = sigma (sum_jp s u - sum_slots) + lam x (+ the p.q partials of the step)
// Rounding: a regrouping of the same products (the noise-band check of this form on all
// golden solves is in DESIGN.md 3.2).
constexpr int kRB = 16;  // atoms per edge of a pair block
constexpr int kRG = 16;  // query points per workgroup (G accumulators per thread)
constexpr int kRJ = 8;   // (j, p) per batch of Zt loads
constexpr int kWC = 32;  // (j, p) per chunk of w staged in LDS
static_assert(kRG % kRJ == 0 && kWC % kRJ == 0, "batches tile the point groups and chunks");

// Zt_jp[d] = (J_j x_j)[P_p d] (z_entry, general permutation)
__device__ __forceinline__ double rec_zt(const double *__restrict__ Rdd,
                                         const double *__restrict__ xc,
                                         const int32_t *__restrict__ Pt,
                                         const int32_t *__restrict__ ps,
                                         const int32_t *__restrict__ pt, int64_t D, int n,
                                         int64_t j, int p, int64_t d) {
  const int64_t e = Pt[(int64_t)p * D + d];
  const int s = ps[e], t = pt[e];
  const double *r = Rdd + (j * D + e) * 3;
  const double *xj = xc + j * 3 * (int64_t)n;
  double z = 0.0;
#pragma unroll
  for (int c = 0; c < 3; ++c) z = fma(r[c], xj[3 * t + c] - xj[3 * s + c], z);
  return z;
}

struct RecArgs {
  const double *Rdd;   // M x D x 3
  const double *Zt;    // (M n_perms) x D, precomputed (ZM == kZStored)
  const double *xc;    // contiguous operand (global index)
  const int32_t *Pt;   // n_perms x D
  const int32_t *ps, *pt;
  const double *uvk;   // records, ni x M x n_perms x (6 n + 2)
  int64_t M, D, i0, ni, MP;
  int64_t ldw;         // row length of wt (ngrp kRG, zero padded)
  int n, n_perms, nblk;
  double *rpart;       // nblk x ni x 3n
  double *sv;          // ni x MP
  // fused search-direction update (one rank, PCG iteration): the operand is
  // p = z + (rho / rho1) p_old (p = z at ITER 1) formed on the fly from xc = p_old and pz,
  // rho the fixed-order sum of rho_part (k_update_p's arithmetic, the same bits); k_rec_fin
  // writes p.  pz == nullptr: xc is the operand itself
  const double *pz = nullptr;
  const double *rho_part = nullptr;
  DevState *st = nullptr;
  long long it = 0;
  // the stop test of the previous iteration (its rr partials written by k_lr_fin's folded
  // k_update_xr), done by workgroup 0; beta's rho1 is then the state's rho (the stop test
  // copies it into rho1 in this same launch)
  StopFold sf;
};

// the operand entry of a fused update (k_update_p: p = fma(beta, p_old, z), p = z at ITER 1)

// wt: w transposed, round_up(MP, kRJ) rows of ldw = ngrp kRG entries, zero padded, so
// the accumulation runs unguarded over whole batches and point groups
// grid: nsw8 pair-scalar workgroups first (dispatched first, off the tail), then the
// pair blocks.  Zt of a batch: gathered from Rdd / x per permutation (kZGather), from the
// LDS-staged x of the block's atoms (kZIdent: one identity permutation), or read from the
// Zt table (kZStored: several point groups, where k_mf_z's one pass over Rdd beats a
// recomputation per group)
#ifdef MLFF_REC_TRACE
// phase timestamps of k_rec_g (a variant build, scripts/experiments/gpu_r03_rectrace.sh):
// per workgroup [start, staged, G loop done, end] of the 100 MHz wall clock, plus the XCC /
// CU the workgroup ran on
__device__ unsigned long long g_rec_trace[8192][5];
#define REC_STAMP(slot)                                                                  \
  do {                                                                                   \
    if (threadIdx.x == 0 && blockIdx.x < 8192)                                           \
      g_rec_trace[blockIdx.x][slot] = __builtin_amdgcn_s_memrealtime();                  \
  } while (0)
#else
#define REC_STAMP(slot) \
  do {                  \
  } while (0)
#endif
enum { kZGather = 0, kZIdent = 1, kZStored = 2 };
// CAP: with one identity permutation the query points' Rdd rows are captured from the Zt
// batches into registers for the epilogue (CAP = false: re-read per epilogue round, fewer
// registers live across the loop)
// FP: the fused search-direction update (RecArgs::pz; identity permutation)
template <int ZM, bool CAP = true, int RG = kRG, int RR = 8, int WC = kWC, bool FP = false>
__global__ __launch_bounds__(256) void k_rec_g(RecArgs a, const double *__restrict__ wt,
                                               int64_t nbp, int64_t ngrp, int64_t nsw8,
                                               const int *__restrict__ status) {
  REC_STAMP(0);
  // the status gate is read here and tested once the first loads are in flight (it only has
  // to hold back the stores of an iteration past convergence)
  const int st0 = status != nullptr ? *status : ST_RUNNING;
  __shared__ double red[RR][3][kRB][kRB + 1];
  __shared__ double sW[WC][RG];
  __shared__ double shp[8];
  const int tid = threadIdx.x;
  const int n3 = 3 * a.n;
  static_assert(!FP || ZM == kZIdent, "fused p: identity permutation");
  // fused p: rho1 and this thread's share of the rho partials, requested first
  const bool first = FP && a.it <= 1;
  const bool sfold = FP && a.sf.rr_part != nullptr;
  const double rho1 = FP ? (sfold ? a.st->rho : a.st->rho1) : 1.0;
  const double rshare = FP ? parts_thread_sum(a.rho_part, kVecGrid) : 0.0;
  if ((int64_t)blockIdx.x < nsw8) {  // pair scalars: one wave per (local point, j, p)
    // (fused p: beta first, by all four waves; the scalar waves are off the critical path)
    const double rho = FP ? parts_bcast(rshare, shp) : 0.0;
    const double beta = rho / rho1;
    if (FP && blockIdx.x == 0 && tid == 0) a.st->rho_new = rho;  // for k_rec_fin
    // the previous iteration's stop test (gated like k_stoptest: a solver stopped before this
    // iteration keeps its state); uniform in block 0, whose thread 0 writes the state
    if (sfold && blockIdx.x == 0 && st0 == ST_RUNNING)
      stop_decide(a.sf, reduce_parts_bcast(a.sf.rr_part, kVecGrid, shp));
    const int64_t q = (int64_t)blockIdx.x * 4 + (tid >> 6);
    if (q >= a.ni * a.MP) return;
    const int64_t il = q / a.MP, jp = q % a.MP, j = jp / a.n_perms;
    const double *vv = a.uvk + q * (int64_t)(6 * a.n + 2) + n3;
    const double *xj = a.xc + j * n3;
    const double *zj = FP ? a.pz + j * n3 : xj;
    double acc = 0.0;
    int t = tid & 63;
    for (; t + 7 * 64 < n3; t += 8 * 64) {  // 16 loads in flight, summed in t order
      double va[8], xa[8], za[FP ? 8 : 1];
#pragma unroll
      for (int u = 0; u < 8; ++u) {
        va[u] = vv[t + u * 64];
        xa[u] = xj[t + u * 64];
        if (FP) za[u % (FP ? 8 : 1)] = zj[t + u * 64];
      }
      if (FP) {
#pragma unroll
        for (int u = 0; u < 8; ++u) xa[u] = fused_p(xa[u], za[u % (FP ? 8 : 1)], beta, first);
      }
#pragma unroll
      for (int u = 0; u < 8; ++u) acc = fma(va[u], xa[u], acc);
    }
    for (; t < n3; t += 64)
      acc = fma(vv[t], FP ? fused_p(xj[t], zj[t], beta, first) : xj[t], acc);
    if (st0 != ST_RUNNING) return;
    acc = wave_sum(acc);
    if ((tid & 63) == 0) a.sv[il * a.MP + jp] = 5.0 * vv[3 * a.n] * acc;  // 5 m (v . x_j)
    REC_STAMP(3);
    return;
  }
  // XCD-aware order: the point groups of one pair block run on one XCD (workgroup L on
  // XCD L mod 8), so they share its L2 for the block's Rdd / x lines
  const int64_t wg = (int64_t)blockIdx.x - nsw8;
  const int64_t slot = wg / 8, grp = slot % ngrp;
  const int64_t bp = (slot / ngrp) * 8 + wg % 8;
  if (bp >= nbp) return;
  int A = (int)((sqrt(8.0 * (double)bp + 1.0) - 1.0) * 0.5);
  while ((int64_t)A * (A + 1) / 2 > bp) --A;
  while ((int64_t)(A + 1) * (A + 2) / 2 <= bp) ++A;
  const int B = (int)(bp - (int64_t)A * (A + 1) / 2);
  const int la = tid >> 4, lb = tid & 15;
  const int aa = A * kRB + la, bb = B * kRB + lb;
  const bool valid = aa < a.n && bb < a.n && aa > bb;
  const int64_t d = valid ? (int64_t)aa * (aa - 1) / 2 + bb : 0;
  // batch slots beyond the last (j, p) and lanes without a pair load in-bounds stand-ins
  // (d = 0, the last j) unconditionally, so no branch separates a batch's loads
  const int64_t g0 = grp * RG;
  const int ng = (int)((a.ni - g0) < RG ? (a.ni - g0) : RG);
  double acc[RG];
#pragma unroll
  for (int k = 0; k < RG; ++k) acc[k] = 0.0;
  const double *wp = wt + g0;
  const int64_t MPp = (a.MP + kRJ - 1) / kRJ * kRJ;  // rows of wt
  const int64_t rs = 3 * a.D;
  const double *rj = a.Rdd + d * 3;
  // identity: x of the chunk's points at the block's 2 x 16 atoms, staged in LDS (in the
  // space of the epilogue's reduction buffer), so a batch loads only its Rdd rows
  double *sx = &red[0][0][0][0];  // [WC][2][kRB][3]
  // one identity permutation, point groups aligned to the batches: the query points are
  // training points j = i0 + g0 + k, so their Rdd rows pass through the batches and are
  // kept for the epilogue instead of being read a second time
  constexpr int kCap = CAP ? RG : 1;
  double rg[kCap][3];
#pragma unroll
  for (int k = 0; k < kCap; ++k) rg[k][0] = rg[k][1] = rg[k][2] = 0.0;
  const bool capture = CAP && ZM == kZIdent && a.i0 % kRJ == 0;
  static_assert(RG % RR == 0 && RG <= 16, "point groups are whole epilogue rounds");
  constexpr bool IDENT = ZM == kZIdent;
  static_assert(RR * 3 * kRB * (kRB + 1) >= WC * 2 * kRB * 3, "x stage fits in red");
  // CAP = false: the query points' Rdd rows of the next epilogue round, prefetched (round 0
  // during the G loop, round r + 1 during round r)
  double rn[CAP ? 1 : RR][3];
  auto load_rows = [&](int k0) {
    if (!CAP) {
#pragma unroll
      for (int kk = 0; kk < (CAP ? 1 : RR); ++kk) {
        const int k = k0 + kk;
        const bool ok = k < ng && valid;
        const double *r = a.Rdd + ((a.i0 + g0 + (ok ? k : 0)) * a.D + (ok ? d : 0)) * 3;
        rn[kk][0] = ok ? r[0] : 0.0;
        rn[kk][1] = ok ? r[1] : 0.0;
        rn[kk][2] = ok ? r[2] : 0.0;
      }
    }
  };
  int64_t jn = 0;  // general permutations: (j, p) of the next batch slot
  int pn = 0;
  for (int64_t c0 = 0; c0 < MPp; c0 += WC) {
    // w of the chunk's (j, p) for the group's points, LDS broadcast operands
    const int cn = (int)((MPp - c0) < WC ? (MPp - c0) : WC);
    // (every thread's staging loads issued together, then stored)
    constexpr int kWL = (WC * RG + 255) / 256, kXL = WC * 2 * kRB * 3 / 256;
    double wl[kWL], xl[IDENT ? kXL : 1], zl[FP ? kXL : 1];
#pragma unroll
    for (int q = 0; q < kWL; ++q) {
      const int e = tid + q * 256;
      wl[q] = e < cn * RG ? wp[(c0 + e / RG) * a.ldw + e % RG] : 0.0;
    }
    if (IDENT) {
#pragma unroll
      for (int q = 0; q < kXL; ++q) {
        const int e = tid + q * 256;
        const int jj = e / (2 * kRB * 3), r = e % (2 * kRB * 3);
        const int atom = (r < kRB * 3 ? A : B) * kRB + (r % (kRB * 3)) / 3;
        const int64_t j = c0 + jj;
        const bool ok = jj < cn && j < a.MP && atom < a.n;
        xl[q] = ok ? a.xc[j * n3 + 3 * atom + r % 3] : 0.0;
        if (FP) zl[q % (FP ? kXL : 1)] = ok ? a.pz[j * n3 + 3 * atom + r % 3] : 0.0;
      }
    }
    if (c0 == 0 && st0 != ST_RUNNING) return;  // uniform: before the first barrier
    if (FP) {  // the operand at the block's atoms: p = z + beta p_old (every load in flight)
      const double beta = parts_bcast(rshare, shp) / rho1;
#pragma unroll
      for (int q = 0; q < kXL; ++q) xl[q] = fused_p(xl[q], zl[q % (FP ? kXL : 1)], beta, first);
    }
    __syncthreads();
#pragma unroll
    for (int q = 0; q < kWL; ++q)
      if (WC * RG % 256 == 0 || tid + q * 256 < WC * RG) (&sW[0][0])[tid + q * 256] = wl[q];
    if (IDENT) {
#pragma unroll
      for (int q = 0; q < kXL; ++q) sx[tid + q * 256] = xl[q];
    }
    __syncthreads();
    REC_STAMP(1);
    if (!CAP && c0 == 0) load_rows(0);  // the epilogue's first rows arrive during the loop
    for (int jb = 0; jb < cn; jb += kRJ) {
      double z[kRJ];
      if (ZM == kZStored) {
        double zv[kRJ];
#pragma unroll
        for (int u = 0; u < kRJ; ++u) {
          const int64_t jp = c0 + jb + u;
          zv[u] = a.Zt[(jp < a.MP ? jp : a.MP - 1) * a.D + d];
        }
#pragma unroll
        for (int u = 0; u < kRJ; ++u) z[u] = (valid && c0 + jb + u < a.MP) ? zv[u] : 0.0;
      } else if (ZM == kZIdent) {
        // Zt_j[d] = sum_c Rdd_j[d, c] (x_j[bb, c] - x_j[aa, c])  (z_entry, s = aa, t = bb)
        double rv[kRJ][3];
#pragma unroll
        for (int u = 0; u < kRJ; ++u) {
          const int64_t j = c0 + jb + u, jc = j < a.MP ? j : a.MP - 1;
          const double *r = rj + jc * rs;
          rv[u][0] = r[0];
          rv[u][1] = r[1];
          rv[u][2] = r[2];
        }
        asm volatile("" ::: "memory");  // the batch's loads are issued together
        if (CAP && capture) {
          const int64_t off = c0 + jb - (a.i0 + g0);
#pragma unroll
          for (int h = 0; h < RG / kRJ; ++h)
            if (off == h * kRJ) {
#pragma unroll
              for (int u = 0; u < kRJ; ++u) {
                rg[(h * kRJ + u) % kCap][0] = rv[u][0];
                rg[(h * kRJ + u) % kCap][1] = rv[u][1];
                rg[(h * kRJ + u) % kCap][2] = rv[u][2];
              }
            }
        }
#pragma unroll
        for (int u = 0; u < kRJ; ++u) {
          const double *xs = sx + (jb + u) * (2 * kRB * 3);
          double zz = 0.0;
#pragma unroll
          for (int c = 0; c < 3; ++c)
            zz = fma(rv[u][c], xs[kRB * 3 + lb * 3 + c] - xs[la * 3 + c], zz);
          z[u] = (valid && c0 + jb + u < a.MP) ? zz : 0.0;
        }
      } else {
#pragma unroll
        for (int u = 0; u < kRJ; ++u) {
          const bool ok = valid && jn < a.M;
          const double zz = rec_zt(a.Rdd, a.xc, a.Pt, a.ps, a.pt, a.D, a.n,
                                   jn < a.M ? jn : a.M - 1, pn, d);
          z[u] = ok ? zz : 0.0;
          if (++pn == a.n_perms) {
            pn = 0;
            ++jn;
          }
        }
      }
      // the w reads of one (j, p) at a time (hoisting all 8 x 16 of them costs 256 VGPRs)
      asm volatile("" ::: "memory");
#pragma unroll
      for (int u = 0; u < kRJ; ++u) {
#pragma unroll
        for (int k = 0; k < RG; ++k) acc[k] = fma(sW[jb + u][k], z[u], acc[k]);
        asm volatile("" ::: "memory");
      }
    }
  }
  // J_i^T G over the block: pair d = (s = aa, t = bb), J[d, t] = +Rdd, J[d, s] = -Rdd;
  // the query points' Rdd rows are loaded together (one round trip), mostly L2 hits
  REC_STAMP(2);
  const int64_t pstride = a.ni * n3;
  if (CAP && !capture) {
#pragma unroll
    for (int k = 0; k < kCap; ++k) {
      if (k < ng && valid) {
        const double *r = a.Rdd + ((a.i0 + g0 + k) * a.D + d) * 3;
        rg[k][0] = r[0];
        rg[k][1] = r[1];
        rg[k][2] = r[2];
      }
    }
  }
#pragma unroll
  for (int k0 = 0; k0 < RG; k0 += RR) {
    if (k0 >= ng) break;
    double rr[RR][3];
#pragma unroll
    for (int kk = 0; kk < RR; ++kk) {
      const int k = k0 + kk;
      if (CAP) {
        rr[kk][0] = rg[k % kCap][0];
        rr[kk][1] = rg[k % kCap][1];
        rr[kk][2] = rg[k % kCap][2];
      } else {
        rr[kk][0] = rn[kk % (CAP ? 1 : RR)][0];
        rr[kk][1] = rn[kk % (CAP ? 1 : RR)][1];
        rr[kk][2] = rn[kk % (CAP ? 1 : RR)][2];
      }
    }
    if (!CAP && k0 + RR < RG && k0 + RR < ng) load_rows(k0 + RR);
    __syncthreads();
#pragma unroll
    for (int kk = 0; kk < RR; ++kk) {
      const int k = k0 + kk;
      red[kk][0][la][lb] = rr[kk][0] * acc[k];
      red[kk][1][la][lb] = rr[kk][1] * acc[k];
      red[kk][2][la][lb] = rr[kk][2] * acc[k];
    }
    __syncthreads();
    // RR points x (rows of A | columns of B) x 16 atoms x 3 components
    for (int e = tid; e < RR * 2 * kRB * 3; e += 256) {
      const int kk = e / (2 * kRB * 3), rem = e % (2 * kRB * 3);
      const int side = rem / (kRB * 3), q = rem % (kRB * 3);
      const int ao = q / 3, c = q % 3;
      if (k0 + kk >= ng) continue;
      if (side == 1 && A == B) continue;  // the diagonal block's columns join its rows
      double v = 0.0;
      int atom, sl;
      if (side == 0) {
        double rs = 0.0;
#pragma unroll
        for (int x = 0; x < kRB; ++x) rs += red[kk][c][ao][x];
        v = -rs;
        if (A == B) {
          double cs = 0.0;
#pragma unroll
          for (int x = 0; x < kRB; ++x) cs += red[kk][c][x][ao];
          v += cs;
        }
        atom = A * kRB + ao;
        sl = B;
      } else {
        double cs = 0.0;
#pragma unroll
        for (int x = 0; x < kRB; ++x) cs += red[kk][c][x][ao];
        v = cs;
        atom = B * kRB + ao;
        sl = A;
      }
      if (atom < a.n) a.rpart[sl * pstride + (g0 + k0 + kk) * n3 + 3 * atom + c] = v;
    }
  }
#ifdef MLFF_REC_TRACE
  __syncthreads();
  REC_STAMP(3);
  if (threadIdx.x == 0 && blockIdx.x < 8192) {
    unsigned hw = 0;
    asm volatile("s_getreg_b32 %0, hwreg(HW_REG_HW_ID)" : "=s"(hw));
    g_rec_trace[blockIdx.x][4] = hw;
  }
#endif
}

// rows of this rank: y = sigma (sum_jp s_ijp u_ijp[t] - sum_slots J^T G) + lam x;
// PQ: the x . y partials of the CG step on the kVecGrid layout (as k_mf_jt_fin).
// 2^lg lanes per row (a lane sums every 2^lg-th term of both series, then a butterfly
// over the group: every lane of it holds the same bits), so the few rows of a small
// system still spread over the whole grid.
// fused search-direction update (k_rec_g FP): the operand rows are p = z + beta p_old,
// written back to p here (after k_rec_g has read p_old), with k_rec_g's rho (st->rho_new)
// and rho1; rho stored in the state
struct FinFuse {
  const double *z = nullptr;  // nullptr: not fused
  DevState *st = nullptr;
  long long it = 0;
  double *p = nullptr;        // = xloc
};

template <bool PQ>
__global__ __launch_bounds__(256) void k_rec_fin(const double *__restrict__ uvk,
                                                 const double *__restrict__ sv,
                                                 const double *__restrict__ rpart, int nblk,
                                                 int64_t MP, int n, int64_t i0, int64_t ni,
                                                 int64_t row0, int64_t nrows, double sigma,
                                                 double lam,
                                                 const double *xloc,  // = ff.p when fused: no restrict
                                                 double *__restrict__ y,
                                                 double *__restrict__ pq_part, int lg,
                                                 const int *__restrict__ status, FinFuse ff) {
  // the status word only gates the stores: tested once the row's loads are issued
  const int st0 = status != nullptr ? *status : ST_RUNNING;
  __shared__ double sh[8];
  const bool fp = ff.z != nullptr, first = ff.it <= 1;
  double beta = 0.0;
  if (fp) {  // rho as k_rec_g summed it, rho1 as its stop test left it: the same beta bits
    const double rho = ff.st->rho_new, rho1 = ff.st->rho1;
    beta = rho / rho1;
    if (st0 == ST_RUNNING && blockIdx.x == 0 && threadIdx.x == 0) ff.st->rho = rho;
  }
  const int64_t n3 = 3 * (int64_t)n, stride = 6 * (int64_t)n + 2, pstride = ni * n3;
  const int G = 1 << lg, sub = threadIdx.x & (G - 1);
  const int64_t pass = (int64_t)gridDim.x * (256 >> lg);
  double pq = 0.0;
  for (int64_t r = ((int64_t)blockIdx.x * 256 + threadIdx.x) >> lg; r < nrows; r += pass) {
    const int64_t g = row0 + r, i = g / n3, t = g - i * n3, il = i - i0, pr = il * n3 + t;
    const double *u = uvk + il * MP * stride + t;
    const double *s = sv + il * MP;
    double acc = 0.0, sl = 0.0;
    int64_t jp = sub;
    for (; jp + 3 * G < MP; jp += 4 * G) {
      double uu[4];
#pragma unroll
      for (int q = 0; q < 4; ++q) uu[q] = u[(jp + q * G) * stride];
#pragma unroll
      for (int q = 0; q < 4; ++q) acc = fma(s[jp + q * G], uu[q], acc);
    }
    for (; jp < MP; jp += G) acc = fma(s[jp], u[jp * stride], acc);
    int q = sub;
    for (; q + 3 * G < nblk; q += 4 * G) {
      double pp[4];
#pragma unroll
      for (int e = 0; e < 4; ++e) pp[e] = rpart[(q + e * G) * pstride + pr];
#pragma unroll
      for (int e = 0; e < 4; ++e) sl += pp[e];
    }
    for (; q < nblk; q += G) sl += rpart[q * pstride + pr];
    double xv = xloc != nullptr ? xloc[r] : 0.0;
    if (fp) xv = fused_p(xv, ff.z[r], beta, first);
    if (st0 != ST_RUNNING) return;  // uniform
    for (int m = G >> 1; m > 0; m >>= 1) {
      acc += __shfl_xor(acc, m, G);
      sl += __shfl_xor(sl, m, G);
    }
    if (sub == 0) {
      double yv = sigma * (acc - sl);
      if (xloc != nullptr) yv += lam * xv;
      y[r] = yv;
      if (fp) ff.p[r] = xv;
      if (PQ) pq = fma(xv, yv, pq);
    }
  }
  if (st0 != ST_RUNNING) return;  // uniform (a block without rows)
  if (PQ) {
    const double t = block_sum256(pq, sh);
    if (threadIdx.x == 0) pq_part[blockIdx.x] = t;
  }
}

// w of the records, transposed for k_rec_g's point-group loads (ldw-long rows, the
// padding zeroed beforehand)
__global__ void k_rec_wt(const double *__restrict__ uvk, int64_t ni, int64_t MP, int n,
                         int64_t ldw, double *__restrict__ wt) {
  const int64_t e = (int64_t)blockIdx.x * 256 + threadIdx.x;
  if (e >= ni * MP) return;
  wt[(e % MP) * ldw + e / MP] = uvk[e * (6 * (int64_t)n + 2) + 6 * n + 1];
}

}  // namespace

int mf_setup(mlff_ctx *ctx, const double *R_desc, const double *R_d_desc, int64_t M, int n_atoms,
             const int32_t *perms, int n_perms, double sig) {
  MfData &mf = ctx->mf;
  mf_free(mf);
  const int n = n_atoms;
  const int64_t D = (int64_t)n * (n - 1) / 2, n3 = 3 * (int64_t)n;
  if (n < 2 || M < 1 || n_perms < 1) return set_error(ctx, MLFF_ERR_ARG, "sgdml operator: bad sizes");
  const bool E = ctx->use_E_cstr;
  if (n3 * M + (E ? M : 0) != ctx->N)
    return set_error(ctx, MLFF_ERR_ARG, E ? "sgdml operator: N != 3 * n_atoms * M + M (use_E_cstr)"
                                          : "sgdml operator: N != 3 * n_atoms * M");
  if (E && ctx->world > 1)
    return set_error(ctx, MLFF_ERR_ARG, "sgdml operator: use_E_cstr runs on one rank");
  std::vector<int32_t> Pt, piinv;
  MLFF_TRY(desc_perm_tables(ctx, perms, n, n_perms, Pt, piinv));
  std::vector<int32_t> ps(D), pt(D);
  for (int a = 1; a < n; ++a)
    for (int b = 0; b < a; ++b) {
      ps[(int64_t)a * (a - 1) / 2 + b] = a;
      pt[(int64_t)a * (a - 1) / 2 + b] = b;
    }
  if (M * n_perms > 65535 || M > 65535)  // grid y / z extents of the pair and J^T kernels
    return set_error(ctx, MLFF_ERR_ARG, "sgdml operator: M * n_perms > 65535 is not supported");
  mf.M = M;
  mf.n = n;
  mf.D = D;
  mf.n_perms = n_perms;
  mf.sig = sig;
  mf.i0 = ctx->row0 / n3;
  mf.ni = ctx->nrows > 0 ? std::min<int64_t>((ctx->row0 + ctx->nrows + n3 - 1) / n3, M) - mf.i0 : 0;
  mf.E = E;
  mf.nF = n3 * M;
  const int64_t MP = M * n_perms;
  const int64_t nic = std::max<int64_t>(mf.ni, 1);
  hipStream_t s = ctx->stream;
  MLFF_HIP(ctx, hipMalloc(&mf.Rd, sizeof(double) * M * D));
  MLFF_HIP(ctx, hipMalloc(&mf.Rdd, sizeof(double) * M * D * 3));
  MLFF_HIP(ctx, hipMalloc(&mf.Rt, sizeof(double) * MP * D));
  MLFF_HIP(ctx, hipMalloc(&mf.Zt, sizeof(double) * MP * D));
  MLFF_HIP(ctx, hipMalloc(&mf.Pt, sizeof(int32_t) * n_perms * D));
  MLFF_HIP(ctx, hipMalloc(&mf.ps, sizeof(int32_t) * D));
  MLFF_HIP(ctx, hipMalloc(&mf.pt, sizeof(int32_t) * D));
  MLFF_HIP(ctx, hipMalloc(&mf.m5, sizeof(double) * nic * MP));
  MLFF_HIP(ctx, hipMalloc(&mf.w, sizeof(double) * nic * MP));
  MLFF_HIP(ctx, hipMalloc(&mf.c, sizeof(double) * nic * MP));
  MLFF_HIP(ctx, hipMalloc(&mf.F, sizeof(double) * nic * D));
  if (ctx->world > 1) MLFF_HIP(ctx, hipMalloc(&mf.xc, sizeof(double) * ctx->N));
  MLFF_HIP(ctx, hipMalloc(&mf.ypart, sizeof(double) * kJSMax * std::max<int64_t>(ctx->nrows, 1)));
  MLFF_HIP(ctx, hipMemcpyAsync(mf.Rd, R_desc, sizeof(double) * M * D, hipMemcpyHostToDevice, s));
  MLFF_HIP(ctx, hipMemcpyAsync(mf.Rdd, R_d_desc, sizeof(double) * M * D * 3, hipMemcpyHostToDevice, s));
  MLFF_HIP(ctx, hipMemcpyAsync(mf.Pt, Pt.data(), sizeof(int32_t) * n_perms * D, hipMemcpyHostToDevice, s));
  MLFF_HIP(ctx, hipMemcpyAsync(mf.ps, ps.data(), sizeof(int32_t) * D, hipMemcpyHostToDevice, s));
  MLFF_HIP(ctx, hipMemcpyAsync(mf.pt, pt.data(), sizeof(int32_t) * D, hipMemcpyHostToDevice, s));
  mf.perms.assign(perms, perms + (size_t)n_perms * n);
  mf.ident = n_perms == 1;
  for (int a = 0; a < n && mf.ident; ++a) mf.ident = perms[a] == a;
  mf.piinv = piinv;
  const unsigned gx = (unsigned)std::min<int64_t>((D + 255) / 256, 1024);
  hipLaunchKernelGGL(k_mf_rt, dim3(gx, (unsigned)MP), dim3(256), 0, s, mf.Rd, mf.Pt, M, n_perms, D,
                     mf.Rt);
  // descriptor slices of the pair sums: enough workgroups to cover the chip in ONE round
  // of resident workgroups (k_mf_pair: 96 VGPRs, 5 waves per SIMD = 5 workgroups per CU;
  // at 4 per CU the nanotube's 1067 slices ran as 1024 + a second round of 43)
  const int64_t tiles = ((MP + kPT - 1) / kPT) * ((mf.ni + kPT - 1) / kPT);
  int64_t nz = (5 * 256 + tiles - 1) / std::max<int64_t>(tiles, 1);
  nz = std::max<int64_t>(1, std::min<int64_t>(nz, (D + kDC - 1) / kDC));
  mf.dslice = round_up((D + nz - 1) / nz, kDC);
  mf.nz = (int)((D + mf.dslice - 1) / mf.dslice);
  nz = mf.nz;
  MLFF_HIP(ctx, hipMalloc(&mf.part, sizeof(double) * nz * nic * MP));
  // operator form: the pair-tile one where it exists (few atoms), else the record-factored one
  // where the records fit, else the pair sums; MLFF_MF_FORM=pt|rec|pair asks for one (A/B, tests).
  // Decided from the sizes every rank shares (not the local point count), so that the ranks of
  // a sharded operator model the same form (mf_seconds, resolve_storage); a rank without
  // points allocates nothing for it
  const char *ef = std::getenv("MLFF_MF_FORM");
  const std::string form = ef != nullptr ? ef : "";
  if ((form.empty() || form == "pt") && !E && pt_supported(D)) {
    mf.ptile = true;
    if (mf.ni > 0) {
      mf.pt_S = pt_chunks(D, mf.ni, MP);
      MLFF_HIP(ctx, hipMalloc(&mf.ptpart, sizeof(double) * mf.pt_S * mf.ni * pt_padded_d(D)));
    }
  }
  // single-column path: the (r = i, s = j) pair records of the local points (3.5 MB for
  // the nanotube, M = 14; ni M n_perms (6 n + 2) doubles in general)
  const double col_bytes = 8.0 * (double)mf.ni * (double)MP * (double)(6 * n + 2);
  if (E) {  // energy tables; columns go through the whole operator (K_op e_g)
    MLFF_HIP(ctx, hipMalloc(&mf.kee, sizeof(double) * nic * M));
    MLFF_HIP(ctx, hipMalloc(&mf.eterm, sizeof(double) * nic * MP));
    launch_sgdml_kee(mf.Rd, M, D, mf.i0, mf.ni, mf.Pt, n_perms, sig, mf.kee, s);
  } else if (mf.ni > 0 && col_bytes <= col_table_cap()) {
    MLFF_HIP(ctx, hipMalloc(&mf.uvk, (size_t)col_bytes));
    MLFF_HIP(ctx, hipMalloc(&mf.pi_d, sizeof(int32_t) * n_perms * n));
    MLFF_HIP(ctx, hipMalloc(&mf.piinv_d, sizeof(int32_t) * n_perms * n));
    MLFF_HIP(ctx, hipMemcpyAsync(mf.pi_d, perms, sizeof(int32_t) * n_perms * n, hipMemcpyHostToDevice, s));
    MLFF_HIP(ctx, hipMemcpyAsync(mf.piinv_d, piinv.data(), sizeof(int32_t) * n_perms * n,
                                 hipMemcpyHostToDevice, s));
    launch_sgdml_records(mf.Rd, mf.Rdd, M, n, D, mf.i0, mf.ni, mf.Pt, mf.piinv_d, n_perms, sig,
                         mf.uvk, s);
    // the record-factored operator (MLFF_MF_REC=0: the five-kernel pair/F/J^T path); its
    // tables only where that form runs (not under the pair-tile form or MLFF_MF_FORM=pair)
    const char *ev = std::getenv("MLFF_MF_REC");
    if ((ev == nullptr || std::atoi(ev) != 0) && !mf.ptile && form != "pair") {
      mf.rblk = (n + kRB - 1) / kRB;
      mf.ldw = round_up(mf.ni, kRG);
      const int64_t wrows = round_up(MP, kRJ);
      MLFF_HIP(ctx, hipMalloc(&mf.wt, sizeof(double) * wrows * mf.ldw));
      MLFF_HIP(ctx, hipMemsetAsync(mf.wt, 0, sizeof(double) * wrows * mf.ldw, s));
      MLFF_HIP(ctx, hipMalloc(&mf.sv, sizeof(double) * MP * mf.ni));
      MLFF_HIP(ctx, hipMalloc(&mf.rpart, sizeof(double) * mf.rblk * mf.ni * n3));
      hipLaunchKernelGGL(k_rec_wt, dim3((unsigned)((mf.ni * MP + 255) / 256)), dim3(256), 0, s,
                         mf.uvk, mf.ni, MP, n, mf.ldw, mf.wt);
      mf.rec = true;
      const char *e3 = std::getenv("MLFF_REC_RG");
      mf.rec_rg = e3 != nullptr ? std::atoi(e3) : 8;
      const char *e4 = std::getenv("MLFF_REC_WC16");
      mf.rec_wc16 = e4 == nullptr || std::atoi(e4) != 0;
    }
  }
  if (mf.ni > 0) {
    hipLaunchKernelGGL(k_mf_pair<0>, dim3((unsigned)((MP + kPT - 1) / kPT),
                       (unsigned)((mf.ni + kPT - 1) / kPT), (unsigned)nz), dim3(256), 0,
                       s, mf.Rd, mf.Rt, (const double *)nullptr, D, mf.dslice, mf.i0, mf.ni, MP,
                       mf.part, (const int *)nullptr);
    hipLaunchKernelGGL(k_mf_pair_fin<0>, dim3((unsigned)((mf.ni * MP + 3) / 4)), dim3(256), 0,
                       s, mf.part, mf.nz, mf.ni * MP, sig, (const double *)nullptr, mf.m5, mf.w,
                       (const int *)nullptr);
  }
  MLFF_HIP(ctx, hipGetLastError());
  MLFF_HIP(ctx, hipStreamSynchronize(s));
  mf.ready = true;
  return MLFF_OK;
}

// the fused p update: one rank holding every row, in the pair-tile form (few atoms) or in the
// default record-factored form with one identity permutation, <= 16 local points, w in one
// 16-slot chunk (the nanotube configs[1] system)
bool mf_can_fuse_p(const mlff_ctx *ctx) {
  const MfData &mf = ctx->mf;
  if (!ctx->fuse_p || ctx->world != 1 || mf.ni <= 0 || ctx->nrows != ctx->N) return false;
  // the pair-tile form: k_mf_z forms p, k_pt_fin writes it (any permutation set)
  if (mf.ptile) return !mf.E;
  return mf.rec && mf.ident && mf.ni <= kRG &&
         mf.rec_rg == 8 && round_up(mf.M * mf.n_perms, kRJ) <= 16 && mf.rec_wc16 &&
         ctx->nrows == ctx->N;
}

void launch_mf_operator(const mlff_ctx *ctx, const double *x_full, double *y_loc,
                        const double *x_loc, const int *status, double sigma, double lam,
                        double *pq_part, const PFuse *pf) {
  const MfData &mf = ctx->mf;
  hipStream_t s = ctx->stream;
  const int64_t MP = mf.M * mf.n_perms;
  const int js = mf_jt_slices(mf.n);
  // on one rank the padded layout is the global index itself (rows_per = N)
  const double *xc = x_full;
  if (ctx->world > 1) {
    hipLaunchKernelGGL(k_mf_contig, dim3((unsigned)((ctx->N + 255) / 256)), dim3(256), 0, s, x_full,
                       ctx->N, ctx->rows_per, ctx->blk, mf.xc, status);
    xc = mf.xc;
  }
  if (mf.ni == 0) {  // no points here: Zt is not needed either
    if (pq_part != nullptr)  // zero partials of an empty shard
      hipLaunchKernelGGL(k_mf_jt_fin<true>, dim3(kVecGrid), dim3(256), 0, s, mf.ypart, js,
                         (int64_t)0, sigma, lam, x_loc, y_loc, pq_part, status);
    return;
  }
  if (mf.ptile) {
    launch_pt_operator(mf, mf.ident ? mf.Rd : mf.Rt, xc, ctx->row0, ctx->nrows, x_loc, y_loc, status,
                       sigma, lam, pq_part, s, pf);
    return;
  }
#ifdef MLFF_REC_TRACE
  static int rec_launches = 0;
#endif
  if (mf.rec) {
    RecArgs ra{mf.Rdd, mf.Zt, xc, mf.Pt, mf.ps, mf.pt, mf.uvk, mf.M, mf.D, mf.i0, mf.ni,
               MP, mf.ldw, (int)mf.n, (int)mf.n_perms, mf.rblk, mf.rpart, mf.sv};
    FinFuse ff;
    if (pf != nullptr) {  // mf_can_fuse_p(ctx) holds (the caller checked)
      ra.pz = pf->z;
      ra.rho_part = pf->rho_part;
      ra.st = pf->st;
      ra.it = pf->it;
      ra.sf = pf->sf;
      ff = FinFuse{pf->z, pf->st, pf->it, const_cast<double *>(x_loc)};
    }
    const int64_t nbp = (int64_t)mf.rblk * (mf.rblk + 1) / 2, ngrp = (mf.ni + kRG - 1) / kRG;
    const int64_t nbp8 = (nbp + 7) / 8 * 8, nsw8 = (mf.ni * MP + 31) / 32 * 8;
    const dim3 grid((unsigned)(nsw8 + nbp8 * ngrp));
    const double *wt = mf.wt;
    if (ngrp > 1) {  // Zt once (k_mf_z), read by every point group
      const unsigned gx = (unsigned)std::min<int64_t>((mf.D + 255) / 256, 1024);
      hipLaunchKernelGGL(k_mf_z<false>, dim3(gx, (unsigned)MP), dim3(256), 0, s, mf.Rdd,
                         mf.ident ? (const int32_t *)nullptr : (const int32_t *)mf.Pt, mf.ps, mf.pt,
                         mf.M, (int)mf.n, (int)mf.n_perms, mf.D, xc, mf.Zt, status, PFuse{});
      hipLaunchKernelGGL(k_rec_g<kZStored>, grid, dim3(256), 0, s, ra, wt, nbp, ngrp, nsw8, status);
    } else if (mf.ident) {
      if (mf.rec_rg == 8 || mf.rec_rg == 4) {
        // smaller point groups per pair block: more waves (the kernel is latency-bound, with
        // ~1.4 workgroups per CU at 16 points), 4-point epilogue rounds (a third of the LDS),
        // the query points' rows re-read from L2 (registers for 3-4 waves per SIMD)
        const int64_t ng = (mf.ni + mf.rec_rg - 1) / mf.rec_rg;
        const dim3 gridg((unsigned)(nsw8 + nbp8 * ng));
        if (pf != nullptr)  // one 16-slot chunk, the p update fused
          hipLaunchKernelGGL((k_rec_g<kZIdent, false, 8, 4, 16, true>), gridg, dim3(256), 0, s, ra, wt,
                             nbp, ng, nsw8, status);
        else if (mf.rec_rg == 8 && round_up(MP, kRJ) <= 16 && mf.rec_wc16)  // one 16-slot chunk
          hipLaunchKernelGGL((k_rec_g<kZIdent, false, 8, 4, 16>), gridg, dim3(256), 0, s, ra, wt, nbp,
                             ng, nsw8, status);
        else if (mf.rec_rg == 8)
          hipLaunchKernelGGL((k_rec_g<kZIdent, false, 8, 4>), gridg, dim3(256), 0, s, ra, wt, nbp,
                             ng, nsw8, status);
        else
          hipLaunchKernelGGL((k_rec_g<kZIdent, false, 4, 4>), gridg, dim3(256), 0, s, ra, wt, nbp,
                             ng, nsw8, status);
      } else {  // 16-point groups, rows captured from the Zt batches (MLFF_REC_RG=16)
        hipLaunchKernelGGL(k_rec_g<kZIdent>, grid, dim3(256), 0, s, ra, wt, nbp, ngrp, nsw8, status);
      }
    } else {
      hipLaunchKernelGGL(k_rec_g<kZGather>, grid, dim3(256), 0, s, ra, wt, nbp, ngrp, nsw8, status);
    }
#ifdef MLFF_REC_TRACE
    static const int trace_at = [] {
      const char *e = std::getenv("MLFF_REC_TRACE_AT");
      return e ? std::atoi(e) : 20;
    }();
    if (++rec_launches == trace_at) {  // after the build and warmup: one application's phases
      static unsigned long long h[8192][5];
      (void)hipStreamSynchronize(s);
      (void)hipMemcpyFromSymbol(h, HIP_SYMBOL(g_rec_trace), sizeof(h));
      if (const char *fn = std::getenv("MLFF_REC_TRACE_FILE")) {
        if (FILE *f = std::fopen(fn, "w")) {
          for (int i = 0; i < 8192; ++i)
            if (h[i][0] != 0)
              std::fprintf(f, "%d %llu %llu %llu %llu %llu\n", i, h[i][0], h[i][1], h[i][2], h[i][3], h[i][4]);
          std::fclose(f);
        }
      }
    }
#endif
    // lanes per row: fill the finisher's grid (kVecGrid workgroups with the p.q partials)
    int lg = 0;
    const int64_t threads = (pq_part != nullptr ? (int64_t)kVecGrid : 1024) * 256;
    while (lg < 4 && ctx->nrows * (2LL << lg) <= threads) ++lg;
    if (pq_part != nullptr) {
      hipLaunchKernelGGL(k_rec_fin<true>, dim3(kVecGrid), dim3(256), 0, s, mf.uvk, mf.sv, mf.rpart,
                         mf.rblk, MP, (int)mf.n, mf.i0, mf.ni, ctx->row0, ctx->nrows, sigma, lam,
                         x_loc, y_loc, pq_part, lg, status, ff);
    } else if (ctx->nrows > 0) {
      const int64_t nb = std::min<int64_t>((ctx->nrows << lg) / 256 + 1, 1024);
      hipLaunchKernelGGL(k_rec_fin<false>, dim3((unsigned)nb), dim3(256), 0, s, mf.uvk, mf.sv,
                         mf.rpart, mf.rblk, MP, (int)mf.n, mf.i0, mf.ni, ctx->row0, ctx->nrows,
                         sigma, lam, x_loc, y_loc, (double *)nullptr, lg, status, FinFuse{});
    }
    return;
  }
  const unsigned gi = (unsigned)((mf.ni + kIC - 1) / kIC);
  // identity permutation: Rt is Rd (same bits), read from the same lines, and the
  // descriptor map is skipped in the Zt gathers (one dependent load less)
  const double *Rt = mf.ident ? mf.Rd : mf.Rt;
  const ZSrc zs{mf.Rdd, mf.ident ? nullptr : mf.Pt, mf.ps, mf.pt, (int)mf.n, (int)mf.n_perms, xc,
                mf.Zt};
  hipLaunchKernelGGL((k_mf_pair<1, true>), dim3((unsigned)((MP + kPT - 1) / kPT),
                     (unsigned)((mf.ni + kPT - 1) / kPT), (unsigned)mf.nz), dim3(256), 0, s,
                     mf.Rd, Rt, (const double *)nullptr, mf.D, mf.dslice, mf.i0, mf.ni, MP,
                     mf.part, status, zs);
  EPair ep;
  ERows er;
  if (mf.E) {  // one rank: the operand's energy entries follow its nF force entries
    ep = EPair{xc + mf.nF, mf.w, mf.eterm, MP, (int)mf.n_perms};
    er = ERows{mf.nF, mf.eterm, mf.kee, xc + mf.nF, mf.M, MP};
  }
  hipLaunchKernelGGL(k_mf_pair_fin<1>, dim3((unsigned)((mf.ni * MP + 3) / 4)), dim3(256), 0, s,
                     mf.part, mf.nz, mf.ni * MP, mf.sig, mf.m5, mf.c, (double *)nullptr, status, ep);
  const int64_t dblk = (mf.D + 63) / 64, dblk8 = (dblk + 7) / 8 * 8;
  if (dblk * (int64_t)gi >= 4096) {
    hipLaunchKernelGGL(k_mf_h<kIC>, dim3((unsigned)(dblk8 * gi)), dim3(64), 0, s, mf.Rd, Rt,
                       mf.Zt, mf.D, mf.i0, mf.ni, MP, mf.c, mf.w, mf.F, status);
  } else {
    hipLaunchKernelGGL(k_mf_h<4>, dim3((unsigned)(dblk8 * ((mf.ni + 3) / 4))), dim3(64), 0, s,
                       mf.Rd, Rt, mf.Zt, mf.D, mf.i0, mf.ni, MP, mf.c, mf.w, mf.F, status);
  }
  {
    const int64_t total = (int64_t)((mf.n + kAB - 1) / kAB) * mf.ni * js;
    hipLaunchKernelGGL(k_mf_jt, dim3((unsigned)((total + 7) / 8 * 8)), dim3(256), 0, s, mf.Rdd,
                       mf.F, mf.D, (int)mf.n, mf.i0, mf.ni, js, ctx->row0, ctx->nrows, mf.ypart,
                       status);
  }
  if (pq_part != nullptr) {
    hipLaunchKernelGGL(k_mf_jt_fin<true>, dim3(kVecGrid), dim3(256), 0, s, mf.ypart, js, ctx->nrows,
                       sigma, lam, x_loc, y_loc, pq_part, status, er);
    return;
  }
  if (ctx->nrows <= 0) return;
  hipLaunchKernelGGL(k_mf_jt_fin<false>, dim3((unsigned)((ctx->nrows + 255) / 256)), dim3(256), 0,
                     s, mf.ypart, js, ctx->nrows, sigma, lam, x_loc, y_loc, (double *)nullptr, status,
                     er);
}

// Training-set energies of the model with coefficients `alphas` (contiguous global
// vector, N), as GDMLPredict predicts them (predict.py:172-220, E_F[0] before the std
// scale, flipped sign as in the reference): E_i = sum_jp (Rd_i - Rt[jp]) . Zt[jp] w_ijp
// with Zt = J alphas.  Points [mf.i0, mf.i0 + mf.ni) of this rank; per-pair products in
// E_pairs (ni x M n_perms, host), summed by the caller in pair order.
int mf_energies(mlff_ctx *ctx, const double *alphas, double *E_pairs_host) {
  MfData &mf = ctx->mf;
  if (mf.E) return set_error(ctx, MLFF_ERR_STATE, "sgdml_energies: not with use_E_cstr");
  hipStream_t s = ctx->stream;
  const int64_t MP = mf.M * mf.n_perms;
  double *da = nullptr;
  MLFF_HIP(ctx, hipMalloc(&da, sizeof(double) * ctx->N));
  MLFF_HIP(ctx, hipMemcpyAsync(da, alphas, sizeof(double) * ctx->N, hipMemcpyHostToDevice, s));
  const unsigned gx = (unsigned)std::min<int64_t>((mf.D + 255) / 256, 1024);
  hipLaunchKernelGGL(k_mf_z<false>, dim3(gx, (unsigned)MP), dim3(256), 0, s, mf.Rdd, mf.Pt, mf.ps, mf.pt,
                     mf.M, mf.n, mf.n_perms, mf.D, da, mf.Zt, (const int *)nullptr, PFuse{});
  if (mf.ni > 0) {
    hipLaunchKernelGGL(k_mf_pair<1>, dim3((unsigned)((MP + kPT - 1) / kPT),
                       (unsigned)((mf.ni + kPT - 1) / kPT), (unsigned)mf.nz), dim3(256), 0, s,
                       mf.Rd, mf.Rt, mf.Zt, mf.D, mf.dslice, mf.i0, mf.ni, MP, mf.part,
                       (const int *)nullptr);
    hipLaunchKernelGGL(k_mf_pair_fin<2>, dim3((unsigned)((mf.ni * MP + 3) / 4)), dim3(256), 0, s,
                       mf.part, mf.nz, mf.ni * MP, mf.sig, mf.w, mf.c, (double *)nullptr,
                       (const int *)nullptr);
    MLFF_HIP(ctx, hipMemcpyAsync(E_pairs_host, mf.c, sizeof(double) * mf.ni * MP,
                                 hipMemcpyDeviceToHost, s));
  }
  MLFF_HIP(ctx, hipGetLastError());
  MLFF_HIP(ctx, hipStreamSynchronize(s));
  hipFree(da);
  return MLFF_OK;
}

// diag(sigma K) of this rank's rows (assembly kernels on the diagonal blocks only)
int mf_diag(mlff_ctx *ctx, double *out) {
  MfData &mf = ctx->mf;
  MLFF_TRY(sgdml_diag(ctx, mf.Rd, mf.Rdd, mf.M, mf.n, mf.Pt, mf.perms.data(), mf.piinv.data(),
                      mf.n_perms, mf.sig, out));
  if (mf.E)  // K[E_i, E_i] = -kee[i, i] (one rank)
    hipLaunchKernelGGL(k_mf_ediag, dim3((unsigned)((mf.M + 255) / 256)), dim3(256), 0, ctx->stream,
                       mf.kee, mf.M, out + mf.nF);
  if (ctx->nrows > 0) launch_scale_copy(out, out, ctx->nrows, ctx->sigma_K, ctx->stream);
  MLFF_HIP(ctx, hipGetLastError());
  return MLFF_OK;
}

bool mf_columns(const mlff_ctx *ctx, const int64_t *cols, int64_t ncols, double sigma,
                double *out, int64_t ldo) {
  const MfData &mf = ctx->mf;
  if (mf.uvk == nullptr) return ctx->nrows == 0 && mf.ready;  // an empty shard has no rows
  launch_sgdml_columns(mf.Rdd, mf.M, mf.n, mf.D, mf.i0, mf.pi_d, mf.piinv_d, mf.n_perms, mf.uvk,
                       ctx->row0, ctx->nrows, cols, ncols, ctx->st, sigma, out, ldo, ctx->stream);
  return true;
}

void launch_mf_zt(const MfData &mf, const double *xc, const int *status, hipStream_t s,
                  const PFuse *pf) {
  const int64_t MP = mf.M * mf.n_perms;
  const int32_t *Pt = mf.ident ? (const int32_t *)nullptr : (const int32_t *)mf.Pt;
  // D <= 128: several (j, p) rows per workgroup (ethanol D = 36: 7), else a row per grid row
  const int rows = mf.D <= 128 ? (int)(256 / mf.D) : 1;
  const dim3 grid = rows > 1 ? dim3((unsigned)((MP + rows - 1) / rows))
                             : dim3((unsigned)std::min<int64_t>((mf.D + 255) / 256, 1024), (unsigned)MP);
  if (pf != nullptr)
    hipLaunchKernelGGL(k_mf_z<true>, grid, dim3(256), 0, s, mf.Rdd, Pt, mf.ps, mf.pt, mf.M, (int)mf.n,
                       (int)mf.n_perms, mf.D, xc, mf.Zt, status, *pf, rows);
  else
    hipLaunchKernelGGL(k_mf_z<false>, grid, dim3(256), 0, s, mf.Rdd, Pt, mf.ps, mf.pt, mf.M, (int)mf.n,
                       (int)mf.n_perms, mf.D, xc, mf.Zt, status, PFuse{}, rows);
}

double mf_seconds(const mlff_ctx *ctx) {
  const MfData &mf = ctx->mf;
  if (mf.ptile) {  // fp64-vector bound: ~40 TFLOP/s of 9 D + 8 flops per pair + 3 launches
    const double pairs = (double)mf.ni * (double)(mf.M * mf.n_perms);
    return 10e-6 + pairs * (9.0 * (double)mf.D + 8.0) / 40e12;
  }
  // latency-bound streams: the record-factored form (2 launches) at ~1.4 TB/s of its
  // algorithmic bytes (nanotube 32.8 MB in 23 us), the pair sums (5 launches) at ~0.5 TB/s
  return mf.rec ? 10e-6 + mf_bytes(ctx) / 1.4e12 : 20e-6 + mf_bytes(ctx) / 0.5e12;
}

int mf_form(const mlff_ctx *ctx) { return ctx->mf.ptile ? 2 : ctx->mf.rec ? 1 : 0; }

double mf_bytes(const mlff_ctx *ctx) {
  const MfData &mf = ctx->mf;
  const double MP = (double)(mf.M * mf.n_perms), D = (double)mf.D;
  if (mf.ptile) {
    // Zt formed from Rdd and x and written; Rt, Zt read (once: the point blocks re-read them
    // from L2); the local points' Rd and Rdd rows; the chunk partials written and read; the
    // operand, the rows and the result.  The kernel is bound by the fp64 vector pipe, not by
    // these bytes
    const double ni = (double)mf.ni, DP = (double)pt_padded_d(mf.D);
    return 8.0 * (3.0 * (double)mf.M * D + 3.0 * MP * D + 4.0 * ni * D +
                  2.0 * mf.pt_S * ni * DP + (double)ctx->N + 2.0 * ctx->nrows);
  }
  if (mf.rec) {
    // Rdd of every point once per point group (Zt on the fly; the query points' own rows
    // are the same lines), the u and v halves of the records, the slot partials written
    // and read, s, the operand and the result
    const double ngrp = (double)((mf.ni + kRG - 1) / kRG), ni = (double)mf.ni;
    const double n3 = 3.0 * mf.n;
    // one point group: Zt formed on the fly from Rdd; several: Zt written once by k_mf_z
    // and read by every group, the groups' own Rdd rows read by their J^T step
    const double zt = ngrp > 1 ? 3.0 * (double)mf.M * D + MP * D * (1.0 + ngrp) + 3.0 * ni * D
                               : 3.0 * (double)mf.M * D;
    return 8.0 * (zt + ni * MP * (2.0 * n3 + 2.0) + 2.0 * mf.rblk * ni * n3 + 2.0 * ni * MP +
                  (double)ctx->N + 2.0 * ctx->nrows);
  }
  const double chunks = (double)((mf.ni + kIC - 1) / kIC);
  // Zt written once; Rt, Zt read by every point chunk in two kernels; Rd, Rdd, F
  return 8.0 * (MP * D * (1.0 + 4.0 * chunks) + (double)mf.ni * D * 6.0 + 16.0 * ctx->nrows);
}

void mf_free(MfData &mf) {
  for (void *p : {(void *)mf.Rd, (void *)mf.Rdd, (void *)mf.Rt, (void *)mf.Zt, (void *)mf.Pt,
                  (void *)mf.ps, (void *)mf.pt, (void *)mf.m5, (void *)mf.w, (void *)mf.c,
                  (void *)mf.F, (void *)mf.part, (void *)mf.ypart, (void *)mf.xc,
                  (void *)mf.uvk, (void *)mf.pi_d, (void *)mf.piinv_d, (void *)mf.kee,
                  (void *)mf.eterm, (void *)mf.wt, (void *)mf.sv, (void *)mf.rpart,
                  (void *)mf.ptpart})
    if (p) (void)hipFree(p);
  mf = MfData();
}

}  // namespace mlff
