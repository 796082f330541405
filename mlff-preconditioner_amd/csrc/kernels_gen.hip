// On-device kernel-matrix generation.
//  - synthetic RBF kernel (tools/utils.py:173-187, sklearn RBF: exp(-0.5 * sqeuclidean(X/l)))
//  - sGDML Matern-5/2 Hessian kernel (train.py:81-236 worker, 1121-1308 driver)
//  - sGDML inverse-distance descriptors (utils/desc.py:80-234)
// Column positions use the padded rank-block layout of the context:
//   pos(g) = (g / rows_per) * blk + g % rows_per.
#include "common.h"
#include "sgdml_col.h"

namespace mlff {

__device__ __forceinline__ int64_t col_pos(int64_t g, int64_t rows_per, int64_t blk) {
  return (g / rows_per) * blk + (g % rows_per);
}

// ---------------------------------------------------------------------------
// K[i, pos(g)] = exp(-0.5 * sum_d (xs_i - xs_g)^2), diag = 1 + jitter.  The squared
// distance is formed without FMA contraction (scipy pdist 'sqeuclidean' order).
__global__ __launch_bounds__(256) void k_gen_rbf(double *__restrict__ K, int64_t ld,
                                                 int64_t nrows, int64_t row0, int64_t rows_per,
                                                 int64_t blk, int64_t N,
                                                 const double *__restrict__ Xs, int d,
                                                 double jitter) {
  const int64_t i = blockIdx.y;
  if (i >= nrows) return;
  const int64_t gi = row0 + i;
  double xi[8];
#pragma unroll
  for (int t = 0; t < 8; ++t) xi[t] = (t < d) ? Xs[gi * d + t] : 0.0;
  double *row = K + i * ld;
  for (int64_t pos = (int64_t)blockIdx.x * 256 + threadIdx.x; pos < ld;
       pos += (int64_t)gridDim.x * 256) {
    const int64_t rk = pos / blk, off = pos % blk;
    const int64_t g = rk * rows_per + off;
    double val = 0.0;
    if (off < rows_per && g < N) val = (g == gi) ? 1.0 + jitter : rbf_value(xi, Xs, g, d);
    __builtin_nontemporal_store(val, row + pos);
  }
}

// columns of the RBF kernel for the local rows (the Nystrom / pivoted-Cholesky column
// fetch of the RBF source): out[jc * ldo + r] = sigma K[row0 + r, g_jc]
__global__ __launch_bounds__(256) void k_rbf_cols(const double *__restrict__ Xs, int d,
                                                  double jitter, int64_t row0, int64_t nrows,
                                                  const int64_t *__restrict__ cols,
                                                  const DevState *__restrict__ st, double sigma,
                                                  double *__restrict__ out, int64_t ldo) {
  const int64_t g = cols != nullptr ? cols[blockIdx.y] : (int64_t)st->m_pi;
  if (g < 0) return;
  double xg[8];
#pragma unroll
  for (int t = 0; t < 8; ++t) xg[t] = (t < d) ? Xs[g * d + t] : 0.0;
  double *o = out + (int64_t)blockIdx.y * ldo;
  for (int64_t r = (int64_t)blockIdx.x * 256 + threadIdx.x; r < nrows;
       r += (int64_t)gridDim.x * 256) {
    const int64_t gi = row0 + r;
    // K[gi, g] = K[g, gi]: evaluated with the column point first, as the tiles store it
    // for gi > g and the rows for g > gi -- the same bits either way
    o[r] = sigma * ((gi == g) ? 1.0 + jitter : rbf_value(xg, Xs, gi, d));
  }
}

void launch_rbf_cols(const RbfData &rbf, int64_t N, int64_t row0, int64_t nrows,
                     const int64_t *cols, int64_t ncols, const DevState *st, double sigma,
                     double *out, int64_t ldo, hipStream_t s) {
  (void)N;
  if (nrows <= 0 || ncols <= 0) return;
  const unsigned gx = (unsigned)std::min<int64_t>((nrows + 255) / 256, 64);
  hipLaunchKernelGGL(k_rbf_cols, dim3(gx, (unsigned)ncols), dim3(256), 0, s, rbf.Xs, rbf.d,
                     rbf.jitter, row0, nrows, cols, st, sigma, out, ldo);
}

__global__ void k_fill(double *__restrict__ y, int64_t n, double v) {
  for (int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x; i < n; i += (int64_t)gridDim.x * 256)
    y[i] = v;
}

void launch_fill(double *y, int64_t n, double v, hipStream_t s) {
  if (n <= 0) return;
  hipLaunchKernelGGL(k_fill, dim3((unsigned)std::min<int64_t>((n + 255) / 256, 1024)), dim3(256), 0, s,
                     y, n, v);
}

void launch_gen_rbf(double *K, int64_t ld, int64_t nrows, int64_t row0, int64_t rows_per,
                    int64_t blk, int64_t N, const double *Xs, int d, double jitter,
                    hipStream_t s) {
  if (nrows <= 0) return;
  const unsigned gx = (unsigned)std::min<int64_t>((ld + 255) / 256, 16);
  hipLaunchKernelGGL(k_gen_rbf, dim3(gx, (unsigned)nrows), dim3(256), 0, s, K, ld, nrows, row0,
                     rows_per, blk, N, Xs, d, jitter);
}

__global__ void k_diag_of(const double *__restrict__ K, int64_t ld, int64_t nrows, int64_t row0,
                          int64_t rows_per, int64_t blk, double sigma, double *__restrict__ out) {
  const int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x;
  if (i >= nrows) return;
  out[i] = sigma * K[i * ld + col_pos(row0 + i, rows_per, blk)];
}

void launch_diag_of(const double *K, int64_t ld, int64_t nrows, int64_t row0, int64_t rows_per,
                    int64_t blk, double sigma, double *out, hipStream_t s) {
  if (nrows <= 0) return;
  hipLaunchKernelGGL(k_diag_of, dim3((unsigned)((nrows + 255) / 256)), dim3(256), 0, s, K, ld,
                     nrows, row0, rows_per, blk, sigma, out);
}

// W[j, i] = sigma * K[i, pos(idx_j)] for local rows i (the column panel K[:, idx]
// transposed; by symmetry of K these are the rows idx of S = sigma K).
__global__ __launch_bounds__(256) void k_gather_cols(const double *__restrict__ K, int64_t ld,
                                                     int64_t nrows,
                                                     const int64_t *__restrict__ idx, int64_t k,
                                                     int64_t rows_per, int64_t blk, double sigma,
                                                     double *__restrict__ W, int64_t ldw) {
  const int64_t j = blockIdx.y;
  const int64_t pos = col_pos(idx[j], rows_per, blk);
  for (int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x; i < nrows;
       i += (int64_t)gridDim.x * 256)
    W[j * ldw + i] = sigma * K[i * ld + pos];
}

void launch_gather_cols(const double *K, int64_t ld, int64_t nrows, const int64_t *idx,
                        int64_t k, int64_t rows_per, int64_t blk, double sigma, double *W,
                        int64_t ldw, hipStream_t s) {
  if (nrows <= 0) return;
  const unsigned gx = (unsigned)std::min<int64_t>((nrows + 255) / 256, 64);
  hipLaunchKernelGGL(k_gather_cols, dim3(gx, (unsigned)k), dim3(256), 0, s, K, ld, nrows, idx, k,
                     rows_per, blk, sigma, W, ldw);
}

__global__ void k_gather_mm(const double *__restrict__ W, int64_t ldw,
                            const int64_t *__restrict__ idx, int64_t k, int64_t row0,
                            int64_t nrows, double *__restrict__ Smm) {
  const int64_t e = (int64_t)blockIdx.x * 256 + threadIdx.x;
  if (e >= k * k) return;
  const int64_t j = e / k, jj = e % k;
  const int64_t g = idx[jj] - row0;
  Smm[e] = (g >= 0 && g < nrows) ? W[j * ldw + g] : 0.0;
}

void launch_gather_mm(const double *W, int64_t ldw, const int64_t *idx, int64_t k, int64_t row0,
                      int64_t nrows, double *Smm, hipStream_t s) {
  hipLaunchKernelGGL(k_gather_mm, dim3((unsigned)((k * k + 255) / 256)), dim3(256), 0, s, W, ldw,
                     idx, k, row0, nrows, Smm);
}

// ---------------------------------------------------------------------------
// sGDML kernel assembly.
//
// For training points i (rows) and j (columns), permutation p with atom map pi
// (descriptor map P_p[pair(a,b)] = pair(pi a, pi b), desc.py:360-389) the
// reference block (train.py:172-205) is
//   K[b, a] = sum_d J_i[d, b] O[d, a],
//   O[d, a] = sum_p 5 m_p diff[p,d] v[p,a] - sum_p w_p J_j[P_p d, a],
//   v[p, a] = sum_d diff[p,d] J_j[P_p d, a],  diff[p,d] = Rd_i[d] - Rd_j[P_p d],
//   m_p = exp(-sqrt5 |diff_p| / sig) / (3 sig^4) * 5,  w_p = (sig^2 + sig sqrt5 |diff_p|) m_p.
// Contracting J_i first gives, with u[p, b] = sum_d J_i[d, b] diff[p, d] and
// G_p = J_i^T J_j[P_p], the equivalent
//   K[b, a] = sum_p 5 m_p u[p, b] v[p, a] - sum_p w_p G_p[b, a],
// where every Jacobian row d = pair(s, t) (s > t) has only two non-zero atoms:
// J[d, t] = +Rdd[d], J[d, s] = -Rdd[d] (desc.py:444-462).

// pair_idx / pair_sign: sgdml_col.h

// The reference assembles the lower block triangle and mirrors it
// (train.py:172-210, exploit_sym): block (i, j) = Blk(r=i, s=j) for j < i and
// Blk(r=j, s=i)^T for j >= i (a diagonal block is stored transposed, which only
// matters for permutation sets that are not a group).  A record (i_loc, j)
// therefore holds the quantities of the pair (r, s) = (i, j) if j < i else (j, i).
//
// one workgroup per (j, i_loc, p): norm, m_p, w_p, u[p, :] (row point r), v[p, :] (col point s)
__global__ __launch_bounds__(256) void k_sgdml_uv(const double *__restrict__ Rd,
                                                  const double *__restrict__ Rdd, int64_t M,
                                                  int n, int64_t D, int64_t i0,
                                                  const int32_t *__restrict__ Pt,  // n_perms x D
                                                  const int32_t *__restrict__ piinv,
                                                  double sig, double *__restrict__ uv,
                                                  int jdiag, int mirror = 1) {
  // jdiag: only the diagonal blocks j = i (records indexed with j slot 0, M = 1)
  // mirror = 0: the record of (r, s) = (i, j) for every j -- the block the reference's
  // matrix-free K_op applies (the query point i, the column point j), used for single
  // columns of the operator (launch_sgdml_columns)
  const int64_t iloc = blockIdx.y;
  const int64_t i = i0 + iloc;
  const int64_t j = jdiag ? i : (int64_t)blockIdx.x;
  const int64_t jslot = jdiag ? 0 : j;
  const int p = blockIdx.z;
  const int n_perms = gridDim.z;
  const int n3 = 3 * n;
  const int64_t rp = (!mirror || j < i) ? i : j;
  const int64_t sp = (!mirror || j < i) ? j : i;
  __shared__ double sh[8];
  const double *rdr = Rd + rp * D;
  const double *rds = Rd + sp * D;
  const int32_t *P = Pt + (int64_t)p * D;
  double acc = 0.0;
  for (int64_t d = threadIdx.x; d < D; d += 256) {
    const double df = rdr[d] - rds[P[d]];
    acc = fma(df, df, acc);
  }
  acc += __shfl_down(acc, 32, 64);
  acc += __shfl_down(acc, 16, 64);
  acc += __shfl_down(acc, 8, 64);
  acc += __shfl_down(acc, 4, 64);
  acc += __shfl_down(acc, 2, 64);
  acc += __shfl_down(acc, 1, 64);
  if ((threadIdx.x & 63) == 0) sh[threadIdx.x >> 6] = acc;
  __syncthreads();
  const double nrm2 = (sh[0] + sh[1]) + (sh[2] + sh[3]);
  const double sqrt5 = sqrt(5.0);
  const double norm = sqrt5 * sqrt(nrm2);
  const double mat52 = exp(-norm / sig) / (3.0 * sig * sig * sig * sig) * 5.0;
  const double w = (sig * sig + sig * norm) * mat52;
  double *rec = uv + ((iloc * M + jslot) * n_perms + p) * (int64_t)(6 * n + 2);
  if (threadIdx.x == 0) {
    rec[6 * n] = mat52;
    rec[6 * n + 1] = w;
  }
  const double *rddr = Rdd + rp * D * 3;
  const double *rdds = Rdd + sp * D * 3;
  const int32_t *pq = piinv + (int64_t)p * n;
  for (int t = threadIdx.x; t < n3; t += 256) {
    const int at = t / 3, c = t % 3;
    // u[(at, c)] = sum_{g != at} sgn(pair(at,g), at) Rdd_r[pair(at,g), c] diff[pair(at,g)]
    double uu = 0.0;
    // v[(at, c)] = sum_{g != at} diff[pair(pi^-1 at, pi^-1 g)] sgn(pair(at,g), at) Rdd_s[pair(at,g), c]
    double vv = 0.0;
    const int ati = pq[at];
    for (int g = 0; g < n; ++g) {
      if (g == at) continue;
      const int64_t d = pair_idx(at, g);
      const double sg = pair_sign(at, g);
      const double dfu = rdr[d] - rds[P[d]];
      uu = fma(sg * rddr[d * 3 + c], dfu, uu);
      const int64_t dv = pair_idx(ati, pq[g]);
      const double dfv = rdr[dv] - rds[P[dv]];
      vv = fma(dfv, sg * rdds[d * 3 + c], vv);
    }
    rec[t] = uu;
    rec[n3 + t] = vv;
  }
}

// diagonal atom block of G_p = J_r^T J_s[P_p] for row atom x (column atom pi_p(x)):
//   sum_{g != x} sgn(pair(x,g),x) Rdd_r[pair(x,g),c1] * sgn(pair(pi x, pi g), pi x) Rdd_s[pair(pi x, pi g), c2]
__device__ void sgdml_gdiag(const double *__restrict__ rddr, const double *__restrict__ rdds,
                            const int32_t *__restrict__ pp, int n, int x, double (*red)[9],
                            double *out9) {
  const int px = pp[x];
  double a9[9];
#pragma unroll
  for (int e = 0; e < 9; ++e) a9[e] = 0.0;
  for (int g = threadIdx.x; g < n; g += 256) {
    if (g == x) continue;
    const int64_t d = pair_idx(x, g);
    const double sd = pair_sign(x, g);
    const int pg = pp[g];
    const int64_t e = pair_idx(px, pg);
    const double se = pair_sign(px, pg);
#pragma unroll
    for (int c = 0; c < 3; ++c)
#pragma unroll
      for (int cc = 0; cc < 3; ++cc)
        a9[c * 3 + cc] = fma(sd * rddr[d * 3 + c], se * rdds[e * 3 + cc], a9[c * 3 + cc]);
  }
#pragma unroll
  for (int e = 0; e < 9; ++e) {
    double v = a9[e];
    v += __shfl_down(v, 32, 64);
    v += __shfl_down(v, 16, 64);
    v += __shfl_down(v, 8, 64);
    v += __shfl_down(v, 4, 64);
    v += __shfl_down(v, 2, 64);
    v += __shfl_down(v, 1, 64);
    if ((threadIdx.x & 63) == 0) red[threadIdx.x >> 6][e] = v;
  }
  __syncthreads();
  if (threadIdx.x < 9)
    out9[threadIdx.x] = (red[0][threadIdx.x] + red[1][threadIdx.x]) +
                        (red[2][threadIdx.x] + red[3][threadIdx.x]);
  __syncthreads();
}

// one workgroup per (atom beta, i_loc, j): rows (i, beta, 0..2) x columns (j, :)
__global__ __launch_bounds__(256) void k_sgdml_block(double *__restrict__ K, int64_t ld,
                                                     int64_t row0, int64_t nrows,
                                                     int64_t rows_per, int64_t blk,
                                                     const double *__restrict__ Rdd, int64_t M,
                                                     int n, int64_t D, int64_t i0,
                                                     const int32_t *__restrict__ pi,
                                                     const int32_t *__restrict__ piinv,
                                                     int n_perms,
                                                     const double *__restrict__ uv, int jdiag,
                                                     double *__restrict__ diag_out) {
  const int beta = blockIdx.x;
  const int64_t iloc = blockIdx.y;
  const int64_t i = i0 + iloc;
  // jdiag: only the diagonal block j = i, written as its diagonal into diag_out
  const int64_t j = jdiag ? i : (int64_t)blockIdx.z;
  const int64_t jslot = jdiag ? 0 : j;
  const int n3 = 3 * n;
  const int64_t grow0 = i * n3 + 3 * beta;  // global row of c = 0
  bool any = false;
  for (int c = 0; c < 3; ++c) {
    const int64_t g = grow0 + c;
    if (g >= row0 && g < row0 + nrows) any = true;
  }
  if (!any) return;
  const bool modeA = j < i;  // block = Blk(r=i, s=j); else Blk(r=j, s=i)^T
  const int64_t rp = modeA ? i : j, sp = modeA ? j : i;
  extern __shared__ double gdiag[];  // n_perms x 9
  __shared__ double red[4][9];
  const double *rddr = Rdd + rp * D * 3;
  const double *rdds = Rdd + sp * D * 3;
  for (int p = 0; p < n_perms; ++p) {
    const int32_t *pp = pi + (int64_t)p * n;
    // mode A: row atom beta; mode B: the row atom of r mapped onto beta
    const int x = modeA ? beta : piinv[(int64_t)p * n + beta];
    sgdml_gdiag(rddr, rdds, pp, n, x, red, gdiag + p * 9);
  }
  const int64_t rec_stride = 6 * n + 2;
  for (int t = threadIdx.x; t < n3; t += 256) {
    const int alpha = t / 3, cc = t % 3;
    double acc0 = 0.0, acc1 = 0.0, acc2 = 0.0;
    for (int p = 0; p < n_perms; ++p) {
      const double *rec = uv + ((iloc * M + jslot) * n_perms + p) * rec_stride;
      const double m5 = 5.0 * rec[6 * n];
      const double w = rec[6 * n + 1];
      const int32_t *pp = pi + (int64_t)p * n;
      const int32_t *pq = piinv + (int64_t)p * n;
      double g0, g1, g2, t0, t1, t2;
      if (modeA) {
        // K[(beta,c),(alpha,cc)] = m5 u[beta,c] v[alpha,cc] - w G(beta,c; alpha,cc)
        const double vv = rec[n3 + t];
        t0 = m5 * rec[3 * beta] * vv;
        t1 = m5 * rec[3 * beta + 1] * vv;
        t2 = m5 * rec[3 * beta + 2] * vv;
        const int ai = pq[alpha];
        if (ai == beta) {
          g0 = gdiag[p * 9 + 0 * 3 + cc];
          g1 = gdiag[p * 9 + 1 * 3 + cc];
          g2 = gdiag[p * 9 + 2 * 3 + cc];
        } else {
          const int64_t d = pair_idx(beta, ai);
          const double sd = pair_sign(beta, ai);
          const int pb = pp[beta];
          const int64_t e = pair_idx(alpha, pb);
          const double jv = pair_sign(alpha, pb) * rdds[e * 3 + cc];
          g0 = sd * rddr[d * 3 + 0] * jv;
          g1 = sd * rddr[d * 3 + 1] * jv;
          g2 = sd * rddr[d * 3 + 2] * jv;
        }
      } else {
        // K[(beta,c),(alpha,cc)] = Blk_{r=j,s=i}[(alpha,cc),(beta,c)]
        //   = m5 u[alpha,cc] v[beta,c] - w G(alpha,cc; beta,c)
        const double uu = m5 * rec[t];
        t0 = uu * rec[n3 + 3 * beta];
        t1 = uu * rec[n3 + 3 * beta + 1];
        t2 = uu * rec[n3 + 3 * beta + 2];
        const int xs = pq[beta];  // row atom of r whose image is beta
        if (alpha == xs) {
          g0 = gdiag[p * 9 + cc * 3 + 0];
          g1 = gdiag[p * 9 + cc * 3 + 1];
          g2 = gdiag[p * 9 + cc * 3 + 2];
        } else {
          const int64_t d = pair_idx(alpha, xs);
          const double sd = pair_sign(alpha, xs);
          const double dv = sd * rddr[d * 3 + cc];
          const int pa = pp[alpha];
          const int64_t e = pair_idx(beta, pa);
          const double se = pair_sign(beta, pa);
          g0 = dv * (se * rdds[e * 3 + 0]);
          g1 = dv * (se * rdds[e * 3 + 1]);
          g2 = dv * (se * rdds[e * 3 + 2]);
        }
      }
      acc0 += t0 - w * g0;
      acc1 += t1 - w * g1;
      acc2 += t2 - w * g2;
    }
    const int64_t gcol = j * n3 + t;
    const int64_t pos = col_pos(gcol, rows_per, blk);
    const double accs[3] = {acc0, acc1, acc2};
    for (int c = 0; c < 3; ++c) {
      const int64_t g = grow0 + c;
      if (g < row0 || g >= row0 + nrows) continue;
      if (diag_out != nullptr) {
        if (gcol == g) diag_out[g - row0] = accs[c];
      } else {
        K[(g - row0) * ld + pos] = accs[c];
      }
    }
  }
}

// ---------------------------------------------------------------------------
// Energy constraints (use_E_cstr).  The reference appends M energy rows / columns to K
// (train.py:212-236) and its K_op predicts energies with energy coefficients
// (iterative_solver.py:423-440, predict.py:206-218):
//   K[E_i, E_j] = -sum_p Kee(nrm_ijp),  Kee(r) = (1 + r/sig (1 + r/(3 sig))) exp(-r/sig),
//   nrm_ijp = sqrt5 |Rd_i - Rd_j[P_p]|.
// kee[il * M + j] = sum_p Kee(nrm_ijp) for i = i0 + il (p summed in order)
__global__ __launch_bounds__(256) void k_sgdml_kee(const double *__restrict__ Rd, int64_t M,
                                                   int64_t D, int64_t i0,
                                                   const int32_t *__restrict__ Pt, int n_perms,
                                                   double sig, double *__restrict__ kee) {
  const int64_t j = blockIdx.x, il = blockIdx.y;
  const double *ri = Rd + (i0 + il) * D;
  const double *rj = Rd + j * D;
  __shared__ double sh[4];
  double total = 0.0;
  for (int p = 0; p < n_perms; ++p) {
    const int32_t *P = Pt + (int64_t)p * D;
    double acc = 0.0;
    for (int64_t d = threadIdx.x; d < D; d += 256) {
      const double df = ri[d] - rj[P[d]];
      acc = fma(df, df, acc);
    }
    acc = wave_sum(acc);
    __syncthreads();  // sh is reused per permutation
    if ((threadIdx.x & 63) == 0) sh[threadIdx.x >> 6] = acc;
    __syncthreads();
    const double nrm = sqrt(5.0) * sqrt((sh[0] + sh[1]) + (sh[2] + sh[3]));
    total += (1.0 + (nrm / sig) * (1.0 + nrm / (3.0 * sig))) * exp(-nrm / sig);
  }
  if (threadIdx.x == 0) kee[il * M + j] = total;
}

// Border of the assembled K for the energy constraints (one rank), from the (r = i, s = j)
// point-pair records of every pair (k_sgdml_uv, mirror = 0) and kee:
//   K[j 3n + t, nF + i] = K[nF + i, j 3n + t] = -sum_p w_p v_p[t]   (train.py:221-230:
//     K_fe = -sum_{p,d} w_p diff_p[d] J_j[P_p d, t] with diff_p = Rd_i - Rd_j[P_p])
//   K[nF + i, nF + j] = -kee[min(i,j), max(i,j)]   (train.py:232-234; column worker
//     max(i, j) writes the pair last)
__global__ __launch_bounds__(256) void k_sgdml_eborder(double *__restrict__ K, int64_t ld,
                                                       const double *__restrict__ uv0,
                                                       const double *__restrict__ kee, int64_t M,
                                                       int n, int n_perms, int64_t nF) {
  const int64_t j = blockIdx.x, i = blockIdx.y;
  const int n3 = 3 * n;
  const int64_t rs = 6 * n + 2;
  const double *rec = uv0 + (i * M + j) * n_perms * rs;
  for (int t = threadIdx.x; t < n3; t += 256) {
    double acc = 0.0;
    for (int p = 0; p < n_perms; ++p) acc = fma(rec[p * rs + 6 * n + 1], rec[p * rs + n3 + t], acc);
    const int64_t g = j * n3 + t;
    K[g * ld + nF + i] = -acc;
    K[(nF + i) * ld + g] = -acc;
  }
  if (threadIdx.x == 0) {
    const int64_t a = i < j ? i : j, b = i < j ? j : i;
    K[(nF + i) * ld + nF + j] = -kee[a * M + b];
  }
}

// descriptor permutations P_p[pair(a,b)] = pair(pi a, pi b) (Desc.perm, desc.py:360-389)
// and inverse atom maps; validates that every row of perms is a permutation
int desc_perm_tables(mlff_ctx *ctx, const int32_t *perms, int n, int n_perms,
                     std::vector<int32_t> &Pt, std::vector<int32_t> &piinv) {
  const int64_t D = (int64_t)n * (n - 1) / 2;
  Pt.assign((size_t)n_perms * D, 0);
  piinv.assign((size_t)n_perms * n, 0);
  for (int p = 0; p < n_perms; ++p) {
    const int32_t *pp = perms + (size_t)p * n;
    std::vector<int> seen(n, 0);
    for (int a = 0; a < n; ++a) {
      if (pp[a] < 0 || pp[a] >= n || seen[pp[a]])
        return set_error(ctx, MLFF_ERR_ARG, "sgdml: perms row is not a permutation");
      seen[pp[a]] = 1;
      piinv[(size_t)p * n + pp[a]] = a;
    }
    for (int a = 1; a < n; ++a)
      for (int b = 0; b < a; ++b) {
        const int pa = pp[a], pb = pp[b];
        const int64_t e = pa > pb ? (int64_t)pa * (pa - 1) / 2 + pb : (int64_t)pb * (pb - 1) / 2 + pa;
        Pt[(size_t)p * D + (int64_t)a * (a - 1) / 2 + b] = (int32_t)e;
      }
  }
  return MLFF_OK;
}

int assemble_sgdml(mlff_ctx *ctx, const double *R_desc, const double *R_d_desc, int64_t M,
                   int n_atoms, const int32_t *perms, int n_perms, double sig) {
  const int n = n_atoms;
  const int64_t D = (int64_t)n * (n - 1) / 2;
  const int64_t n3 = 3 * n;
  if (n < 2 || M < 1 || n_perms < 1) return set_error(ctx, MLFF_ERR_ARG, "assemble_sgdml: bad sizes");
  const bool E = ctx->use_E_cstr;
  const int64_t nF = n3 * M;
  if (nF + (E ? M : 0) != ctx->N)
    return set_error(ctx, MLFF_ERR_ARG, E ? "assemble_sgdml: N != 3 * n_atoms * M + M (use_E_cstr)"
                                          : "assemble_sgdml: N != 3 * n_atoms * M");
  if (E && ctx->world > 1)
    return set_error(ctx, MLFF_ERR_ARG, "assemble_sgdml: use_E_cstr runs on one rank");
  if (n_perms > 1024) return set_error(ctx, MLFF_ERR_ARG, "assemble_sgdml: too many permutations");
  std::vector<int32_t> Pt, piinv;
  MLFF_TRY(desc_perm_tables(ctx, perms, n, n_perms, Pt, piinv));
  // training points whose rows intersect this rank
  const int64_t i0 = std::min<int64_t>(ctx->row0 / n3, M);
  const int64_t i1 = std::min<int64_t>((ctx->row0 + ctx->nrows + n3 - 1) / n3, M);  // exclusive
  const int64_t mi = i1 - i0;
  double *dRd = nullptr, *dRdd = nullptr, *uv = nullptr;
  int32_t *dP = nullptr, *dpi = nullptr, *dpiinv = nullptr;
  const int64_t rec = 6 * n + 2;
  hipStream_t s = ctx->stream;
  ScratchScope scope(ctx);
  MLFF_TRY(scratch_alloc(ctx, &dRd, M * D));
  MLFF_TRY(scratch_alloc(ctx, &dRdd, M * D * 3));
  MLFF_TRY(scratch_alloc(ctx, &dP, n_perms * D));
  MLFF_TRY(scratch_alloc(ctx, &dpi, n_perms * n));
  MLFF_TRY(scratch_alloc(ctx, &dpiinv, n_perms * n));
  MLFF_TRY(scratch_alloc(ctx, &uv, mi * M * n_perms * rec));
  MLFF_HIP(ctx, hipMemcpyAsync(dRd, R_desc, sizeof(double) * M * D, hipMemcpyHostToDevice, s));
  MLFF_HIP(ctx, hipMemcpyAsync(dRdd, R_d_desc, sizeof(double) * M * D * 3, hipMemcpyHostToDevice, s));
  MLFF_HIP(ctx, hipMemcpyAsync(dP, Pt.data(), sizeof(int32_t) * n_perms * D, hipMemcpyHostToDevice, s));
  MLFF_HIP(ctx, hipMemcpyAsync(dpi, perms, sizeof(int32_t) * n_perms * n, hipMemcpyHostToDevice, s));
  MLFF_HIP(ctx, hipMemcpyAsync(dpiinv, piinv.data(), sizeof(int32_t) * n_perms * n, hipMemcpyHostToDevice, s));
  MLFF_HIP(ctx, hipMemsetAsync(ctx->K, 0, sizeof(double) * ctx->blk * ctx->ld, s));
  if (mi > 0) {
    hipLaunchKernelGGL(k_sgdml_uv, dim3((unsigned)M, (unsigned)mi, (unsigned)n_perms), dim3(256), 0,
                       s, dRd, dRdd, M, n, D, i0, dP, dpiinv, sig, uv, 0);
    hipLaunchKernelGGL(k_sgdml_block, dim3((unsigned)n, (unsigned)mi, (unsigned)M), dim3(256),
                       sizeof(double) * 9 * n_perms, s, ctx->K, ctx->ld, ctx->row0, ctx->nrows,
                       ctx->rows_per, ctx->blk, dRdd, M, n, D, i0, dpi, dpiinv, n_perms, uv, 0,
                       (double *)nullptr);
  }
  if (E) {  // one rank: rows and columns are global indices
    const double rec_bytes = 8.0 * (double)M * (double)M * n_perms * (double)rec;
    if (rec_bytes > 4.0e9)
      return set_error(ctx, MLFF_ERR_ARG, "assemble_sgdml: use_E_cstr pair records exceed 4 GB");
    double *uv0 = nullptr, *kee = nullptr;
    MLFF_TRY(scratch_alloc(ctx, &uv0, M * M * n_perms * rec));
    MLFF_TRY(scratch_alloc(ctx, &kee, M * M));
    hipLaunchKernelGGL(k_sgdml_uv, dim3((unsigned)M, (unsigned)M, (unsigned)n_perms), dim3(256), 0,
                       s, dRd, dRdd, M, n, D, (int64_t)0, dP, dpiinv, sig, uv0, 0, 0);
    hipLaunchKernelGGL(k_sgdml_kee, dim3((unsigned)M, (unsigned)M), dim3(256), 0, s, dRd, M, D,
                       (int64_t)0, dP, n_perms, sig, kee);
    hipLaunchKernelGGL(k_sgdml_eborder, dim3((unsigned)M, (unsigned)M), dim3(256), 0, s, ctx->K,
                       ctx->ld, uv0, kee, M, n, n_perms, nF);
  }
  MLFF_HIP(ctx, hipGetLastError());
  MLFF_HIP(ctx, hipStreamSynchronize(s));
  return MLFF_OK;
}

// diag(sigma K) of this rank's rows from the sGDML inputs without assembling K:
// the assembly kernels restricted to the diagonal blocks (diag_K of
// iterative_cholesky.py:241-380, _assemble_kernel_mat_diag).
int sgdml_diag(mlff_ctx *ctx, const double *dRd, const double *dRdd, int64_t M, int n,
               const int32_t *dP, const int32_t *perms_host, const int32_t *piinv_host,
               int n_perms, double sig, double *diag_out) {
  const int64_t D = (int64_t)n * (n - 1) / 2, n3 = 3 * (int64_t)n;
  // force rows only (the energy rows of use_E_cstr follow them; mf_diag fills those)
  const int64_t nrows = std::max<int64_t>(0, std::min<int64_t>(ctx->nrows, n3 * M - ctx->row0));
  if (nrows == 0) return MLFF_OK;
  const int64_t i0 = ctx->row0 / n3;
  const int64_t mi = (ctx->row0 + nrows + n3 - 1) / n3 - i0;
  hipStream_t s = ctx->stream;
  double *uv = nullptr;
  int32_t *dpi = nullptr, *dpiinv = nullptr;
  const int64_t rec = 6 * n + 2;
  ScratchScope scope(ctx);
  MLFF_TRY(scratch_alloc(ctx, &uv, mi * n_perms * rec));
  MLFF_TRY(scratch_alloc(ctx, &dpi, n_perms * n));
  MLFF_TRY(scratch_alloc(ctx, &dpiinv, n_perms * n));
  MLFF_HIP(ctx, hipMemcpyAsync(dpi, perms_host, sizeof(int32_t) * n_perms * n, hipMemcpyHostToDevice, s));
  MLFF_HIP(ctx, hipMemcpyAsync(dpiinv, piinv_host, sizeof(int32_t) * n_perms * n, hipMemcpyHostToDevice, s));
  hipLaunchKernelGGL(k_sgdml_uv, dim3(1, (unsigned)mi, (unsigned)n_perms), dim3(256), 0, s, dRd, dRdd,
                     (int64_t)1, n, D, i0, dP, dpiinv, sig, uv, 1);
  hipLaunchKernelGGL(k_sgdml_block, dim3((unsigned)n, (unsigned)mi, 1), dim3(256),
                     sizeof(double) * 9 * n_perms, s, (double *)nullptr, ctx->ld, ctx->row0,
                     nrows, ctx->rows_per, ctx->blk, dRdd, (int64_t)1, n, D, i0, dpi, dpiinv,
                     n_perms, uv, 1, diag_out);
  MLFF_HIP(ctx, hipGetLastError());
  return MLFF_OK;
}

// ---------------------------------------------------------------------------
// Single columns of the matrix-free operator, S[:, g] = sigma K_op e_g, from the (r = i,
// s = j) records of the point pairs (mirror = 0 above).  e_g (g = j 3n + 3a + c) touches
// one training point j, so K_op e_g (predict.py:72-234 with alphas = e_g; the reference's
// get_col, iterative_cholesky.py:152-156) reduces to the j-column of every query point's
// Hessian block:
//   K[(i,b,c'), g] = sum_p 5 m_p u_p[(b,c')] v_p[(a,c)] - w_p G_p[(b,c'), (a,c)],
//   G_p = J_i^T J_j[P_p]: atom b = pi_p^-1(a) sums over all partners (sgdml_gdiag), every
//   other atom b has the single partner pi_p^-1(a).
// O(rows x n_perms) per column instead of a full operator application (O(M^2 D)).
// Column index: cols[blockIdx.y] (host-chosen sets), or st->m_pi (the device-side pivot
// of the pivoted Cholesky; no host round trip).  Rows: this rank's [row0, row0 + nrows).
// One wave per (64 rows of a query point, column): the rows of atom b = pi_p^-1 a (the
// diagonal atom of permutation p) need its partner series, which the wave sums
// lane-parallel first when its rows include that atom; then every lane writes one row.
// ~250 waves for the nanotube (14 points x 18 row chunks), two dependent load rounds each.
__global__ __launch_bounds__(64) void k_sgdml_col(const double *__restrict__ Rdd, int64_t M,
                                                  int n, int64_t D, int64_t i0,
                                                  const int32_t *__restrict__ pi,
                                                  const int32_t *__restrict__ piinv,
                                                  int n_perms, const double *__restrict__ uvk,
                                                  int64_t row0, int64_t nrows,
                                                  const int64_t *__restrict__ cols,
                                                  const DevState *__restrict__ st, double sigma,
                                                  double *__restrict__ out, int64_t ldo) {
  const int64_t g = cols != nullptr ? cols[blockIdx.y] : (int64_t)st->m_pi;
  if (g < 0) return;
  const int chunks = (3 * n + kColRows - 1) / kColRows;
  bool act;
  int64_t r;
  const double acc = sgdml_col_acc(Rdd, M, n, D, i0, pi, piinv, n_perms, uvk, row0, nrows, g,
                                   blockIdx.x / chunks, (int)(blockIdx.x % chunks) * kColRows,
                                   threadIdx.x, act, r);
  if (act) out[(int64_t)blockIdx.y * ldo + r] = sigma * acc;
}

void launch_sgdml_kee(const double *Rd, int64_t M, int64_t D, int64_t i0, int64_t ni,
                      const int32_t *Pt, int n_perms, double sig, double *kee, hipStream_t s) {
  if (ni <= 0) return;
  hipLaunchKernelGGL(k_sgdml_kee, dim3((unsigned)M, (unsigned)ni), dim3(256), 0, s, Rd, M, D, i0, Pt,
                     n_perms, sig, kee);
}

void launch_sgdml_records(const double *Rd, const double *Rdd, int64_t M, int n, int64_t D,
                          int64_t i0, int64_t ni, const int32_t *Pt, const int32_t *piinv,
                          int n_perms, double sig, double *uvk, hipStream_t s) {
  if (ni <= 0) return;
  hipLaunchKernelGGL(k_sgdml_uv, dim3((unsigned)M, (unsigned)ni, (unsigned)n_perms), dim3(256), 0,
                     s, Rd, Rdd, M, n, D, i0, Pt, piinv, sig, uvk, 0, 0);
}

void launch_sgdml_columns(const double *Rdd, int64_t M, int n, int64_t D, int64_t i0,
                          const int32_t *pi, const int32_t *piinv, int n_perms,
                          const double *uvk, int64_t row0, int64_t nrows, const int64_t *cols,
                          int64_t ncols, const DevState *st, double sigma, double *out,
                          int64_t ldo, hipStream_t s) {
  if (nrows <= 0 || ncols <= 0) return;
  const int64_t n3 = 3 * (int64_t)n;
  const int64_t ni = (row0 + nrows + n3 - 1) / n3 - i0;  // local query points
  const int64_t chunks = (n3 + kColRows - 1) / kColRows;
  hipLaunchKernelGGL(k_sgdml_col, dim3((unsigned)(ni * chunks), (unsigned)ncols), dim3(64), 0, s, Rdd,
                     M, n, D, i0, pi, piinv, n_perms, uvk, row0, nrows, cols, st, sigma, out, ldo);
}

// ---------------------------------------------------------------------------
// Descriptors: R_desc[m, d] = 1 / |r_a - r_b|, R_d_desc[m, d, :] = (r_a - r_b) / |r_a - r_b|^3
// for d = pair(a, b), a > b (desc.py:80-200 without cutoff / PBC).
__global__ __launch_bounds__(256) void k_desc(const double *__restrict__ R, int64_t M, int n,
                                              double *__restrict__ Rd, double *__restrict__ Rdd) {
  const int64_t D = (int64_t)n * (n - 1) / 2;
  const int64_t m = blockIdx.y;
  const double *r = R + m * n * 3;
  for (int64_t d = (int64_t)blockIdx.x * 256 + threadIdx.x; d < D;
       d += (int64_t)gridDim.x * 256) {
    // invert d = a(a-1)/2 + b
    int a = (int)((1.0 + sqrt(1.0 + 8.0 * (double)d)) * 0.5);
    while ((int64_t)a * (a - 1) / 2 > d) --a;
    while ((int64_t)(a + 1) * a / 2 <= d) ++a;
    const int b = (int)(d - (int64_t)a * (a - 1) / 2);
    const double dx = r[a * 3 + 0] - r[b * 3 + 0];
    const double dy = r[a * 3 + 1] - r[b * 3 + 1];
    const double dz = r[a * 3 + 2] - r[b * 3 + 2];
    const double dist = sqrt(__dadd_rn(__dadd_rn(__dmul_rn(dx, dx), __dmul_rn(dy, dy)), __dmul_rn(dz, dz)));
    Rd[m * D + d] = 1.0 / dist;
    const double d3 = dist * dist * dist;
    Rdd[(m * D + d) * 3 + 0] = dx / d3;
    Rdd[(m * D + d) * 3 + 1] = dy / d3;
    Rdd[(m * D + d) * 3 + 2] = dz / d3;
  }
}

int sgdml_descriptors(const double *R, int64_t M, int n, double *R_desc, double *R_d_desc) {
  const int64_t D = (int64_t)n * (n - 1) / 2;
  double *dR = nullptr, *dRd = nullptr, *dRdd = nullptr;
  if (hipMalloc(&dR, sizeof(double) * M * n * 3) != hipSuccess) return MLFF_ERR_NOMEM;
  if (hipMalloc(&dRd, sizeof(double) * M * D) != hipSuccess) return MLFF_ERR_NOMEM;
  if (hipMalloc(&dRdd, sizeof(double) * M * D * 3) != hipSuccess) return MLFF_ERR_NOMEM;
  if (hipMemcpy(dR, R, sizeof(double) * M * n * 3, hipMemcpyHostToDevice) != hipSuccess)
    return MLFF_ERR_HIP;
  const unsigned gx = (unsigned)std::min<int64_t>((D + 255) / 256, 64);
  hipLaunchKernelGGL(k_desc, dim3(gx, (unsigned)M), dim3(256), 0, 0, dR, M, n, dRd, dRdd);
  if (hipGetLastError() != hipSuccess) return MLFF_ERR_HIP;
  if (hipMemcpy(R_desc, dRd, sizeof(double) * M * D, hipMemcpyDeviceToHost) != hipSuccess)
    return MLFF_ERR_HIP;
  if (hipMemcpy(R_d_desc, dRdd, sizeof(double) * M * D * 3, hipMemcpyDeviceToHost) != hipSuccess)
    return MLFF_ERR_HIP;
  hipFree(dR);
  hipFree(dRd);
  hipFree(dRdd);
  return MLFF_OK;
}

}  // namespace mlff
