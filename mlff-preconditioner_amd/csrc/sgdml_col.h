// Device helpers shared by the sGDML kernels of kernels_gen.hip and the persistent pivoted
// Cholesky of kernels_pivchol.hip: the descriptor-pair index / Jacobian sign and one wave's
// rows of a single operator column (the body of k_sgdml_col, so both produce the same bits).
#pragma once

#include "common.h"

namespace mlff {

__device__ __forceinline__ int64_t pair_idx(int a, int b) {
  // tril_indices(n, -1) ordering, a != b
  return a > b ? (int64_t)a * (a - 1) / 2 + b : (int64_t)b * (b - 1) / 2 + a;
}
__device__ __forceinline__ double pair_sign(int a, int b) {  // sign of J[pair(a,b), atom a]
  return a > b ? -1.0 : 1.0;
}

constexpr int kColRows = 64;

// K_op[(i, t), g] / sigma for the 64 rows t = t0 + lane of local query point il (one wave, all
// 64 lanes call it: the partner series of the diagonal atom is a wave sum).  e_g (g = j 3n + 3a
// + c) touches one training point j, so the column is the j-column of every query point's Hessian
// block (predict.py:72-234 with alphas = e_g; iterative_cholesky.py:152-156):
//   K[(i,b,c'), g] = sum_p 5 m_p u_p[(b,c')] v_p[(a,c)] - w_p G_p[(b,c'), (a,c)],
// G_p = J_i^T J_j[P_p]: atom b = pi_p^-1(a) sums over all partners, every other atom b has the
// single partner pi_p^-1(a).  act / r: the lane's row is one of this rank's rows (local index r).
__device__ __forceinline__ double sgdml_col_acc(const double *__restrict__ Rdd, int64_t M, int n,
                                                int64_t D, int64_t i0,
                                                const int32_t *__restrict__ pi,
                                                const int32_t *__restrict__ piinv, int n_perms,
                                                const double *__restrict__ uvk, int64_t row0,
                                                int64_t nrows, int64_t g, int64_t il, int t0,
                                                int lane, bool &act, int64_t &r) {
  const int n3 = 3 * n;
  const int64_t i = i0 + il;
  const int t = t0 + lane;                  // row of the point's 3n block
  r = i * n3 + t - row0;                    // local row
  const int64_t j = g / n3;
  const int a = (int)((g % n3) / 3), c = (int)(g % 3);
  const int64_t rec_stride = 6 * n + 2;
  const double *rdds = Rdd + j * D * 3;
  const double *rddr = Rdd + i * D * 3;
  const double *recs = uvk + (il * M + j) * n_perms * rec_stride;
  act = t < n3 && r >= 0 && r < nrows;
  const int b = t / 3, cr = t % 3;
  double acc = 0.0;
  for (int p = 0; p < n_perms; ++p) {
    const int32_t *pp = pi + (int64_t)p * n;
    const int bd = piinv[(int64_t)p * n + a];  // the row atom whose image is a
    double gdv = 0.0;
    if (3 * bd + 2 >= t0 && 3 * bd < t0 + kColRows) {  // wave-uniform: this chunk holds bd
      double s0 = 0.0, s1 = 0.0, s2 = 0.0;
      for (int x = lane; x < n; x += 64) {
        if (x == bd) continue;
        const int64_t d = pair_idx(bd, x);
        const int px = pp[x];
        const double js = pair_sign(a, px) * rdds[pair_idx(a, px) * 3 + c];
        const double sd = pair_sign(bd, x);
        s0 = fma(sd * rddr[d * 3 + 0], js, s0);
        s1 = fma(sd * rddr[d * 3 + 1], js, s1);
        s2 = fma(sd * rddr[d * 3 + 2], js, s2);
      }
      s0 = wave_sum(s0);
      s1 = wave_sum(s1);
      s2 = wave_sum(s2);
      const double s0b = __shfl(s0, 0, 64), s1b = __shfl(s1, 0, 64), s2b = __shfl(s2, 0, 64);
      gdv = cr == 0 ? s0b : (cr == 1 ? s1b : s2b);
    }
    if (act) {
      const double *rec = recs + (int64_t)p * rec_stride;
      const double m5 = 5.0 * rec[6 * n];
      const double w = rec[6 * n + 1];
      const double tv = m5 * rec[3 * b + cr] * rec[n3 + 3 * a + c];
      double gv = gdv;
      if (b != bd) {
        const int64_t d = pair_idx(b, bd);
        const int pb = pp[b];
        gv = pair_sign(b, bd) * rddr[d * 3 + cr] * (pair_sign(a, pb) * rdds[pair_idx(a, pb) * 3 + c]);
      }
      acc += tv - w * gv;
    }
  }
  return acc;
}

}  // namespace mlff
