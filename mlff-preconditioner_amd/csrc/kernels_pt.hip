// Pair-tile form of the matrix-free sGDML operator, for the many-point / few-atom regime
// (small molecules: n <= 24 atoms, D = n (n - 1) / 2 <= 288 descriptor entries, thousands
// to tens of thousands of training points).
//
// The operator is the reference's K_op (iterative_solver.py:383-445): GDMLPredict's force
// prediction at every training point i with alphas = x (predict.py:172-220):
//   z_j   = J_j x_j,  Zt[jp] = z_j[P_p],  Rt[jp] = Rd_j[P_p]          (k_mf_z, k_mf_rt)
//   diff  = Rd_i - Rt[jp],  nrm = sqrt5 |diff|
//   m     = exp(-nrm / sig) 5 / (3 sig^4),  w = (sig^2 + sig nrm) m
//   F_i   = sum_jp 5 m (diff . Zt[jp]) diff - w Zt[jp]
//   y_i   = J_i^T F_i
// In this regime the work is O(M^2 n_perms D) flops on O(M n_perms D) bytes (ethanol,
// M = 5833: 34 M pairs x 36 entries against 3.4 MB of Rt / Zt): an N-body problem in a
// D-dimensional space, bound by the fp64 vector pipe, not by HBM.  The record-factored form
// (kernels_mf.hip k_rec_g) streams O(M^2 n) bytes of pair records instead and, with one 16 x 16
// atom-pair block for a 9-atom molecule, runs M / 8 workgroups.
//
// k_pt_pair<L, DL>: a workgroup holds 256 / L query points in registers, L lanes per point,
// each lane DL descriptor entries (interleaved pairs: lane l owns entries 2 (l + L e) and
// 2 (l + L e) + 1), and streams a contiguous chunk of the (j, p) range through LDS in tiles of
// kPtTJ rows of Rt / Zt (every group of the workgroup reads the same row: LDS broadcast).  Per
// pair: the lane's partial |diff|^2 and diff . Zt, an xor butterfly over the L lanes (every lane
// ends with the same bits), m, w and c = 5 m (diff . Zt) computed by every lane, F += c diff -
// w Zt on the lane's entries.  The chunk's partial F of each point goes to part[s][i][:]; the
// chunks split the (j, p) range so that the grid fills the chip.
// k_pt_fin: F_i = sum_s part[s][i] (fixed chunk order), y rows = J_i^T F_i (partners b in
// increasing order), y = sigma y + lam x, and the x . y partials of the PCG step.
// Rounding: another summation order of the reference's products.
#include "common.h"

#include <algorithm>
#include <cstdlib>

namespace mlff {

namespace {

constexpr int kPtTJ = 32;       // (j, p) rows per LDS tile
constexpr int kPtThreads = 256;
constexpr double kSqrt5 = 2.23606797749978969640917366873127623544;

struct PtArgs {
  const double *Rd;  // M x D, query rows i0 + il
  const double *Rt;  // MP x D
  const double *Zt;  // MP x D
  int64_t D, i0, ni, MP;
  int S;             // chunks of the (j, p) range (gridDim.y)
  double sig, sig2, inv_sig, k5;  // k5 = 5 / (3 sig^4)
  double *part;      // S x ni x DP
};

// xor-partner sum over the L lanes of a point with DPP moves (VALU, no LDS round trip):
// quad_perm [1,0,3,2] and [2,3,0,1] pair lanes 1 and 2 apart, row_half_mirror pairs every lane
// of a quad with one of the other quad of its 8 (each step adds a commutative pair: every lane
// of the group ends with the same bits)
template <int CTRL>
__device__ __forceinline__ double dpp_f64(double v) {
  const int lo = __builtin_amdgcn_update_dpp(0, __double2loint(v), CTRL, 0xF, 0xF, false);
  const int hi = __builtin_amdgcn_update_dpp(0, __double2hiint(v), CTRL, 0xF, 0xF, false);
  return __hiloint2double(hi, lo);
}
template <int L>
__device__ __forceinline__ double group_sum(double v) {
  static_assert(L == 1 || L == 2 || L == 4 || L == 8, "DPP butterfly for L <= 8");
  if (L >= 2) v += dpp_f64<0xB1>(v);   // quad_perm(1, 0, 3, 2)
  if (L >= 4) v += dpp_f64<0x4E>(v);   // quad_perm(2, 3, 0, 1)
  if (L >= 8) v += dpp_f64<0x141>(v);  // row_half_mirror
  return v;
}

// rows of Rt / Zt per LDS tile: 32, fewer for long descriptors (<= 18 KB per array)
constexpr int pt_tile_rows(int DP) { return DP <= 72 ? 32 : DP <= 144 ? 16 : 8; }

// NJ independent (j, p) rows per step (their dependent chains -- partial sums, butterfly,
// sqrt, exp -- interleave); KEEP_DF / KEEP_Z: diff / the Zt row kept in registers between
// the two passes over the lane's entries (else formed / read from LDS again)
template <int L, int DL, int NJ, bool KEEP_DF, bool KEEP_Z, int WPE = 1>
__global__ __launch_bounds__(kPtThreads) __attribute__((amdgpu_waves_per_eu(WPE, 8)))
void k_pt_pair(PtArgs a, const int *__restrict__ status) {
  static_assert(DL % 2 == 0 && 64 % L == 0, "lane layout");
  constexpr int DP = L * DL;              // padded descriptor length
  constexpr int G = kPtThreads / L;       // query points per workgroup
  constexpr int TJ = pt_tile_rows(DP);
  static_assert(TJ % NJ == 0, "steps tile the LDS rows");
  constexpr int kStage = TJ * DP;         // doubles per staged array
  constexpr int kPer = (kStage + kPtThreads - 1) / kPtThreads;
  constexpr int KD = KEEP_DF ? DL : 2, KZ = KEEP_Z ? DL : 2;
  // the status word is tested once the point rows and the first tile are requested
  const int st0 = status != nullptr ? *status : ST_RUNNING;
  __shared__ double sR[kStage];
  __shared__ double sZ[kStage];
  const int tid = threadIdx.x;
  const int l = tid % L, g = tid / L;
  const int64_t il = (int64_t)blockIdx.x * G + g;
  const bool live = il < a.ni;
  // the point's descriptor entries in registers (zero past D and for idle lanes)
  double rd[DL], f[DL];
  {
    const double *row = a.Rd + (a.i0 + (live ? il : 0)) * a.D;
#pragma unroll
    for (int e = 0; e < DL / 2; ++e) {
      const int64_t d = 2 * (l + L * e);
      rd[2 * e] = (live && d < a.D) ? row[d] : 0.0;
      rd[2 * e + 1] = (live && d + 1 < a.D) ? row[d + 1] : 0.0;
      f[2 * e] = f[2 * e + 1] = 0.0;
    }
  }
  const int64_t s = blockIdx.y;
  const int64_t jb0 = (a.MP * s) / a.S, jb1 = (a.MP * (s + 1)) / a.S;
  const int64_t ntile = (jb1 - jb0 + TJ - 1) / TJ;
  // staging of tile t: rows jb0 + t TJ ..., entries past D and rows past jb1 zero (a zero row
  // adds exact zeros: a = 0 so c = 0, and w * 0)
  double vr[kPer], vz[kPer];
  auto load_tile = [&](int64_t t) {
#pragma unroll
    for (int u = 0; u < kPer; ++u) {
      const int e = tid + kPtThreads * u;
      const int jj = e / DP, d = e % DP;
      const int64_t jp = jb0 + t * TJ + jj;
      const bool ok = e < kStage && jp < jb1 && d < a.D;
      vr[u] = ok ? a.Rt[jp * a.D + d] : 0.0;
      vz[u] = ok ? a.Zt[jp * a.D + d] : 0.0;
    }
  };
  if (ntile > 0) load_tile(0);
  if (st0 != ST_RUNNING) return;  // uniform: before the first barrier
  for (int64_t t = 0; t < ntile; ++t) {
    __syncthreads();  // the previous tile is consumed
#pragma unroll
    for (int u = 0; u < kPer; ++u) {
      const int e = tid + kPtThreads * u;
      if (kStage % kPtThreads == 0 || e < kStage) {
        sR[e] = vr[u];
        sZ[e] = vz[u];
      }
    }
    __syncthreads();
    if (t + 1 < ntile) load_tile(t + 1);  // in flight during this tile's pairs
    const int64_t rem = jb1 - jb0 - t * TJ;
    const int cnt = (int)(rem < TJ ? rem : TJ);
#pragma unroll 1
    for (int j0 = 0; j0 < cnt; j0 += NJ) {
      double df[NJ][KD], zz[NJ][KZ], r2[NJ], ad[NJ];
#pragma unroll
      for (int q = 0; q < NJ; ++q) {
        const double *rr = sR + (j0 + q) * DP + 2 * l;
        const double *zr = sZ + (j0 + q) * DP + 2 * l;
        double r2a = 0.0, r2b = 0.0, aa = 0.0, ab = 0.0;
#pragma unroll
        for (int e = 0; e < DL / 2; ++e) {
          const double2 tv = *reinterpret_cast<const double2 *>(rr + 2 * L * e);
          const double2 zv = *reinterpret_cast<const double2 *>(zr + 2 * L * e);
          const double d0 = rd[2 * e] - tv.x, d1 = rd[2 * e + 1] - tv.y;
          if (KEEP_DF) {
            df[q][(2 * e) % KD] = d0;
            df[q][(2 * e + 1) % KD] = d1;
          }
          if (KEEP_Z) {
            zz[q][(2 * e) % KZ] = zv.x;
            zz[q][(2 * e + 1) % KZ] = zv.y;
          }
          r2a = fma(d0, d0, r2a);
          r2b = fma(d1, d1, r2b);
          aa = fma(d0, zv.x, aa);
          ab = fma(d1, zv.y, ab);
        }
        r2[q] = r2a + r2b;
        ad[q] = aa + ab;
      }
      double c[NJ], w[NJ];
#pragma unroll
      for (int q = 0; q < NJ; ++q) {
        const double rs = group_sum<L>(r2[q]), as = group_sum<L>(ad[q]);
        const double nrm = kSqrt5 * sqrt(rs);
        const double m = exp(-nrm * a.inv_sig) * a.k5;
        w[q] = fma(a.sig, nrm, a.sig2) * m;
        c[q] = 5.0 * m * as;
      }
      // the second pass re-reads what it does not keep (no CSE of the LDS loads across this)
      if (!KEEP_DF || !KEEP_Z) asm volatile("" ::: "memory");
#pragma unroll
      for (int q = 0; q < NJ; ++q) {
        const double *rr = sR + (j0 + q) * DP + 2 * l;
        const double *zr = sZ + (j0 + q) * DP + 2 * l;
#pragma unroll
        for (int e = 0; e < DL / 2; ++e) {
          double d0, d1, z0, z1;
          if (KEEP_DF) {
            d0 = df[q][(2 * e) % KD];
            d1 = df[q][(2 * e + 1) % KD];
          } else {
            const double2 tv = *reinterpret_cast<const double2 *>(rr + 2 * L * e);
            d0 = rd[2 * e] - tv.x;
            d1 = rd[2 * e + 1] - tv.y;
          }
          if (KEEP_Z) {
            z0 = zz[q][(2 * e) % KZ];
            z1 = zz[q][(2 * e + 1) % KZ];
          } else {
            const double2 zv = *reinterpret_cast<const double2 *>(zr + 2 * L * e);
            z0 = zv.x;
            z1 = zv.y;
          }
          f[2 * e] = fma(-w[q], z0, fma(c[q], d0, f[2 * e]));
          f[2 * e + 1] = fma(-w[q], z1, fma(c[q], d1, f[2 * e + 1]));
        }
      }
    }
  }
  if (!live) return;
  double *out = a.part + (s * a.ni + il) * DP;
#pragma unroll
  for (int e = 0; e < DL / 2; ++e)
    *reinterpret_cast<double2 *>(out + 2 * (l + L * e)) = make_double2(f[2 * e], f[2 * e + 1]);
}

// k_pt_mfma<DR, NT, DZM>: the force sum on the matrix cores.  |diff|^2 stays on the VALU with
// direct differences (no |a|^2 + |b|^2 - 2 a.b cancellation: the self pair keeps nrm = 0), each
// pair formed by ONE lane (no butterfly, no redundant sqrt / exp); the accumulation
//   F_i = sum_jp c (Rd_i - Rt_jp) - w Zt_jp = Rd'_i sum_jp c  -  sum_jp [c | w] [Rt' ; Zt]
// is a (points x 2 rows) x (2 rows x D) product on v_mfma_f64_16x16x4f64, and with DZM so is
//   diff . Zt_jp = Rd'_i . Zt_jp - Rt'_jp . Zt_jp      (rows x D) x (D x points), minus q_jp,
// with the descriptors centred on training point 0 (Rd' = Rd - mu, Rt' = Rt - mu: for
// geometries of one molecule every entry lies within a factor 2 of mu's, so the centring is
// exact (Sterbenz) and Rd' - Rt' has the bits of Rd - Rt, while |Rd'| ~ |diff| keeps the
// expansions' cancellation at O(1): their error is eps |Rd'| |Zt| per product, the size of the
// direct form's own rounding against the operator's scale).  A wave holds 16 query points
// (lane & 15; Rd' row in registers); lane kk = lane >> 4 forms the pairs with rows 4 r + kk of
// each 16-row block -- the A operand layout of the force MFMA's k-step r and the output layout
// of the (rows x points) diff . Zt product, so dz, c and w never change lanes.  The four waves
// of a workgroup (64 points) share the LDS tiles of Rt' / Zt (32 rows, stride DS); q_jp is
// summed while the tile is staged (8 threads per row, DPP butterfly: fixed order).
constexpr int kMfPts = 64;
constexpr int kMfTJ = 32;
typedef double v4d __attribute__((ext_vector_type(4)));
template <int DR, int NT, bool DZM>
__global__ __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(2, 8))) void k_pt_mfma(PtArgs a, const int *__restrict__ status) {
  static_assert(DR % 4 == 0 && DR <= 16 * NT, "register row within the n-tiles");
  constexpr int DC = 16 * NT;        // staged columns (zero past D)
  constexpr int DS = DC + 2;         // LDS row stride: the 4 rows a wave reads sit in 4 bank groups
  constexpr int EPT = DC / 8;        // staged entries per thread: 8 threads per row, 32 rows
  static_assert(DC % 8 == 0 && kMfTJ * 8 == 256, "staging");
  if (status != nullptr && *status != ST_RUNNING) return;
  __shared__ double sR[kMfTJ * DS];
  __shared__ double sZ[kMfTJ * DS];
  __shared__ double sQ[kMfTJ];
  __shared__ double sMu[DC];
  __shared__ double sC[4][16];
  __shared__ double sCW[4][2][4][64];
  const int tid = threadIdx.x, wv = tid >> 6, lane = tid & 63;
  const int pi = lane & 15, kk = lane >> 4;
  for (int d = tid; d < DC; d += 256) sMu[d] = d < a.D ? a.Rd[d] : 0.0;
  __syncthreads();
  const int64_t ib = (int64_t)blockIdx.x * kMfPts + wv * 16;
  const int64_t il = ib + pi;
  const bool live = il < a.ni;
  double rd[DR];
  {
    const double *row = a.Rd + (a.i0 + (live ? il : 0)) * a.D;
#pragma unroll
    for (int d = 0; d < DR; ++d) rd[d] = (live && d < a.D) ? row[d] - sMu[d] : 0.0;
  }
  double rdB[DR / 4];  // B operand of the diff . Zt product: Rd'[pi][4 s + kk]
  if (DZM) {
#pragma unroll
    for (int s4 = 0; s4 < DR / 4; ++s4)
      rdB[s4] = kk == 0 ? rd[4 * s4] : kk == 1 ? rd[4 * s4 + 1] : kk == 2 ? rd[4 * s4 + 2] : rd[4 * s4 + 3];
  }
  const int64_t s = blockIdx.y;
  const int64_t jb0 = (a.MP * s) / a.S, jb1 = (a.MP * (s + 1)) / a.S;
  const int64_t ntile = (jb1 - jb0 + kMfTJ - 1) / kMfTJ;
  const int srow = tid >> 3, sd0 = (tid & 7) * EPT;  // staging: row, first entry
  double vr[EPT], vz[EPT];
  auto load_tile = [&](int64_t t) {
    const int64_t jp = jb0 + t * kMfTJ + srow;
#pragma unroll
    for (int u = 0; u < EPT; ++u) {
      const int d = sd0 + u;
      const bool ok = jp < jb1 && d < a.D;
      vr[u] = ok ? a.Rt[jp * a.D + d] : 0.0;
      vz[u] = ok ? a.Zt[jp * a.D + d] : 0.0;
    }
  };
  v4d acc[NT];
#pragma unroll
  for (int t = 0; t < NT; ++t) acc[t] = v4d{0.0, 0.0, 0.0, 0.0};
  double csum = 0.0;
  if (ntile > 0) load_tile(0);
  for (int64_t t = 0; t < ntile; ++t) {
    __syncthreads();  // the previous tile is consumed
    {
      const bool rok = jb0 + t * kMfTJ + srow < jb1;
      double q = 0.0;
#pragma unroll
      for (int u = 0; u < EPT; ++u) {
        const int d = sd0 + u;
        // padded rows stay zero (not -mu): diff . 0 = 0 gives c = 0, and w meets Zt = 0
        const double rv = (rok && d < a.D) ? vr[u] - sMu[d] : 0.0;
        sR[srow * DS + d] = rv;
        sZ[srow * DS + d] = vz[u];
        q = fma(rv, vz[u], q);
      }
      if (DZM) {
        q = group_sum<8>(q);
        if ((tid & 7) == 0) sQ[srow] = q;
      }
    }
    __syncthreads();
    if (t + 1 < ntile) load_tile(t + 1);  // in flight during this tile's pairs
#pragma unroll 1
    for (int b = 0; b < kMfTJ / 16; ++b) {
      if (DZM) {  // dz[q] of rows b 16 + kk + 4 q, point pi
        v4d dz = v4d{0.0, 0.0, 0.0, 0.0};
#pragma unroll
        for (int s4 = 0; s4 < DR / 4; ++s4)
          dz = __builtin_amdgcn_mfma_f64_16x16x4f64(sZ[(b * 16 + pi) * DS + 4 * s4 + kk], rdB[s4], dz,
                                                    0, 0, 0);
#pragma unroll
        for (int r = 0; r < 4; ++r) sCW[wv][0][r][lane] = dz[r] - sQ[b * 16 + 4 * r + kk];
      }
      // one pair row at a time (one inlined exp; dz, c, w through this lane's LDS slots)
#pragma unroll 2
      for (int r = 0; r < 4; ++r) {
        const double *rr = sR + (b * 16 + 4 * r + kk) * DS;
        const double *zr = sZ + (b * 16 + 4 * r + kk) * DS;
        double r2a = 0.0, r2b = 0.0, aa = 0.0, ab = 0.0;
#pragma unroll
        for (int e = 0; e < DR / 2; ++e) {
          const double2 tv = *reinterpret_cast<const double2 *>(rr + 2 * e);
          const double d0 = rd[2 * e] - tv.x, d1 = rd[2 * e + 1] - tv.y;
          r2a = fma(d0, d0, r2a);
          r2b = fma(d1, d1, r2b);
          if (!DZM) {
            const double2 zv = *reinterpret_cast<const double2 *>(zr + 2 * e);
            aa = fma(d0, zv.x, aa);
            ab = fma(d1, zv.y, ab);
          }
        }
        const double dz = DZM ? sCW[wv][0][r][lane] : aa + ab;
        const double nrm = kSqrt5 * sqrt(r2a + r2b);
        const double m = exp(-nrm * a.inv_sig) * a.k5;
        const double c = 5.0 * m * dz;
        sCW[wv][0][r][lane] = -c;
        sCW[wv][1][r][lane] = -(fma(a.sig, nrm, a.sig2) * m);
        csum += c;
      }
      double cA[4], wA[4];
#pragma unroll
      for (int r = 0; r < 4; ++r) {  // the lane's own slots: no barrier
        cA[r] = sCW[wv][0][r][lane];
        wA[r] = sCW[wv][1][r][lane];
      }
#pragma unroll
      for (int nt = 0; nt < NT; ++nt) {
#pragma unroll
        for (int r = 0; r < 4; ++r)
          acc[nt] = __builtin_amdgcn_mfma_f64_16x16x4f64(
              cA[r], sR[(b * 16 + 4 * r + kk) * DS + 16 * nt + pi], acc[nt], 0, 0, 0);
#pragma unroll
        for (int r = 0; r < 4; ++r)
          acc[nt] = __builtin_amdgcn_mfma_f64_16x16x4f64(
              wA[r], sZ[(b * 16 + 4 * r + kk) * DS + 16 * nt + pi], acc[nt], 0, 0, 0);
      }
    }
  }
  // sum_jp c of point pi: the four row-lanes' partials in a commutative pair order
  csum += __shfl_xor(csum, 16);
  csum += __shfl_xor(csum, 32);
  if (kk == 0) sC[wv][pi] = csum;
  __syncthreads();
  // acc[nt][q] = F'[point kk + 4 q][entry 16 nt + pi]
  constexpr int64_t DP = DR;  // chunk partial stride: the variant's L * DL (pt_padded_d)
#pragma unroll
  for (int q = 0; q < 4; ++q) {
    const int pq = kk + 4 * q;
    const int64_t ilq = ib + pq;
    if (ilq >= a.ni) continue;
    const double cs = sC[wv][pq];
    const double *row = a.Rd + (a.i0 + ilq) * a.D;
    double *out = a.part + (s * a.ni + ilq) * DP;
#pragma unroll
    for (int nt = 0; nt < NT; ++nt) {
      const int d = 16 * nt + pi;
      if (d < a.D) out[d] = fma(row[d] - sMu[d], cs, acc[nt][q]);
    }
  }
}

// k_pt_mfma_sp<DR, NT>: k_pt_mfma<DR, NT, false> software-pipelined so that the matrix pipe and
// the VALU work at once: the force MFMAs of 16-row group g - 1 are issued between the VALU pair
// rows of group g (row r of g, then group g - 1's k-step r: 2 NT MFMAs, independent of the row's
// VALU chain), so each wave keeps both pipes busy instead of alternating VALU and MFMA phases.
// Groups of 16 (j, p) rows are staged one per step into a 3-slot LDS ring (g - 1 read by the
// MFMAs, g by the VALU, g + 1 written by the next step: one barrier per step orders them); c, w
// of group g go to this lane's slots of a 2-deep buffer.  The (0 x zero rows) MFMAs of the first
// step add exact zeros.  Same pairs, same operands as k_pt_mfma; the force sum's k-steps in
// (group, row, c then w) order.
template <int DR, int NT>
__global__ __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(2, 8))) void k_pt_mfma_sp(PtArgs a, const int *__restrict__ status) {
  static_assert(DR % 2 == 0 && DR <= 16 * NT, "register row within the n-tiles");
  constexpr int DC = 16 * NT;        // staged columns (zero past D)
  constexpr int DS = DC + 2;         // LDS row stride
  constexpr int kG = 16;             // rows per group
  constexpr int EPT = kG * DC / 256; // staged entries per thread and array
  static_assert(kG * DC % 256 == 0 && DC % EPT == 0, "staging");
  if (status != nullptr && *status != ST_RUNNING) return;
  __shared__ double sR[3][kG * DS];
  __shared__ double sZ[3][kG * DS];
  __shared__ double sMu[DC];
  __shared__ double sC[4][16];
  __shared__ double sCW[2][4][2][4][64];
  const int tid = threadIdx.x, wv = tid >> 6, lane = tid & 63;
  const int pi = lane & 15, kk = lane >> 4;
  for (int d = tid; d < DC; d += 256) sMu[d] = d < a.D ? a.Rd[d] : 0.0;
  // the step-0 MFMAs read group "-1": slot 2 rows and buffer 1 c, w, all zero
  for (int e = tid; e < kG * DS; e += 256) sR[2][e] = sZ[2][e] = 0.0;
#pragma unroll
  for (int u = 0; u < 8; ++u) (&sCW[1][wv][0][0][0])[lane + 64 * u] = 0.0;
  __syncthreads();
  const int64_t ib = (int64_t)blockIdx.x * kMfPts + wv * 16;
  const int64_t il = ib + pi;
  const bool live = il < a.ni;
  double rd[DR];
  {
    const double *row = a.Rd + (a.i0 + (live ? il : 0)) * a.D;
#pragma unroll
    for (int d = 0; d < DR; ++d) rd[d] = (live && d < a.D) ? row[d] - sMu[d] : 0.0;
  }
  const int64_t s = blockIdx.y;
  const int64_t jb0 = (a.MP * s) / a.S, jb1 = (a.MP * (s + 1)) / a.S;
  const int64_t ngr = (jb1 - jb0 + kG - 1) / kG;
  const int srow = tid / (DC / EPT), sd0 = (tid % (DC / EPT)) * EPT;
  double vr[EPT], vz[EPT];
  auto load_group = [&](int64_t g) {
    const int64_t jp = jb0 + g * kG + srow;
#pragma unroll
    for (int u = 0; u < EPT; ++u) {
      const int d = sd0 + u;
      const bool ok = g < ngr && jp < jb1 && d < a.D;
      vr[u] = ok ? a.Rt[jp * a.D + d] : 0.0;
      vz[u] = ok ? a.Zt[jp * a.D + d] : 0.0;
    }
  };
  v4d acc[NT];
#pragma unroll
  for (int t = 0; t < NT; ++t) acc[t] = v4d{0.0, 0.0, 0.0, 0.0};
  double csum = 0.0;
  load_group(0);
  for (int64_t g = 0; g <= ngr; ++g) {
    const int cur = (int)(g % 3), prv = (int)((g + 2) % 3);
    const int cb = (int)(g & 1), pb = cb ^ 1;
    if (g < ngr) {
      const bool rok = jb0 + g * kG + srow < jb1;
#pragma unroll
      for (int u = 0; u < EPT; ++u) {
        const int d = sd0 + u;
        // padded rows stay zero (not -mu): diff . 0 = 0 gives c = 0, and w meets Zt = 0
        sR[cur][srow * DS + d] = (rok && d < a.D) ? vr[u] - sMu[d] : 0.0;
        sZ[cur][srow * DS + d] = vz[u];
      }
    }
    __syncthreads();
    if (g + 1 < ngr) load_group(g + 1);  // in flight during this step
    if (g == ngr) {  // drain: the last group's force MFMAs
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const double cp = sCW[pb][wv][0][r][lane], wp = sCW[pb][wv][1][r][lane];
#pragma unroll
        for (int nt = 0; nt < NT; ++nt) {
          acc[nt] = __builtin_amdgcn_mfma_f64_16x16x4f64(cp, sR[prv][(4 * r + kk) * DS + 16 * nt + pi],
                                                         acc[nt], 0, 0, 0);
          acc[nt] = __builtin_amdgcn_mfma_f64_16x16x4f64(wp, sZ[prv][(4 * r + kk) * DS + 16 * nt + pi],
                                                         acc[nt], 0, 0, 0);
        }
      }
      break;
    }
#pragma unroll 1
    for (int r = 0; r < 4; ++r) {
      // group g - 1's k-step r on the matrix pipe (its operands are ready), one MFMA after every
      // few entries of pair row r of group g on the VALU: an MFMA the busy matrix pipe cannot
      // take stalls the wave's in-order issue, so back-to-back MFMAs would idle the VALU
      const double cp = sCW[pb][wv][0][r][lane], wp = sCW[pb][wv][1][r][lane];
      double bR[NT], bZ[NT];
#pragma unroll
      for (int nt = 0; nt < NT; ++nt) {
        bR[nt] = sR[prv][(4 * r + kk) * DS + 16 * nt + pi];
        bZ[nt] = sZ[prv][(4 * r + kk) * DS + 16 * nt + pi];
      }
      constexpr int kStep = DR / 2 / (2 * NT) > 0 ? DR / 2 / (2 * NT) : 1;
      const double *rr = sR[cur] + (4 * r + kk) * DS;
      const double *zr = sZ[cur] + (4 * r + kk) * DS;
      double r2a = 0.0, r2b = 0.0, aa = 0.0, ab = 0.0;
#pragma unroll
      for (int e = 0; e < DR / 2; ++e) {
        const double2 tv = *reinterpret_cast<const double2 *>(rr + 2 * e);
        const double2 zv = *reinterpret_cast<const double2 *>(zr + 2 * e);
        const double d0 = rd[2 * e] - tv.x, d1 = rd[2 * e + 1] - tv.y;
        r2a = fma(d0, d0, r2a);
        r2b = fma(d1, d1, r2b);
        aa = fma(d0, zv.x, aa);
        ab = fma(d1, zv.y, ab);
        if (e % kStep == kStep - 1 && e / kStep < 2 * NT) {
          const int i = e / kStep, nt = i >> 1;
          acc[nt] = __builtin_amdgcn_mfma_f64_16x16x4f64((i & 1) ? wp : cp, (i & 1) ? bZ[nt] : bR[nt],
                                                         acc[nt], 0, 0, 0);
          __builtin_amdgcn_sched_barrier(0);
        }
      }
#pragma unroll
      for (int i = DR / 2 / kStep; i < 2 * NT; ++i) {  // short rows: the remaining k-steps
        const int nt = i >> 1;
        acc[nt] = __builtin_amdgcn_mfma_f64_16x16x4f64((i & 1) ? wp : cp, (i & 1) ? bZ[nt] : bR[nt],
                                                       acc[nt], 0, 0, 0);
      }
      const double nrm = kSqrt5 * sqrt(r2a + r2b);
      const double m = exp(-nrm * a.inv_sig) * a.k5;
      const double c = 5.0 * m * (aa + ab);
      sCW[cb][wv][0][r][lane] = -c;
      sCW[cb][wv][1][r][lane] = -(fma(a.sig, nrm, a.sig2) * m);
      csum += c;
    }
  }
  csum += __shfl_xor(csum, 16);
  csum += __shfl_xor(csum, 32);
  if (kk == 0) sC[wv][pi] = csum;
  __syncthreads();
  constexpr int64_t DP = DR;
#pragma unroll
  for (int q = 0; q < 4; ++q) {
    const int pq = kk + 4 * q;
    const int64_t ilq = ib + pq;
    if (ilq >= a.ni) continue;
    const double cs = sC[wv][pq];
    const double *row = a.Rd + (a.i0 + ilq) * a.D;
    double *out = a.part + (s * a.ni + ilq) * DP;
#pragma unroll
    for (int nt = 0; nt < NT; ++nt) {
      const int d = 16 * nt + pi;
      if (d < a.D) out[d] = fma(row[d] - sMu[d], cs, acc[nt][q]);
    }
  }
}

__device__ __forceinline__ int64_t pt_pair(int a, int b) {
  return a > b ? (int64_t)a * (a - 1) / 2 + b : (int64_t)b * (b - 1) / 2 + a;
}

struct PtFin {
  const double *part;   // S x ni x DP
  const double *Rdd;    // M x D x 3
  int64_t D, DP, i0, ni, row0, nrows;
  int S, n;
  double sigma, lam;
  const double *xloc;   // this rank's operand rows (nullptr: no lam term); p_old when fused
  double *y;
  double *pq_part;      // kVecGrid partials of x . y (nullptr: none)
  // fused search-direction update (launch_pt_operator's pf): the operand rows are
  // p = fused_p(xloc, z) with k_mf_z's rho (st->rho_new) and rho1, written back to xloc here
  // (k_mf_z, the only other reader of p_old, has finished); rho stored in the state
  const double *z = nullptr;
  DevState *st = nullptr;
  long long it = 0;
};

// a workgroup per training point (grid-stride over the points): F_i = sum of the S chunk
// partials, the chunks split over Q = 256 / D groups of D threads (each group sums its
// contiguous run of chunks in chunk order -- batches of 8 predicated loads in flight, the padding
// adds exact zeros -- and the Q group sums are then added in group order: a fixed order, one
// dependent load round for S <= 8 Q instead of S / 8); the point's Rdd row is staged in LDS in the
// same round; then one thread per row forms J_i^T F_i (partners b in increasing order),
// sigma y + lam x and the x . y partials
constexpr int kPtFinMaxF = 512;  // LDS doubles of the group partials (Q D <= 256, or D <= 288)
__global__ __launch_bounds__(256) void k_pt_fin(PtFin a, const int *__restrict__ status) {
  // the status word gates the state write and the stores: tested once the first point's
  // loads are issued
  const int st0 = status != nullptr ? *status : ST_RUNNING;
  __shared__ double sP[kPtFinMaxF];
  __shared__ double sF[kPtFinMaxF];
  __shared__ double sR[3 * 288];
  __shared__ double sh[8];
  const int n3 = 3 * a.n;
  const int D = (int)a.D;
  const int Q = D <= 256 ? 256 / D : 1;           // chunk groups
  const int64_t zs = a.ni * a.DP;                 // stride between chunks
  const bool fp = a.z != nullptr, first = a.it <= 1;
  double beta = 0.0;
  if (fp) {  // rho as k_mf_z summed it, rho1 as its folded stop test left it: k_update_p's beta
    const double rho = a.st->rho_new;
    beta = rho / a.st->rho1;
    if (st0 == ST_RUNNING && blockIdx.x == 0 && threadIdx.x == 0) a.st->rho = rho;
  }
  double pq = 0.0;
  for (int64_t il = blockIdx.x; il < a.ni; il += gridDim.x) {
    const int64_t i = a.i0 + il;
    const double *src = a.part + il * a.DP;
    // the operand entries of this thread's row (n3 <= 72 < 256), requested with the partials
    // (not after the barriers: one dependent load round less)
    const int64_t rl0 = i * n3 + threadIdx.x - a.row0;
    const bool rown = threadIdx.x < n3 && rl0 >= 0 && rl0 < a.nrows && a.xloc != nullptr;
    const double xpre = rown ? a.xloc[rl0] : 0.0;
    const double zpre = rown && fp ? a.z[rl0] : 0.0;
    for (int e = threadIdx.x; e < 3 * D; e += 256) sR[e] = a.Rdd[i * a.D * 3 + e];
    for (int e = threadIdx.x; e < Q * D; e += 256) {  // D > 256: Q = 1, two entries per thread
      const int g = e / D, d = e % D;
      const int z0 = (int)(((int64_t)a.S * g) / Q), z1 = (int)(((int64_t)a.S * (g + 1)) / Q);
      double sum = 0.0;
      for (int z = z0; z < z1; z += 8) {
        double t[8];
#pragma unroll
        for (int u = 0; u < 8; ++u) t[u] = z + u < z1 ? src[(int64_t)(z + u) * zs + d] : 0.0;
#pragma unroll
        for (int u = 0; u < 8; ++u) sum += t[u];
      }
      sP[e] = sum;
    }
    if (st0 != ST_RUNNING) return;  // uniform: before the first barrier and any global store
    __syncthreads();
    for (int d = threadIdx.x; d < D; d += 256) {
      double f = sP[d];
      for (int g = 1; g < Q; ++g) f += sP[g * D + d];
      sF[d] = f;
    }
    __syncthreads();
    for (int r = threadIdx.x; r < n3; r += 256) {
      const int64_t rl = i * n3 + r - a.row0;
      if (rl < 0 || rl >= a.nrows) continue;
      const int at = r / 3, c = r % 3;
      double xv = 0.0;
      if (a.xloc != nullptr) {
        xv = r < 256 ? xpre : a.xloc[rl];  // r < n3 <= 72: the prefetched entry
        if (fp) xv = fused_p(xv, r < 256 ? zpre : a.z[rl], beta, first);
      }
      double acc = 0.0;
      for (int b = 0; b < a.n; ++b) {
        if (b == at) continue;
        const int64_t d = pt_pair(at, b);
        const double rv = sR[d * 3 + c];
        acc = fma(at > b ? -rv : rv, sF[d], acc);
      }
      double yv = a.sigma * acc;
      if (a.xloc != nullptr) {
        if (fp) const_cast<double *>(a.xloc)[rl] = xv;
        yv = fma(a.lam, xv, yv);
        if (a.pq_part != nullptr) pq = fma(xv, yv, pq);
      }
      a.y[rl] = yv;
    }
    __syncthreads();
  }
  if (st0 != ST_RUNNING) return;  // uniform (a block without points)
  if (a.pq_part != nullptr) {
    const double t = block_sum256(pq, sh);
    if (threadIdx.x == 0) a.pq_part[blockIdx.x] = t;
  }
}

using PairFn = void (*)(PtArgs, const int *);

struct PtVariant {
  int L, DL;
  PairFn fn;
  int G;  // query points per workgroup
};

// L lanes per point (partial sums joined by the DPP butterfly), DL entries per lane; the
// first variant that covers D is the default.  MLFF_PT_VARIANT=<index> forces one (sweeps; it
// must cover D)
const PtVariant kPtVariants[] = {
    {2, 18, k_pt_pair<2, 18, 1, true, true>, 128},    // D <= 36  (n <= 9: ethanol)
    {4, 18, k_pt_pair<4, 18, 1, true, false>, 64},   // D <= 72  (n <= 12: uracil)
    {4, 28, k_pt_pair<4, 28, 1, false, false>, 64},  // D <= 112 (n <= 15: toluene)
    {8, 28, k_pt_pair<8, 28, 1, false, false>, 32},  // D <= 224 (n <= 21: aspirin)
    {8, 36, k_pt_pair<8, 36, 1, false, false>, 32},  // D <= 288 (n <= 24: azobenzene)
    // sweep variants of the ethanol shape (MLFF_PT_VARIANT)
    {2, 18, k_pt_pair<2, 18, 2, true, false>, 128},
    {2, 18, k_pt_pair<2, 18, 2, true, true>, 128},
    {4, 10, k_pt_pair<4, 10, 2, true, true>, 64},
    {4, 10, k_pt_pair<4, 10, 1, true, true>, 64},
    {1, 36, k_pt_pair<1, 36, 2, false, false>, 256},
    {2, 18, k_pt_pair<2, 18, 1, true, false, 3>, 128},   // 10: 3 waves per SIMD
    {2, 18, k_pt_pair<2, 18, 1, true, true, 3>, 128},
    {2, 18, k_pt_pair<2, 18, 1, false, false, 3>, 128},
    {2, 18, k_pt_pair<2, 18, 1, false, false, 4>, 128},
    // 14, 15: the force sum (and 15: diff . Zt) on the matrix cores (D <= 36; MLFF_PT_MFMA=1 / 2)
    {1, 36, k_pt_mfma<36, 3, false>, kMfPts},
    {1, 36, k_pt_mfma<36, 3, true>, kMfPts},
    // 16: 14 software-pipelined (the force MFMAs of one row group beside the next one's VALU rows;
    // MLFF_PT_MFMA=3)
    {1, 36, k_pt_mfma_sp<36, 3>, kMfPts},
};

const PtVariant *pt_variant(int64_t D) {
  const char *ev = std::getenv("MLFF_PT_VARIANT");
  int forced = ev != nullptr ? std::atoi(ev) : -1;
  constexpr int nv = (int)(sizeof(kPtVariants) / sizeof(kPtVariants[0]));
  if (forced < 0 && D <= 36)
    if (const char *em = std::getenv("MLFF_PT_MFMA"); em != nullptr && std::atoi(em) != 0)
      forced = nv - 4 + std::min(std::max(std::atoi(em), 1), 3);
  if (forced >= 0 && forced < nv && D <= (int64_t)kPtVariants[forced].L * kPtVariants[forced].DL)
    return &kPtVariants[forced];
  for (int i = 0; i < 5; ++i)
    if (D <= (int64_t)kPtVariants[i].L * kPtVariants[i].DL) return &kPtVariants[i];
  return nullptr;
}

}  // namespace

bool pt_supported(int64_t D) { return pt_variant(D) != nullptr; }

// chunks of the (j, p) range: about two workgroups per CU in all (each a few waves of one
// point block), chunks of at least 16 rows so that the partial F traffic (S x ni x DP x 16
// bytes) stays small against the pairs
int pt_chunks(int64_t D, int64_t ni, int64_t MP) {
  const PtVariant *v = pt_variant(D);
  if (v == nullptr || ni <= 0) return 1;
  const int64_t G = v->G, blocks = (ni + G - 1) / G;
  // one round of resident workgroups: the chip holds CUs x (workgroups per CU at this
  // kernel's registers) at once, and a grid one workgroup past that runs a second round of
  // the same length (M = 2777: 528 workgroups on 512 slots took 120 us, 506 take ~60)
  int dev = 0, cus = 256, per_cu = 2;
  if (hipGetDevice(&dev) == hipSuccess) {
    hipDeviceProp_t prop;
    if (hipGetDeviceProperties(&prop, dev) == hipSuccess) cus = prop.multiProcessorCount;
    int nb = 0;
    if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&nb, reinterpret_cast<const void *>(v->fn),
                                                     kPtThreads, 0) == hipSuccess && nb > 0)
      per_cu = nb;
  }
  const int64_t slots = (int64_t)cus * per_cu;
  int64_t S = std::max<int64_t>(1, slots / blocks);
  // chunks of at least 16 rows -- unless that leaves the grid under a quarter of the CUs (few
  // training points: configs[0]'s M = 111 ran 7 workgroups); then at least 4 rows (M = 111:
  // 28 chunks, operator 20.3 -> 16.4 us, PCG step 38.7 -> 35.1 us; M = 583 keeps 37 x 5 = 185
  // workgroups, where 52 / 74 chunks were slower; profiles/r05/pt_small/)
  if (blocks * std::min<int64_t>(S, (MP + 15) / 16) < cus / 4)
    S = std::min<int64_t>(S, (MP + 3) / 4);
  else
    S = std::min<int64_t>(S, (MP + 15) / 16);
  if (const char *e = std::getenv("MLFF_PT_CHUNKS")) S = std::atoi(e);  // sweeps
  return (int)std::max<int64_t>(1, std::min<int64_t>(S, MP));
}

int64_t pt_padded_d(int64_t D) {
  const PtVariant *v = pt_variant(D);
  return v == nullptr ? D : (int64_t)v->L * v->DL;
}

void launch_pt_operator(const MfData &mf, const double *Rt, const double *xc, int64_t row0,
                        int64_t nrows, const double *x_loc, double *y_loc, const int *status,
                        double sigma, double lam, double *pq_part, hipStream_t s,
                        const PFuse *pf) {
  const PtVariant *v = pt_variant(mf.D);
  const int64_t MP = mf.M * mf.n_perms;
  // Zt = (J_j x_j)[P_p] once per application (k_mf_z, kernels_mf.hip); fused: of p = z + beta x
  launch_mf_zt(mf, xc, status, s, pf);
  PtArgs a;
  a.Rd = mf.Rd;
  a.Rt = Rt;
  a.Zt = mf.Zt;
  a.D = mf.D;
  a.i0 = mf.i0;
  a.ni = mf.ni;
  a.MP = MP;
  a.S = mf.pt_S;
  a.sig = mf.sig;
  a.sig2 = mf.sig * mf.sig;
  a.inv_sig = 1.0 / mf.sig;
  a.k5 = 5.0 / (3.0 * mf.sig * mf.sig * mf.sig * mf.sig);
  a.part = mf.ptpart;
  const int64_t G = v->G;
  hipLaunchKernelGGL(v->fn, dim3((unsigned)((mf.ni + G - 1) / G), (unsigned)mf.pt_S), dim3(kPtThreads),
                     0, s, a, status);
  PtFin fa;
  fa.part = mf.ptpart;
  fa.Rdd = mf.Rdd;
  fa.D = mf.D;
  fa.DP = (int64_t)v->L * v->DL;
  fa.i0 = mf.i0;
  fa.ni = mf.ni;
  fa.row0 = row0;
  fa.nrows = nrows;
  fa.S = mf.pt_S;
  fa.n = mf.n;
  fa.sigma = sigma;
  fa.lam = lam;
  fa.xloc = x_loc;
  fa.y = y_loc;
  fa.pq_part = pq_part;
  if (pf != nullptr) {  // one rank holding every row (mf_can_fuse_p): x_loc is p_old
    fa.z = pf->z;
    fa.st = pf->st;
    fa.it = pf->it;
  }
  const unsigned grid = pq_part != nullptr ? (unsigned)kVecGrid
                                           : (unsigned)std::min<int64_t>(mf.ni, 2048);
  hipLaunchKernelGGL(k_pt_fin, dim3(std::max(grid, 1u)), dim3(256), 0, s, fa, status);
}

}  // namespace mlff
