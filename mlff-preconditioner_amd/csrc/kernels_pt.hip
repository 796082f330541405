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
  if (status != nullptr && *status != ST_RUNNING) return;
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
  if (status != nullptr && *status != ST_RUNNING) return;
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
    if (blockIdx.x == 0 && threadIdx.x == 0) a.st->rho = rho;
  }
  double pq = 0.0;
  for (int64_t il = blockIdx.x; il < a.ni; il += gridDim.x) {
    const int64_t i = a.i0 + il;
    const double *src = a.part + il * a.DP;
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
      if (a.xloc != nullptr) {  // requested before the J^T sum
        xv = a.xloc[rl];
        if (fp) xv = fused_p(xv, a.z[rl], beta, first);
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
  if (a.pq_part != nullptr) {
    const double t = block_sum256(pq, sh);
    if (threadIdx.x == 0) a.pq_part[blockIdx.x] = t;
  }
}

using PairFn = void (*)(PtArgs, const int *);

struct PtVariant {
  int L, DL;
  PairFn fn;
};

// L lanes per point (partial sums joined by the DPP butterfly), DL entries per lane; the
// first variant that covers D is the default.  MLFF_PT_VARIANT=<index> forces one (sweeps; it
// must cover D)
const PtVariant kPtVariants[] = {
    {2, 18, k_pt_pair<2, 18, 1, true, true>},    // D <= 36  (n <= 9: ethanol)
    {4, 18, k_pt_pair<4, 18, 1, true, false>},   // D <= 72  (n <= 12: uracil)
    {4, 28, k_pt_pair<4, 28, 1, false, false>},  // D <= 112 (n <= 15: toluene)
    {8, 28, k_pt_pair<8, 28, 1, false, false>},  // D <= 224 (n <= 21: aspirin)
    {8, 36, k_pt_pair<8, 36, 1, false, false>},  // D <= 288 (n <= 24: azobenzene)
    // sweep variants of the ethanol shape (MLFF_PT_VARIANT)
    {2, 18, k_pt_pair<2, 18, 2, true, false>},
    {2, 18, k_pt_pair<2, 18, 2, true, true>},
    {4, 10, k_pt_pair<4, 10, 2, true, true>},
    {4, 10, k_pt_pair<4, 10, 1, true, true>},
    {1, 36, k_pt_pair<1, 36, 2, false, false>},
    {2, 18, k_pt_pair<2, 18, 1, true, false, 3>},   // 10: 3 waves per SIMD
    {2, 18, k_pt_pair<2, 18, 1, true, true, 3>},
    {2, 18, k_pt_pair<2, 18, 1, false, false, 3>},
    {2, 18, k_pt_pair<2, 18, 1, false, false, 4>},
};

const PtVariant *pt_variant(int64_t D) {
  const char *ev = std::getenv("MLFF_PT_VARIANT");
  const int forced = ev != nullptr ? std::atoi(ev) : -1;
  constexpr int nv = (int)(sizeof(kPtVariants) / sizeof(kPtVariants[0]));
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
  const int64_t G = kPtThreads / v->L, blocks = (ni + G - 1) / G;
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
  const int64_t G = kPtThreads / v->L;
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
