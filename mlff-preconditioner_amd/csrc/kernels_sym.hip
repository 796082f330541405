// Symmetric tiled kernel operator: y = sigma * K v + lam * v reading only the
// lower block triangle of K (half the HBM bytes of the dense row GEMV).
//
// Reference operator: K_op (src/sGDML/sgdml/solvers/iterative_solver.py:383-445),
// the sGDML kernel is symmetric by construction (train.py:81-236 mirrors the lower
// block triangle); the RBF kernel (src/tools/utils.py:173-187) is symmetric entry
// by entry.  SURVEY §8d: "if symmetric (half) storage is ever used, still report
// against 8 N^2 and state it".
//
// Storage: the padded global index space [0, Np) (Np = nb * B, the rank-block
// `pos` coordinates of the dense layout) is cut into B x B tiles; tile (I, J),
// I >= J, is stored contiguously (B x B row-major) once, by exactly one rank.
// Diagonal tiles are stored full.
//
// Mat-vec: one workgroup per stored tile.  Each wave streams B/4 rows of the tile
// (lane = 4 double2 columns, non-temporal 16-B loads) and forms
//   row partials  s_i = sum_c A[i, c] v[J B + c]      -> slot J of row I B + i
//   column partials t_c = sum_i A[i, c] v[I B + i]    -> slot I of row J B + c (I > J)
// Row partials of a batch of 8 rows are summed across the 64 lanes through a
// wave-private LDS transpose (8 stores, 4 loads, 3 exchanges per batch); column
// partials stay in registers for the whole tile and are combined across the 4
// waves through LDS.
// Every (slot, row) of the slot buffer P (nb x Np) is written by exactly one tile
// (no atomics), and a second kernel sums the nb slots of each row in a fixed
// order -> the result is bitwise deterministic.
#include "common.h"

namespace mlff {

typedef double d2 __attribute__((ext_vector_type(2)));

namespace {

constexpr int B = kSymTile;  // 512
constexpr int kRowsPerWave = B / 4;
constexpr int kRB = 8;  // rows per batch (loads in flight per wave: kRB x 4 KB)

template <bool DIAG>
__device__ __forceinline__ void tile_body(const double *__restrict__ A, int I, int J,
                                          const double *__restrict__ v,
                                          double *__restrict__ P, int64_t Np,
                                          double *__restrict__ sh) {
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  const d2 *v2 = reinterpret_cast<const d2 *>(v + (int64_t)J * B);
  d2 pc[4];
#pragma unroll
  for (int q = 0; q < 4; ++q) pc[q] = v2[lane + 64 * q];
  double *vrow = sh;                       // v[I B .. I B + B)
  double *rows = sh + B;                   // row partials of the tile
  double *cs = sh + 2 * B;                 // 4 x B column partials
  double *red = sh + 6 * B + w * kRB * 64; // wave-private kRB x 64 transpose buffer
  if (!DIAG)
    for (int i = threadIdx.x; i < B; i += 256) vrow[i] = v[(int64_t)I * B + i];
  __syncthreads();
  d2 acc[4];
#pragma unroll
  for (int q = 0; q < 4; ++q) acc[q] = d2{0.0, 0.0};
#pragma unroll 1
  for (int g = 0; g < kRowsPerWave / kRB; ++g) {
    const int rbase = (g * 4 + w) * kRB;  // batches interleaved across the 4 waves
    const d2 *rowp = reinterpret_cast<const d2 *>(A + (int64_t)rbase * B) + lane;
    d2 a[kRB][4];
#pragma unroll
    for (int rr = 0; rr < kRB; ++rr)
#pragma unroll
      for (int q = 0; q < 4; ++q) a[rr][q] = __builtin_nontemporal_load(rowp + rr * (B / 2) + 64 * q);
#pragma unroll
    for (int rr = 0; rr < kRB; ++rr) {
      double s0 = a[rr][0].x * pc[0].x;
      double s1 = a[rr][0].y * pc[0].y;
#pragma unroll
      for (int q = 1; q < 4; ++q) {
        s0 = fma(a[rr][q].x, pc[q].x, s0);
        s1 = fma(a[rr][q].y, pc[q].y, s1);
      }
      red[rr * 64 + lane] = s0 + s1;
      if (!DIAG) {
        const double pr = vrow[rbase + rr];
#pragma unroll
        for (int q = 0; q < 4; ++q) {
          acc[q].x = fma(a[rr][q].x, pr, acc[q].x);
          acc[q].y = fma(a[rr][q].y, pr, acc[q].y);
        }
      }
    }
    // row sums: lane 8 r + c adds lanes 8c .. 8c + 7 of row r, then xor over c
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
    const d2 *rp = reinterpret_cast<const d2 *>(red + (lane >> 3) * 64 + (lane & 7) * 8);
    const d2 t0 = rp[0], t1 = rp[1], t2 = rp[2], t3 = rp[3];
    double t = ((t0.x + t0.y) + (t1.x + t1.y)) + ((t2.x + t2.y) + (t3.x + t3.y));
    t += __shfl_xor(t, 1, 64);
    t += __shfl_xor(t, 2, 64);
    t += __shfl_xor(t, 4, 64);
    if ((lane & 7) == 0) rows[rbase + (lane >> 3)] = t;
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
  }
  if (!DIAG) {
    d2 *cs2 = reinterpret_cast<d2 *>(cs);
#pragma unroll
    for (int q = 0; q < 4; ++q) cs2[w * (B / 2) + lane + 64 * q] = acc[q];
  }
  __syncthreads();
  // slot stores are non-temporal: interleaved with the tile stream they cost ~4 %
  // of the kernel as ordinary stores (scripts/probe_symv.hip)
  double *Prow = P + (int64_t)J * Np + (int64_t)I * B;
  for (int c = threadIdx.x; c < B; c += 256) __builtin_nontemporal_store(rows[c], Prow + c);
  if (!DIAG) {
    double *Pcol = P + (int64_t)I * Np + (int64_t)J * B;
    for (int c = threadIdx.x; c < B; c += 256)
      __builtin_nontemporal_store((cs[c] + cs[B + c]) + (cs[2 * B + c] + cs[3 * B + c]), Pcol + c);
  }
}

__global__ __launch_bounds__(256) void k_symv_tiles(const double *__restrict__ tiles,
                                                    const int2 *__restrict__ list,
                                                    const double *__restrict__ v,
                                                    double *__restrict__ P, int64_t Np,
                                                    const int *__restrict__ status) {
  if (status != nullptr && *status != ST_RUNNING) return;
  __shared__ double sh[6 * B + 4 * kRB * 64];
  const int2 t = list[blockIdx.x];
  const double *A = tiles + (int64_t)blockIdx.x * B * B;
  if (t.x == t.y)
    tile_body<true>(A, t.x, t.y, v, P, Np, sh);
  else
    tile_body<false>(A, t.x, t.y, v, P, Np, sh);
}

__device__ __forceinline__ int owner_of(int I, int J, int tiles_per_rank) {
  const int a = I / tiles_per_rank, c = J / tiles_per_rank;
  if (a == c) return a;
  return ((I + J) & 1) ? a : c;
}

// y[i] = sum_{t=0}^{nb-1} P[t, i] over the slots whose tile this rank owns
// (all slots on one rank); EPI: y = sigma * y + lam * vloc for rows < n_out
template <bool ALL, bool EPI>
__global__ __launch_bounds__(256) void k_sym_reduce(const double *__restrict__ P, int64_t Np,
                                                    int nb, int rank, int tiles_per_rank,
                                                    int64_t n_out, double *__restrict__ y,
                                                    double sigma, double lam,
                                                    const double *__restrict__ vloc,
                                                    const int *__restrict__ status) {
  if (status != nullptr && *status != ST_RUNNING) return;
  const int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x;
  if (i >= n_out) return;
  const int bi = (int)(i / B);
  double s = 0.0;
  if (ALL) {
    // 8 slot loads in flight per thread; the additions stay in slot order
    int t = 0;
    for (; t + 7 < nb; t += 8) {
      double v[8];
#pragma unroll
      for (int u = 0; u < 8; ++u) v[u] = __builtin_nontemporal_load(P + (int64_t)(t + u) * Np + i);
#pragma unroll
      for (int u = 0; u < 8; ++u) s += v[u];
    }
    for (; t < nb; ++t) s += P[(int64_t)t * Np + i];
  } else {
    for (int t = 0; t < nb; ++t) {
      const int I = bi > t ? bi : t, J = bi > t ? t : bi;
      if (owner_of(I, J, tiles_per_rank) != rank) continue;
      s += P[(int64_t)t * Np + i];
    }
  }
  if (EPI) {
    double yv = sigma * s;
    if (vloc != nullptr) yv += lam * vloc[i];
    y[i] = yv;
  } else {
    y[i] = s;
  }
}

__global__ __launch_bounds__(256) void k_axpby_loc(double *__restrict__ y, int64_t n, double sigma,
                                                   double lam, const double *__restrict__ vloc,
                                                   const int *__restrict__ status) {
  if (status != nullptr && *status != ST_RUNNING) return;
  const int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x;
  if (i >= n) return;
  double yv = sigma * y[i];
  if (vloc != nullptr) yv += lam * vloc[i];
  y[i] = yv;
}

// Pack (COMPARE = false) or verify symmetry (COMPARE = true) of one stored tile per
// workgroup, 64 x 64 sub-blocks through LDS.  Source rows are this rank's dense
// rows (row stride ld, global row g at local row g - rowbase).  TRANS: the tile is
// read from rows J B + c (symmetric mirror) instead of rows I B + r.
template <bool COMPARE>
__global__ __launch_bounds__(256) void k_sym_pack(const double *__restrict__ K, int64_t ld,
                                                  int64_t rowbase, int64_t nloc, const int2 *__restrict__ list,
                                                  const unsigned char *__restrict__ trans,
                                                  double *__restrict__ tiles,
                                                  int *__restrict__ mismatch) {
  __shared__ double S[64][65];
  const int2 t = list[blockIdx.x];
  const bool tr = trans[blockIdx.x] != 0;
  double *T = tiles + (int64_t)blockIdx.x * B * B;
  const int tx = threadIdx.x & 63, ty = threadIdx.x >> 6;
  int bad = 0;
  for (int sb = 0; sb < (B / 64) * (B / 64); ++sb) {
    const int br = (sb / (B / 64)) * 64, bc = (sb % (B / 64)) * 64;  // sub-block of the tile
    // source sub-block rows / cols
    const int64_t srow = tr ? (int64_t)t.y * B + bc : (int64_t)t.x * B + br;
    const int64_t scol = tr ? (int64_t)t.x * B + br : (int64_t)t.y * B + bc;
    __syncthreads();
    // outside the dense block (rows beyond this rank's, columns beyond ld: the
    // padding of Np = round_up(ld, B) on one rank) the matrix is zero
    for (int a = ty; a < 64; a += 4) {
      const int64_t lr = srow + a - rowbase, c = scol + tx;
      S[a][tx] = (lr >= 0 && lr < nloc && c < ld) ? K[lr * ld + c] : 0.0;
    }
    __syncthreads();
    for (int a = ty; a < 64; a += 4) {
      const double val = tr ? S[tx][a] : S[a][tx];  // tile(br + a, bc + tx)
      double *dst = T + (int64_t)(br + a) * B + bc + tx;
      if (COMPARE) {
        if (*dst != val) bad = 1;
      } else {
        *dst = val;
      }
    }
  }
  if (COMPARE && bad) atomicOr(mismatch, 1);
}

}  // namespace

void launch_symv(const SymPack &sp, const double *v_full, double *P, const int *status,
                 hipStream_t s) {
  if (sp.ntiles == 0) return;
  hipLaunchKernelGGL(k_symv_tiles, dim3((unsigned)sp.ntiles), dim3(256), 0, s, sp.tiles, sp.list,
                     v_full, P, sp.Np, status);
}

void launch_sym_reduce(const SymPack &sp, int rank, int world, int64_t n_out, double *y,
                       bool epilogue, double sigma, double lam, const double *vloc,
                       const int *status, hipStream_t s) {
  if (n_out <= 0) return;
  const dim3 grid((unsigned)((n_out + 255) / 256));
  if (world == 1) {
    if (epilogue)
      hipLaunchKernelGGL((k_sym_reduce<true, true>), grid, dim3(256), 0, s, sp.P, sp.Np, (int)sp.nb,
                         rank, (int)sp.tiles_per_rank, n_out, y, sigma, lam, vloc, status);
    else
      hipLaunchKernelGGL((k_sym_reduce<true, false>), grid, dim3(256), 0, s, sp.P, sp.Np,
                         (int)sp.nb, rank, (int)sp.tiles_per_rank, n_out, y, sigma, lam, vloc,
                         status);
  } else {
    hipLaunchKernelGGL((k_sym_reduce<false, false>), grid, dim3(256), 0, s, sp.P, sp.Np,
                       (int)sp.nb, rank, (int)sp.tiles_per_rank, n_out, y, sigma, lam, vloc,
                       status);
  }
}

void launch_axpby_loc(double *y, int64_t n, double sigma, double lam, const double *vloc,
                      const int *status, hipStream_t s) {
  if (n <= 0) return;
  hipLaunchKernelGGL(k_axpby_loc, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, s, y, n, sigma,
                     lam, vloc, status);
}

// host-side tile assignment (same rule as owner_of)
static int owner_host(int I, int J, int tpr) {
  const int a = I / tpr, c = J / tpr;
  if (a == c) return a;
  return ((I + J) & 1) ? a : c;
}

int sym_build(mlff_ctx *ctx, bool check_symmetry, bool *symmetric_out) {
  SymPack &sp = ctx->sym;
  hipStream_t s = ctx->stream;
  const int64_t Np = round_up(ctx->ld, B);
  const int nb = (int)(Np / B);
  // tiles per rank block: blk is a multiple of B when world > 1 (mlff_ctx_create)
  const int tpr = ctx->world > 1 ? (int)(ctx->blk / B) : nb;
  std::vector<int2> list;
  std::vector<unsigned char> trans;
  for (int I = 0; I < nb; ++I)
    for (int J = 0; J <= I; ++J) {
      if (owner_host(I, J, tpr) != ctx->rank) continue;
      list.push_back(make_int2(I, J));
      trans.push_back(ctx->world > 1 && (I / tpr) != ctx->rank ? 1 : 0);
    }
  const int64_t nt = (int64_t)list.size();
  if (sp.tiles == nullptr || sp.ntiles != nt || sp.Np != Np) {
    sym_free(sp);
    if (nt > 0) {
      MLFF_HIP(ctx, hipMalloc(&sp.tiles, sizeof(double) * nt * B * B));
      MLFF_HIP(ctx, hipMalloc(&sp.list, sizeof(int2) * nt));
    }
    MLFF_HIP(ctx, hipMalloc(&sp.P, sizeof(double) * (int64_t)nb * Np));
    MLFF_HIP(ctx, hipMalloc(&sp.yg, sizeof(double) * Np));
    MLFF_HIP(ctx, hipMemsetAsync(sp.P, 0, sizeof(double) * (int64_t)nb * Np, s));
    MLFF_HIP(ctx, hipMemsetAsync(sp.yg, 0, sizeof(double) * Np, s));
  }
  sp.ntiles = nt;
  sp.Np = Np;
  sp.nb = nb;
  sp.tiles_per_rank = tpr;
  unsigned char *dtrans = nullptr;
  int *dflag = nullptr;
  if (nt > 0) {
    MLFF_HIP(ctx, hipMemcpyAsync(sp.list, list.data(), sizeof(int2) * nt, hipMemcpyHostToDevice, s));
    MLFF_HIP(ctx, hipMalloc(&dtrans, nt));
    MLFF_HIP(ctx, hipMalloc(&dflag, sizeof(int)));
    MLFF_HIP(ctx, hipMemcpyAsync(dtrans, trans.data(), nt, hipMemcpyHostToDevice, s));
    MLFF_HIP(ctx, hipMemsetAsync(dflag, 0, sizeof(int), s));
    const int64_t rowbase = (int64_t)ctx->rank * ctx->blk;
    const double *Ksrc = ctx->K;
    const int64_t ldsrc = ctx->ld;
    hipLaunchKernelGGL(k_sym_pack<false>, dim3((unsigned)nt), dim3(256), 0, s, Ksrc, ldsrc, rowbase,
                       ctx->blk, sp.list, dtrans, sp.tiles, dflag);
    int mism = 0;
    if (check_symmetry) {
      // mirror read: every tile compared against rows J B + c (one rank holds all rows)
      MLFF_HIP(ctx, hipMemsetAsync(dtrans, 1, nt, s));
      hipLaunchKernelGGL(k_sym_pack<true>, dim3((unsigned)nt), dim3(256), 0, s, Ksrc, ldsrc, rowbase,
                         ctx->blk, sp.list, dtrans, sp.tiles, dflag);
      MLFF_HIP(ctx, hipMemcpyAsync(&mism, dflag, sizeof(int), hipMemcpyDeviceToHost, s));
    }
    MLFF_HIP(ctx, hipGetLastError());
    MLFF_HIP(ctx, hipStreamSynchronize(s));
    hipFree(dtrans);
    hipFree(dflag);
    if (symmetric_out) *symmetric_out = (mism == 0);
  } else if (symmetric_out) {
    *symmetric_out = true;
  }
  sp.ready = true;
  return MLFF_OK;
}

void sym_free(SymPack &sp) {
  for (void *p : {(void *)sp.tiles, (void *)sp.list, (void *)sp.P, (void *)sp.yg})
    if (p) (void)hipFree(p);
  sp.tiles = nullptr;
  sp.list = nullptr;
  sp.P = nullptr;
  sp.yg = nullptr;
  sp.ntiles = 0;
  sp.ready = false;
}

}  // namespace mlff
