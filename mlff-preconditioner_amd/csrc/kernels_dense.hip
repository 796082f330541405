// Dense fp64 building blocks of the low-rank preconditioner builds (SYRK, POTRF,
// TRSM on "wide" k x N panels).  They replace the numpy/LAPACK calls of
//   iterative_cholesky.py:141-143   kernel = lam I + L^T L; L2 = cholesky; T = L2^-1 L^T
//   iterative_solver.py:218-283     Nystrom: cho_factor / solve_triangular / K_nm^T K_nm
//   iterative_solver.py:370-374     _sb variant
//   iterative_solver.py:507-550     leverage scores
// Panels are stored k x ncols row-major ("wide"), so every panel operation reads
// contiguous 512-B row segments.
#include "common.h"

#include <cstdlib>

namespace mlff {

// ---------------------------------------------------------------------------
// Tiled fp64 GEMM, 64 x 64 output tile per 256-thread workgroup, 4 x 4 per
// thread, BK = 16.  blockIdx.z = K split (slab = C + z * slab_stride).
template <bool TA, bool TB>
__global__ __launch_bounds__(256) void k_gemm(int64_t M, int64_t N, int64_t K, double alpha,
                                              const double *__restrict__ A, int64_t lda,
                                              const double *__restrict__ B, int64_t ldb,
                                              double beta, double *__restrict__ C, int64_t ldc,
                                              int64_t kchunk, int64_t slab_stride, int tri) {
  constexpr int BM = 64, BN = 64, BK = 16;
  // tri: only the tiles touching the lower triangle (a symmetric product, mirrored after)
  if (tri && (int64_t)blockIdx.x * BN >= (int64_t)blockIdx.y * BM + BM) return;
  __shared__ double As[BK][BM + 1];
  __shared__ double Bs[BK][BN + 1];
  const int tid = threadIdx.x;
  const int tx = tid & 15, ty = tid >> 4;
  const int64_t m0 = (int64_t)blockIdx.y * BM, n0 = (int64_t)blockIdx.x * BN;
  const int64_t kb = (int64_t)blockIdx.z * kchunk;
  int64_t ke = kb + kchunk;
  if (ke > K) ke = K;
  C += (int64_t)blockIdx.z * slab_stride;
  double acc[4][4];
#pragma unroll
  for (int i = 0; i < 4; ++i)
#pragma unroll
    for (int j = 0; j < 4; ++j) acc[i][j] = 0.0;

  for (int64_t k0 = kb; k0 < ke; k0 += BK) {
#pragma unroll
    for (int l = 0; l < 4; ++l) {
      const int e = tid + 256 * l;
      int mm, kk;
      if (TA) { kk = e >> 6; mm = e & 63; } else { mm = e >> 4; kk = e & 15; }
      const int64_t gm = m0 + mm, gk = k0 + kk;
      double a = 0.0;
      if (gm < M && gk < ke) a = TA ? A[gk * lda + gm] : A[gm * lda + gk];
      As[kk][mm] = a;
      int nn, kb2;
      if (TB) { nn = e >> 4; kb2 = e & 15; } else { kb2 = e >> 6; nn = e & 63; }
      const int64_t gn = n0 + nn, gk2 = k0 + kb2;
      double bv = 0.0;
      if (gn < N && gk2 < ke) bv = TB ? B[gn * ldb + gk2] : B[gk2 * ldb + gn];
      Bs[kb2][nn] = bv;
    }
    __syncthreads();
#pragma unroll
    for (int kk = 0; kk < BK; ++kk) {
      double a[4], bb[4];
#pragma unroll
      for (int i = 0; i < 4; ++i) a[i] = As[kk][ty + 16 * i];
#pragma unroll
      for (int j = 0; j < 4; ++j) bb[j] = Bs[kk][tx + 16 * j];
#pragma unroll
      for (int i = 0; i < 4; ++i)
#pragma unroll
        for (int j = 0; j < 4; ++j) acc[i][j] = fma(a[i], bb[j], acc[i][j]);
    }
    __syncthreads();
  }
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    const int64_t gm = m0 + ty + 16 * i;
    if (gm >= M) continue;
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      const int64_t gn = n0 + tx + 16 * j;
      if (gn >= N) continue;
      double v = alpha * acc[i][j];
      if (beta != 0.0) v = fma(beta, C[gm * ldc + gn], v);
      C[gm * ldc + gn] = v;
    }
  }
}

// ---------------------------------------------------------------------------
// The same GEMM on the matrix cores (v_mfma_f64_16x16x4_f64): BM x 128 output tile per
// 256-thread workgroup (BM = 64 or 128), the four waves 2 x 2 over it, each wave BM/2 x 64
// as (BM/32) x 4 blocks of 16 x 16; K staged through LDS 16 at a time exactly as k_gemm
// stages it.  Lane l of a 16x16x4 step holds A[row l&15][k l>>4] and B[k l>>4][col l&15];
// register r of its result is C[row (l>>4) + 4r][col l&15] (cdna_hip_programming.md, f64
// MFMA layout).  LDS rows padded to 144 doubles (288 dwords = 32 mod 64 banks): the four
// k rows one step reads fall on disjoint bank halves pairwise (2 passes, the minimum).
// Fixed summation order (k ascending, 4 per instruction): deterministic.
typedef double v4d __attribute__((ext_vector_type(4)));
template <int BM, bool TA, bool TB, int NTH = 256>
__global__ __launch_bounds__(NTH) void k_gemm_mfma(int64_t M, int64_t N, int64_t K, double alpha,
                                                   const double *__restrict__ A, int64_t lda,
                                                   const double *__restrict__ B, int64_t ldb,
                                                   double beta, double *__restrict__ C,
                                                   int64_t ldc, int64_t kchunk,
                                                   int64_t slab_stride, int tri) {
  constexpr int BN = 128, BK = 16, LP = 144;
  if (tri && (int64_t)blockIdx.x * BN >= (int64_t)blockIdx.y * BM + BM) return;
  constexpr int WR = NTH / 128;        // wave rows (two wave columns of 64)
  constexpr int IM = BM / WR / 16, JN = 4;  // 16 x 16 blocks per wave
  static_assert(IM >= 1, "tile too small for the wave grid");
  constexpr int LA = BM * BK / NTH, LB = BN * BK / NTH;  // staged elements per thread
  __shared__ double As[BK][LP];
  __shared__ double Bs[BK][LP];
  const int tid = threadIdx.x, lane = tid & 63, wv = tid >> 6;
  const int wm = (wv >> 1) * (BM / WR), wn = (wv & 1) * 64;
  const int64_t m0 = (int64_t)blockIdx.y * BM, n0 = (int64_t)blockIdx.x * BN;
  const int64_t kb = (int64_t)blockIdx.z * kchunk;
  int64_t ke = kb + kchunk;
  if (ke > K) ke = K;
  C += (int64_t)blockIdx.z * slab_stride;
  v4d acc[IM][JN];
#pragma unroll
  for (int i = 0; i < IM; ++i)
#pragma unroll
    for (int j = 0; j < JN; ++j) acc[i][j] = v4d{0.0, 0.0, 0.0, 0.0};
  // software pipeline: the next K tile's global loads are in flight while the matrix
  // cores work on the current one (one wave per SIMD at this register count)
  double va[LA], vb[LB];
  auto load_tile = [&](int64_t k0) {
#pragma unroll
    for (int l = 0; l < LA; ++l) {
      const int e = tid + NTH * l;
      const int mm = TA ? (e % BM) : (e / BK), kk = TA ? (e / BM) : (e % BK);
      const int64_t gm = m0 + mm, gk = k0 + kk;
      va[l] = (gm < M && gk < ke) ? (TA ? A[gk * lda + gm] : A[gm * lda + gk]) : 0.0;
    }
#pragma unroll
    for (int l = 0; l < LB; ++l) {
      const int e = tid + NTH * l;
      const int nn = TB ? (e / BK) : (e % BN), kk = TB ? (e % BK) : (e / BN);
      const int64_t gn = n0 + nn, gk = k0 + kk;
      vb[l] = (gn < N && gk < ke) ? (TB ? B[gn * ldb + gk] : B[gk * ldb + gn]) : 0.0;
    }
  };
  if (kb < ke) load_tile(kb);
  for (int64_t k0 = kb; k0 < ke; k0 += BK) {
    __syncthreads();  // the previous step's fragment reads are done
#pragma unroll
    for (int l = 0; l < LA; ++l) {
      const int e = tid + NTH * l;
      As[TA ? (e / BM) : (e % BK)][TA ? (e % BM) : (e / BK)] = va[l];
    }
#pragma unroll
    for (int l = 0; l < LB; ++l) {
      const int e = tid + NTH * l;
      Bs[TB ? (e % BK) : (e / BN)][TB ? (e / BK) : (e % BN)] = vb[l];
    }
    __syncthreads();
    if (k0 + BK < ke) load_tile(k0 + BK);
#pragma unroll
    for (int ks = 0; ks < BK / 4; ++ks) {
      const int kr = 4 * ks + (lane >> 4);
      double a[IM], b[JN];
#pragma unroll
      for (int i = 0; i < IM; ++i) a[i] = As[kr][wm + 16 * i + (lane & 15)];
#pragma unroll
      for (int j = 0; j < JN; ++j) b[j] = Bs[kr][wn + 16 * j + (lane & 15)];
#pragma unroll
      for (int i = 0; i < IM; ++i)
#pragma unroll
        for (int j = 0; j < JN; ++j)
          acc[i][j] = __builtin_amdgcn_mfma_f64_16x16x4f64(a[i], b[j], acc[i][j], 0, 0, 0);
    }
  }
#pragma unroll
  for (int i = 0; i < IM; ++i)
#pragma unroll
    for (int j = 0; j < JN; ++j)
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int64_t gm = m0 + wm + 16 * i + (lane >> 4) + 4 * r;
        const int64_t gn = n0 + wn + 16 * j + (lane & 15);
        if (gm >= M || gn >= N) continue;
        double v = alpha * acc[i][j][r];
        if (beta != 0.0) v = fma(beta, C[gm * ldc + gn], v);
        C[gm * ldc + gn] = v;
      }
}

template <int BM, int NTH>
static void gemm_mfma_launch_t(bool ta, bool tb, int64_t M, int64_t Nc, int64_t Kd, double alpha,
                               const double *A, int64_t lda, const double *B, int64_t ldb,
                               double beta, double *C, int64_t ldc, int64_t kchunk, int splits,
                               int64_t slab_stride, hipStream_t s, int tri) {
  dim3 grid((unsigned)((Nc + 127) / 128), (unsigned)((M + BM - 1) / BM), (unsigned)splits);
  if (!ta && !tb)
    hipLaunchKernelGGL((k_gemm_mfma<BM, false, false, NTH>), grid, dim3(NTH), 0, s, M, Nc, Kd, alpha,
                       A, lda, B, ldb, beta, C, ldc, kchunk, slab_stride, tri);
  else if (!ta && tb)
    hipLaunchKernelGGL((k_gemm_mfma<BM, false, true, NTH>), grid, dim3(NTH), 0, s, M, Nc, Kd, alpha,
                       A, lda, B, ldb, beta, C, ldc, kchunk, slab_stride, tri);
  else if (ta && !tb)
    hipLaunchKernelGGL((k_gemm_mfma<BM, true, false, NTH>), grid, dim3(NTH), 0, s, M, Nc, Kd, alpha,
                       A, lda, B, ldb, beta, C, ldc, kchunk, slab_stride, tri);
  else
    hipLaunchKernelGGL((k_gemm_mfma<BM, true, true, NTH>), grid, dim3(NTH), 0, s, M, Nc, Kd, alpha,
                       A, lda, B, ldb, beta, C, ldc, kchunk, slab_stride, tri);
}

// workgroup size of the matrix-core GEMM (MLFF_GEMM_NTH = 256 / 512 for A/B sweeps)
static int gemm_nth() {
  static const int nth = [] {
    const char *e = std::getenv("MLFF_GEMM_NTH");
    return (e != nullptr && std::atoi(e) == 256) ? 256 : 512;
  }();
  return nth;
}

template <int BM>
static void gemm_mfma_launch(bool ta, bool tb, int64_t M, int64_t Nc, int64_t Kd, double alpha,
                             const double *A, int64_t lda, const double *B, int64_t ldb,
                             double beta, double *C, int64_t ldc, int64_t kchunk, int splits,
                             int64_t slab_stride, hipStream_t s, int tri) {
  if (gemm_nth() == 512)
    gemm_mfma_launch_t<BM, 512>(ta, tb, M, Nc, Kd, alpha, A, lda, B, ldb, beta, C, ldc, kchunk,
                                splits, slab_stride, s, tri);
  else
    gemm_mfma_launch_t<BM, 256>(ta, tb, M, Nc, Kd, alpha, A, lda, B, ldb, beta, C, ldc, kchunk,
                                splits, slab_stride, s, tri);
}

// the matrix-core path for every GEMM at least 64 x 128 with a K of 32 or more
// (MLFF_GEMM_VALU=1 keeps the VALU kernel for A/B sweeps)
static bool use_mfma(int64_t M, int64_t Nc, int64_t Kd) {
  static const bool valu = [] {
    const char *e = std::getenv("MLFF_GEMM_VALU");
    return e != nullptr && e[0] == '1';
  }();
  return !valu && M >= 64 && Nc >= 128 && Kd >= 32;
}

static void gemm_launch(bool ta, bool tb, int64_t M, int64_t Nc, int64_t Kd, double alpha,
                        const double *A, int64_t lda, const double *B, int64_t ldb, double beta,
                        double *C, int64_t ldc, int splits, int64_t slab_stride, hipStream_t s,
                        int tri = 0) {
  if (M <= 0 || Nc <= 0) return;
  int64_t kchunk = (Kd + splits - 1) / splits;
  kchunk = round_up(kchunk < 1 ? 1 : kchunk, 16);
  if (use_mfma(M, Nc, Kd)) {
    if (M >= 128)
      gemm_mfma_launch<128>(ta, tb, M, Nc, Kd, alpha, A, lda, B, ldb, beta, C, ldc, kchunk, splits,
                            slab_stride, s, tri);
    else
      gemm_mfma_launch<64>(ta, tb, M, Nc, Kd, alpha, A, lda, B, ldb, beta, C, ldc, kchunk, splits,
                           slab_stride, s, tri);
    return;
  }
  dim3 grid((unsigned)((Nc + 63) / 64), (unsigned)((M + 63) / 64), (unsigned)splits);
  if (!ta && !tb)
    hipLaunchKernelGGL((k_gemm<false, false>), grid, dim3(256), 0, s, M, Nc, Kd, alpha, A, lda, B,
                       ldb, beta, C, ldc, kchunk, slab_stride, tri);
  else if (!ta && tb)
    hipLaunchKernelGGL((k_gemm<false, true>), grid, dim3(256), 0, s, M, Nc, Kd, alpha, A, lda, B,
                       ldb, beta, C, ldc, kchunk, slab_stride, tri);
  else if (ta && !tb)
    hipLaunchKernelGGL((k_gemm<true, false>), grid, dim3(256), 0, s, M, Nc, Kd, alpha, A, lda, B,
                       ldb, beta, C, ldc, kchunk, slab_stride, tri);
  else
    hipLaunchKernelGGL((k_gemm<true, true>), grid, dim3(256), 0, s, M, Nc, Kd, alpha, A, lda, B,
                       ldb, beta, C, ldc, kchunk, slab_stride, tri);
}

void launch_gemm(bool ta, bool tb, int64_t M, int64_t Nc, int64_t Kd, double alpha,
                 const double *A, int64_t lda, const double *B, int64_t ldb, double beta,
                 double *C, int64_t ldc, hipStream_t s) {
  gemm_launch(ta, tb, M, Nc, Kd, alpha, A, lda, B, ldb, beta, C, ldc, 1, 0, s);
}

// deterministic slab sum: G[i] = sum_s slab[s][i]
__global__ __launch_bounds__(256) void k_sum_slabs(const double *__restrict__ slabs, int splits,
                                                   int64_t n, double *__restrict__ out) {
  for (int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x; i < n;
       i += (int64_t)gridDim.x * 256) {
    double a = 0.0;
    for (int s = 0; s < splits; ++s) a += slabs[(int64_t)s * n + i];
    out[i] = a;
  }
}

int syrk_wide(mlff_ctx *ctx, const double *W, int64_t k, int64_t ncols, int64_t ldw, double *G) {
  return gram_wide(ctx, W, W, k, ncols, ldw, G);
}

// C (M x N, ld ldc) = sum_s slab_s (M x N each, ld N), fixed slab order
__global__ __launch_bounds__(256) void k_sum_slabs_ld(const double *__restrict__ slabs, int splits,
                                                      int64_t M, int64_t N, double *__restrict__ C,
                                                      int64_t ldc) {
  const int64_t n = M * N;
  for (int64_t e = (int64_t)blockIdx.x * 256 + threadIdx.x; e < n; e += (int64_t)gridDim.x * 256) {
    double a = 0.0;
    for (int sp = 0; sp < splits; ++sp) a += slabs[(int64_t)sp * n + e];
    C[(e / N) * ldc + e % N] = a;
  }
}

int gemm_splitk(mlff_ctx *ctx, bool ta, bool tb, int64_t M, int64_t N, int64_t K, const double *A,
                int64_t lda, const double *B, int64_t ldb, double *C, int64_t ldc) {
  if (M <= 0 || N <= 0) return MLFF_OK;
  const bool mf = use_mfma(M, N, K);
  const int64_t tiles = ((M + (mf ? (M >= 128 ? 127 : 63) : 63)) / (mf ? (M >= 128 ? 128 : 64) : 64)) *
                        ((N + (mf ? 127 : 63)) / (mf ? 128 : 64));
  int64_t splits = std::min<int64_t>((512 + tiles - 1) / tiles, std::max<int64_t>(1, K / 256));
  if (splits > 64) splits = 64;
  if (splits <= 1) {
    gemm_launch(ta, tb, M, N, K, 1.0, A, lda, B, ldb, 0.0, C, ldc, 1, 0, ctx->stream);
    MLFF_HIP(ctx, hipGetLastError());
    return MLFF_OK;
  }
  ScratchScope scope(ctx);
  double *slabs = nullptr;
  MLFF_TRY(scratch_alloc(ctx, &slabs, (size_t)(splits * M * N)));
  gemm_launch(ta, tb, M, N, K, 1.0, A, lda, B, ldb, 0.0, slabs, N, (int)splits, M * N, ctx->stream);
  hipLaunchKernelGGL(k_sum_slabs_ld, dim3((unsigned)std::min<int64_t>((M * N + 255) / 256, 4096)),
                     dim3(256), 0, ctx->stream, slabs, (int)splits, M, N, C, ldc);
  MLFF_HIP(ctx, hipGetLastError());
  return MLFF_OK;
}

// G[j, i] = G[i, j] for i > j (the lower triangle of a symmetric product mirrored up)
__global__ __launch_bounds__(256) void k_mirror_lower(double *__restrict__ G, int64_t k) {
  for (int64_t e = (int64_t)blockIdx.x * 256 + threadIdx.x; e < k * k;
       e += (int64_t)gridDim.x * 256) {
    const int64_t i = e / k, j = e % k;
    if (j > i) G[e] = G[j * k + i];
  }
}

// G = A B^T over ncols (k x k; A, B "wide" k x ncols panels).  A == B (a Gram matrix / SYRK):
// only the tiles touching the lower triangle are computed and mirrored -- each entry is the
// same sum in the same order either way, so G is bitwise what the full product gives
int gram_wide(mlff_ctx *ctx, const double *A, const double *Bm, int64_t k, int64_t ncols,
              int64_t ldw, double *G) {
  const double *W = A;
  const int tri = A == Bm ? 1 : 0;
  // workgroup tiles of the GEMM path taken (matrix cores: up to 128 x 128, VALU: 64 x 64)
  const int64_t tm = use_mfma(k, k, ncols) ? (k >= 128 ? 128 : 64) : 64;
  const int64_t tn = use_mfma(k, k, ncols) ? 128 : 64;
  int64_t tiles = ((k + tm - 1) / tm) * ((k + tn - 1) / tn);
  if (tri) tiles = (tiles + (k + tm - 1) / tm) / 2;
  int64_t splits = (1024 + tiles - 1) / tiles;
  const int64_t max_splits = (ncols + 511) / 512;
  if (splits > max_splits) splits = max_splits;
  if (splits < 1) splits = 1;
  if (splits > 256) splits = 256;
  const unsigned gm = (unsigned)std::min<int64_t>((k * k + 255) / 256, 4096);
  if (splits == 1) {
    gemm_launch(false, true, k, k, ncols, 1.0, W, ldw, Bm, ldw, 0.0, G, k, 1, 0, ctx->stream, tri);
    if (tri) hipLaunchKernelGGL(k_mirror_lower, dim3(gm), dim3(256), 0, ctx->stream, G, k);
    MLFF_HIP(ctx, hipGetLastError());
    return MLFF_OK;
  }
  ScratchScope scope(ctx);
  double *slabs = nullptr;
  MLFF_TRY(scratch_alloc(ctx, &slabs, splits * k * k));
  gemm_launch(false, true, k, k, ncols, 1.0, W, ldw, Bm, ldw, 0.0, slabs, k, (int)splits, k * k,
              ctx->stream, tri);
  const int64_t n = k * k;
  // (the skipped upper tiles of the slabs hold stale scratch; their sums are overwritten)
  hipLaunchKernelGGL(k_sum_slabs, dim3((unsigned)std::min<int64_t>((n + 255) / 256, 2048)),
                     dim3(256), 0, ctx->stream, slabs, (int)splits, n, G);
  if (tri) hipLaunchKernelGGL(k_mirror_lower, dim3(gm), dim3(256), 0, ctx->stream, G, k);
  MLFF_HIP(ctx, hipGetLastError());
  return MLFF_OK;
}

// ---------------------------------------------------------------------------
// Unblocked Cholesky of the jb x jb diagonal block A[j0.., j0..] in LDS.
__global__ __launch_bounds__(256) void k_potrf_diag(double *__restrict__ A, int64_t lda,
                                                    int64_t j0, int jb, int *err) {
  __shared__ double L[64][65];
  const int tid = threadIdx.x;
  for (int e = tid; e < jb * jb; e += 256) {
    const int i = e / jb, j = e % jb;
    L[i][j] = A[(j0 + i) * lda + j0 + j];
  }
  __syncthreads();
  for (int c = 0; c < jb; ++c) {
    if (tid == 0) {
      const double d = L[c][c];
      if (!(d > 0.0)) atomicExch(err, 1);
      L[c][c] = sqrt(d);
    }
    __syncthreads();
    const double dc = L[c][c];
    for (int i = c + 1 + tid; i < jb; i += 256) L[i][c] = L[i][c] / dc;
    __syncthreads();
    const int nt = jb - c - 1;
    for (int e = tid; e < nt * nt; e += 256) {
      const int i = c + 1 + e / nt, j = c + 1 + e % nt;
      if (j <= i) L[i][j] = fma(-L[i][c], L[j][c], L[i][j]);
    }
    __syncthreads();
  }
  for (int e = tid; e < jb * jb; e += 256) {
    const int i = e / jb, j = e % jb;
    if (j <= i) A[(j0 + i) * lda + j0 + j] = L[i][j];
  }
}

// The same diagonal block in ONE wave (round 6): lane i holds row i in registers, the column c
// entries L[j][c] it needs come from lane j by readlane -- k_potrf_diag's operations in its order
// (sqrt of the pivot, the column divided by it, then the right-looking fma update of the lower
// triangle), so the same bits, without its 3 x jb workgroup barriers (83 us per 64 x 64 block at
// k = 2701, profiles/r06/bench/nanotube_kernel_stats.txt)
__global__ __launch_bounds__(64) void k_potrf_diag_wave(double *__restrict__ A, int64_t lda,
                                                        int64_t j0, int jb, int *err) {
  const int i = threadIdx.x;
  double r[64];
#pragma unroll
  for (int j = 0; j < 64; ++j) r[j] = (i < jb && j < jb) ? A[(j0 + i) * lda + j0 + j] : 0.0;
  bool bad = false;
#pragma unroll
  for (int c = 0; c < 64; ++c) {
    if (c < jb) {
      const unsigned long long dbits = __builtin_bit_cast(unsigned long long, r[c]);
      const double d = __builtin_bit_cast(
          double, ((unsigned long long)(unsigned)__builtin_amdgcn_readlane((int)(dbits >> 32), c) << 32) |
                      (unsigned)__builtin_amdgcn_readlane((int)(dbits & 0xffffffffull), c));
      bad = bad || !(d > 0.0);
      const double dc = sqrt(d);
      if (i == c) r[c] = dc;
      if (i > c) r[c] = r[c] / dc;
#pragma unroll
      for (int j = c + 1; j < 64; ++j) {
        // L[j][c] from lane j: two v_readlane (compile-time lane) into scalar registers
        const unsigned long long bits = __builtin_bit_cast(unsigned long long, r[c]);
        const unsigned lo = (unsigned)__builtin_amdgcn_readlane((int)(bits & 0xffffffffull), j);
        const unsigned hi = (unsigned)__builtin_amdgcn_readlane((int)(bits >> 32), j);
        const double ljc = __builtin_bit_cast(double, ((unsigned long long)hi << 32) | lo);
        if (j < jb && j <= i) r[j] = fma(-r[c], ljc, r[j]);
      }
    }
  }
  if (bad && i == 0) atomicExch(err, 1);
  if (i < jb) {
#pragma unroll
    for (int j = 0; j < 64; ++j)
      if (j < jb && j <= i) A[(j0 + i) * lda + j0 + j] = r[j];
  }
}

// Panel solve: rows i >= j0 + jb:  A[i, j0:j0+jb] <- A[i, j0:j0+jb] * L_dd^-T
__global__ __launch_bounds__(64) void k_trsm_panel(double *__restrict__ A, int64_t lda,
                                                   int64_t k, int64_t j0, int jb) {
  __shared__ double L[64][65];
  for (int e = threadIdx.x; e < jb * jb; e += 64) {
    const int i = e / jb, j = e % jb;
    L[i][j] = A[(j0 + i) * lda + j0 + j];
  }
  __syncthreads();
  const int64_t i = j0 + jb + (int64_t)blockIdx.x * 64 + threadIdx.x;
  if (i >= k) return;
  double x[64];
  double *row = A + i * lda + j0;
#pragma unroll
  for (int c = 0; c < 64; ++c) x[c] = (c < jb) ? row[c] : 0.0;
#pragma unroll
  for (int c = 0; c < 64; ++c) {
    if (c < jb) {
      double v = x[c];
#pragma unroll
      for (int cc = 0; cc < c; ++cc) v = fma(-x[cc], L[c][cc], v);
      x[c] = v / L[c][c];
    }
  }
#pragma unroll
  for (int c = 0; c < 64; ++c)
    if (c < jb) row[c] = x[c];
}

__global__ void k_zero_upper(double *A, int64_t k) {
  for (int64_t e = (int64_t)blockIdx.x * 256 + threadIdx.x; e < k * k;
       e += (int64_t)gridDim.x * 256) {
    const int64_t i = e / k, j = e % k;
    if (j > i) A[e] = 0.0;
  }
}

void launch_zero_upper(double *A, int64_t k, hipStream_t s) {
  const int64_t n = k * k;
  hipLaunchKernelGGL(k_zero_upper, dim3((unsigned)std::min<int64_t>((n + 255) / 256, 4096)),
                     dim3(256), 0, s, A, k);
}

__global__ void k_add_diag(double *A, int64_t k, double v) {
  const int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x;
  if (i < k) A[i * k + i] += v;
}

void launch_add_diag(double *A, int64_t k, double v, hipStream_t s) {
  hipLaunchKernelGGL(k_add_diag, dim3((unsigned)((k + 255) / 256)), dim3(256), 0, s, A, k, v);
}

int potrf_lower(mlff_ctx *ctx, double *A, int64_t k, bool *ok_out) {
  int *err = &ctx->st->linalg_err;
  MLFF_HIP(ctx, hipMemsetAsync(err, 0, sizeof(int), ctx->stream));
  for (int64_t j0 = 0; j0 < k; j0 += 64) {
    const int jb = (int)std::min<int64_t>(64, k - j0);
    const char *e_diag = std::getenv("MLFF_POTRF_DIAG");  // 0: the workgroup form (A/B, tests)
    const bool wave_diag = e_diag == nullptr || std::atoi(e_diag) != 0;
    if (wave_diag)
      hipLaunchKernelGGL(k_potrf_diag_wave, dim3(1), dim3(64), 0, ctx->stream, A, k, j0, jb, err);
    else
      hipLaunchKernelGGL(k_potrf_diag, dim3(1), dim3(256), 0, ctx->stream, A, k, j0, jb, err);
    const int64_t rest = k - j0 - jb;
    if (rest > 0) {
      hipLaunchKernelGGL(k_trsm_panel, dim3((unsigned)((rest + 63) / 64)), dim3(64), 0,
                         ctx->stream, A, k, k, j0, jb);
      const double *P = A + (j0 + jb) * k + j0;
      // the lower block triangle only (tri): the upper blocks are never read and are zeroed at
      // the end; every lower entry gets the same update (round 6: half the trailing GEMM)
      gemm_launch(false, true, rest, rest, jb, -1.0, P, k, P, k, 1.0, A + (j0 + jb) * k + j0 + jb,
                  k, 1, 0, ctx->stream, 1);
    }
  }
  launch_zero_upper(A, k, ctx->stream);
  MLFF_HIP(ctx, hipGetLastError());
  int h_err = 0;
  MLFF_HIP(ctx, hipMemcpyAsync(&h_err, err, sizeof(int), hipMemcpyDeviceToHost, ctx->stream));
  MLFF_HIP(ctx, hipStreamSynchronize(ctx->stream));
  if (ok_out != nullptr) {
    *ok_out = h_err == 0;
    return MLFF_OK;
  }
  if (h_err) return set_error(ctx, MLFF_ERR_LINALG, "Cholesky factorization failed: matrix is not positive definite");
  return MLFF_OK;
}

// ---------------------------------------------------------------------------
// W[i0:i0+ib, :] <- L_ii^-1 W[i0:i0+ib, :], one thread per column.
__global__ __launch_bounds__(256) void k_trsm_diag_wide(const double *__restrict__ Lm, int64_t k,
                                                        int64_t i0, int ib,
                                                        double *__restrict__ W, int64_t ldw,
                                                        int64_t ncols) {
  __shared__ double L[64][65];
  for (int e = threadIdx.x; e < ib * ib; e += 256) {
    const int i = e / ib, j = e % ib;
    L[i][j] = Lm[(i0 + i) * k + i0 + j];
  }
  __syncthreads();
  const int64_t c = (int64_t)blockIdx.x * 256 + threadIdx.x;
  if (c >= ncols) return;
  double x[64];
#pragma unroll
  for (int r = 0; r < 64; ++r) x[r] = (r < ib) ? W[(i0 + r) * ldw + c] : 0.0;
#pragma unroll
  for (int r = 0; r < 64; ++r) {
    if (r < ib) {
      double v = x[r];
#pragma unroll
      for (int rr = 0; rr < r; ++rr) v = fma(-L[r][rr], x[rr], v);
      x[r] = v / L[r][r];
    }
  }
#pragma unroll
  for (int r = 0; r < 64; ++r)
    if (r < ib) W[(i0 + r) * ldw + c] = x[r];
}

// W_blk -= sum_s slab_s (deterministic order), ib x ncols
__global__ __launch_bounds__(256) void k_sub_slabs(const double *__restrict__ slabs, int splits,
                                                   int ib, int64_t ncols, double *__restrict__ W,
                                                   int64_t ldw) {
  const int64_t n = (int64_t)ib * ncols;
  for (int64_t e = (int64_t)blockIdx.x * 256 + threadIdx.x; e < n; e += (int64_t)gridDim.x * 256) {
    double a = 0.0;
    for (int sp = 0; sp < splits; ++sp) a += slabs[(int64_t)sp * n + e];
    const int64_t r = e / ncols, c = e % ncols;
    W[r * ldw + c] -= a;
  }
}

int trsm_lower_wide(mlff_ctx *ctx, const double *L, int64_t k, double *W, int64_t ncols,
                    int64_t ldw) {
  ScratchScope scope(ctx);
  double *slabs = nullptr;
  int64_t slab_cap = 0;
  for (int64_t i0 = 0; i0 < k; i0 += 64) {
    const int ib = (int)std::min<int64_t>(64, k - i0);
    if (i0 > 0) {
      // W[i0 : i0 + ib] -= L[i0 : i0 + ib, :i0] W[:i0]: one 64-row band, so split K until
      // the band's tiles (ncols / 128 of them) fill the chip
      const int64_t tiles = (ncols + 127) / 128;
      int64_t splits = std::min<int64_t>((512 + tiles - 1) / tiles, (i0 + 63) / 64);
      if (!use_mfma(ib, ncols, i0) || splits < 2) {
        gemm_launch(false, false, ib, ncols, i0, -1.0, L + i0 * k, k, W, ldw, 1.0, W + i0 * ldw,
                    ldw, 1, 0, ctx->stream);
      } else {
        const int64_t need = splits * ib * ncols;
        if (need > slab_cap) {
          MLFF_TRY(scratch_alloc(ctx, &slabs, (size_t)need));
          slab_cap = need;
        }
        gemm_launch(false, false, ib, ncols, i0, 1.0, L + i0 * k, k, W, ldw, 0.0, slabs, ncols,
                    (int)splits, ib * ncols, ctx->stream);
        hipLaunchKernelGGL(k_sub_slabs, dim3((unsigned)std::min<int64_t>((ib * ncols + 255) / 256, 4096)),
                           dim3(256), 0, ctx->stream, slabs, (int)splits, ib, ncols, W + i0 * ldw, ldw);
      }
    }
    hipLaunchKernelGGL(k_trsm_diag_wide, dim3((unsigned)((ncols + 255) / 256)), dim3(256), 0,
                       ctx->stream, L, k, i0, ib, W, ldw, ncols);
  }
  MLFF_HIP(ctx, hipGetLastError());
  return MLFF_OK;
}

__global__ __launch_bounds__(256) void k_colsumsq(const double *__restrict__ W, int64_t k,
                                                  int64_t ncols, int64_t ldw,
                                                  double *__restrict__ out) {
  const int64_t c = (int64_t)blockIdx.x * 256 + threadIdx.x;
  if (c >= ncols) return;
  double a = 0.0;
  for (int64_t j = 0; j < k; ++j) {
    const double v = W[j * ldw + c];
    a = fma(v, v, a);
  }
  out[c] = a;
}

void launch_colsumsq(const double *W, int64_t k, int64_t ncols, int64_t ldw, double *out,
                     hipStream_t s) {
  if (ncols <= 0) return;
  hipLaunchKernelGGL(k_colsumsq, dim3((unsigned)((ncols + 255) / 256)), dim3(256), 0, s, W, k,
                     ncols, ldw, out);
}

int test_gemm(mlff_ctx *ctx, int ta, int tb, int64_t M, int64_t Nc, int64_t Kd, double alpha,
              const double *A, int64_t lda, const double *B, int64_t ldb, double beta, double *C,
              int64_t ldc, int splits) {
  hipStream_t s = ctx->stream;
  const int64_t na = (ta ? Kd : M) * lda, nb = (tb ? Nc : Kd) * ldb, nc = M * ldc;
  ScratchScope scope(ctx);
  double *dA = nullptr, *dB = nullptr, *dC = nullptr, *slabs = nullptr;
  MLFF_TRY(scratch_alloc(ctx, &dA, (size_t)na));
  MLFF_TRY(scratch_alloc(ctx, &dB, (size_t)nb));
  MLFF_TRY(scratch_alloc(ctx, &dC, (size_t)nc));
  MLFF_HIP(ctx, hipMemcpyAsync(dA, A, sizeof(double) * na, hipMemcpyHostToDevice, s));
  MLFF_HIP(ctx, hipMemcpyAsync(dB, B, sizeof(double) * nb, hipMemcpyHostToDevice, s));
  MLFF_HIP(ctx, hipMemcpyAsync(dC, C, sizeof(double) * nc, hipMemcpyHostToDevice, s));
  if (splits <= 1) {
    gemm_launch(ta != 0, tb != 0, M, Nc, Kd, alpha, dA, lda, dB, ldb, beta, dC, ldc, 1, 0, s);
  } else {  // the split-K slab path of gram_wide / trsm_lower_wide: C = beta C + alpha sum_s
    MLFF_TRY(scratch_alloc(ctx, &slabs, (size_t)splits * M * ldc));
    gemm_launch(ta != 0, tb != 0, M, Nc, Kd, alpha, dA, lda, dB, ldb, 0.0, slabs, ldc, splits,
                M * ldc, s);
    if (beta != 1.0) return set_error(ctx, MLFF_ERR_ARG, "test_gemm: split path needs beta = 1");
    hipLaunchKernelGGL(k_sub_slabs, dim3(256), dim3(256), 0, s, slabs, splits, (int)M, ldc, dC, ldc);
    // k_sub_slabs subtracts: report C - alpha AB for the caller to compare
  }
  MLFF_HIP(ctx, hipGetLastError());
  MLFF_HIP(ctx, hipMemcpyAsync(C, dC, sizeof(double) * nc, hipMemcpyDeviceToHost, s));
  MLFF_HIP(ctx, hipStreamSynchronize(s));
  return MLFF_OK;
}

}  // namespace mlff
