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

#include <algorithm>
#include <cstdlib>
#include <cstring>

namespace mlff {

typedef double d2 __attribute__((ext_vector_type(2)));

namespace {

constexpr int B = kSymTile;  // 512
constexpr int kRowsPerWave = B / 4;
constexpr int kRB = 8;  // rows per batch (loads in flight per wave: kRB x 4 KB)

// 8-row batches [gb0, gb1) of tile (I, J) (64 batches = the whole tile), the batches
// interleaved over the 4 waves; row partials of those rows to slot J, the segment's
// column partials to plane Pc (P, or a second plane for a segment that does not start
// the tile, see sym_build)
template <bool DIAG>
__device__ __forceinline__ void tile_body(const double *__restrict__ A, int I, int J,
                                          const double *__restrict__ v,
                                          double *__restrict__ P, double *__restrict__ Pc,
                                          int64_t Np, int gb0, int gb1,
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
  const int row0 = gb0 * kRB, nrows = (gb1 - gb0) * kRB;
  if (!DIAG)
    for (int i = threadIdx.x; i < nrows; i += 256) vrow[row0 + i] = v[(int64_t)I * B + row0 + i];
  __syncthreads();
  d2 acc[4];
#pragma unroll
  for (int q = 0; q < 4; ++q) acc[q] = d2{0.0, 0.0};
#pragma unroll 1
  for (int g = gb0 + w; g < gb1; g += 4) {
    const int rbase = g * kRB;  // batches interleaved across the 4 waves
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
  double *Prow = P + (int64_t)J * Np + (int64_t)I * B + row0;
  for (int c = threadIdx.x; c < nrows; c += 256) __builtin_nontemporal_store(rows[row0 + c], Prow + c);
  if (!DIAG) {
    double *Pcol = Pc + (int64_t)I * Np + (int64_t)J * B;
    for (int c = threadIdx.x; c < B; c += 256)
      __builtin_nontemporal_store((cs[c] + cs[B + c]) + (cs[2 * B + c] + cs[3 * B + c]), Pcol + c);
  }
}

constexpr int kBatches = B / kRB;  // 8-row batches per tile

// workgroups [0, nwhole): one whole tile each; then 2^lsub workgroups per remaining tile,
// one row slice (512 >> lsub rows) each, so the launch ends on sub-tile units instead of a
// partial round of whole tiles (a lone 2-MB tile streams at one CU's rate)
__global__ __launch_bounds__(256) void k_symv_tiles(const double *__restrict__ tiles,
                                                    const int2 *__restrict__ list,
                                                    const double *__restrict__ v,
                                                    double *__restrict__ P,
                                                    double *__restrict__ Pq, int64_t Np,
                                                    int nwhole, int nb, int lsub,
                                                    const int *__restrict__ status) {
  if (status != nullptr && *status != ST_RUNNING) return;
  __shared__ double sh[6 * B + 4 * kRB * 64];
  int tile = blockIdx.x, h = 0, gb0 = 0, gb1 = kBatches;
  if (tile >= nwhole) {
    const int u = tile - nwhole;
    tile = nwhole + (u >> lsub);
    h = u & ((1 << lsub) - 1);
    gb0 = h * (kBatches >> lsub);
    gb1 = gb0 + (kBatches >> lsub);
  }
  const int2 t = list[tile];
  const double *A = tiles + (int64_t)tile * B * B;
  double *Pc = h == 0 ? P : Pq + (int64_t)(h - 1) * nb * Np;
  if (t.x == t.y)
    tile_body<true>(A, t.x, t.y, v, P, Pc, Np, gb0, gb1, sh);
  else
    tile_body<false>(A, t.x, t.y, v, P, Pc, Np, gb0, gb1, sh);
}

// Dynamic persistent schedule with cross-tile prefetch: C resident workgroups take work
// units (whole tiles, then the quarter units of the tail) from a ticket counter; before
// finishing a tile (LDS combine + slot stores) a workgroup already has the first batch
// of its next unit and the next p segment in flight, so the HBM stream of a workgroup
// slot does not stop at tile boundaries.  The counter is reset by the slot reduction.
__device__ __forceinline__ void decode_unit(long long u, int nwhole, int lsub, int &tile, int &h,
                                            int &gb0, int &gb1) {
  if (u < nwhole) {
    tile = (int)u;
    h = 0;
    gb0 = 0;
    gb1 = kBatches;
  } else {
    const long long q = u - nwhole;
    tile = nwhole + (int)(q >> lsub);
    h = (int)(q & ((1 << lsub) - 1));
    gb0 = h * (kBatches >> lsub);
    gb1 = gb0 + (kBatches >> lsub);
  }
}

// rho of the gathered partials (every rank's kVecGrid rho partials in its gb block, after z):
// k_update_p_gathered's sum -- thread f adds partials f, f + 256, ... in order (8 in flight),
// then block_sum256 -- so every workgroup that forms it holds the same bits
__device__ __forceinline__ double gathered_rho(const PGather &pg, double *sh) {
  double v = 0.0;
  const int np = pg.world * kVecGrid;
  int f = threadIdx.x;
  for (; f + 7 * 256 < np; f += 8 * 256) {
    double t[8];
#pragma unroll
    for (int u = 0; u < 8; ++u) {
      const int g = f + u * 256;
      t[u] = pg.gb[(int64_t)(g / kVecGrid) * pg.gstride + pg.blk + (g % kVecGrid)];
    }
#pragma unroll
    for (int u = 0; u < 8; ++u) v += t[u];
  }
  for (; f < np; f += 256) v += pg.gb[(int64_t)(f / kVecGrid) * pg.gstride + pg.blk + (f % kVecGrid)];
  v = block_sum256(v, sh);
  __syncthreads();
  if (threadIdx.x == 0) sh[4] = v;
  __syncthreads();
  const double rho = sh[4];
  __syncthreads();
  return rho;
}

// operand entries of the fused form: p = fma(beta, p_old, z) (z at iteration 1), z from the
// gather buffer -- k_update_p_gathered's arithmetic, the same bits.  Entries past the ranks'
// blocks (one rank: blk = round_up(n, 64) < Np = round_up(n, 512), the tile padding) are zero,
// as the unfused operand's padding is: the gather buffer holds world blocks only.  blk is a
// multiple of 64, so a d2 pair never straddles two blocks.
__device__ __forceinline__ double pg_z(const PGather &pg, int64_t i) {
  const int64_t rk = i / pg.blk;
  return rk < pg.world ? pg.gb[rk * pg.gstride + i % pg.blk] : 0.0;
}
__device__ __forceinline__ double pg_val(const PGather &pg, const double *v, int64_t i, double beta) {
  return pg.it > 1 ? fma(beta, v[i], pg_z(pg, i)) : pg_z(pg, i);
}
__device__ __forceinline__ d2 pg_val2(const PGather &pg, const double *v, int64_t i, double beta) {
  if (pg.gb == nullptr) return *reinterpret_cast<const d2 *>(v + i);
  const int64_t rk = i / pg.blk;
  const d2 z = rk < pg.world ? *reinterpret_cast<const d2 *>(pg.gb + rk * pg.gstride + i % pg.blk)
                             : d2{0.0, 0.0};
  if (pg.it <= 1) return z;
  const d2 po = *reinterpret_cast<const d2 *>(v + i);
  return d2{fma(beta, po.x, z.x), fma(beta, po.y, z.y)};
}

__global__ __launch_bounds__(256) void k_symv_dyn(const double *__restrict__ tiles,
                                                  const int2 *__restrict__ list,
                                                  const double *__restrict__ v,
                                                  double *__restrict__ P,
                                                  double *__restrict__ Pq, int64_t Np,
                                                  int nwhole, long long nunits, int nb,
                                                  int lsub,
                                                  unsigned long long *__restrict__ ticket,
                                                  const int *__restrict__ status, PGather pg,
                                                  unsigned long long *wgtrace = nullptr) {
  if (status != nullptr && *status != ST_RUNNING) return;
  // MLFF_SYM_TRACE (diagnostic): per workgroup its start, end and units taken
  if (wgtrace != nullptr && threadIdx.x == 0) wgtrace[3 * blockIdx.x] = wall_clock64();
  long long units_done = 0;
  __shared__ double sh[6 * B + 4 * kRB * 64];
  __shared__ long long s_next;
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  double *vrow = sh, *rows = sh + B, *cs = sh + 2 * B;
  double *red = sh + 6 * B + w * kRB * 64;
  // first unit = blockIdx.x (no atomic burst at launch: one counter word serves ~90
  // grabs per us); later grabs come from the counter, offset by the grid
  const long long G = gridDim.x;
  long long u = blockIdx.x;
  if (u >= nunits) return;
  // fused p update: beta from the gathered rho partials (block 0 publishes rho for the slot
  // reduction, which writes p after every tile has read p_old)
  double beta = 0.0;
  if (pg.gb != nullptr) {
    const double rho = gathered_rho(pg, sh);
    if (pg.it > 1) beta = rho / pg.st->rho1;
    if (blockIdx.x == 0 && threadIdx.x == 0) pg.st->rho_new = rho;
  }
  int tile, h, gb0, gb1;
  decode_unit(u, nwhole, lsub, tile, h, gb0, gb1);
  int2 t = list[tile];
  const double *A = tiles + (int64_t)tile * B * B;
  d2 pc[4], a[kRB][4];
  {
#pragma unroll
    for (int q = 0; q < 4; ++q) pc[q] = pg_val2(pg, v, (int64_t)t.y * B + 2 * (lane + 64 * q), beta);
    const d2 *rowp = reinterpret_cast<const d2 *>(A + (int64_t)(gb0 + w) * kRB * B) + lane;
#pragma unroll
    for (int rr = 0; rr < kRB; ++rr)
#pragma unroll
      for (int q = 0; q < 4; ++q) a[rr][q] = __builtin_nontemporal_load(rowp + rr * (B / 2) + 64 * q);
  }
  if (threadIdx.x == 0) s_next = G + (long long)atomicAdd(ticket, 1ull);
  for (int i = threadIdx.x; i < (gb1 - gb0) * kRB; i += 256) {
    const int64_t gi = (int64_t)t.x * B + gb0 * kRB + i;
    vrow[gb0 * kRB + i] = pg.gb != nullptr ? pg_val(pg, v, gi, beta) : v[gi];
  }
  __syncthreads();
  while (true) {
    const bool diag = t.x == t.y;
    d2 acc[4];
#pragma unroll
    for (int q = 0; q < 4; ++q) acc[q] = d2{0.0, 0.0};
#pragma unroll 1
    for (int g = gb0 + w; g < gb1; g += 4) {
      const int rbase = g * kRB;
      if (g != gb0 + w) {
        const d2 *rowp = reinterpret_cast<const d2 *>(A + (int64_t)rbase * B) + lane;
#pragma unroll
        for (int rr = 0; rr < kRB; ++rr)
#pragma unroll
          for (int q = 0; q < 4; ++q)
            a[rr][q] = __builtin_nontemporal_load(rowp + rr * (B / 2) + 64 * q);
      }
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
        if (!diag) {
          const double pr = vrow[rbase + rr];
#pragma unroll
          for (int q = 0; q < 4; ++q) {
            acc[q].x = fma(a[rr][q].x, pr, acc[q].x);
            acc[q].y = fma(a[rr][q].y, pr, acc[q].y);
          }
        }
      }
      __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
      __builtin_amdgcn_wave_barrier();
      __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
      const d2 *rp = reinterpret_cast<const d2 *>(red + (lane >> 3) * 64 + (lane & 7) * 8);
      const d2 t0 = rp[0], t1 = rp[1], t2 = rp[2], t3 = rp[3];
      double tt = ((t0.x + t0.y) + (t1.x + t1.y)) + ((t2.x + t2.y) + (t3.x + t3.y));
      tt += __shfl_xor(tt, 1, 64);
      tt += __shfl_xor(tt, 2, 64);
      tt += __shfl_xor(tt, 4, 64);
      if ((lane & 7) == 0) rows[rbase + (lane >> 3)] = tt;
      __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
      __builtin_amdgcn_wave_barrier();
      __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
    }
    if (!diag) {
      d2 *cs2 = reinterpret_cast<d2 *>(cs);
#pragma unroll
      for (int q = 0; q < 4; ++q) cs2[w * (B / 2) + lane + 64 * q] = acc[q];
    }
    __syncthreads();  // rows / cs complete; s_next visible
    const long long un = s_next;
    int tile2 = 0, h2 = 0, gb02 = 0, gb12 = 0;
    int2 t2 = t;
    const double *A2 = A;
    if (un < nunits) {  // next unit: p segment and first batch in flight during the stores
      decode_unit(un, nwhole, lsub, tile2, h2, gb02, gb12);
      t2 = list[tile2];
      A2 = tiles + (int64_t)tile2 * B * B;
#pragma unroll
      for (int q = 0; q < 4; ++q)
        pc[q] = pg_val2(pg, v, (int64_t)t2.y * B + 2 * (lane + 64 * q), beta);
      const d2 *rowp = reinterpret_cast<const d2 *>(A2 + (int64_t)(gb02 + w) * kRB * B) + lane;
#pragma unroll
      for (int rr = 0; rr < kRB; ++rr)
#pragma unroll
        for (int q = 0; q < 4; ++q)
          a[rr][q] = __builtin_nontemporal_load(rowp + rr * (B / 2) + 64 * q);
    }
    {
      const int row0 = gb0 * kRB, nr = (gb1 - gb0) * kRB;
      double *Prow = P + (int64_t)t.y * Np + (int64_t)t.x * B + row0;
      for (int c = threadIdx.x; c < nr; c += 256) __builtin_nontemporal_store(rows[row0 + c], Prow + c);
      if (!diag) {
        double *Pc = h == 0 ? P : Pq + (int64_t)(h - 1) * nb * Np;
        double *Pcol = Pc + (int64_t)t.x * Np + (int64_t)t.y * B;
        for (int c = threadIdx.x; c < B; c += 256)
          __builtin_nontemporal_store((cs[c] + cs[B + c]) + (cs[2 * B + c] + cs[3 * B + c]), Pcol + c);
      }
    }
    __syncthreads();  // LDS consumed, s_next read by everyone
    ++units_done;
    if (un >= nunits) break;
    if (threadIdx.x == 0) s_next = G + (long long)atomicAdd(ticket, 1ull);
    tile = tile2;
    h = h2;
    gb0 = gb02;
    gb1 = gb12;
    t = t2;
    A = A2;
    for (int i = threadIdx.x; i < (gb1 - gb0) * kRB; i += 256) {
      const int64_t gi = (int64_t)t.x * B + gb0 * kRB + i;
      vrow[gb0 * kRB + i] = pg.gb != nullptr ? pg_val(pg, v, gi, beta) : v[gi];
    }
    __syncthreads();
  }
  if (wgtrace != nullptr && threadIdx.x == 0) {
    wgtrace[3 * blockIdx.x + 1] = wall_clock64();
    wgtrace[3 * blockIdx.x + 2] = (unsigned long long)units_done;
  }
}

// column partials of slot t for rows of block bi: tile (t, bi), t > bi; a split tile
// adds its sub-units 1..nq (planes Pq) to sub-unit 0 (P) in sub-unit order
constexpr int kOwnSplit = 1 << 24;  // flag bit of an owned-slot entry: the tile is split

// y[i] = sum_{t=0}^{nb-1} P[t, i] over the slots whose tile this rank owns
// (all slots on one rank); EPI: y = sigma * y + lam * vloc for rows < n_out
// y[i] = sum_{t=0}^{nb-1} of the slots of row i (one rank); EPI: y = sigma y + lam vloc;
// PQ (with EPI): also the p.q partial sums (vloc = p) of each workgroup -> pq_part
// (grid = kVecGrid workgroups, grid-stride over the rows)
template <bool EPI, bool PQ>
__global__ __launch_bounds__(256) void k_sym_reduce(const double *__restrict__ P,
                                                    const double *__restrict__ Pq,
                                                    const unsigned char *__restrict__ split,
                                                    int t_split, int64_t Np, int nb, int nq,
                                                    int64_t n_out, double *__restrict__ y,
                                                    double sigma, double lam,
                                                    const double *__restrict__ vloc,
                                                    double *__restrict__ pq_part,
                                                    unsigned long long *__restrict__ ticket,
                                                    const int *__restrict__ status,
                                                    PGather pg = PGather{},
                                                    double *pw = nullptr) {
  if (status != nullptr && *status != ST_RUNNING) return;
  if (blockIdx.x == 0 && threadIdx.x == 0) *ticket = 0ull;  // k_symv_dyn's counter
  double apq = 0.0;
  // one rank, fused p update (PGather): rho as k_symv_dyn summed it, p = fma(beta, p_old, z)
  // written here (every tile has read p_old) and used as the epilogue's v -- k_update_p's bits
  double beta = 0.0;
  if (PQ && pg.gb != nullptr) {
    const double rho = pg.st->rho_new;
    if (pg.it > 1) beta = rho / pg.st->rho1;
    if (blockIdx.x == 0 && threadIdx.x == 0) pg.st->rho = rho;
  }
  const int64_t pl = (int64_t)nb * Np;
  for (int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x; i < n_out;
       i += (int64_t)gridDim.x * 256) {
    const int bi = (int)(i / B);
    double s = 0.0;
    // slots below t_split hold no split tile for this row block (t_split: the smallest
    // row-block index of a split tile, nb if none).  8 slot loads in flight per
    // thread; the additions stay in slot order
    const int tend = t_split > bi ? t_split : bi + 1;
    const int t8 = tend < nb ? tend : nb;
    // (16 in flight: at one row per thread the 512-workgroup PQ grid leaves 1 wave per SIMD,
    // so the slot loads' round trips are the kernel's time)
    int t = 0;
    for (; t + 15 < t8; t += 16) {
      double v[16];
#pragma unroll
      for (int u = 0; u < 16; ++u) v[u] = __builtin_nontemporal_load(P + (int64_t)(t + u) * Np + i);
#pragma unroll
      for (int u = 0; u < 16; ++u) s += v[u];
    }
    for (; t + 7 < t8; t += 8) {
      double v[8];
#pragma unroll
      for (int u = 0; u < 8; ++u) v[u] = __builtin_nontemporal_load(P + (int64_t)(t + u) * Np + i);
#pragma unroll
      for (int u = 0; u < 8; ++u) s += v[u];
    }
    // the remaining slots (split tiles among them) in batches of 8 as well; every slot
    // value is ((P + Pq0) + Pq1) + ... + Pq_{nq-1}, added in slot order
    for (; t < nb; t += 8) {
      double v[8];
#pragma unroll
      for (int u = 0; u < 8; ++u) {
        v[u] = 0.0;
        const int tu = t + u;
        if (tu < nb) {
          v[u] = P[(int64_t)tu * Np + i];
          if (tu > bi && split[(int64_t)tu * nb + bi])
            for (int hq = 0; hq < nq; ++hq) v[u] += Pq[hq * pl + (int64_t)tu * Np + i];
        }
      }
#pragma unroll
      for (int u = 0; u < 8; ++u)
        if (t + u < nb) s += v[u];
    }
    if (EPI) {
      double pv = 0.0;
      if (PQ && pg.gb != nullptr) {  // (vloc is p itself: read through pw only)
        pv = pg_val(pg, pw, i, beta);
        pw[i] = pv;
      } else if (vloc != nullptr) {
        pv = vloc[i];
      }
      double yv = sigma * s;
      if (vloc != nullptr) yv += lam * pv;
      y[i] = yv;
      if (PQ) apq = fma(pv, yv, apq);
    } else {
      y[i] = s;
    }
  }
  if (PQ) {
    __shared__ double sh[4];
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) apq += __shfl_down(apq, o, 64);
    if ((threadIdx.x & 63) == 0) sh[threadIdx.x >> 6] = apq;
    __syncthreads();
    if (threadIdx.x == 0) pq_part[blockIdx.x] = (sh[0] + sh[1]) + (sh[2] + sh[3]);
  }
}

// several ranks: y_g = sum over this rank's slots for every row of [0, ld), written
// into rank blocks of stride `bstride` (= blk + tail: the reduce-scatter operand).
// PQ: also the partial p.y_g (all rows) + (lam/sigma-free) ||p_loc||^2 partials, one
// pair per workgroup (fixed order), for k_pq_publish.
// PQ: the last workgroup to finish (arrival counter ticket[1], reset by it) also does
// k_pq_publish's work -- the same sums in the same order, so the same share bits -- one launch
// less per sharded iteration (the publish was a 4.9 us single-workgroup launch at W = 8)
struct PqPublish {
  double sigma = 0.0, lam = 0.0;
  int world = 0;
};

template <bool PQ>
__global__ __launch_bounds__(256) void k_sym_reduce_w(const double *__restrict__ P,
                                                      const double *__restrict__ Pq,
                                                      const unsigned char *__restrict__ split,
                                                      int64_t Np, int nq,
                                                      int nb, int rank,
                                                      const int *__restrict__ own,
                                                      int64_t ld, int64_t blk, int64_t bstride,
                                                      double *__restrict__ yg,
                                                      double *p,  // read, and written when fused
                                                      double *__restrict__ pq_part,
                                                      double *__restrict__ pp_part,
                                                      unsigned long long *__restrict__ ticket,
                                                      const int *__restrict__ status,
                                                      PGather pg, PqPublish pub) {
  if (status != nullptr && *status != ST_RUNNING) return;
  if (blockIdx.x == 0 && threadIdx.x == 0) *ticket = 0ull;  // k_symv_dyn's counter
  __shared__ double sh[8];
  __shared__ int s_last;
  double apq = 0.0, app = 0.0;
  // fused p update: rho as k_symv_dyn summed it, p written here (every tile has read p_old)
  double beta = 0.0;
  if (PQ && pg.gb != nullptr) {
    const double rho = pg.st->rho_new;
    if (pg.it > 1) beta = rho / pg.st->rho1;
    if (blockIdx.x == 0 && threadIdx.x == 0) pg.st->rho = rho;
  }
  const int64_t lo = (int64_t)rank * blk, hi = lo + blk;
  for (int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x; i < ld;
       i += (int64_t)gridDim.x * 256) {
    // a wave's 64 rows lie in one 512-row block: bi, the slot list and its split flags are
    // wave-uniform (scalar loads), so no slot load waits on a flag or index load
    const int bi = __builtin_amdgcn_readfirstlane((int)(i / B));
    double s = 0.0;
    // this rank's slots of row block bi (own: ascending slots, kOwnSplit marks a split
    // tile; built at setup) in batches of 16 whose loads are all in flight before the
    // first addition; every slot value is ((P + Pq0) + Pq1) + ... (nq planes), added in
    // slot order
    const int *ol = own + (int64_t)bi * nb;
    const int cnt = own[(int64_t)nb * nb + bi];
    const int64_t pl = (int64_t)nb * Np;
    for (int c = 0; c < cnt; c += 16) {
      double v[16];
#pragma unroll
      for (int u = 0; u < 16; ++u) {
        v[u] = 0.0;
        if (c + u < cnt) {
          const int e = ol[c + u];
          const int64_t at = (int64_t)(e & (kOwnSplit - 1)) * Np + i;
          v[u] = P[at];
          if (e & kOwnSplit)
            for (int hq = 0; hq < nq; ++hq) v[u] += Pq[hq * pl + at];
        }
      }
#pragma unroll
      for (int u = 0; u < 16; ++u)
        if (c + u < cnt) s += v[u];
    }
    yg[(i / blk) * bstride + i % blk] = s;
    if (PQ) {
      double pv;
      if (pg.gb != nullptr) {
        pv = pg_val(pg, p, i, beta);
        p[i] = pv;
      } else {
        pv = p[i];
      }
      apq = fma(pv, s, apq);
      if (i >= lo && i < hi) app = fma(pv, pv, app);
    }
  }
  if (PQ) {
    double t = apq;
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) t += __shfl_down(t, o, 64);
    double u = app;
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) u += __shfl_down(u, o, 64);
    const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
    if (lane == 0) {
      sh[w] = t;
      sh[4 + w] = u;
    }
    __syncthreads();
    if (threadIdx.x == 0) {
      pq_part[blockIdx.x] = (sh[0] + sh[1]) + (sh[2] + sh[3]);
      pp_part[blockIdx.x] = (sh[4] + sh[5]) + (sh[6] + sh[7]);
      __builtin_amdgcn_fence(__ATOMIC_RELEASE, "agent");
      s_last = atomicAdd(ticket + 1, 1ull) == (unsigned long long)(gridDim.x - 1);
    }
    __syncthreads();
    if (!s_last) return;
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");
    // k_pq_publish: s_rank = sigma sum(pq_part) + lam sum(pp_part), into tail slot `rank` of
    // every rank block of the reduce-scatter operand
    const int np = (int)gridDim.x;
    double a = 0.0, b = 0.0;
    for (int i = threadIdx.x; i < np; i += 256) {
      a += pq_part[i];
      b += pp_part[i];
    }
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) {
      a += __shfl_down(a, o, 64);
      b += __shfl_down(b, o, 64);
    }
    __syncthreads();
    if (lane == 0) {
      sh[w] = a;
      sh[4 + w] = b;
    }
    __syncthreads();
    const double share = pub.sigma * ((sh[0] + sh[1]) + (sh[2] + sh[3])) +
                         pub.lam * ((sh[4] + sh[5]) + (sh[6] + sh[7]));
    for (int g = threadIdx.x; g < pub.world; g += 256) yg[(int64_t)g * bstride + blk + rank] = share;
    if (threadIdx.x == 0) ticket[1] = 0ull;
  }
}

// k_sym_reduce_w with the slot loads of a row all in flight (round 6): at
// W = 8 a rank's own row blocks hold 72 slots (+ the split tiles' planes) against 8 elsewhere,
// and k_sym_reduce_w took them as 5 dependent batches of 16, each behind a scalar load of its
// slot entries and a wait per split plane -- 25 us of the 0.38 ms per-rank step.  Here the
// workgroup's row block (256 rows lie in one 512-row block) stages its flat load list (every
// slot and, after a split slot, its planes: SymPack::plist) in LDS once, and a row's loads go
// out in batches of kRwBatch with the next batch in flight while the current one is added:
// unconditional loads (entries past the count re-read the last one), the additions in list
// order -- each slot ((P + Pq0) + Pq1) + ..., the slots in ascending order: k_sym_reduce_w's
// sums, the same bits (MLFF_SYM_REDUCE_LIST=0 restores it; test_sym_reduce_list_bitwise)
constexpr int kRwBatch = 32;
constexpr int kRwMaxList = 2048;

template <bool PQ>
__global__ __launch_bounds__(256) void k_sym_reduce_wl(const double *__restrict__ P,
                                                       const double *__restrict__ Pq,
                                                       int64_t Np, int nb,
                                                       const int *__restrict__ plist,
                                                       int64_t pstride, int rank,
                                                       int64_t ld, int64_t blk, int64_t bstride,
                                                       double *__restrict__ yg, double *p,
                                                       double *__restrict__ pq_part,
                                                       double *__restrict__ pp_part,
                                                       unsigned long long *__restrict__ ticket,
                                                       const int *__restrict__ status,
                                                       PGather pg, PqPublish pub) {
  if (status != nullptr && *status != ST_RUNNING) return;
  if (blockIdx.x == 0 && threadIdx.x == 0) *ticket = 0ull;  // k_symv_dyn's counter
  __shared__ double sh[8];
  __shared__ int s_last;
  __shared__ int sl[kRwMaxList];
  double apq = 0.0, app = 0.0;
  double beta = 0.0;
  if (PQ && pg.gb != nullptr) {
    const double rho = pg.st->rho_new;
    if (pg.it > 1) beta = rho / pg.st->rho1;
    if (blockIdx.x == 0 && threadIdx.x == 0) pg.st->rho = rho;
  }
  const int64_t lo = (int64_t)rank * blk, hi = lo + blk;
  const int64_t plane = (int64_t)nb * Np;
  for (int64_t c0 = (int64_t)blockIdx.x * 256; c0 < ld; c0 += (int64_t)gridDim.x * 256) {
    const int64_t i = c0 + threadIdx.x;
    const int bi = (int)(c0 / B);  // the workgroup's 256 rows lie in one row block
    // the list, its count and the p update's operands are requested together (none waits for
    // another): the list's whole stride (entries past the count are zeros, slot 0 of P)
    const int cnt = plist[(int64_t)nb * pstride + bi];
    int le[kRwMaxList / 256];
#pragma unroll
    for (int q = 0; q < kRwMaxList / 256; ++q) {
      const int e = threadIdx.x + 256 * q;
      le[q] = e < pstride ? plist[(int64_t)bi * pstride + e] : 0;
    }
    double pz = 0.0, pold = 0.0;
    if (PQ && i < ld) {
      if (pg.gb != nullptr) {
        pz = pg_z(pg, i);
        if (pg.it > 1) pold = p[i];
      } else {
        pold = p[i];
      }
    }
    __syncthreads();  // the previous chunk's list reads are done
#pragma unroll
    for (int q = 0; q < kRwMaxList / 256; ++q)
      if (threadIdx.x + 256 * q < pstride) sl[threadIdx.x + 256 * q] = le[q];
    __syncthreads();
    // a batch's list entries one per lane (lane & 31), read out with v_readlane: no LDS round
    // trip between a batch's loads
    const int lane32 = (int)(threadIdx.x & 31);
    auto entries = [&](int e0) { return sl[e0 + lane32 < cnt ? e0 + lane32 : cnt - 1]; };
    auto load = [&](int ent, int u) {
      const int x = __builtin_amdgcn_readlane(ent, u);
      const int h = x >> 16;
      const double *base = h == 0 ? P : Pq + (int64_t)(h - 1) * plane;
      return base[(int64_t)(x & 0xffff) * Np + i];
    };
    double s = 0.0, cur = 0.0;
    if (cnt > 0 && i < ld) {
      double v[kRwBatch];
      int ev = entries(0);
#pragma unroll
      for (int u = 0; u < kRwBatch; ++u) v[u] = load(ev, u);
      for (int e0 = 0; e0 < cnt; e0 += kRwBatch) {
        double w[kRwBatch];
        const int ew = entries(e0 + kRwBatch < cnt ? e0 + kRwBatch : e0);
        if (e0 + kRwBatch < cnt) {  // uniform: the whole next batch in flight
#pragma unroll
          for (int u = 0; u < kRwBatch; ++u) w[u] = load(ew, u);
        } else {
#pragma unroll
          for (int u = 0; u < kRwBatch; ++u) w[u] = 0.0;
        }
#pragma unroll
        for (int u = 0; u < kRwBatch; ++u) {
          if (e0 + u < cnt) {
            if (__builtin_amdgcn_readlane(ev, u) >> 16) {
              cur += v[u];  // a split slot's next plane
            } else {
              s += cur;  // the previous slot is complete
              cur = v[u];
            }
          }
        }
#pragma unroll
        for (int u = 0; u < kRwBatch; ++u) v[u] = w[u];
        ev = ew;
      }
    }
    s += cur;
    if (i >= ld) continue;
    yg[(i / blk) * bstride + i % blk] = s;
    if (PQ) {
      double pv;
      if (pg.gb != nullptr) {  // pg_val's arithmetic on the operands loaded above
        pv = pg.it > 1 ? fma(beta, pold, pz) : pz;
        p[i] = pv;
      } else {
        pv = pold;
      }
      apq = fma(pv, s, apq);
      if (i >= lo && i < hi) app = fma(pv, pv, app);
    }
  }
  if (PQ) {
    double t = apq;
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) t += __shfl_down(t, o, 64);
    double u = app;
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) u += __shfl_down(u, o, 64);
    const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
    if (lane == 0) {
      sh[w] = t;
      sh[4 + w] = u;
    }
    __syncthreads();
    // the last-arriving workgroup publishes this rank's share.  Each workgroup's two partials are
    // stored write-through (sc1: agent-scope relaxed atomic stores) and drained before its ticket
    // add, and the last arriver reads them with sc1 loads only, so no agent-scope release fence
    // (an L2 write-back per workgroup: k_sym_reduce_w's form) and no acquire are needed
    // (cdna_hip_programming.md Guideline 16, R1 / the counter form)
    if (threadIdx.x == 0) {
      const double a0 = (sh[0] + sh[1]) + (sh[2] + sh[3]);
      const double b0 = (sh[4] + sh[5]) + (sh[6] + sh[7]);
      if (pub.world > 0) {
        __hip_atomic_store(reinterpret_cast<unsigned long long *>(pq_part) + blockIdx.x,
                           __builtin_bit_cast(unsigned long long, a0), __ATOMIC_RELAXED,
                           __HIP_MEMORY_SCOPE_AGENT);
        __hip_atomic_store(reinterpret_cast<unsigned long long *>(pp_part) + blockIdx.x,
                           __builtin_bit_cast(unsigned long long, b0), __ATOMIC_RELAXED,
                           __HIP_MEMORY_SCOPE_AGENT);
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        s_last = __hip_atomic_fetch_add(ticket + 1, 1ull, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) ==
                 (unsigned long long)(gridDim.x - 1);
      } else {
        pq_part[blockIdx.x] = a0;
        pp_part[blockIdx.x] = b0;
      }
    }
    if (pub.world == 0) return;  // the separate k_pq_publish launch follows
    __syncthreads();
    if (!s_last) return;
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");  // no loads above the ticket
    const int np = (int)gridDim.x;
    double a = 0.0, b = 0.0;
    for (int q = threadIdx.x; q < np; q += 256) {
      a += __builtin_bit_cast(double, __hip_atomic_load(reinterpret_cast<unsigned long long *>(pq_part) + q,
                                                        __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT));
      b += __builtin_bit_cast(double, __hip_atomic_load(reinterpret_cast<unsigned long long *>(pp_part) + q,
                                                        __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT));
    }
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) {
      a += __shfl_down(a, o, 64);
      b += __shfl_down(b, o, 64);
    }
    __syncthreads();
    if (lane == 0) {
      sh[w] = a;
      sh[4 + w] = b;
    }
    __syncthreads();
    const double share = pub.sigma * ((sh[0] + sh[1]) + (sh[2] + sh[3])) +
                         pub.lam * ((sh[4] + sh[5]) + (sh[6] + sh[7]));
    for (int g = threadIdx.x; g < pub.world; g += 256) yg[(int64_t)g * bstride + blk + rank] = share;
    if (threadIdx.x == 0) __hip_atomic_store(ticket + 1, 0ull, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  }
}

// s_rank = sigma * sum(pq_part) + lam * sum(pp_part) (this rank's share of p.q), put
// into tail slot `rank` of every rank block of the reduce-scatter operand; the other
// tail slots stay zero, so the reduce-scatter hands every rank the exact vector of
// shares (x + 0 is exact in any order) and each rank sums it in rank order: p.q is
// bitwise identical on all ranks without a separate allreduce.
__global__ __launch_bounds__(256) void k_pq_publish(const double *__restrict__ pq_part,
                                                    const double *__restrict__ pp_part, int np,
                                                    double sigma, double lam, int rank, int world,
                                                    int64_t blk, int64_t bstride,
                                                    double *__restrict__ yg,
                                                    const int *__restrict__ status) {
  if (status != nullptr && *status != ST_RUNNING) return;
  __shared__ double sh[8];
  double a = 0.0, b = 0.0;
  for (int i = threadIdx.x; i < np; i += 256) {
    a += pq_part[i];
    b += pp_part[i];
  }
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) {
    a += __shfl_down(a, o, 64);
    b += __shfl_down(b, o, 64);
  }
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  if (lane == 0) {
    sh[w] = a;
    sh[4 + w] = b;
  }
  __syncthreads();
  const double share = sigma * ((sh[0] + sh[1]) + (sh[2] + sh[3])) +
                       lam * ((sh[4] + sh[5]) + (sh[6] + sh[7]));
  for (int g = threadIdx.x; g < world; g += 256) yg[(int64_t)g * bstride + blk + rank] = share;
}

// y[i] = sigma * src[i] + lam * vloc[i]  (src may alias y)
__global__ __launch_bounds__(256) void k_axpby_loc(const double *__restrict__ src, double *y,
                                                   int64_t n, double sigma, double lam,
                                                   const double *__restrict__ vloc,
                                                   const int *__restrict__ status) {
  if (status != nullptr && *status != ST_RUNNING) return;
  const int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x;
  if (i >= n) return;
  double yv = sigma * src[i];
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

// Generate one stored tile per workgroup directly from the RBF points (no dense rows):
// tile (I, J) element (r, c) = K[pos I B + r, pos J B + c] in the padded rank-block index
// space (zero outside [0, N)); each thread owns 2 columns and walks the 512 rows
// (non-temporal 4-KB row stores)
__global__ __launch_bounds__(256) void k_sym_gen_rbf(const int2 *__restrict__ list,
                                                     const double *__restrict__ Xs, int d,
                                                     double jitter, int64_t N, int64_t rows_per,
                                                     int64_t blk, double *__restrict__ tiles) {
  const int2 t = list[blockIdx.x];
  double *T = tiles + (int64_t)blockIdx.x * B * B;
  double xc[2][8];
  int64_t gc[2];
  bool vc[2];
#pragma unroll
  for (int h = 0; h < 2; ++h) {
    const int64_t pos = (int64_t)t.y * B + threadIdx.x + 256 * h;
    const int64_t off = pos % blk;
    gc[h] = (pos / blk) * rows_per + off;
    vc[h] = off < rows_per && gc[h] < N;
#pragma unroll
    for (int u = 0; u < 8; ++u) xc[h][u] = (vc[h] && u < d) ? Xs[gc[h] * d + u] : 0.0;
  }
  for (int r = 0; r < B; ++r) {
    const int64_t pos = (int64_t)t.x * B + r;
    const int64_t off = pos % blk;
    const int64_t gr = (pos / blk) * rows_per + off;
    const bool vr = off < rows_per && gr < N;
#pragma unroll
    for (int h = 0; h < 2; ++h) {
      double val = 0.0;
      // K[gr, gc] evaluated from the column point (rbf_value(x_gc, gr)): bitwise the same
      // as from the row point, see common.h
      if (vr && vc[h]) val = (gr == gc[h]) ? 1.0 + jitter : rbf_value(xc[h], Xs, gr, d);
      __builtin_nontemporal_store(val, T + (int64_t)r * B + threadIdx.x + 256 * h);
    }
  }
}

}  // namespace

void launch_symv(const SymPack &sp, const double *v_full, double *P, const int *status,
                 hipStream_t s, PGather pg) {
  if (sp.ntiles == 0) return;
  const int64_t grid = sp.nwhole + ((sp.ntiles - sp.nwhole) << sp.lsub);
  if (sp.dyn > 0) {
    const unsigned G = (unsigned)std::min<int64_t>(sp.dyn, grid);
    // MLFF_SYM_TRACE=<n> (diagnostic): the n-th launch of the process records
    // each workgroup's start / end / units and prints where the tile stream's time goes (the
    // ramp until every workgroup runs, the tail after the median one is done); one sync
    static const long long trace_at = [] {
      const char *e = std::getenv("MLFF_SYM_TRACE");
      return e ? std::atoll(e) : 0ll;
    }();
    static long long launches = 0;
    unsigned long long *tr = nullptr;
    if (trace_at > 0 && ++launches == trace_at &&
        hipMalloc(&tr, sizeof(unsigned long long) * 3 * G) == hipSuccess)
      (void)hipMemsetAsync(tr, 0, sizeof(unsigned long long) * 3 * G, s);
    hipLaunchKernelGGL(k_symv_dyn, dim3(G), dim3(256), 0, s,
                       sp.tiles, sp.list, v_full, P, sp.Pq, sp.Np, (int)sp.nwhole, (long long)grid,
                       (int)sp.nb, sp.lsub, sp.ticket, status, pg, tr);
    if (tr != nullptr) {
      std::vector<unsigned long long> h((size_t)3 * G);
      if (hipStreamSynchronize(s) == hipSuccess &&
          hipMemcpy(h.data(), tr, sizeof(unsigned long long) * h.size(), hipMemcpyDeviceToHost) ==
              hipSuccess) {
        unsigned long long t0 = ~0ull, t1 = 0;
        std::vector<double> st, en, un;
        for (unsigned g = 0; g < G; ++g) {
          if (h[3 * g] == 0) continue;
          t0 = std::min(t0, h[3 * g]);
          t1 = std::max(t1, h[3 * g + 1]);
        }
        double idle = 0.0;
        for (unsigned g = 0; g < G; ++g) {
          if (h[3 * g] == 0) continue;
          st.push_back(10.0 * (double)(h[3 * g] - t0));
          en.push_back(10.0 * (double)(h[3 * g + 1] - t0));
          un.push_back((double)h[3 * g + 2]);
          idle += 10.0 * (double)(t1 - h[3 * g + 1]) + 10.0 * (double)(h[3 * g] - t0);
        }
        auto q = [](std::vector<double> v, double f) {
          std::sort(v.begin(), v.end());
          return v.empty() ? 0.0 : v[(size_t)(f * (double)(v.size() - 1))];
        };
        const double span = 10.0 * (double)(t1 - t0);
        std::fprintf(stderr,
                     "[sym trace] units %lld on %zu workgroups (units per wg p0/p50/p100 %.0f/%.0f/%.0f); "
                     "span %.1f us; starts p50/p100 %.1f/%.1f us; ends p0/p10/p50/p90/p100 "
                     "%.1f/%.1f/%.1f/%.1f/%.1f us; idle (ramp + tail) %.1f %% of wg-time\n",
                     (long long)grid, st.size(), q(un, 0.0), q(un, 0.5), q(un, 1.0), 1e-3 * span,
                     1e-3 * q(st, 0.5), 1e-3 * q(st, 1.0), 1e-3 * q(en, 0.0), 1e-3 * q(en, 0.1),
                     1e-3 * q(en, 0.5), 1e-3 * q(en, 0.9), 1e-3 * q(en, 1.0),
                     100.0 * idle / (span * (double)st.size()));
      }
      (void)hipFree(tr);
    }
    return;
  }
  hipLaunchKernelGGL(k_symv_tiles, dim3((unsigned)grid), dim3(256), 0, s, sp.tiles, sp.list, v_full,
                     P, sp.Pq, sp.Np, (int)sp.nwhole, (int)sp.nb, sp.lsub, status);
}

void launch_sym_reduce(const SymPack &sp, int64_t n_out, double *y, bool epilogue, double sigma,
                       double lam, const double *vloc, const int *status, hipStream_t s) {
  if (n_out <= 0) return;
  const dim3 grid((unsigned)((n_out + 255) / 256));
  if (epilogue)
    hipLaunchKernelGGL((k_sym_reduce<true, false>), grid, dim3(256), 0, s, sp.P, sp.Pq, sp.split,
                       (int)sp.t_split, sp.Np, (int)sp.nb, (1 << sp.lsub) - 1, n_out, y, sigma, lam, vloc,
                       (double *)nullptr, sp.ticket, status);
  else
    hipLaunchKernelGGL((k_sym_reduce<false, false>), grid, dim3(256), 0, s, sp.P, sp.Pq, sp.split,
                       (int)sp.t_split, sp.Np, (int)sp.nb, (1 << sp.lsub) - 1, n_out, y, sigma, lam, vloc,
                       (double *)nullptr, sp.ticket, status);
}

void launch_sym_reduce_pq(const SymPack &sp, int64_t n_out, double *y, double sigma, double lam,
                          const double *p, double *pq_part, const int *status, hipStream_t s,
                          PGather pg) {
  hipLaunchKernelGGL((k_sym_reduce<true, true>), dim3(kVecGrid), dim3(256), 0, s, sp.P, sp.Pq,
                     sp.split, (int)sp.t_split, sp.Np, (int)sp.nb, (1 << sp.lsub) - 1, n_out, y, sigma,
                     lam, p, pq_part,
                     sp.ticket, status, pg, pg.gb != nullptr ? const_cast<double *>(p) : nullptr);
}

// k_sym_reduce_wl unless MLFF_SYM_REDUCE_LIST=0 at the operator's build (A/B: k_sym_reduce_w);
// the list form needs the row block's list in LDS (kRwMaxList)
static bool sym_reduce_list(const SymPack &sp) {
  return sp.plist != nullptr && sp.pstride <= kRwMaxList && sp.nb <= 0xffff;
}

void launch_sym_reduce_ranks(const SymPack &sp, int rank, int world, int64_t blk,
                             const double *p_full, double *pq_part, double *pp_part,
                             double sigma, double lam, const int *status, hipStream_t s,
                             PGather pg, bool separate_publish) {
  const int64_t ld = (int64_t)world * blk;
  const dim3 grid(kVecGrid);
  double *pw = const_cast<double *>(p_full);  // written only when the p update is fused
  const PqPublish pub = p_full == nullptr ? PqPublish{}
                                          : PqPublish{sigma, lam, separate_publish ? 0 : world};
  const PGather pgu = p_full == nullptr ? PGather{} : pg;
  if (sym_reduce_list(sp)) {
    if (p_full == nullptr)
      hipLaunchKernelGGL((k_sym_reduce_wl<false>), grid, dim3(256), 0, s, sp.P, sp.Pq, sp.Np,
                         (int)sp.nb, sp.plist, sp.pstride, rank, ld, blk, sp.ystride, sp.yg, pw,
                         pq_part, pp_part, sp.ticket, status, pgu, pub);
    else
      hipLaunchKernelGGL((k_sym_reduce_wl<true>), grid, dim3(256), 0, s, sp.P, sp.Pq, sp.Np,
                         (int)sp.nb, sp.plist, sp.pstride, rank, ld, blk, sp.ystride, sp.yg, pw,
                         pq_part, pp_part, sp.ticket, status, pgu, pub);
  } else if (p_full == nullptr) {
    hipLaunchKernelGGL((k_sym_reduce_w<false>), grid, dim3(256), 0, s, sp.P, sp.Pq, sp.split, sp.Np,
                       (1 << sp.lsub) - 1, (int)sp.nb, rank,
                       sp.own, ld, blk, sp.ystride, sp.yg, pw, pq_part, pp_part,
                       sp.ticket, status, PGather{}, PqPublish{});
  } else {
    hipLaunchKernelGGL((k_sym_reduce_w<true>), grid, dim3(256), 0, s, sp.P, sp.Pq, sp.split, sp.Np,
                       (1 << sp.lsub) - 1, (int)sp.nb, rank,
                       sp.own, ld, blk, sp.ystride, sp.yg, pw, pq_part, pp_part,
                       sp.ticket, status, pg, pub);
  }
  if (p_full != nullptr && separate_publish)  // MLFF_PQ_PUBLISH=1 (ctx->pq_publish): A/B
    hipLaunchKernelGGL(k_pq_publish, dim3(1), dim3(256), 0, s, pq_part, pp_part, kVecGrid, sigma, lam,
                       rank, world, blk, sp.ystride, sp.yg, status);
}

void launch_axpby_loc(const double *src, double *y, int64_t n, double sigma, double lam,
                      const double *vloc, const int *status, hipStream_t s) {
  if (n <= 0) return;
  hipLaunchKernelGGL(k_axpby_loc, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, s, src, y, n,
                     sigma, lam, vloc, status);
}

// tile assignment: tile (I, J), I >= J, is stored by the rank of row block I when both
// blocks are one rank's, else by I's or J's rank by the parity of I + J (balanced to a tile)
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
  // Tail split: with C workgroups resident at once (2 per CU: 208 VGPRs -> 2 waves per
  // SIMD), whole tiles fill floor(nt / C) full rounds and the nt mod C remaining tiles
  // run as quarters instead of a partial round of lone 2-MB tiles.  Measured (one
  // MI355X, round 1): 1035 tiles 0.354 -> 0.338 ms, 528 tiles 0.198 -> 0.181 ms; more
  // quarters cost more than they save (all tiles as quarters: 2.51 -> 2.67 ms at 8256).
  int cus = 0;
  if (hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, ctx->device) != hipSuccess ||
      cus < 1)
    cus = 256;
  const int64_t C = 2 * (int64_t)cus;
  int64_t nwhole = (nt / C) * C;
  // MLFF_SYM_WHOLE_ROUNDS=<r> (A/B): at most r rounds of whole tiles, the rest split (finer units
  // for the dynamic schedule where a rank holds only ~2 tiles per resident workgroup, W = 8)
  if (const char *e = std::getenv("MLFF_SYM_WHOLE_ROUNDS"))
    nwhole = std::min<int64_t>(nwhole, std::max<int64_t>(0, std::atoll(e)) * C);
  // launch schedule: k_symv_dyn (C resident workgroups taking units from a counter, next
  // unit prefetched across tile boundaries) -- measured on one MI355X: 2.51 ms at 8256
  // tiles where one-workgroup-per-unit launches took 2.51-2.61 ms (bimodal across runs),
  // equal at 528 / 1035 tiles.  MLFF_SYM_SCHED=static selects the one-workgroup-per-unit
  // launch (k_symv_tiles).
  // Sub-units per split tile: 4 (quarters).  MLFF_SYM_LSUB=3|4 slices the split tiles
  // into 8 / 16 row slices instead (the count that would fill the C slots when the nt mod
  // C tail tiles are few, e.g. 8 of a rank's 1032 at 8 ranks).  Measured on one MI355X
  // (scripts/gpu_sym_lsub_ab.sh, profiles/r02/final3e): no gain -- the dynamic schedule
  // already overlaps the tail (k_symv_dyn 323.9 vs 323.6 us at W = 8) while the reduce
  // reads 15 instead of 3 planes of the split slots (12.7 -> 17.9 us): the step got 1 %
  // slower at W = 8 / 4, 0.2 % at W = 1.  Kept selectable, not default.
  int lsub = 2;
  if (const char *e = std::getenv("MLFF_SYM_LSUB")) {
    const int v = std::atoi(e);
    if (v >= 1 && v <= 4) lsub = v;
  }
  const int64_t nq = ((int64_t)1 << lsub) - 1;
  int64_t dyn = C;
  if (const char *e = std::getenv("MLFF_SYM_SCHED"))
    if (std::strcmp(e, "static") == 0) dyn = 0;
  // (A persistent schedule -- exactly C workgroups streaming equal batch ranges, tiles
  // cut at range boundaries -- measured slower at every size on one MI355X: 2.67 vs
  // 2.61 ms at 8256 tiles, 0.366 vs 0.338 ms at 1035: the hardware dispatcher's dynamic
  // whole-tile balance beats a static equal-byte split.)
  if (sp.tiles == nullptr || sp.ntiles != nt || sp.Np != Np || sp.pq_planes != nq) {
    sym_free(sp);
    if (nt > 0) {
      MLFF_HIP(ctx, hipMalloc(&sp.tiles, sizeof(double) * nt * B * B));
      MLFF_HIP(ctx, hipMalloc(&sp.list, sizeof(int2) * nt));
    }
    MLFF_HIP(ctx, hipMalloc(&sp.P, sizeof(double) * (int64_t)nb * Np));
    MLFF_HIP(ctx, hipMemsetAsync(sp.P, 0, sizeof(double) * (int64_t)nb * Np, s));
    MLFF_HIP(ctx, hipMalloc(&sp.Pq, sizeof(double) * nq * (int64_t)nb * Np));
    MLFF_HIP(ctx, hipMemsetAsync(sp.Pq, 0, sizeof(double) * nq * (int64_t)nb * Np, s));
    sp.pq_planes = nq;
    MLFF_HIP(ctx, hipMalloc(&sp.split, (size_t)nb * nb));
    MLFF_HIP(ctx, hipMalloc(&sp.own, sizeof(int) * (size_t)nb * (nb + 1)));
    // [k_symv_dyn's work counter, k_sym_reduce_w's arrival counter]
    MLFF_HIP(ctx, hipMalloc(&sp.ticket, 2 * sizeof(unsigned long long)));
    MLFF_HIP(ctx, hipMemsetAsync(sp.ticket, 0, 2 * sizeof(unsigned long long), s));
    if (ctx->world > 1) {
      // reduce-scatter operand: rank blocks of blk rows + a tail of p.q shares
      sp.ystride = ctx->blk + round_up(ctx->world, kPad);
      const int64_t ny = (int64_t)ctx->world * sp.ystride;
      MLFF_HIP(ctx, hipMalloc(&sp.yg, sizeof(double) * ny));
      MLFF_HIP(ctx, hipMalloc(&sp.yr, sizeof(double) * sp.ystride));
      MLFF_HIP(ctx, hipMemsetAsync(sp.yg, 0, sizeof(double) * ny, s));
      MLFF_HIP(ctx, hipMemsetAsync(sp.yr, 0, sizeof(double) * sp.ystride, s));
    }
  }
  sp.ntiles = nt;
  sp.Np = Np;
  sp.nb = nb;
  sp.tiles_per_rank = tpr;
  sp.nwhole = nwhole;
  sp.lsub = lsub;
  sp.dyn = dyn;
  {
    std::vector<unsigned char> split((size_t)nb * nb, 0);
    sp.t_split = nb;
    for (int64_t t = nwhole; t < nt; ++t) {
      split[(size_t)list[t].x * nb + list[t].y] = 1;
      sp.t_split = std::min<int64_t>(sp.t_split, list[t].x);
    }
    MLFF_HIP(ctx, hipMemcpyAsync(sp.split, split.data(), split.size(), hipMemcpyHostToDevice, s));
    // owned slots per row block (k_sym_reduce_w): row bi's slot t is this rank's when it
    // stores tile (max(bi, t), min(bi, t)); rows of nb ascending entries, then nb counts
    std::vector<int> own((size_t)nb * (nb + 1), 0);
    for (int bi = 0; bi < nb; ++bi) {
      int c = 0;
      for (int t = 0; t < nb; ++t)
        if (owner_host(std::max(bi, t), std::min(bi, t), tpr) == ctx->rank)
          own[(size_t)bi * nb + c++] = t | (t > bi && split[(size_t)t * nb + bi] ? kOwnSplit : 0);
      own[(size_t)nb * nb + bi] = c;
    }
    MLFF_HIP(ctx, hipMemcpyAsync(sp.own, own.data(), sizeof(int) * own.size(), hipMemcpyHostToDevice, s));
    // the flat load list of k_sym_reduce_wl: each owned slot, a split slot followed by its planes;
    // row blocks at a stride of the longest list (rounded to 64 entries)
    std::vector<std::vector<int>> lists((size_t)nb);
    sp.pmax = 0;
    for (int bi = 0; bi < nb; ++bi) {
      for (int j = 0; j < own[(size_t)nb * nb + bi]; ++j) {
        const int e = own[(size_t)bi * nb + j];
        const int t = e & (kOwnSplit - 1);
        lists[bi].push_back(t);
        if (e & kOwnSplit)
          for (int h = 1; h <= nq; ++h) lists[bi].push_back(t | (h << 16));
      }
      sp.pmax = std::max(sp.pmax, (int)lists[bi].size());
    }
    sp.pstride = round_up(std::max(sp.pmax, 1), 64);
    std::vector<int> plist((size_t)nb * (sp.pstride + 1), 0);
    for (int bi = 0; bi < nb; ++bi) {
      std::copy(lists[bi].begin(), lists[bi].end(), plist.begin() + (size_t)bi * sp.pstride);
      plist[(size_t)nb * sp.pstride + bi] = (int)lists[bi].size();
    }
    if (sp.plist != nullptr) (void)hipFree(sp.plist);
    sp.plist = nullptr;
    const char *rl = std::getenv("MLFF_SYM_REDUCE_LIST");
    if (ctx->world > 1 && (rl == nullptr || std::atoi(rl) != 0)) {
      MLFF_HIP(ctx, hipMalloc(&sp.plist, sizeof(int) * plist.size()));
      MLFF_HIP(ctx, hipMemcpyAsync(sp.plist, plist.data(), sizeof(int) * plist.size(),
                                   hipMemcpyHostToDevice, s));
    }
    MLFF_HIP(ctx, hipStreamSynchronize(s));
  }
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
    if (!ctx->has_matrix && ctx->rbf.ready) {  // generated from the points (no dense rows)
      hipLaunchKernelGGL(k_sym_gen_rbf, dim3((unsigned)nt), dim3(256), 0, s, sp.list, ctx->rbf.Xs,
                         ctx->rbf.d, ctx->rbf.jitter, ctx->N, ctx->rows_per, ctx->blk, sp.tiles);
      check_symmetry = false;
    } else {
      hipLaunchKernelGGL(k_sym_pack<false>, dim3((unsigned)nt), dim3(256), 0, s, Ksrc, ldsrc, rowbase,
                         ctx->blk, sp.list, dtrans, sp.tiles, dflag);
    }
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
  for (void *p : {(void *)sp.tiles, (void *)sp.list, (void *)sp.P, (void *)sp.yg, (void *)sp.yr,
                  (void *)sp.Pq, (void *)sp.split, (void *)sp.ticket, (void *)sp.own,
                  (void *)sp.plist})
    if (p) (void)hipFree(p);
  sp.own = nullptr;
  sp.plist = nullptr;
  sp.pmax = 0;
  sp.Pq = nullptr;
  sp.split = nullptr;
  sp.ticket = nullptr;
  sp.tiles = nullptr;
  sp.list = nullptr;
  sp.P = nullptr;
  sp.yg = nullptr;
  sp.yr = nullptr;
  sp.ntiles = 0;
  sp.pq_planes = 0;
  sp.ready = false;
}

}  // namespace mlff
