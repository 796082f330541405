// Development probe: variants of the symmetric tiled mat-vec (csrc/kernels_sym.hip)
// at N = 65536 on one MI355X, timed with hipEvents.  Not part of the library.
//   hipcc -O3 --offload-arch=gfx950 -std=c++17 scripts/probe_symv.hip -o probe_symv
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cmath>
#include <cstdlib>
#include <vector>

#define CK(x)                                                                  \
  do {                                                                         \
    hipError_t e = (x);                                                        \
    if (e != hipSuccess) {                                                     \
      printf("HIP error %s at %s:%d\n", hipGetErrorString(e), __FILE__, __LINE__); \
      exit(1);                                                                 \
    }                                                                          \
  } while (0)

typedef double d2 __attribute__((ext_vector_type(2)));
constexpr int B = 512;

template <int RB>
__device__ __forceinline__ double batch_reduce(double (&v)[RB], int lane) {
#pragma unroll
  for (int s = 0, half = RB / 2; half >= 1; ++s, half >>= 1) {
    const bool hi = (lane >> s) & 1;
#pragma unroll
    for (int k = 0; k < half; ++k) {
      const double keep = hi ? v[k + half] : v[k];
      const double send = hi ? v[k] : v[k + half];
      v[k] = keep + __shfl_xor(send, 1 << s, 64);
    }
  }
  double r = v[0];
#pragma unroll
  for (int m = RB; m < 64; m <<= 1) r += __shfl_xor(r, m, 64);
  return r;
}

template <int RB>
__device__ __forceinline__ int row_of_lane(int lane) {
  int row = 0;
#pragma unroll
  for (int s = 0, half = RB / 2; half >= 1; ++s, half >>= 1)
    if ((lane >> s) & 1) row += half;
  return row;
}

// NW waves per workgroup, each streams B/NW rows of the tile in batches of RB rows.
// PF: software prefetch of the next batch.
template <int RB, int NW, bool PF, bool DIAG>
__device__ __forceinline__ void body(const double *__restrict__ A, int I, int J,
                                     const double *__restrict__ v, double *__restrict__ P,
                                     long Np, double *sh) {
  constexpr int RPW = B / NW;
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  const d2 *v2 = reinterpret_cast<const d2 *>(v + (long)J * B);
  d2 pc[4];
#pragma unroll
  for (int q = 0; q < 4; ++q) pc[q] = v2[lane + 64 * q];
  double *vrow = sh;
  if (!DIAG) {
    for (int i = threadIdx.x; i < B; i += NW * 64) vrow[i] = v[(long)I * B + i];
    __syncthreads();
  }
  d2 acc[4];
#pragma unroll
  for (int q = 0; q < 4; ++q) acc[q] = d2{0.0, 0.0};
  double *Prow = P + (long)J * Np + (long)I * B;
  const d2 *base = reinterpret_cast<const d2 *>(A + (long)(w * RPW) * B) + lane;
  d2 a[RB][4], nx[RB][4];
  if (PF) {
#pragma unroll
    for (int rr = 0; rr < RB; ++rr)
#pragma unroll
      for (int q = 0; q < 4; ++q) nx[rr][q] = __builtin_nontemporal_load(base + rr * (B / 2) + 64 * q);
  }
#pragma unroll 1
  for (int g = 0; g < RPW / RB; ++g) {
    const int rbase = w * RPW + g * RB;
    const d2 *rowp = base + (long)g * RB * (B / 2);
    if (PF) {
#pragma unroll
      for (int rr = 0; rr < RB; ++rr)
#pragma unroll
        for (int q = 0; q < 4; ++q) a[rr][q] = nx[rr][q];
      if (g + 1 < RPW / RB) {
#pragma unroll
        for (int rr = 0; rr < RB; ++rr)
#pragma unroll
          for (int q = 0; q < 4; ++q)
            nx[rr][q] = __builtin_nontemporal_load(rowp + (RB + rr) * (B / 2) + 64 * q);
      }
    } else {
#pragma unroll
      for (int rr = 0; rr < RB; ++rr)
#pragma unroll
        for (int q = 0; q < 4; ++q) a[rr][q] = __builtin_nontemporal_load(rowp + rr * (B / 2) + 64 * q);
    }
    double vals[RB];
#pragma unroll
    for (int rr = 0; rr < RB; ++rr) {
      double s0 = a[rr][0].x * pc[0].x;
      double s1 = a[rr][0].y * pc[0].y;
#pragma unroll
      for (int q = 1; q < 4; ++q) {
        s0 = fma(a[rr][q].x, pc[q].x, s0);
        s1 = fma(a[rr][q].y, pc[q].y, s1);
      }
      vals[rr] = s0 + s1;
      if (!DIAG) {
        const double pr = vrow[rbase + rr];
#pragma unroll
        for (int q = 0; q < 4; ++q) {
          acc[q].x = fma(a[rr][q].x, pr, acc[q].x);
          acc[q].y = fma(a[rr][q].y, pr, acc[q].y);
        }
      }
    }
    const double rs = batch_reduce<RB>(vals, lane);
    if (lane < RB) Prow[rbase + row_of_lane<RB>(lane)] = rs;
  }
  if (!DIAG) {
    d2 *cs = reinterpret_cast<d2 *>(sh + B);
    __syncthreads();
#pragma unroll
    for (int q = 0; q < 4; ++q) cs[w * (B / 2) + lane + 64 * q] = acc[q];
    __syncthreads();
    double *Pcol = P + (long)I * Np + (long)J * B;
    const double *csd = sh + B;
    for (int c = threadIdx.x; c < B; c += NW * 64) {
      double t = 0.0;
      for (int ww = 0; ww < NW; ++ww) t += csd[ww * B + c];
      Pcol[c] = t;
    }
  }
}

template <int RB, int NW, bool PF>
__global__ __launch_bounds__(NW * 64) void k_symv(const double *__restrict__ tiles,
                                                  const int2 *__restrict__ list,
                                                  const double *__restrict__ v,
                                                  double *__restrict__ P, long Np,
                                                  long pitch = (long)B * B) {
  __shared__ double sh[(NW + 1) * B];
  const int2 t = list[blockIdx.x];
  const double *A = tiles + (long)blockIdx.x * pitch;
  if (t.x == t.y)
    body<RB, NW, PF, true>(A, t.x, t.y, v, P, Np, sh);
  else
    body<RB, NW, PF, false>(A, t.x, t.y, v, P, Np, sh);
}


// variant: LDSROWS = row sums staged in LDS and written once per tile (coalesced);
// IL = rows interleaved across waves (wave w takes batches w, w+NW, ...)
template <int RB, bool LDSROWS, bool IL, bool DIAG>
__device__ __forceinline__ void body2(const double *__restrict__ A, int I, int J,
                                      const double *__restrict__ v, double *__restrict__ P,
                                      long Np, double *sh) {
  constexpr int NW = 4;
  constexpr int RPW = B / NW;
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  const d2 *v2 = reinterpret_cast<const d2 *>(v + (long)J * B);
  d2 pc[4];
#pragma unroll
  for (int q = 0; q < 4; ++q) pc[q] = v2[lane + 64 * q];
  double *vrow = sh;
  double *rows = sh + (NW + 1) * B;  // B row sums
  if (!DIAG) {
    for (int i = threadIdx.x; i < B; i += NW * 64) vrow[i] = v[(long)I * B + i];
  }
  __syncthreads();
  d2 acc[4];
#pragma unroll
  for (int q = 0; q < 4; ++q) acc[q] = d2{0.0, 0.0};
  double *Prow = P + (long)J * Np + (long)I * B;
#pragma unroll 1
  for (int g = 0; g < RPW / RB; ++g) {
    const int rbase = IL ? (g * NW + w) * RB : w * RPW + g * RB;
    const d2 *rowp = reinterpret_cast<const d2 *>(A + (long)rbase * B) + lane;
    d2 a[RB][4];
#pragma unroll
    for (int rr = 0; rr < RB; ++rr)
#pragma unroll
      for (int q = 0; q < 4; ++q) a[rr][q] = __builtin_nontemporal_load(rowp + rr * (B / 2) + 64 * q);
    double vals[RB];
#pragma unroll
    for (int rr = 0; rr < RB; ++rr) {
      double s0 = a[rr][0].x * pc[0].x;
      double s1 = a[rr][0].y * pc[0].y;
#pragma unroll
      for (int q = 1; q < 4; ++q) {
        s0 = fma(a[rr][q].x, pc[q].x, s0);
        s1 = fma(a[rr][q].y, pc[q].y, s1);
      }
      vals[rr] = s0 + s1;
      if (!DIAG) {
        const double pr = vrow[rbase + rr];
#pragma unroll
        for (int q = 0; q < 4; ++q) {
          acc[q].x = fma(a[rr][q].x, pr, acc[q].x);
          acc[q].y = fma(a[rr][q].y, pr, acc[q].y);
        }
      }
    }
    const double rs = batch_reduce<RB>(vals, lane);
    if (lane < RB) {
      if (LDSROWS) rows[rbase + row_of_lane<RB>(lane)] = rs;
      else Prow[rbase + row_of_lane<RB>(lane)] = rs;
    }
  }
  if (LDSROWS || !DIAG) __syncthreads();
  if (LDSROWS)
    for (int c = threadIdx.x; c < B; c += NW * 64) Prow[c] = rows[c];
  if (!DIAG) {
    d2 *cs = reinterpret_cast<d2 *>(sh + B);
#pragma unroll
    for (int q = 0; q < 4; ++q) cs[w * (B / 2) + lane + 64 * q] = acc[q];
    __syncthreads();
    double *Pcol = P + (long)I * Np + (long)J * B;
    const double *csd = sh + B;
    for (int c = threadIdx.x; c < B; c += NW * 64)
      Pcol[c] = (csd[c] + csd[B + c]) + (csd[2 * B + c] + csd[3 * B + c]);
  }
}

template <int RB, bool LDSROWS, bool IL>
__global__ __launch_bounds__(256) void k_symv2(const double *__restrict__ tiles,
                                               const int2 *__restrict__ list,
                                               const double *__restrict__ v,
                                               double *__restrict__ P, long Np) {
  __shared__ double sh[6 * B];
  const int2 t = list[blockIdx.x];
  const double *A = tiles + (long)blockIdx.x * B * B;
  if (t.x == t.y)
    body2<RB, LDSROWS, IL, true>(A, t.x, t.y, v, P, Np, sh);
  else
    body2<RB, LDSROWS, IL, false>(A, t.x, t.y, v, P, Np, sh);
}

// variant 3 (GEMV-like): the 4 waves share every row; thread t owns columns 2t, 2t+1
// (column partials stay in registers, no cross-wave column reduction); row sums
// = wave butterfly + 4-way LDS sum per batch of RB rows.
template <int RB, bool DIAG>
__device__ __forceinline__ void body3(const double *__restrict__ A, int I, int J,
                                      const double *__restrict__ v, double *__restrict__ P,
                                      long Np, double *sh) {
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6, t = threadIdx.x;
  const d2 pc = reinterpret_cast<const d2 *>(v + (long)J * B)[t];
  double *vrow = sh;            // B
  double *part = sh + B;        // 2 x 4 x RB
  double *rows = part + 8 * RB; // B
  if (!DIAG)
    for (int i = t; i < B; i += 256) vrow[i] = v[(long)I * B + i];
  __syncthreads();
  d2 acc = {0.0, 0.0};
  const d2 *base = reinterpret_cast<const d2 *>(A) + t;
#pragma unroll 1
  for (int g = 0; g < B / RB; ++g) {
    d2 a[RB];
#pragma unroll
    for (int rr = 0; rr < RB; ++rr) a[rr] = __builtin_nontemporal_load(base + (long)(g * RB + rr) * (B / 2));
    double vals[RB];
#pragma unroll
    for (int rr = 0; rr < RB; ++rr) {
      vals[rr] = fma(a[rr].x, pc.x, a[rr].y * pc.y);
      if (!DIAG) {
        const double pr = vrow[g * RB + rr];
        acc.x = fma(a[rr].x, pr, acc.x);
        acc.y = fma(a[rr].y, pr, acc.y);
      }
    }
    const double rs = batch_reduce<RB>(vals, lane);
    double *pb = part + (g & 1) * 4 * RB;
    if (lane < RB) pb[w * RB + row_of_lane<RB>(lane)] = rs;
    __syncthreads();
    if (t < RB) rows[g * RB + t] = (pb[t] + pb[RB + t]) + (pb[2 * RB + t] + pb[3 * RB + t]);
  }
  __syncthreads();
  double *Prow = P + (long)J * Np + (long)I * B;
  for (int c = t; c < B; c += 256) Prow[c] = rows[c];
  if (!DIAG) {
    d2 *Pcol = reinterpret_cast<d2 *>(P + (long)I * Np + (long)J * B);
    Pcol[t] = acc;
  }
}

template <int RB>
__global__ __launch_bounds__(256) void k_symv3(const double *__restrict__ tiles,
                                               const int2 *__restrict__ list,
                                               const double *__restrict__ v,
                                               double *__restrict__ P, long Np) {
  __shared__ double sh[2 * B + 8 * RB];
  const int2 t = list[blockIdx.x];
  const double *A = tiles + (long)blockIdx.x * B * B;
  if (t.x == t.y)
    body3<RB, true>(A, t.x, t.y, v, P, Np, sh);
  else
    body3<RB, false>(A, t.x, t.y, v, P, Np, sh);
}

// variant 4: symv2 (IL, LDS rows) with p columns read from LDS and an occupancy target
template <int RB, bool DIAG>
__device__ __forceinline__ void body4(const double *__restrict__ A, int I, int J,
                                      const double *__restrict__ v, double *__restrict__ P,
                                      long Np, double *sh) {
  constexpr int NW = 4;
  constexpr int RPW = B / NW;
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  double *vrow = sh;                // B
  d2 *vcol = reinterpret_cast<d2 *>(sh + B);  // B doubles
  double *rows = sh + 2 * B;        // B
  double *cs = sh + 3 * B;          // 4 x B
  for (int i = threadIdx.x; i < B; i += 256) {
    if (!DIAG) vrow[i] = v[(long)I * B + i];
    sh[B + i] = v[(long)J * B + i];
  }
  __syncthreads();
  d2 acc[4];
#pragma unroll
  for (int q = 0; q < 4; ++q) acc[q] = d2{0.0, 0.0};
#pragma unroll 1
  for (int g = 0; g < RPW / RB; ++g) {
    const int rbase = (g * NW + w) * RB;
    const d2 *rowp = reinterpret_cast<const d2 *>(A + (long)rbase * B) + lane;
    d2 a[RB][4];
#pragma unroll
    for (int rr = 0; rr < RB; ++rr)
#pragma unroll
      for (int q = 0; q < 4; ++q) a[rr][q] = __builtin_nontemporal_load(rowp + rr * (B / 2) + 64 * q);
    double vals[RB];
#pragma unroll
    for (int rr = 0; rr < RB; ++rr) {
      double s0 = 0.0, s1 = 0.0;
#pragma unroll
      for (int q = 0; q < 4; ++q) {
        const d2 pc = vcol[lane + 64 * q];
        s0 = fma(a[rr][q].x, pc.x, s0);
        s1 = fma(a[rr][q].y, pc.y, s1);
      }
      vals[rr] = s0 + s1;
      if (!DIAG) {
        const double pr = vrow[rbase + rr];
#pragma unroll
        for (int q = 0; q < 4; ++q) {
          acc[q].x = fma(a[rr][q].x, pr, acc[q].x);
          acc[q].y = fma(a[rr][q].y, pr, acc[q].y);
        }
      }
    }
    const double rs = batch_reduce<RB>(vals, lane);
    if (lane < RB) rows[rbase + row_of_lane<RB>(lane)] = rs;
  }
  if (!DIAG) {
    d2 *cs2 = reinterpret_cast<d2 *>(cs);
#pragma unroll
    for (int q = 0; q < 4; ++q) cs2[w * (B / 2) + lane + 64 * q] = acc[q];
  }
  __syncthreads();
  double *Prow = P + (long)J * Np + (long)I * B;
  for (int c = threadIdx.x; c < B; c += 256) Prow[c] = rows[c];
  if (!DIAG) {
    double *Pcol = P + (long)I * Np + (long)J * B;
    for (int c = threadIdx.x; c < B; c += 256)
      Pcol[c] = (cs[c] + cs[B + c]) + (cs[2 * B + c] + cs[3 * B + c]);
  }
}

template <int RB, int WPE>
__global__ __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(WPE)))
void k_symv4(const double *__restrict__ tiles, const int2 *__restrict__ list,
             const double *__restrict__ v, double *__restrict__ P, long Np) {
  __shared__ double sh[7 * B];
  const int2 t = list[blockIdx.x];
  const double *A = tiles + (long)blockIdx.x * B * B;
  if (t.x == t.y)
    body4<RB, true>(A, t.x, t.y, v, P, Np, sh);
  else
    body4<RB, false>(A, t.x, t.y, v, P, Np, sh);
}

// variant 6: row sums reduced through a wave-private LDS transpose instead of the
// select-heavy butterfly (8 ds_write_b64 + 4 ds_read_b128 + 7 adds + 3 xor-shuffles
// per 8 rows); rows interleaved across waves, row sums staged for one coalesced write.
template <bool DIAG, bool NOWRITE, bool NOCOL, bool NTST = false>
__device__ __forceinline__ void body6(const double *__restrict__ A, int I, int J,
                                      const double *__restrict__ v, double *__restrict__ P,
                                      long Np, double *sh) {
  constexpr int NW = 4, RB = 8;
  constexpr int RPW = B / NW;
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  const d2 *v2 = reinterpret_cast<const d2 *>(v + (long)J * B);
  d2 pc[4];
#pragma unroll
  for (int q = 0; q < 4; ++q) pc[q] = v2[lane + 64 * q];
  double *vrow = sh;                  // B
  double *rows = sh + B;              // B
  double *cs = sh + 2 * B;            // 4 x B
  double *red = sh + 6 * B + w * RB * 64;  // wave-private 8 x 64
  if (!DIAG)
    for (int i = threadIdx.x; i < B; i += 256) vrow[i] = v[(long)I * B + i];
  __syncthreads();
  d2 acc[4];
#pragma unroll
  for (int q = 0; q < 4; ++q) acc[q] = d2{0.0, 0.0};
#pragma unroll 1
  for (int g = 0; g < RPW / RB; ++g) {
    const int rbase = (g * NW + w) * RB;
    const d2 *rowp = reinterpret_cast<const d2 *>(A + (long)rbase * B) + lane;
    d2 a[RB][4];
#pragma unroll
    for (int rr = 0; rr < RB; ++rr)
#pragma unroll
      for (int q = 0; q < 4; ++q) a[rr][q] = __builtin_nontemporal_load(rowp + rr * (B / 2) + 64 * q);
#pragma unroll
    for (int rr = 0; rr < RB; ++rr) {
      double s0 = a[rr][0].x * pc[0].x;
      double s1 = a[rr][0].y * pc[0].y;
#pragma unroll
      for (int q = 1; q < 4; ++q) {
        s0 = fma(a[rr][q].x, pc[q].x, s0);
        s1 = fma(a[rr][q].y, pc[q].y, s1);
      }
      red[rr * 64 + lane] = s0 + s1;
      if (!DIAG && !NOCOL) {
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
    // lane = 8 * row + c: sums red[row][8c .. 8c + 8)
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
  double *Prow = P + (long)J * Np + (long)I * B;
  if (NOWRITE) {
    double t = 0.0;
    for (int c = threadIdx.x; c < B; c += 256) t += rows[c] + cs[c];
    if (t == 1234.5678) Prow[0] = t;
    return;
  }
  if (NTST) {
    for (int c = threadIdx.x; c < B; c += 256) __builtin_nontemporal_store(rows[c], Prow + c);
    if (!DIAG) {
      double *Pcol = P + (long)I * Np + (long)J * B;
      for (int c = threadIdx.x; c < B; c += 256)
        __builtin_nontemporal_store((cs[c] + cs[B + c]) + (cs[2 * B + c] + cs[3 * B + c]), Pcol + c);
    }
    return;
  }
  for (int c = threadIdx.x; c < B; c += 256) Prow[c] = rows[c];
  if (!DIAG) {
    double *Pcol = P + (long)I * Np + (long)J * B;
    for (int c = threadIdx.x; c < B; c += 256)
      Pcol[c] = (cs[c] + cs[B + c]) + (cs[2 * B + c] + cs[3 * B + c]);
  }
}

__global__ __launch_bounds__(256) void k_symv6nt(const double *__restrict__ tiles,
                                                 const int2 *__restrict__ list,
                                                 const double *__restrict__ v,
                                                 double *__restrict__ P, long Np) {
  __shared__ double sh[6 * B + 4 * 8 * 64];
  const int2 t = list[blockIdx.x];
  const double *A = tiles + (long)blockIdx.x * B * B;
  if (t.x == t.y)
    body6<true, false, false, true>(A, t.x, t.y, v, P, Np, sh);
  else
    body6<false, false, false, true>(A, t.x, t.y, v, P, Np, sh);
}

// writes only (same P pattern, no tile reads): what do the slot writes cost alone?
__global__ __launch_bounds__(256) void k_pwrite(const int2 *__restrict__ list, double *__restrict__ P,
                                                long Np) {
  const int2 t = list[blockIdx.x];
  double *Prow = P + (long)t.y * Np + (long)t.x * B;
  for (int c = threadIdx.x; c < B; c += 256) Prow[c] = 1.0;
  if (t.x != t.y) {
    double *Pcol = P + (long)t.x * Np + (long)t.y * B;
    for (int c = threadIdx.x; c < B; c += 256) Pcol[c] = 2.0;
  }
}

template <bool NOWRITE, bool NOCOL>
__global__ __launch_bounds__(256) void k_symv6x(const double *__restrict__ tiles,
                                                const int2 *__restrict__ list,
                                                const double *__restrict__ v,
                                                double *__restrict__ P, long Np) {
  __shared__ double sh[6 * B + 4 * 8 * 64];
  const int2 t = list[blockIdx.x];
  const double *A = tiles + (long)blockIdx.x * B * B;
  if (t.x == t.y)
    body6<true, NOWRITE, NOCOL>(A, t.x, t.y, v, P, Np, sh);
  else
    body6<false, NOWRITE, NOCOL>(A, t.x, t.y, v, P, Np, sh);
}

__global__ __launch_bounds__(256) void k_symv6(const double *__restrict__ tiles,
                                               const int2 *__restrict__ list,
                                               const double *__restrict__ v,
                                               double *__restrict__ P, long Np) {
  __shared__ double sh[6 * B + 4 * 8 * 64];
  const int2 t = list[blockIdx.x];
  const double *A = tiles + (long)blockIdx.x * B * B;
  if (t.x == t.y)
    body6<true, false, false>(A, t.x, t.y, v, P, Np, sh);
  else
    body6<false, false, false>(A, t.x, t.y, v, P, Np, sh);
}

__global__ void k_reduce(const double *__restrict__ P, long Np, int nb, long n,
                         double *__restrict__ y) {
  const long i = (long)blockIdx.x * 256 + threadIdx.x;
  if (i >= n) return;
  double s = 0.0;
  for (int t = 0; t < nb; ++t) s += P[(long)t * Np + i];
  y[i] = s;
}

// plain streaming read of the same bytes (upper bound for this access pattern)
__global__ __launch_bounds__(256) void k_stream(const d2 *__restrict__ A, long n2,
                                                double *__restrict__ out) {
  d2 acc = {0.0, 0.0};
  for (long i = (long)blockIdx.x * 256 + threadIdx.x; i < n2; i += (long)gridDim.x * 256) {
    const d2 a = __builtin_nontemporal_load(A + i);
    acc += a;
  }
  if (acc.x == 12345.678) out[0] = acc.y;
}

template <int U>
__global__ __launch_bounds__(256) void k_stream_u(const d2 *__restrict__ A, long n2,
                                                  double *__restrict__ out) {
  d2 acc = {0.0, 0.0};
  const long stride = (long)gridDim.x * 256;
  long i = (long)blockIdx.x * 256 + threadIdx.x;
  for (; i + (U - 1) * stride < n2; i += U * stride) {
    d2 a[U];
#pragma unroll
    for (int u = 0; u < U; ++u) a[u] = __builtin_nontemporal_load(A + i + u * stride);
#pragma unroll
    for (int u = 0; u < U; ++u) acc += a[u];
  }
  if (acc.x == 12345.678) out[0] = acc.y;
}

// copy of the library's dense row GEMV k_gemv<4,4,1>
template <int R, int U>
__global__ __launch_bounds__(256) void k_gemv(const double *__restrict__ M, long ld, long rows,
                                              const double *__restrict__ v, double *__restrict__ y) {
  __shared__ double sh[4 * R];
  const long r0 = (long)blockIdx.x * R;
  const long n2 = ld / 2;
  const d2 *v2 = reinterpret_cast<const d2 *>(v);
  const d2 *rowp[R];
#pragma unroll
  for (int r = 0; r < R; ++r) rowp[r] = reinterpret_cast<const d2 *>(M + (r0 + r) * ld);
  double acc[R];
#pragma unroll
  for (int r = 0; r < R; ++r) acc[r] = 0.0;
  for (long c = threadIdx.x; c + (long)(U - 1) * 256 < n2; c += 256L * U) {
    d2 xv[U];
    d2 kv[R][U];
#pragma unroll
    for (int u = 0; u < U; ++u) xv[u] = v2[c + u * 256];
#pragma unroll
    for (int r = 0; r < R; ++r)
#pragma unroll
      for (int u = 0; u < U; ++u) kv[r][u] = __builtin_nontemporal_load(rowp[r] + c + u * 256);
#pragma unroll
    for (int r = 0; r < R; ++r)
#pragma unroll
      for (int u = 0; u < U; ++u) {
        acc[r] = fma(kv[r][u].x, xv[u].x, acc[r]);
        acc[r] = fma(kv[r][u].y, xv[u].y, acc[r]);
      }
  }
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
#pragma unroll
  for (int r = 0; r < R; ++r) {
    double s = acc[r];
    for (int o = 32; o > 0; o >>= 1) s += __shfl_down(s, o, 64);
    if (lane == 0) sh[w * R + r] = s;
  }
  __syncthreads();
  if (threadIdx.x < R) y[r0 + threadIdx.x] = (sh[threadIdx.x] + sh[R + threadIdx.x]) + (sh[2 * R + threadIdx.x] + sh[3 * R + threadIdx.x]);
}

__global__ void k_fill(double *A, long n, unsigned seed) {
  for (long i = (long)blockIdx.x * 256 + threadIdx.x; i < n; i += (long)gridDim.x * 256) {
    unsigned h = (unsigned)(i * 2654435761u) ^ seed;
    h ^= h >> 13;
    h *= 0x5bd1e995u;
    A[i] = (double)(h & 0xffff) / 65536.0 - 0.5;
  }
}

template <typename F>
float time_it(F f, int reps) {
  hipEvent_t a, b;
  CK(hipEventCreate(&a));
  CK(hipEventCreate(&b));
  f();
  CK(hipDeviceSynchronize());
  CK(hipEventRecord(a, 0));
  for (int r = 0; r < reps; ++r) f();
  CK(hipEventRecord(b, 0));
  CK(hipEventSynchronize(b));
  float ms = 0;
  CK(hipEventElapsedTime(&ms, a, b));
  return ms / reps;
}

int main(int argc, char **argv) {
  const long N = argc > 1 ? atol(argv[1]) : 65536;
  const int nb = (int)((N + B - 1) / B);
  const long Np = (long)nb * B;
  std::vector<int2> list;
  for (int I = 0; I < nb; ++I)
    for (int J = 0; J <= I; ++J) list.push_back(make_int2(I, J));
  const long nt = (long)list.size();
  double *tiles, *v, *P, *y, *out;
  int2 *dl;
  CK(hipMalloc(&tiles, sizeof(double) * nt * B * B));
  CK(hipMalloc(&v, sizeof(double) * Np));
  CK(hipMalloc(&P, sizeof(double) * nb * Np));
  CK(hipMalloc(&y, sizeof(double) * Np * 2));
  CK(hipMalloc(&out, sizeof(double)));
  CK(hipMalloc(&dl, sizeof(int2) * nt));
  CK(hipMemcpy(dl, list.data(), sizeof(int2) * nt, hipMemcpyHostToDevice));
  hipLaunchKernelGGL(k_fill, dim3(4096), dim3(256), 0, 0, tiles, nt * B * B, 1u);
  hipLaunchKernelGGL(k_fill, dim3(256), dim3(256), 0, 0, v, Np, 2u);
  CK(hipDeviceSynchronize());
  const double bytes = 8.0 * nt * B * B;
  printf("N=%ld tiles=%ld bytes=%.3f GB\n", N, nt, bytes / 1e9);
  const int reps = 10;
  float ms = time_it([&] {
    hipLaunchKernelGGL(k_stream, dim3(8192), dim3(256), 0, 0, (const d2 *)tiles, nt * B * B / 2, out);
  }, reps);
  printf("stream-read         %.3f ms  %.0f GB/s\n", ms, bytes / ms / 1e6);
#define RUN(RB, NW, PF)                                                                    \
  ms = time_it([&] {                                                                       \
    hipLaunchKernelGGL((k_symv<RB, NW, PF>), dim3((unsigned)nt), dim3(NW * 64), 0, 0, tiles, \
                       dl, v, P, Np);                                                      \
  }, reps);                                                                                \
  printf("symv RB=%d NW=%d PF=%d  %.3f ms  %.0f GB/s\n", RB, NW, (int)PF, ms, bytes / ms / 1e6);
  RUN(8, 4, true)
#define RUN2(RB, LR, IL)                                                                   \
  ms = time_it([&] {                                                                       \
    hipLaunchKernelGGL((k_symv2<RB, LR, IL>), dim3((unsigned)nt), dim3(256), 0, 0, tiles, dl, v, P, Np); \
  }, reps);                                                                                \
  printf("symv2 RB=%d LDSROWS=%d IL=%d  %.3f ms  %.0f GB/s\n", RB, (int)LR, (int)IL, ms, bytes / ms / 1e6);
  RUN2(8, true, true)
#define RUN3(RB)                                                                           \
  ms = time_it([&] {                                                                       \
    hipLaunchKernelGGL((k_symv3<RB>), dim3((unsigned)nt), dim3(256), 0, 0, tiles, dl, v, P, Np); \
  }, reps);                                                                                \
  printf("symv3 RB=%d  %.3f ms  %.0f GB/s\n", RB, ms, bytes / ms / 1e6);
#define RUN4(RB, WPE)                                                                      \
  ms = time_it([&] {                                                                       \
    hipLaunchKernelGGL((k_symv4<RB, WPE>), dim3((unsigned)nt), dim3(256), 0, 0, tiles, dl, v, P, Np); \
  }, reps);                                                                                \
  printf("symv4 RB=%d WPE=%d  %.3f ms  %.0f GB/s\n", RB, WPE, ms, bytes / ms / 1e6);
  RUN4(8, 1)
  RUN4(8, 2)
  RUN4(8, 3)
  RUN4(12, 2)
  RUN4(6, 3)
  RUN4(4, 4)
  ms = time_it([&] {
    hipLaunchKernelGGL(k_symv6, dim3((unsigned)nt), dim3(256), 0, 0, tiles, dl, v, P, Np);
  }, reps);
  printf("symv6 (LDS transpose rows)  %.3f ms  %.0f GB/s\n", ms, bytes / ms / 1e6);
  ms = time_it([&] {
    hipLaunchKernelGGL(k_symv6nt, dim3((unsigned)nt), dim3(256), 0, 0, tiles, dl, v, P, Np);
  }, reps);
  printf("symv6 nontemporal P stores %.3f ms  %.0f GB/s\n", ms, bytes / ms / 1e6);
  ms = time_it([&] {
    hipLaunchKernelGGL(k_pwrite, dim3((unsigned)nt), dim3(256), 0, 0, dl, P, Np);
  }, reps);
  printf("P writes alone (67 MB)      %.3f ms\n", ms);
  ms = time_it([&] {
    hipLaunchKernelGGL((k_symv6x<true, false>), dim3((unsigned)nt), dim3(256), 0, 0, tiles, dl, v, P, Np);
  }, reps);
  printf("symv6 no P writes           %.3f ms  %.0f GB/s\n", ms, bytes / ms / 1e6);
  ms = time_it([&] {
    hipLaunchKernelGGL((k_symv6x<false, true>), dim3((unsigned)nt), dim3(256), 0, 0, tiles, dl, v, P, Np);
  }, reps);
  printf("symv6 no column FMAs        %.3f ms  %.0f GB/s\n", ms, bytes / ms / 1e6);
  ms = time_it([&] {
    hipLaunchKernelGGL((k_symv6x<true, true>), dim3((unsigned)nt), dim3(256), 0, 0, tiles, dl, v, P, Np);
  }, reps);
  printf("symv6 no writes, no col     %.3f ms  %.0f GB/s\n", ms, bytes / ms / 1e6);
  {  // correctness of symv6 vs symv (row + column partials)
    std::vector<double> h1((size_t)nb * Np), h2((size_t)nb * Np);
    CK(hipMemset(P, 0, sizeof(double) * nb * Np));
    hipLaunchKernelGGL((k_symv<8, 4, true>), dim3((unsigned)nt), dim3(256), 0, 0, tiles, dl, v, P, Np, (long)B * B);
    CK(hipMemcpy(h1.data(), P, sizeof(double) * nb * Np, hipMemcpyDeviceToHost));
    CK(hipMemset(P, 0, sizeof(double) * nb * Np));
    hipLaunchKernelGGL(k_symv6, dim3((unsigned)nt), dim3(256), 0, 0, tiles, dl, v, P, Np);
    CK(hipMemcpy(h2.data(), P, sizeof(double) * nb * Np, hipMemcpyDeviceToHost));
    double md = 0, mx = 0;
    for (size_t i = 0; i < h1.size(); ++i) { md = fmax(md, fabs(h1[i] - h2[i])); mx = fmax(mx, fabs(h1[i])); }
    printf("symv6 vs symv max|diff| %.3e (max %.3e)\n", md, mx);
  }
  // tile pitch experiment: pad each tile by `pad` doubles (alignment phase of the WGs)
  for (long pad : {64L, 512L, 4096L + 64L}) {
    const long pitch = (long)B * B + pad;
    const long nt3 = nt * (long)B * B / pitch;  // same buffer, slightly fewer tiles
    ms = time_it([&] {
      hipLaunchKernelGGL((k_symv<8, 4, true>), dim3((unsigned)nt3), dim3(256), 0, 0, tiles, dl, v, P, Np, pitch);
    }, reps);
    printf("symv 8,4,PF pitch+%ld (%ld tiles) %.3f ms  %.0f GB/s\n", pad, nt3, ms, 8.0 * nt3 * B * B / ms / 1e6);
  }
  // tail test: the first multiple of 512 tiles only
  {
    const long nt2 = nt / 512 * 512;
    ms = time_it([&] {
      hipLaunchKernelGGL((k_symv<8, 4, true>), dim3((unsigned)nt2), dim3(256), 0, 0, tiles, dl, v, P, Np);
    }, reps);
    printf("symv 8,4,PF on %ld tiles  %.3f ms  %.0f GB/s\n", nt2, ms, 8.0 * nt2 * B * B / ms / 1e6);
  }
  ms = time_it([&] {
    hipLaunchKernelGGL((k_stream_u<8>), dim3(4096), dim3(256), 0, 0, (const d2 *)tiles, nt * B * B / 2, out);
  }, reps);
  printf("stream-read U=8 g4096 %.3f ms  %.0f GB/s\n", ms, bytes / ms / 1e6);
  ms = time_it([&] {
    hipLaunchKernelGGL((k_stream_u<8>), dim3(16384), dim3(256), 0, 0, (const d2 *)tiles, nt * B * B / 2, out);
  }, reps);
  printf("stream-read U=8 g16k %.3f ms  %.0f GB/s\n", ms, bytes / ms / 1e6);
  {
    const long ld = 65536, rows = nt * B * B / ld;
    ms = time_it([&] {
      hipLaunchKernelGGL((k_gemv<4, 4>), dim3((unsigned)(rows / 4)), dim3(256), 0, 0, tiles, ld, rows, v, y);
    }, reps);
    printf("dense gemv<4,4> on same bytes (%ld x %ld)  %.3f ms  %.0f GB/s\n", rows, ld, ms,
           8.0 * rows * ld / ms / 1e6);
  }
  ms = time_it([&] {
    hipLaunchKernelGGL(k_reduce, dim3((unsigned)((N + 255) / 256)), dim3(256), 0, 0, P, Np, nb, N, y);
  }, reps);
  printf("reduce              %.3f ms  (%.0f GB/s over %.1f MB)\n", ms,
         8.0 * nb * N / ms / 1e6, 8.0 * nb * N / 1e6);
  return 0;
}
