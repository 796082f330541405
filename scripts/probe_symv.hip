// Development probe: variants of the symmetric tiled mat-vec (csrc/kernels_sym.hip)
// at N = 65536 on one MI355X, timed with hipEvents.  Not part of the library.
//   hipcc -O3 --offload-arch=gfx950 -std=c++17 scripts/probe_symv.hip -o probe_symv
#include <hip/hip_runtime.h>

#include <cstdio>
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
                                                  double *__restrict__ P, long Np) {
  __shared__ double sh[(NW + 1) * B];
  const int2 t = list[blockIdx.x];
  const double *A = tiles + (long)blockIdx.x * B * B;
  if (t.x == t.y)
    body<RB, NW, PF, true>(A, t.x, t.y, v, P, Np, sh);
  else
    body<RB, NW, PF, false>(A, t.x, t.y, v, P, Np, sh);
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
  CK(hipMalloc(&y, sizeof(double) * Np));
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
  RUN(8, 4, false)
  RUN(4, 4, false)
  RUN(4, 4, true)
  RUN(8, 4, true)
  RUN(8, 8, false)
  RUN(4, 8, false)
  RUN(4, 8, true)
  RUN(2, 4, true)
  ms = time_it([&] {
    hipLaunchKernelGGL(k_reduce, dim3((unsigned)((N + 255) / 256)), dim3(256), 0, 0, P, Np, nb, N, y);
  }, reps);
  printf("reduce              %.3f ms  (%.0f GB/s over %.1f MB)\n", ms,
         8.0 * nb * N / ms / 1e6, 8.0 * nb * N / 1e6);
  return 0;
}
