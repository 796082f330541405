// FETCH_SIZE calibration for the access widths of k_rec_g (MI355X_MICROARCH.md, HBM: "FETCH_SIZE
// reports 1/2 of the bytes of a wide coalesced streaming read ... other access widths are
// uncalibrated: calibrate on a known byte count in your own access pattern").
//
//   hipcc --offload-arch=gfx950 -O3 scripts/dev/pmc_calib.hip -o gpurun_out/pmc_calib
//   rocprofv3 --pmc FETCH_SIZE -- gpurun_out/pmc_calib        (one counter group per pass)
//
// Each kernel reads a fresh 256 MiB-beyond-MALL buffer region of BYTES bytes exactly once:
//   k_wide     16 B per lane, consecutive (the calibrated case: expect FETCH_SIZE = BYTES / 2)
//   k_rdd      k_rec_g's Rdd pattern: lanes of a 16-wide row take consecutive pairs d, each lane
//              loads its pair's 3 doubles (r[0], r[1], r[2] at a 24-byte stride, 8 B per load);
//              rows of 16 pairs at the pair-triangle offsets a(a-1)/2 (a = 16 A + la)
//   k_scalar8  8 B per lane, consecutive (k_rec_fin / staging loads)
// FETCH_SIZE / BYTES per kernel is the factor to apply to that pattern's counts.
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdlib>
#include <vector>

typedef double d2v __attribute__((ext_vector_type(2)));

__global__ void k_wide(const d2v *__restrict__ a, size_t n2, double *__restrict__ out) {
  double s = 0.0;
  for (size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x; i < n2; i += (size_t)gridDim.x * blockDim.x) {
    const d2v v = __builtin_nontemporal_load(a + i);
    s += v.x + v.y;
  }
  if (s == 1.2345) out[0] = s;  // keep the loads
}

__global__ void k_scalar8(const double *__restrict__ a, size_t n, double *__restrict__ out) {
  double s = 0.0;
  for (size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (size_t)gridDim.x * blockDim.x)
    s += a[i];
  if (s == 1.2345) out[0] = s;
}

// Rdd of one point: D pairs x 3 doubles.  A workgroup of 256 threads = a 16 x 16 atom block
// (la = tid / 16, lb = tid % 16), pair d = aa (aa - 1) / 2 + bb for aa = 16 A + la > bb = 16 B + lb,
// every (A >= B) block and every point j, as k_rec_g reads it (one load per component).
__global__ void k_rdd(const double *__restrict__ Rdd, int n, long long D, int M, int nblk,
                      double *__restrict__ out) {
  const long long nbp = (long long)nblk * (nblk + 1) / 2;
  double s = 0.0;
  for (long long u = blockIdx.x; u < nbp * M; u += gridDim.x) {
    const long long bp = u % nbp, j = u / nbp;
    int A = 0;
    while ((long long)(A + 1) * (A + 2) / 2 <= bp) ++A;
    const int B = (int)(bp - (long long)A * (A + 1) / 2);
    const int aa = A * 16 + (threadIdx.x >> 4), bb = B * 16 + (threadIdx.x & 15);
    if (aa < n && bb < n && aa > bb) {
      const double *r = Rdd + (j * D + (long long)aa * (aa - 1) / 2 + bb) * 3;
      s += r[0] + r[1] + r[2];
    }
  }
  if (s == 1.2345) out[0] = s;
}

int main() {
  const int n = 370, M = 14;
  const long long D = (long long)n * (n - 1) / 2;
  const size_t rdd = (size_t)M * D * 3;                 // 22.9 MB: the nanotube's Rdd
  const size_t big = (size_t)1 << 28;                   // 2 GiB region: beyond the 256 MiB MALL
  double *a = nullptr, *out = nullptr;
  if (hipMalloc(&a, big * sizeof(double)) != hipSuccess || hipMalloc(&out, 64) != hipSuccess) return 1;
  if (hipMemset(a, 0, big * sizeof(double)) != hipSuccess) return 1;
  const size_t bytes = (size_t)512 << 20;               // 512 MiB per streaming kernel
  if (hipDeviceSynchronize() != hipSuccess) return 1;
  // distinct regions so no kernel finds another's lines in the MALL
  k_wide<<<4096, 256>>>(reinterpret_cast<const d2v *>(a), bytes / 16, out);
  k_scalar8<<<4096, 256>>>(a + bytes / 8, bytes / 8, out);
  const int nblk = (n + 15) / 16;
  k_rdd<<<2048, 256>>>(a + 2 * bytes / 8, n, D, M, nblk, out);
  if (hipDeviceSynchronize() != hipSuccess) return 1;
  printf("k_wide bytes %zu\nk_scalar8 bytes %zu\nk_rdd bytes %zu (M %d x D %lld x 3 doubles)\n", bytes,
         bytes, rdd * 8, M, D);
  (void)hipFree(a);
  (void)hipFree(out);
  return 0;
}
