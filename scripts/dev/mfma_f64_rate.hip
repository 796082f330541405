// Micro-benchmark: issue rate and dependent latency of v_mfma_f64_16x16x4f64 and of v_fma_f64 on
// one MI355X (gfx950).  Build: hipcc --offload-arch=gfx950 -O3 mfma_f64_rate.hip -o mfma_f64_rate
// Prints cycles per instruction per SIMD (clock64 inside the kernel) for
//   chains = 1 (dependent back-to-back: latency) and chains = 4 / 8 (independent: issue rate),
// with 1 and 2 waves per SIMD.
#include <hip/hip_runtime.h>
#include <cstdio>

typedef double v4d __attribute__((ext_vector_type(4)));

template <int CH>
__global__ __launch_bounds__(256) void k_mfma(double *out, int iters, long long *cyc) {
  v4d acc[CH];
  for (int c = 0; c < CH; ++c) acc[c] = v4d{0.0, 0.0, 0.0, 0.0};
  double a = threadIdx.x * 1e-3, b = 1.0 + blockIdx.x * 1e-6;
  const long long t0 = clock64();
  for (int i = 0; i < iters; ++i) {
#pragma unroll
    for (int c = 0; c < CH; ++c) acc[c] = __builtin_amdgcn_mfma_f64_16x16x4f64(a, b, acc[c], 0, 0, 0);
  }
  const long long t1 = clock64();
  double s = 0.0;
  for (int c = 0; c < CH; ++c) s += acc[c][0] + acc[c][1] + acc[c][2] + acc[c][3];
  out[blockIdx.x * 256 + threadIdx.x] = s;
  if (threadIdx.x == 0) cyc[blockIdx.x] = t1 - t0;
}

template <int CH>
__global__ __launch_bounds__(256) void k_fma(double *out, int iters, long long *cyc) {
  double acc[CH];
  for (int c = 0; c < CH; ++c) acc[c] = threadIdx.x + c;
  const double a = 1.0 + threadIdx.x * 1e-9, b = 1e-7;
  const long long t0 = clock64();
  for (int i = 0; i < iters; ++i) {
#pragma unroll
    for (int c = 0; c < CH; ++c) acc[c] = fma(acc[c], a, b);
  }
  const long long t1 = clock64();
  double s = 0.0;
  for (int c = 0; c < CH; ++c) s += acc[c];
  out[blockIdx.x * 256 + threadIdx.x] = s;
  if (threadIdx.x == 0) cyc[blockIdx.x] = t1 - t0;
}

template <typename K>
void run(const char *name, K kern, int ch, int blocks, int iters, double *out, long long *cyc) {
  hipLaunchKernelGGL(kern, dim3(blocks), dim3(256), 0, 0, out, iters, cyc);
  hipDeviceSynchronize();
  hipEvent_t e0, e1;
  hipEventCreate(&e0);
  hipEventCreate(&e1);
  hipEventRecord(e0);
  hipLaunchKernelGGL(kern, dim3(blocks), dim3(256), 0, 0, out, iters, cyc);
  hipEventRecord(e1);
  hipEventSynchronize(e1);
  float ms = 0.f;
  hipEventElapsedTime(&ms, e0, e1);
  long long c0 = 0;
  hipMemcpy(&c0, cyc, sizeof(long long), hipMemcpyDeviceToHost);
  // 4 waves per workgroup, one per SIMD when blocks <= CUs; blocks / 256 workgroups per CU
  const double per_inst = (double)c0 / ((double)iters * ch);
  const double insts = (double)blocks * 4 * iters * ch;
  printf("%-6s chains %d  workgroups %5d  cycles/inst (clock64, one wave) %7.2f  %.3f ms  %.2f G wave-inst/s\n",
         name, ch, blocks, per_inst, ms, insts / (ms * 1e6));
}

int main() {
  double *out;
  long long *cyc;
  hipMalloc(&out, sizeof(double) * 256 * 2048);
  hipMalloc(&cyc, sizeof(long long) * 2048);
  const int iters = 4096;
  for (int blocks : {256, 512, 1024}) {
    run("mfma", k_mfma<1>, 1, blocks, iters, out, cyc);
    run("mfma", k_mfma<4>, 4, blocks, iters, out, cyc);
    run("mfma", k_mfma<8>, 8, blocks, iters, out, cyc);
    run("fma", k_fma<1>, 1, blocks, iters, out, cyc);
    run("fma", k_fma<8>, 8, blocks, iters, out, cyc);
  }
  return 0;
}
