// Microbenchmark: sustained v_mfma_f64_16x16x4_f64 and v_fma_f64 rates on the whole chip.
// Build: hipcc --offload-arch=gfx950 -O3 tools/mfma_f64_peak.hip -o tools/mfma_f64_peak
#include <hip/hip_runtime.h>
#include <cstdio>
typedef double d4 __attribute__((ext_vector_type(4)));

template <int NACC>
__global__ __launch_bounds__(256) void mfma_loop(double* out, int iters, double a0, double b0) {
  d4 acc[NACC];
  for (int i = 0; i < NACC; ++i) acc[i] = d4{0, 0, 0, 0};
  double a = a0 + threadIdx.x * 1e-9, b = b0 - threadIdx.x * 1e-9;
  for (int it = 0; it < iters; ++it) {
#pragma unroll
    for (int i = 0; i < NACC; ++i) acc[i] = __builtin_amdgcn_mfma_f64_16x16x4f64(a, b, acc[i], 0, 0, 0);
  }
  double s = 0;
  for (int i = 0; i < NACC; ++i) s += acc[i][0] + acc[i][1] + acc[i][2] + acc[i][3];
  out[blockIdx.x * blockDim.x + threadIdx.x] = s;
}

__global__ __launch_bounds__(256) void fma_loop(double* out, int iters, double a0, double b0) {
  double x[8];
  for (int i = 0; i < 8; ++i) x[i] = threadIdx.x + i;
  const double a = a0, b = b0;
  for (int it = 0; it < iters; ++it) {
#pragma unroll
    for (int i = 0; i < 8; ++i) x[i] = fma(x[i], a, b);
  }
  double s = 0;
  for (int i = 0; i < 8; ++i) s += x[i];
  out[blockIdx.x * blockDim.x + threadIdx.x] = s;
}

int main() {
  double* out;
  const int blocks = 256 * 4, threads = 256;
  hipMalloc(&out, blocks * threads * sizeof(double));
  hipEvent_t e0, e1;
  hipEventCreate(&e0);
  hipEventCreate(&e1);
  const int iters = 20000;
  for (int rep = 0; rep < 2; ++rep) {
    hipLaunchKernelGGL(mfma_loop<4>, dim3(blocks), dim3(threads), 0, 0, out, iters, 1.0000001, 0.9999999);
    hipEventRecord(e0);
    hipLaunchKernelGGL(mfma_loop<4>, dim3(blocks), dim3(threads), 0, 0, out, iters, 1.0000001, 0.9999999);
    hipEventRecord(e1);
    hipEventSynchronize(e1);
    float ms;
    hipEventElapsedTime(&ms, e0, e1);
    double flop = 2.0 * 16 * 16 * 4 * 4.0 * iters * (blocks * threads / 64);
    printf("mfma_f64_16x16x4 (4 acc/wave, 4 waves/CU): %.2f TFLOP/s\n", flop / ms / 1e9);
    hipLaunchKernelGGL(mfma_loop<8>, dim3(blocks), dim3(threads), 0, 0, out, iters / 2, 1.0000001, 0.9999999);
    hipEventRecord(e0);
    hipLaunchKernelGGL(mfma_loop<8>, dim3(blocks), dim3(threads), 0, 0, out, iters / 2, 1.0000001, 0.9999999);
    hipEventRecord(e1);
    hipEventSynchronize(e1);
    hipEventElapsedTime(&ms, e0, e1);
    flop = 2.0 * 16 * 16 * 4 * 8.0 * (iters / 2) * (blocks * threads / 64);
    printf("mfma_f64_16x16x4 (8 acc/wave): %.2f TFLOP/s\n", flop / ms / 1e9);
    hipEventRecord(e0);
    hipLaunchKernelGGL(fma_loop, dim3(blocks), dim3(threads), 0, 0, out, iters, 1.0000001, 1e-7);
    hipEventRecord(e1);
    hipEventSynchronize(e1);
    hipEventElapsedTime(&ms, e0, e1);
    flop = 2.0 * 8 * iters * (double)blocks * threads;
    printf("v_fma_f64: %.2f TFLOP/s\n", flop / ms / 1e9);
  }
  return 0;
}
