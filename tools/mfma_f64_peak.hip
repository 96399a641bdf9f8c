// Microbenchmark: sustained v_mfma_f64_16x16x4_f64 and v_fma_f64 rates on the whole chip.
// Build: hipcc --offload-arch=gfx950 -O3 tools/mfma_f64_peak.hip -o tools/mfma_f64_peak
#include <hip/hip_runtime.h>
#include <cstdio>
typedef double d4 __attribute__((ext_vector_type(4)));

// clk[0..1]: shader clock (clock64) and 100 MHz wall clock (wall_clock64) of block 0 at start / end,
// so the effective shader frequency under this load is known (the ceiling scales with it)
template <int NACC>
__global__ __launch_bounds__(256) void mfma_loop(double* out, int iters, double a0, double b0,
                                                 unsigned long long* clk) {
  if (blockIdx.x == 0 && threadIdx.x == 0) {
    clk[0] = clock64();
    clk[1] = wall_clock64();
  }
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
  if (blockIdx.x == 0 && threadIdx.x == 0) {
    clk[2] = clock64();
    clk[3] = wall_clock64();
  }
}

static double ghz(unsigned long long* dclk) {
  unsigned long long h[4];
  hipMemcpy(h, dclk, sizeof(h), hipMemcpyDeviceToHost);
  return (double)(h[2] - h[0]) / (double)(h[3] - h[1]) * 0.1;  // wall clock: 100 MHz
}

// Same loop with the accumulators pinned to VGPRs (inline asm "+v"), the form the library's GEMM engine
// compiles to; the builtin loop above keeps them in AGPRs.
template <int NACC>
__global__ __launch_bounds__(256) void mfma_loop_v(double* out, int iters, double a0, double b0,
                                                   unsigned long long* clk) {
  if (blockIdx.x == 0 && threadIdx.x == 0) {
    clk[0] = clock64();
    clk[1] = wall_clock64();
  }
  d4 acc[NACC];
  for (int i = 0; i < NACC; ++i) acc[i] = d4{0, 0, 0, 0};
  double a = a0 + threadIdx.x * 1e-9, b = b0 - threadIdx.x * 1e-9;
  for (int it = 0; it < iters; ++it) {
#pragma unroll
    for (int i = 0; i < NACC; ++i) asm volatile("v_mfma_f64_16x16x4_f64 %0, %1, %2, %0" : "+v"(acc[i]) : "v"(a), "v"(b));
  }
  double s = 0;
  for (int i = 0; i < NACC; ++i) s += acc[i][0] + acc[i][1] + acc[i][2] + acc[i][3];
  out[blockIdx.x * blockDim.x + threadIdx.x] = s;
  if (blockIdx.x == 0 && threadIdx.x == 0) {
    clk[2] = clock64();
    clk[3] = wall_clock64();
  }
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
  unsigned long long* clk;
  hipMalloc(&clk, 4 * sizeof(unsigned long long));
  const int blocks = 256 * 4, threads = 256;
  hipMalloc(&out, blocks * threads * sizeof(double));
  hipEvent_t e0, e1;
  hipEventCreate(&e0);
  hipEventCreate(&e1);
  const int iters = 20000;
  for (int rep = 0; rep < 2; ++rep) {
    hipLaunchKernelGGL(mfma_loop<4>, dim3(blocks), dim3(threads), 0, 0, out, iters, 1.0000001, 0.9999999, clk);
    hipEventRecord(e0);
    hipLaunchKernelGGL(mfma_loop<4>, dim3(blocks), dim3(threads), 0, 0, out, iters, 1.0000001, 0.9999999, clk);
    hipEventRecord(e1);
    hipEventSynchronize(e1);
    float ms;
    hipEventElapsedTime(&ms, e0, e1);
    double flop = 2.0 * 16 * 16 * 4 * 4.0 * iters * (blocks * threads / 64);
    double f = ghz(clk);
    printf("mfma_f64_16x16x4 (4 acc/wave, 4 waves/SIMD): %.2f TFLOP/s at %.2f GHz shader clock (%.2f at 2.4 GHz)\n",
           flop / ms / 1e9, f, flop / ms / 1e9 * 2.4 / f);
    hipLaunchKernelGGL(mfma_loop<8>, dim3(blocks), dim3(threads), 0, 0, out, iters / 2, 1.0000001, 0.9999999, clk);
    hipEventRecord(e0);
    hipLaunchKernelGGL(mfma_loop<8>, dim3(blocks), dim3(threads), 0, 0, out, iters / 2, 1.0000001, 0.9999999, clk);
    hipEventRecord(e1);
    hipEventSynchronize(e1);
    hipEventElapsedTime(&ms, e0, e1);
    flop = 2.0 * 16 * 16 * 4 * 8.0 * (iters / 2) * (blocks * threads / 64);
    f = ghz(clk);
    printf("mfma_f64_16x16x4 (8 acc/wave): %.2f TFLOP/s at %.2f GHz shader clock (%.2f at 2.4 GHz)\n", flop / ms / 1e9,
           f, flop / ms / 1e9 * 2.4 / f);
    hipLaunchKernelGGL(mfma_loop_v<8>, dim3(blocks), dim3(threads), 0, 0, out, iters / 2, 1.0000001, 0.9999999, clk);
    hipEventRecord(e0);
    hipLaunchKernelGGL(mfma_loop_v<8>, dim3(blocks), dim3(threads), 0, 0, out, iters / 2, 1.0000001, 0.9999999, clk);
    hipEventRecord(e1);
    hipEventSynchronize(e1);
    hipEventElapsedTime(&ms, e0, e1);
    f = ghz(clk);
    printf("mfma_f64_16x16x4 VGPR acc (8 acc/wave): %.2f TFLOP/s at %.2f GHz shader clock (%.2f at 2.4 GHz)\n",
           flop / ms / 1e9, f, flop / ms / 1e9 * 2.4 / f);
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
