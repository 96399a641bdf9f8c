// Microbenchmark: v_mfma_f64_16x16x4_f64 throughput with NACC independent accumulator chains per wave (VGPR
// accumulators) at W waves per SIMD -- how many chains one wave needs to keep the FP64 matrix pipe busy.
// Build: hipcc --offload-arch=gfx950 -O3 tools/mfma_chain.hip -o tools/mfma_chain
#include <hip/hip_runtime.h>
#include <cstdio>
typedef double d4 __attribute__((ext_vector_type(4)));

template <int NACC>
__global__ void chain(double* out, int iters, double a0, double b0) {
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
}

template <int NACC>
static void run(double* out, int wps) {
  const int threads = 256 * wps, blocks = 256;   // one workgroup per CU, wps waves per SIMD
  const int iters = 4096 / NACC * 8;
  hipLaunchKernelGGL(chain<NACC>, dim3(blocks), dim3(threads), 0, 0, out, 16, 1.0, 1.0);
  hipDeviceSynchronize();
  hipEvent_t e0, e1;
  hipEventCreate(&e0);
  hipEventCreate(&e1);
  hipEventRecord(e0);
  hipLaunchKernelGGL(chain<NACC>, dim3(blocks), dim3(threads), 0, 0, out, iters, 1.0, 1.0);
  hipEventRecord(e1);
  hipEventSynchronize(e1);
  float ms = 0;
  hipEventElapsedTime(&ms, e0, e1);
  const double flop = 2.0 * 16 * 16 * 4 * (double)NACC * iters * (threads / 64) * blocks;
  printf("chains/wave %d, waves/SIMD %d: %.2f TFLOP/s\n", NACC, wps, flop / (ms * 1e-3) / 1e12);
}

int main() {
  double* out;
  hipMalloc(&out, 256 * 1024 * sizeof(double));
  for (int wps = 1; wps <= 2; ++wps) {
    run<1>(out, wps);
    run<2>(out, wps);
    run<3>(out, wps);
    run<4>(out, wps);
    run<8>(out, wps);
  }
  return 0;
}
