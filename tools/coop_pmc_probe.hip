// Minimal reproducer for the SIGSEGV at process exit seen under `rocprofv3 --pmc` (profiles/r04/pmc_probe*):
// one trivial kernel launched with hipLaunchCooperativeKernel (mode 1) or a plain launch (mode 0), then exit.
//   hipcc --offload-arch=gfx950 -O2 tools/coop_pmc_probe.hip -o tools/coop_pmc_probe
//   rocprofv3 --pmc FETCH_SIZE -- tools/coop_pmc_probe 1
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdlib>

__global__ void touch(double* x, int n) {
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i < n) x[i] = 2.0 * i;
}

int main(int argc, char** argv) {
  const int coop = argc > 1 ? atoi(argv[1]) : 1;
  const int n = 256 * 64;
  double* x = nullptr;
  if (hipMalloc(&x, n * sizeof(double)) != hipSuccess) return 2;
  hipError_t e;
  if (coop) {
    int nn = n;
    void* args[] = {(void*)&x, (void*)&nn};
    e = hipLaunchCooperativeKernel((const void*)touch, dim3(256), dim3(64), args, 0, nullptr);
  } else {
    hipLaunchKernelGGL(touch, dim3(256), dim3(64), 0, nullptr, x, n);
    e = hipGetLastError();
  }
  if (e != hipSuccess) {
    printf("launch failed: %s\n", hipGetErrorString(e));
    return 3;
  }
  if (hipDeviceSynchronize() != hipSuccess) return 4;
  double h = 0;
  if (hipMemcpy(&h, x + 7, sizeof(double), hipMemcpyDeviceToHost) != hipSuccess) return 5;
  (void)hipFree(x);
  printf("coop=%d ok x[7]=%g\n", coop, h);
  return 0;
}
