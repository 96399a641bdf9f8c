// PMC calibration: kernels with exactly known HBM byte counts (256 MiB read, 256 MiB written,
// 16-B per lane, fully coalesced) to convert FETCH_SIZE / WRITE_SIZE into bytes on gfx950.
// Build: hipcc --offload-arch=gfx950 -O3 tools/pmc_calib.hip -o tools/pmc_calib
#include <hip/hip_runtime.h>
#include <cstdio>
typedef double v2 __attribute__((ext_vector_type(2)));
__global__ void write_only(v2* out, size_t n) {
  for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < n; i += (size_t)gridDim.x * blockDim.x)
    out[i] = v2{(double)i, 1.0};
}
__global__ void read_only(const v2* in, size_t n, double* sink) {
  double s = 0;
  for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < n; i += (size_t)gridDim.x * blockDim.x)
    s += in[i].x + in[i].y;
  if (s == 12345.678) sink[0] = s;
}
int main() {
  const size_t bytes = 256ull << 20, n = bytes / 16;
  v2 *a, *b;
  double* sink;
  if (hipMalloc(&a, bytes) || hipMalloc(&b, bytes) || hipMalloc(&sink, 8)) return 1;
  for (int r = 0; r < 2; ++r) {
    hipLaunchKernelGGL(write_only, dim3(4096), dim3(256), 0, 0, a, n);
    hipLaunchKernelGGL(write_only, dim3(4096), dim3(256), 0, 0, b, n);  // evict a from MALL
    hipLaunchKernelGGL(read_only, dim3(4096), dim3(256), 0, 0, a, n, sink);
  }
  if (hipDeviceSynchronize()) return 2;
  printf("pmc_calib: each write_only writes %zu B, read_only reads %zu B\n", bytes, bytes);
  return 0;
}
