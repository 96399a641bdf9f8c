// glf_chunk.hip — Lindblad / GLF runs with more than MAX_NC collapse operators (GLF pairs): the persistent kernel's
// CHUNK instantiations, whose X / k GEMMs walk the segment list MAX_NC segments at a time through the LDS table and
// accumulate in registers (same operand order as one long list: the sum over c runs in the same sequence).
// oqs.liouvillian sums over any c_ops list (oqs.py:697-714); a full set of |i><j| jumps at N = 17 is 272 operators.
#include "glf_kernel.hpp"

namespace qd {

int glf_launch_chunk(const LindbladParams& p, int B, hipStream_t st) {
  const int Np = p.Np;
  const bool herm = p.herm != 0;
  if (Np == 32) {
    if (herm) hipLaunchKernelGGL((lindblad_rk4_kernel<32, true, false, true>), dim3(B), dim3(CG_WG), 0, st, p);
    else hipLaunchKernelGGL((lindblad_rk4_kernel<32, false, false, true>), dim3(B), dim3(CG_WG), 0, st, p);
  } else if (Np == 64) {
    if (herm) hipLaunchKernelGGL((lindblad_rk4_kernel<64, true, false, true>), dim3(B), dim3(CG_WG), 0, st, p);
    else hipLaunchKernelGGL((lindblad_rk4_kernel<64, false, false, true>), dim3(B), dim3(CG_WG), 0, st, p);
  } else {
    // Hermitian: the plain X GEMM (every tile takes every segment; exact for Lindblad as for GLF operands).  The
    // tile-skipping HSEG form, whose accumulators would have to stay live across the chunk loop, spills 496 B / lane.
    if (herm) hipLaunchKernelGGL((lindblad_rk4_kernel<128, true, false, true>), dim3(B), dim3(CG_WG), 0, st, p);
    else hipLaunchKernelGGL((lindblad_rk4_kernel<128, false, false, true>), dim3(B), dim3(CG_WG), 0, st, p);
  }
  QD_HIP(hipGetLastError());
  return QD_OK;
}

}  // namespace qd
