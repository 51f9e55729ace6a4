// Launches of the software-pipelined 64x64 fp32 tile (gemm_pipe.h), one kernel per B operand mode.
#include "gemm_pipe.h"

#if A2M_PIPE_STAMPS
__device__ unsigned long long g_pipe_stamps[kPipeStampBlocks * 6];
#endif
namespace a2m {
void launch_pipe(const GemmArgs& a, int ma, int mb, int batch, hipStream_t st) {
  const dim3 grid((unsigned)cdiv(a.N, 64), (unsigned)cdiv(a.M, 64), (unsigned)(batch * a.splits));
  if (mb == 4) { hipLaunchKernelGGL((gemm_pipe_kernel<4, 0, 4>), grid, dim3(256), 0, st, a); return; }
  if (mb == 1) { hipLaunchKernelGGL((gemm_pipe_kernel<7, 0, 4>), grid, dim3(256), 0, st, a); return; }   // stride-2 runs
  if (ma == 3) {
    if (mb == 3) hipLaunchKernelGGL((gemm_pipe_kernel<3, 0, 3>), grid, dim3(256), 0, st, a);
    else hipLaunchKernelGGL((gemm_pipe_kernel<0, 0, 3>), grid, dim3(256), 0, st, a);
    return;
  }
  if (mb == 5 && a.B.halo) hipLaunchKernelGGL((gemm_pipe_kernel<5, 0>), grid, dim3(256), 0, st, a);
  else if (mb == 5 && a.B.tapconv == 1) hipLaunchKernelGGL((gemm_pipe_kernel<5, 1>), grid, dim3(256), 0, st, a);
  else if (mb == 5 && a.B.tapconv == 2) hipLaunchKernelGGL((gemm_pipe_kernel<5, 2>), grid, dim3(256), 0, st, a);
  else if (mb == 5) hipLaunchKernelGGL((gemm_pipe_kernel<5, 3>), grid, dim3(256), 0, st, a);
  else if (mb == 6) hipLaunchKernelGGL(gemm_pipe_kernel<6>, grid, dim3(256), 0, st, a);
  else if (mb == 3) hipLaunchKernelGGL(gemm_pipe_kernel<3>, grid, dim3(256), 0, st, a);
  else hipLaunchKernelGGL(gemm_pipe_kernel<0>, grid, dim3(256), 0, st, a);
}
}  // namespace a2m

#if A2M_PIPE_STAMPS
// diagnostic builds only (tools/build_variant.sh ... -DA2M_PIPE_STAMPS=1): the stamp table
extern "C" int a2m_debug_pipe_stamps(unsigned long long* out, int n) {
  if (n > kPipeStampBlocks * 6) n = kPipeStampBlocks * 6;
  return hipMemcpyFromSymbol(out, HIP_SYMBOL(g_pipe_stamps), n * sizeof(unsigned long long)) == hipSuccess ? 0 : 1;
}
#endif
