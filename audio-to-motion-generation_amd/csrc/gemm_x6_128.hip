// Instantiation of the GEMM engine's launch_tile<128, 128, 32, 2> (bf16x6: fp32 operands split
// into three bf16 planes, six MFMA products per k-chunk; one translation unit per tile configuration).
#include "gemm_kernel.h"

#ifdef A2M_WITH_X6   // bf16x6 is an experiment (measured slower than fp32): built only on request

namespace a2m {
template void launch_tile<128, 128, 32, 2>(const GemmArgs&, int, int, int, hipStream_t);
}  // namespace a2m
#endif  // A2M_WITH_X6
