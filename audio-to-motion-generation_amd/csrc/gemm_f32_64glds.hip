// Instantiation of the GEMM engine's launch_tile<64, 64, 32, 0, 4> (the 64x64 fp32 tile with
// LDS-DMA operand staging; one translation unit per tile configuration).
#include "gemm_kernel.h"

namespace a2m {
template void launch_tile<64, 64, 32, 0, 4>(const GemmArgs&, int, int, int, hipStream_t);
}  // namespace a2m
