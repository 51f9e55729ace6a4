// Instantiation of the GEMM engine's launch_tile<128, 128, 32, 0, 4> (the 128x128 fp32 tile
// with LDS-DMA operand staging; one translation unit per tile configuration).
#include "gemm_kernel.h"

namespace a2m {
template void launch_tile<128, 128, 32, 0, 4>(const GemmArgs&, int, int, int, hipStream_t);
}  // namespace a2m
