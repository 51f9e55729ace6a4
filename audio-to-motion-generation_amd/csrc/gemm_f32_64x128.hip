// Instantiation of the GEMM engine's launch_tile<64, 128, 32, 0> (the 64x128 fp32 tile;
// one translation unit per tile configuration so the kernels compile in parallel).
#include "gemm_kernel.h"

namespace a2m {
template void launch_tile<64, 128, 32, 0>(const GemmArgs&, int, int, int, hipStream_t);
}  // namespace a2m
