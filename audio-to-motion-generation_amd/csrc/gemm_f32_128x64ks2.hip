// Instantiation of the GEMM engine's launch_tile<128, 64, 32, 0, 2> (the 128x64 fp32 tile with two wave groups splitting each k-tile;
// one translation unit per tile configuration so the kernels compile in parallel).
#include "gemm_kernel.h"

namespace a2m {
template void launch_tile<128, 64, 32, 0, 2>(const GemmArgs&, int, int, int, hipStream_t);
}  // namespace a2m
