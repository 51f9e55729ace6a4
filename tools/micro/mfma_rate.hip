// MFMA issue-rate probe (diagnostic): v_mfma_f32_32x32x2_f32 / v_mfma_f32_16x16x4_f32 chains on
// NACC independent accumulators, W waves per SIMD (256 x W threads per block, one block per CU),
// operands in registers.  Prints the achieved fraction of the f32 MFMA peak per configuration.
//   hipcc --offload-arch=gfx950 -O3 tools/micro/mfma_rate.hip -o /tmp/mfma_rate && /tmp/mfma_rate
#include <hip/hip_runtime.h>
#include <cstdio>

typedef float floatx16 __attribute__((ext_vector_type(16)));
typedef float floatx4 __attribute__((ext_vector_type(4)));

template <int NACC, bool BIG>
__global__ void mfma_loop(float* out, int iters, float a0, float b0) {
  float a = a0 + threadIdx.x * 1e-7f, b = b0 - threadIdx.x * 1e-7f;
  if constexpr (BIG) {
    floatx16 acc[NACC];
    for (int j = 0; j < NACC; ++j)
      for (int q = 0; q < 16; ++q) acc[j][q] = 0.f;
    for (int i = 0; i < iters; ++i) {
#pragma unroll
      for (int s = 0; s < 16 / NACC; ++s)
#pragma unroll
        for (int j = 0; j < NACC; ++j) acc[j] = __builtin_amdgcn_mfma_f32_32x32x2f32(a, b, acc[j], 0, 0, 0);
    }
    float r = 0.f;
    for (int j = 0; j < NACC; ++j)
      for (int q = 0; q < 16; ++q) r += acc[j][q];
    out[blockIdx.x * blockDim.x + threadIdx.x] = r;
  } else {
    floatx4 acc[NACC];
    for (int j = 0; j < NACC; ++j)
      for (int q = 0; q < 4; ++q) acc[j][q] = 0.f;
    for (int i = 0; i < iters; ++i) {
#pragma unroll
      for (int s = 0; s < 32 / NACC; ++s)
#pragma unroll
        for (int j = 0; j < NACC; ++j) acc[j] = __builtin_amdgcn_mfma_f32_16x16x4f32(a, b, acc[j], 0, 0, 0);
    }
    float r = 0.f;
    for (int j = 0; j < NACC; ++j)
      for (int q = 0; q < 4; ++q) r += acc[j][q];
    out[blockIdx.x * blockDim.x + threadIdx.x] = r;
  }
}

template <int NACC, bool BIG>
void run(int W, float* out) {
  const int iters = 2000;
  dim3 grid(256), block(256 * W);
  hipLaunchKernelGGL((mfma_loop<NACC, BIG>), grid, block, 0, 0, out, 10, 1.f, 2.f);
  hipEvent_t e0, e1;
  hipEventCreate(&e0); hipEventCreate(&e1);
  hipEventRecord(e0);
  for (int r = 0; r < 5; ++r) hipLaunchKernelGGL((mfma_loop<NACC, BIG>), grid, block, 0, 0, out, iters, 1.f, 2.f);
  hipEventRecord(e1);
  hipEventSynchronize(e1);
  float ms;
  hipEventElapsedTime(&ms, e0, e1);
  // per wave per iter: 16 (32x32x2: 4096 flop) or 32 (16x16x4: 2048 flop) MFMAs
  const double flop = 5.0 * 256 * 4 * W * (double)iters * (BIG ? 16 * 4096.0 : 32 * 2048.0);
  const double tf = flop / (ms * 1e-3) / 1e12;
  printf("%s NACC=%d waves/SIMD=%d: %.1f TF (%.2f of 157.3)\n", BIG ? "32x32x2" : "16x16x4 ", NACC, W, tf, tf / 157.3);
}

int main() {
  float* out;
  hipMalloc(&out, 256 * 1024 * sizeof(float));
  for (int W = 1; W <= 2; ++W) {
    run<1, true>(W, out); run<2, true>(W, out); run<4, true>(W, out);
    run<1, false>(W, out); run<2, false>(W, out); run<4, false>(W, out);
  }
  return 0;
}
