// VALU issue-rate probe: scalar v_fma_f32 vs packed v_pk_fma_f32 (wave64), several waves per SIMD.
#include <hip/hip_runtime.h>
#include <cstdio>
typedef float f2 __attribute__((ext_vector_type(2)));
constexpr int ITERS = 4096;

__global__ void scalar_fma(float* out, float a, float b) {
  float x[8];
  for (int i = 0; i < 8; ++i) x[i] = threadIdx.x + i;
  for (int it = 0; it < ITERS; ++it)
#pragma unroll
    for (int i = 0; i < 8; ++i) x[i] = __builtin_fmaf(x[i], a, b);
  float s = 0;
  for (int i = 0; i < 8; ++i) s += x[i];
  out[blockIdx.x * blockDim.x + threadIdx.x] = s;
}
__global__ void packed_fma(float* out, float a, float b) {
  f2 x[8];
  for (int i = 0; i < 8; ++i) x[i] = (f2){(float)threadIdx.x + i, (float)i};
  const f2 av = (f2){a, a}, bv = (f2){b, b};
  for (int it = 0; it < ITERS; ++it)
#pragma unroll
    for (int i = 0; i < 8; ++i) x[i] = __builtin_elementwise_fma(x[i], av, bv);
  float s = 0;
  for (int i = 0; i < 8; ++i) s += x[i].x + x[i].y;
  out[blockIdx.x * blockDim.x + threadIdx.x] = s;
}
__global__ void scalar_add(float* out, float a, float b) {
  float x[8];
  for (int i = 0; i < 8; ++i) x[i] = threadIdx.x + i;
  for (int it = 0; it < ITERS; ++it)
#pragma unroll
    for (int i = 0; i < 8; ++i) x[i] = x[i] + a;
  float s = 0;
  for (int i = 0; i < 8; ++i) s += x[i];
  out[blockIdx.x * blockDim.x + threadIdx.x] = s;
}
__global__ void packed_add(float* out, float a, float b) {
  f2 x[8];
  for (int i = 0; i < 8; ++i) x[i] = (f2){(float)threadIdx.x + i, (float)i};
  const f2 av = (f2){a, b};
  for (int it = 0; it < ITERS; ++it)
#pragma unroll
    for (int i = 0; i < 8; ++i) x[i] = x[i] + av;
  float s = 0;
  for (int i = 0; i < 8; ++i) s += x[i].x + x[i].y;
  out[blockIdx.x * blockDim.x + threadIdx.x] = s;
}

int main() {
  float* out;
  hipMalloc(&out, 256 * 8 * 1024 * 4 * sizeof(float));
  hipEvent_t e0, e1;
  hipEventCreate(&e0);
  hipEventCreate(&e1);
  struct K { const char* n; void (*f)(float*, float, float); double flops_per_op; };
  K ks[] = {{"scalar_fma", scalar_fma, 2}, {"packed_fma", packed_fma, 4}, {"scalar_add", scalar_add, 1},
            {"packed_add", packed_add, 2}};
  for (int wps : {1, 2, 4, 8}) {       // waves per SIMD
    const int blocks = 256 * wps;      // 256-thread blocks = 4 waves = one per SIMD
    for (auto& k : ks) {
      hipLaunchKernelGGL(k.f, dim3(blocks), dim3(256), 0, 0, out, 1.0001f, 0.5f);
      hipEventRecord(e0);
      hipLaunchKernelGGL(k.f, dim3(blocks), dim3(256), 0, 0, out, 1.0001f, 0.5f);
      hipEventRecord(e1);
      hipEventSynchronize(e1);
      float ms;
      hipEventElapsedTime(&ms, e0, e1);
      const double insts = (double)blocks * 4 * ITERS * 8;   // wave-instructions
      const double cyc_per_inst_simd = ms * 1e-3 * 2.4e9 * 1024 / insts;  // 1024 SIMDs
      printf("%-11s waves/SIMD %d: %.3f ms, %.2f SIMD-cycles per wave-instruction, %.1f TFLOP/s\n",
             k.n, wps, ms, cyc_per_inst_simd, insts * 64 * k.flops_per_op / (ms * 1e-3) / 1e12);
    }
  }
  return 0;
}
