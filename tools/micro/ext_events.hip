// Probe: kernel timestamps through hipExtLaunchKernelGGL's start/stop events, eagerly and under
// stream capture (graph replay), against a plain event pair around the launch.
#include <hip/hip_runtime.h>
#include <hip/hip_ext.h>
#include <cstdio>
__global__ void spin(float* x, int n, int it) {
  int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i < n) { float v = x[i]; for (int k = 0; k < it; ++k) v = v * 1.0001f + 0.5f; x[i] = v; }
}
#define C(x) do { hipError_t e = (x); if (e != hipSuccess) printf("%-70s -> %s\n", #x, hipGetErrorString(e)); } while (0)
int main() {
  float* x; C(hipMalloc(&x, 1 << 24));
  hipStream_t s; C(hipStreamCreateWithFlags(&s, hipStreamNonBlocking));
  hipEvent_t a, b, p0, p1; C(hipEventCreate(&a)); C(hipEventCreate(&b)); C(hipEventCreate(&p0)); C(hipEventCreate(&p1));
  for (int it : {200, 2000, 20000}) {
    for (int r = 0; r < 3; ++r) {
      C(hipEventRecord(p0, s));
      hipExtLaunchKernelGGL(spin, dim3(4096), dim3(256), 0, s, a, b, 0, x, 1 << 20, it);
      C(hipEventRecord(p1, s));
      C(hipStreamSynchronize(s));
      float ms = -1, mp = -1; C(hipEventElapsedTime(&ms, a, b)); C(hipEventElapsedTime(&mp, p0, p1));
      printf("eager it=%d: ext %.4f ms, plain pair %.4f ms\n", it, ms, mp);
    }
  }
  // under capture: 3 kernels, the middle one with ext events
  hipGraph_t g; hipGraphExec_t ge;
  C(hipStreamBeginCapture(s, hipStreamCaptureModeGlobal));
  hipLaunchKernelGGL(spin, dim3(4096), dim3(256), 0, s, x, 1 << 20, 2000);
  hipExtLaunchKernelGGL(spin, dim3(4096), dim3(256), 0, s, a, b, 0, x, 1 << 20, 2000);
  C(hipGetLastError());
  hipLaunchKernelGGL(spin, dim3(4096), dim3(256), 0, s, x, 1 << 20, 2000);
  hipError_t e = hipStreamEndCapture(s, &g);
  printf("capture end: %s\n", hipGetErrorString(e));
  if (e == hipSuccess) {
    size_t nn = 0; C(hipGraphGetNodes(g, nullptr, &nn)); printf("graph nodes: %zu\n", nn);
    C(hipGraphInstantiate(&ge, g, nullptr, nullptr, 0));
    for (int r = 0; r < 4; ++r) {
      C(hipEventRecord(p0, s));
      C(hipGraphLaunch(ge, s));
      C(hipEventRecord(p1, s));
      C(hipStreamSynchronize(s));
      float ms = -1, mp = -1;
      hipError_t q = hipEventElapsedTime(&ms, a, b);
      C(hipEventElapsedTime(&mp, p0, p1));
      printf("graph replay %d: ext %.4f ms (%s), whole graph %.4f ms\n", r, ms, hipGetErrorString(q), mp);
    }
  }
  C(hipGetLastError());
  return 0;
}
