// Probe: can HIP event records be captured into a graph as timing event nodes
// (hipEventRecordWithFlags(..., hipEventRecordExternal)) and timed after each replay?
#include <hip/hip_runtime.h>
#include <cstdio>
__global__ void spin(float* x, int n) {
  int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i < n) { float v = x[i]; for (int k = 0; k < 2000; ++k) v = v * 1.0001f + 0.5f; x[i] = v; }
}
#define C(x) do { hipError_t e = (x); printf("%-60s -> %s\n", #x, hipGetErrorString(e)); } while (0)
int main() {
  float* x; C(hipMalloc(&x, 1 << 22));
  hipStream_t s; C(hipStreamCreate(&s));
  for (unsigned fl : {0u, (unsigned)hipEventDisableTiming}) {
    hipEvent_t a, b; C(hipEventCreateWithFlags(&a, fl)); C(hipEventCreateWithFlags(&b, fl));
    hipGraph_t g; hipGraphExec_t ge;
    C(hipStreamBeginCapture(s, hipStreamCaptureModeGlobal));
    C(hipEventRecordWithFlags(a, s, hipEventRecordExternal));
    hipLaunchKernelGGL(spin, dim3(4096), dim3(256), 0, s, x, 1 << 20);
    C(hipGetLastError());
    C(hipEventRecordWithFlags(b, s, hipEventRecordExternal));
    C(hipStreamEndCapture(s, &g));
    C(hipGraphInstantiate(&ge, g, nullptr, nullptr, 0));
    for (int r = 0; r < 3; ++r) {
      C(hipGraphLaunch(ge, s)); C(hipStreamSynchronize(s));
      float ms = -1; C(hipEventElapsedTime(&ms, a, b)); printf("flags %u replay %d: %.4f ms\n", fl, r, ms);
    }
  }
  // plain (non-external) record during capture, timing event
  hipEvent_t a, b; C(hipEventCreate(&a)); C(hipEventCreate(&b));
  hipGraph_t g; hipGraphExec_t ge;
  C(hipStreamBeginCapture(s, hipStreamCaptureModeGlobal));
  C(hipEventRecord(a, s));
  hipLaunchKernelGGL(spin, dim3(4096), dim3(256), 0, s, x, 1 << 20);
  C(hipEventRecord(b, s));
  C(hipStreamEndCapture(s, &g));
  C(hipGraphInstantiate(&ge, g, nullptr, nullptr, 0));
  C(hipGraphLaunch(ge, s)); C(hipStreamSynchronize(s));
  float ms = -1; C(hipEventElapsedTime(&ms, a, b)); printf("plain: %.4f ms\n", ms);
  {  // event creation and stream query during a global-mode capture
    hipGraph_t g2; hipEvent_t c;
    hipStreamCaptureStatus cs;
    C(hipStreamBeginCapture(s, hipStreamCaptureModeGlobal));
    C(hipStreamIsCapturing(s, &cs));
    printf("capturing status %d\n", (int)cs);
    C(hipEventCreate(&c));
    C(hipEventRecordWithFlags(c, s, hipEventRecordExternal));
    hipLaunchKernelGGL(spin, dim3(4096), dim3(256), 0, s, x, 1 << 20);
    C(hipStreamEndCapture(s, &g2));
    C(hipGetLastError());
  }
  {  // same in relaxed mode
    hipGraph_t g2; hipEvent_t c;
    C(hipStreamBeginCapture(s, hipStreamCaptureModeRelaxed));
    C(hipEventCreate(&c));
    C(hipEventRecordWithFlags(c, s, hipEventRecordExternal));
    C(hipStreamEndCapture(s, &g2));
    C(hipGetLastError());
  }
  {  // capture-info queries after an external record
    hipGraph_t g2; hipEvent_t c; C(hipEventCreate(&c));
    hipStreamCaptureStatus cs; unsigned long long id;
    const hipGraphNode_t* deps; size_t nd = 0; hipGraph_t cg;
    C(hipStreamBeginCapture(s, hipStreamCaptureModeGlobal));
    C(hipStreamGetCaptureInfo(s, &cs, &id));
    C(hipStreamGetCaptureInfo_v2(s, &cs, &id, &cg, &deps, &nd)); printf("nd=%zu\n", nd);
    C(hipEventRecordWithFlags(c, s, hipEventRecordExternal));
    C(hipStreamGetCaptureInfo(s, &cs, &id));
    C(hipStreamGetCaptureInfo_v2(s, &cs, &id, &cg, &deps, &nd)); printf("nd=%zu\n", nd);
    hipLaunchKernelGGL(spin, dim3(4096), dim3(256), 0, s, x, 1 << 20);
    C(hipStreamGetCaptureInfo_v2(s, &cs, &id, &cg, &deps, &nd)); printf("nd=%zu\n", nd);
    C(hipEventRecordWithFlags(c, s, hipEventRecordExternal));
    C(hipStreamGetCaptureInfo_v2(s, &cs, &id, &cg, &deps, &nd)); printf("nd=%zu\n", nd);
    void* p = nullptr;
    C(hipMallocAsync(&p, 4096, s));
    C(hipStreamEndCapture(s, &g2));
  }
  {  // torch-like streams: non-blocking with priority; the three capture modes
    for (int mode = 0; mode < 3; ++mode)
      for (int nb = 0; nb < 2; ++nb) {
        hipStream_t s2;
        if (nb) C(hipStreamCreateWithPriority(&s2, hipStreamNonBlocking, 0)); else C(hipStreamCreate(&s2));
        hipEvent_t c; C(hipEventCreate(&c));
        hipGraph_t g2;
        C(hipStreamBeginCapture(s2, (hipStreamCaptureMode)mode));
        hipLaunchKernelGGL(spin, dim3(4096), dim3(256), 0, s2, x, 1 << 20);
        hipError_t r = hipEventRecordWithFlags(c, s2, hipEventRecordExternal);
        printf("mode %d nonblocking %d: external record -> %s\n", mode, nb, hipGetErrorString(r));
        C(hipStreamEndCapture(s2, &g2));
        (void)hipGetLastError();
      }
  }
  return 0;
}
