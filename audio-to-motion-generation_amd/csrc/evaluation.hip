// Pose normalisation and the PCK metric, on device so the training
// and inference loops never bring poses back to the host:
//   moments      normalization_tools.py:7-45 (one batch's mean and mean-of-squares, neck-
//                subtracted or plain; the host averages batches as the reference does)
//   normalize    version5_model_train.py:298-304: ((x - neck) - mean) / std, planar [2][52]
//   denormalize  generate_motion_video.py:259-260: x * std + mean (separate roundings, as torch)
//   pck          motion_evaluation.py:4-22 / pose_video/evaluation.py:4-21
//   windows      dataUtils.py:585-665 (PATS sample windows gathered from HBM-resident sequences)
// All bandwidth-trivial element work; the moments pass is a fixed-order fp64 reduction.
#include "a2m_internal.h"

namespace a2m {

constexpr int PF = 104, PJ = 52;

// One 1024-thread workgroup: feature f = tid % 128 (< 104), frame group g = tid / 128 sums
// frames g, g+8, ... in fp64; the 8 partials are combined in a fixed order.
__global__ __launch_bounds__(1024) void pose_moments_kernel(const float* __restrict__ pose,
                                                            int64_t n_frames, int necksub,
                                                            double* __restrict__ acc) {
  __shared__ double r1[8][PF], r2[8][PF];
  const int f = threadIdx.x & 127, g = threadIdx.x >> 7;
  double s1 = 0.0, s2 = 0.0;
  if (f < PF) {
    const int neck = f < PJ ? 0 : PJ;
#pragma unroll 4
    for (int64_t t = g; t < n_frames; t += 8) {
      const float* fr = pose + t * PF;
      const double v = necksub ? (double)(fr[f] - fr[neck]) : (double)fr[f];
      s1 += v;
      s2 += v * v;
    }
    r1[g][f] = s1;
    r2[g][f] = s2;
  }
  __syncthreads();
  if (g == 0 && f < PF) {
    double a = 0.0, b = 0.0;
#pragma unroll
    for (int q = 0; q < 8; ++q) { a += r1[q][f]; b += r2[q][f]; }
    acc[f] += a / (double)n_frames;
    acc[PF + f] += b / (double)n_frames;
  }
}

__global__ void pose_normalize_kernel(const float* __restrict__ pose, int64_t n, const float* mean,
                                      const float* std_, float* __restrict__ out) {
  for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < n * PF;
       i += (int64_t)gridDim.x * blockDim.x) {
    const int64_t fr = i / PF;
    const int j = (int)(i - fr * PF);
    const float neck = pose[fr * PF + (j < PJ ? 0 : PJ)];
    const float c = __fsub_rn(pose[i], neck);
    out[i] = __fdiv_rn(__fsub_rn(c, mean[j]), std_[j]);
  }
}

__global__ void pose_denormalize_kernel(const float* __restrict__ pose, int64_t n, const float* mean,
                                        const float* std_, float* __restrict__ out) {
  for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < n * PF;
       i += (int64_t)gridDim.x * blockDim.x) {
    const int j = (int)(i % PF);
    out[i] = __fadd_rn(__fmul_rn(pose[i], std_[j]), mean[j]);
  }
}

// One wave per sample: extent of gt over the K keypoints (per axis), then per-keypoint
// Euclidean distances against alpha * max(extent_x, extent_y), fp64 on fp32 inputs.
__global__ __launch_bounds__(256) void pck_kernel(const float* __restrict__ pred,
                                                  const float* __restrict__ gt, int N, int K,
                                                  double alpha, double* __restrict__ out) {
  const int n = blockIdx.x * 4 + (threadIdx.x >> 6), lane = threadIdx.x & 63;
  if (n >= N) return;
  const float* g = gt + (int64_t)n * 2 * K;
  const float* p = pred + (int64_t)n * 2 * K;
  float xmax = -INFINITY, xmin = INFINITY, ymax = -INFINITY, ymin = INFINITY;
  for (int k = lane; k < K; k += 64) {
    xmax = fmaxf(xmax, g[k]); xmin = fminf(xmin, g[k]);
    ymax = fmaxf(ymax, g[K + k]); ymin = fminf(ymin, g[K + k]);
  }
  for (int o = 32; o > 0; o >>= 1) {
    xmax = fmaxf(xmax, __shfl_xor(xmax, o)); xmin = fminf(xmin, __shfl_xor(xmin, o));
    ymax = fmaxf(ymax, __shfl_xor(ymax, o)); ymin = fminf(ymin, __shfl_xor(ymin, o));
  }
  const double ext = fmax(fabs((double)xmax - (double)xmin), fabs((double)ymax - (double)ymin));
  const double radius = ext * alpha;
  int hits = 0;
  for (int k = lane; k < K; k += 64) {
    const double dx = (double)g[k] - (double)p[k], dy = (double)g[K + k] - (double)p[K + k];
    hits += sqrt(dx * dx + dy * dy) <= radius;
  }
  for (int o = 32; o > 0; o >>= 1) hits += __shfl_xor(hits, o);
  if (lane == 0) out[n] = (double)hits / (double)K;
}

}  // namespace a2m

using namespace a2m;

extern "C" {

int a2m_pose_moments_f32(const float* pose, int64_t n_frames, int32_t necksub, double* acc,
                         void* stream) {
  A2M_CHECK_ARG(pose && acc && n_frames > 0, "pose_moments: bad args");
  hipLaunchKernelGGL(pose_moments_kernel, dim3(1), dim3(1024), 0, as_stream(stream), pose, n_frames,
                     necksub, acc);
  A2M_LAUNCH_CHECK();
  return A2M_OK;
}

int a2m_pose_normalize_f32(const float* pose, int64_t n_frames, const float* mean, const float* std_,
                           float* out, void* stream) {
  A2M_CHECK_ARG(pose && mean && std_ && out && n_frames >= 0, "pose_normalize: bad args");
  if (n_frames == 0) return A2M_OK;
  const int blocks = (int)std::min<int64_t>(cdiv(n_frames * PF, 256), 4096);
  hipLaunchKernelGGL(pose_normalize_kernel, dim3(blocks), dim3(256), 0, as_stream(stream), pose,
                     n_frames, mean, std_, out);
  A2M_LAUNCH_CHECK();
  return A2M_OK;
}

int a2m_pose_denormalize_f32(const float* pose, int64_t n_frames, const float* mean,
                             const float* std_, float* out, void* stream) {
  A2M_CHECK_ARG(pose && mean && std_ && out && n_frames >= 0, "pose_denormalize: bad args");
  if (n_frames == 0) return A2M_OK;
  const int blocks = (int)std::min<int64_t>(cdiv(n_frames * PF, 256), 4096);
  hipLaunchKernelGGL(pose_denormalize_kernel, dim3(blocks), dim3(256), 0, as_stream(stream), pose,
                     n_frames, mean, std_, out);
  A2M_LAUNCH_CHECK();
  return A2M_OK;
}

int a2m_pck_f32(const float* pred, const float* gt, int32_t N, int32_t K, double alpha,
                double* out, void* stream) {
  A2M_CHECK_ARG(pred && gt && out && N >= 0 && K > 0, "pck: bad args");
  if (N == 0) return A2M_OK;
  hipLaunchKernelGGL(pck_kernel, dim3((unsigned)cdiv(N, 4)), dim3(256), 0, as_stream(stream), pred, gt,
                     N, K, alpha, out);
  A2M_LAUNCH_CHECK();
  return A2M_OK;
}

}  // extern "C"

// ---------------------------------------------------------------------------- windowing
// PATS sample windows (dataUtils.py:585-624, :646-665): out[w][j][c] = data[starts[w] +
// j*interval][c] for j < ceil(window / interval), optionally standardised as (x - mean[c]) /
// (std[c] < 1e-7 ? 1 : std[c]) -- the loader's cached normalisation (:656-662).
namespace a2m {
__global__ void window_gather_kernel(const float* __restrict__ data, int C, const int64_t* starts,
                                     int nw, int nj, int interval, const float* mean,
                                     const float* std_, float* __restrict__ out) {
  const int64_t total = (int64_t)nw * nj * C;
  for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < total;
       i += (int64_t)gridDim.x * blockDim.x) {
    const int c = (int)(i % C);
    const int64_t wj = i / C;
    const int j = (int)(wj % nj), w = (int)(wj / nj);
    float v = data[(starts[w] + (int64_t)j * interval) * C + c];
    if (mean) {
      const float s = std_[c] < 1e-7f ? 1.f : std_[c];
      v = __fdiv_rn(__fsub_rn(v, mean[c]), s);
    }
    out[i] = v;
  }
}
}  // namespace a2m

extern "C" int a2m_window_gather_f32(const float* data, int64_t length, int32_t C,
                                     const int64_t* starts, int32_t n_windows, int32_t window,
                                     int32_t interval, const float* mean, const float* std_,
                                     float* out, void* stream) {
  A2M_CHECK_ARG(data && starts && out && C > 0 && n_windows >= 0 && window > 0 && interval > 0 &&
                    (mean == nullptr) == (std_ == nullptr),
                "window_gather: bad args");
  (void)length;  // the host computed starts < length - window (dataUtils.py:611-618)
  if (n_windows == 0) return A2M_OK;
  const int nj = (window + interval - 1) / interval;
  const int64_t total = (int64_t)n_windows * nj * C;
  const int blocks = (int)std::min<int64_t>(cdiv(total, 256), 4096);
  hipLaunchKernelGGL(window_gather_kernel, dim3(blocks), dim3(256), 0, as_stream(stream), data, C, starts,
                     n_windows, nj, interval, mean, std_, out);
  A2M_LAUNCH_CHECK();
  return A2M_OK;
}
