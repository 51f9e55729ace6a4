// Generator pose losses (real_motion_model.py:307-461) on interleaved (x, y) poses.
//   bone  = MSE over (b, bone) of mean_T ||p[child] - p[parent]||  (gen vs real), 51 bones
//   angle = 0.7 * mean relu(-a) + relu(a - pi)  over 30 hand triples (:350-392)
//         + 0.3 * mean relu(-pi/2 - a) + relu(a - pi) over 5 body triples (:394-447)
//   a = atan2(cross(u, v), dot(u, v)), u = p[j] - p[p], v = p[c] - p[j]
// Two deterministic passes: per-(clip, 16-frame chunk) partial sums, then a single workgroup
// reduction in a fixed order.
#include "a2m_internal.h"

namespace a2m {

// Skeleton2D.parents (pats/data_loading/skeleton.py:94-110)
__constant__ int kParents[52] = {-1, 0, 1, 2, 0, 4, 5, 0, 7, 7, 6,
                                 10, 11, 12, 13, 10, 15, 16, 17, 10, 19, 20, 21, 10, 23, 24, 25,
                                 10, 27, 28, 29, 3, 31, 32, 33, 34, 31, 36, 37, 38, 31, 40, 41,
                                 42, 31, 44, 45, 46, 31, 48, 49, 50};
// Triples produced by _initialize_hand_triples / _initialize_body_triples
// (real_motion_model.py:280-304): (parent, joint, first child) along every chain.
// hand indices are relative to joint 10.
__constant__ int kHandTriples[30][3] = {
    {0, 1, 2}, {1, 2, 3}, {2, 3, 4}, {0, 5, 6}, {5, 6, 7}, {6, 7, 8}, {0, 9, 10}, {9, 10, 11},
    {10, 11, 12}, {0, 13, 14}, {13, 14, 15}, {14, 15, 16}, {0, 17, 18}, {17, 18, 19}, {18, 19, 20},
    {21, 22, 23}, {22, 23, 24}, {23, 24, 25}, {21, 26, 27}, {26, 27, 28}, {27, 28, 29},
    {21, 30, 31}, {30, 31, 32}, {31, 32, 33}, {21, 34, 35}, {34, 35, 36}, {35, 36, 37},
    {21, 38, 39}, {38, 39, 40}, {39, 40, 41}};
__constant__ int kBodyTriples[5][3] = {{0, 1, 2}, {1, 2, 3}, {0, 4, 5}, {4, 5, 6}, {0, 7, 8}};

constexpr int kBones = 51;
constexpr int kPart = 2 * kBones + 2;  // per-clip partials

__device__ __forceinline__ float block_sum(float v, float* red) {
  for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o);
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  __syncthreads();
  if (lane == 0) red[w] = v;
  __syncthreads();
  float s = 0.f;
  if (threadIdx.x == 0)
    for (int i = 0; i < (int)(blockDim.x >> 6); ++i) s += red[i];
  return s;  // valid on thread 0
}

__device__ __forceinline__ float signed_angle(const float* p, int a, int j, int c) {
  const float ux = p[2 * j] - p[2 * a], uy = p[2 * j + 1] - p[2 * a + 1];
  const float vx = p[2 * c] - p[2 * j], vy = p[2 * c + 1] - p[2 * j + 1];
  return atan2f(ux * vy - uy * vx, ux * vx + uy * vy);
}

// One workgroup per (clip, 16-frame chunk): the chunk's poses are staged in LDS with coalesced
// loads, then the 35 joint angles of each frame and the 2 x 51 bone-length partial sums read LDS.
// (One workgroup per clip walking all T * 35 angles was latency-bound: 15 us at B = 64, T = 64.)
constexpr int kTCh = 16;

__global__ __launch_bounds__(256) void pose_loss_partial_kernel(const float* gen, int64_t gs_b,
                                                                int64_t gs_t, const float* real,
                                                                int64_t rs_b, int64_t rs_t, int T,
                                                                float* part) {
  __shared__ float red[4];
  __shared__ float sg[kTCh][104];
  __shared__ float sr[kTCh][104];
  const int b = blockIdx.x, c = blockIdx.y, nch = gridDim.y;
  const int t0 = c * kTCh, tn = min(kTCh, T - t0);
  float* pb = part + ((int64_t)b * nch + c) * kPart;
  for (int i = threadIdx.x; i < tn * 104; i += blockDim.x) {
    const int t = i / 104, f = i % 104;
    sg[t][f] = gen[b * gs_b + (int64_t)(t0 + t) * gs_t + f];
    if (real != nullptr) sr[t][f] = real[b * rs_b + (int64_t)(t0 + t) * rs_t + f];
  }
  __syncthreads();
  // bone-length sums over the chunk's frames, one thread per (bone, pose) series in frame order;
  // without a real pose the bone loss is 0 and the generated lengths are not needed (inference)
  if (real != nullptr && threadIdx.x < 2 * kBones) {
    const int i = threadIdx.x;
    const int jb = (i % kBones) + 1, pj = kParents[jb];
    float s = 0.f;
    for (int t = 0; t < tn; ++t) {
      const float* p = i >= kBones ? sr[t] : sg[t];
      const float dx = p[2 * jb] - p[2 * pj], dy = p[2 * jb + 1] - p[2 * pj + 1];
      s += sqrtf(dx * dx + dy * dy);
    }
    pb[i] = s;
  }
  float hs = 0.f, bs = 0.f;
  for (int i = threadIdx.x; i < tn * 35; i += blockDim.x) {
    const int t = i / 35, q = i % 35;
    if (q < 30) {
      const float a = signed_angle(sg[t] + 20, kHandTriples[q][0], kHandTriples[q][1], kHandTriples[q][2]);
      hs += fmaxf(0.f - a, 0.f) + fmaxf(a - 3.14159265358979f, 0.f);
    } else {
      const int r = q - 30;
      const float a = signed_angle(sg[t], kBodyTriples[r][0], kBodyTriples[r][1], kBodyTriples[r][2]);
      bs += fmaxf(-1.57079632679490f - a, 0.f) + fmaxf(a - 3.14159265358979f, 0.f);
    }
  }
  const float H = block_sum(hs, red);
  const float Bsum = block_sum(bs, red);
  if (threadIdx.x == 0) {
    pb[2 * kBones] = H;
    pb[2 * kBones + 1] = Bsum;
  }
}

// Fixed-order reduction of the (clip, chunk) partials: bone means per clip = chunk sums / T.
__global__ __launch_bounds__(256) void pose_loss_final_kernel(const float* part, int B, int nch,
                                                              int T, int has_real, float hand_w,
                                                              float body_w, float* out) {
  __shared__ float red[4];
  float bone = 0.f, hs = 0.f, bs = 0.f;
  for (int i = threadIdx.x; has_real && i < B * kBones; i += blockDim.x) {
    const float* pb = part + (int64_t)(i / kBones) * nch * kPart;
    const int k = i % kBones;
    float g = 0.f, r = 0.f;
    for (int c = 0; c < nch; ++c) {
      g += pb[c * kPart + k];
      r += pb[c * kPart + kBones + k];
    }
    const float d = g / (float)T - r / (float)T;
    bone += d * d;
  }
  for (int i = threadIdx.x; i < B * nch; i += blockDim.x) {
    hs += part[(int64_t)i * kPart + 2 * kBones];
    bs += part[(int64_t)i * kPart + 2 * kBones + 1];
  }
  const float Bn = block_sum(bone, red);
  const float Hs = block_sum(hs, red);
  const float Bs = block_sum(bs, red);
  if (threadIdx.x == 0) {
    out[0] = has_real ? Bn / (float)(B * kBones) : 0.f;
    out[1] = hand_w * (Hs / (float)(B * T * 30)) + body_w * (Bs / (float)(B * T * 5));
  }
}

}  // namespace a2m

using namespace a2m;

extern "C" int a2m_pose_losses_w_f32(const float* gen, int64_t gs_b, int64_t gs_t, const float* real,
                                     int64_t rs_b, int64_t rs_t, int32_t B, int32_t T, float hand_w,
                                     float body_w, float* out, void* ws, size_t ws_bytes,
                                     void* stream) {
  A2M_CHECK_ARG(gen && out && B > 0 && T > 0, "pose_losses: bad args");
  const int nch = (T + kTCh - 1) / kTCh;
  const size_t need = sizeof(float) * (size_t)B * nch * kPart;
  if (!ws || ws_bytes < need) {
    set_error("pose_losses: workspace too small (%zu < %zu)", ws_bytes, need);
    return A2M_EWS;
  }
  float* part = static_cast<float*>(ws);
  hipStream_t st = as_stream(stream);
  hipLaunchKernelGGL(pose_loss_partial_kernel, dim3(B, nch), dim3(256), 0, st, gen, gs_b, gs_t,
                     real, rs_b, rs_t, T, part);
  A2M_LAUNCH_CHECK();
  hipLaunchKernelGGL(pose_loss_final_kernel, dim3(1), dim3(256), 0, st, part, B, nch, T,
                     real != nullptr ? 1 : 0, hand_w, body_w, out);
  A2M_LAUNCH_CHECK();
  return A2M_OK;
}

extern "C" int a2m_pose_losses_f32(const float* gen, int64_t gs_b, int64_t gs_t, const float* real,
                                   int64_t rs_b, int64_t rs_t, int32_t B, int32_t T, float* out,
                                   void* ws, size_t ws_bytes, void* stream) {
  return a2m_pose_losses_w_f32(gen, gs_b, gs_t, real, rs_b, rs_t, B, T, 0.7f, 0.3f, out, ws,
                               ws_bytes, stream);
}
