// Fused attention core for short sequences (T <= 64) and narrow queries (C/8 <= 64): the
// decoders' SelfAttention(256) at T = 64 (model_layers.py:121-146):
//     S = Q^T K  (no 1/sqrt(d) scaling, :140),  A = softmax_j(S),
//     y[c][i] = gamma * sum_j V[c][j] A[i][j] + x[c][i] (+ res[c][i])
// One workgroup per (clip, 64-channel chunk of V): the 64 x 64 score tile is recomputed per
// chunk (K = C/8 <= 64, a few MFMAs) instead of making a round trip through HBM, the softmax
// runs on the LDS tile, and the PV product + epilogue follow without leaving the workgroup.
// The normalised attention matrix is also written out when the backward pass needs it.
// Replaces three launches (score GEMM, softmax, PV GEMM) of the general path.
#include "a2m_internal.h"

namespace a2m {

typedef float floatx16 __attribute__((ext_vector_type(16)));

constexpr int AT = 64;        // max sequence length / tile edge
constexpr int AP = AT + 4;    // LDS pitch: conflict-free ds_read_b128 rows
constexpr int ACH = 64;       // output channels per workgroup

__global__ __launch_bounds__(256) void attn_core_kernel(const float* __restrict__ qkv, int64_t qs_b,
                                                        int C, int T, const float* __restrict__ gamma,
                                                        const float* __restrict__ x, int64_t x_bs,
                                                        const float* __restrict__ res,
                                                        float* __restrict__ y,
                                                        float* __restrict__ attn_out) {
  __shared__ __attribute__((aligned(16))) float qs[AT * AP];   // Q^T: [i][c]  (c < Cq <= 64)
  __shared__ __attribute__((aligned(16))) float ks[AT * AP];   // K^T: [j][c]
  __shared__ __attribute__((aligned(16))) float ss[AT * AP];   // scores / attention [i][j]
  __shared__ __attribute__((aligned(16))) float vs[ACH * AP];  // V chunk [c][j]
  const int b = blockIdx.y, c0 = blockIdx.x * ACH;
  const int Cq = C / 8;
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int li = lane & 31, lh = lane >> 5;
  const int wm = wave >> 1, wn = wave & 1;
  const float* q = qkv + (int64_t)b * qs_b;
  const float* k = q + (int64_t)Cq * T;
  const float* v = q + (int64_t)2 * Cq * T + (int64_t)c0 * T;

  // stage Q^T, K^T (transposed on the way in: source rows are channels, t contiguous) and V
  {  // every global load of this thread issued before the LDS writes
    constexpr int NE = AT * AT / 256;
    float qv[NE], kv[NE], vv[NE];
#pragma unroll
    for (int j = 0; j < NE; ++j) {
      const int e = tid + j * 256, c = e / AT, t = e % AT;
      const bool ok = c < Cq && t < T;
      qv[j] = ok ? q[(int64_t)c * T + t] : 0.f;
      kv[j] = ok ? k[(int64_t)c * T + t] : 0.f;
      vv[j] = (c0 + c < C && t < T) ? v[(int64_t)c * T + t] : 0.f;
    }
#pragma unroll
    for (int j = 0; j < NE; ++j) {
      const int e = tid + j * 256, c = e / AT, t = e % AT;
      qs[t * AP + c] = qv[j];
      ks[t * AP + c] = kv[j];
      vs[c * AP + t] = vv[j];
    }
  }
  __syncthreads();

  // S[i][j] = sum_c Q^T[i][c] K^T[j][c]: wave (wm, wn) owns the 32 x 32 tile (wm, wn)
  floatx16 acc;
#pragma unroll
  for (int r = 0; r < 16; ++r) acc[r] = 0.f;
  {
    const int ia = wm * 32 + li, jb = wn * 32 + li;
    for (int kc = 0; kc < Cq; kc += 16) {
      const float4 a0 = *reinterpret_cast<const float4*>(qs + ia * AP + kc + lh * 8);
      const float4 a1 = *reinterpret_cast<const float4*>(qs + ia * AP + kc + lh * 8 + 4);
      const float4 b0 = *reinterpret_cast<const float4*>(ks + jb * AP + kc + lh * 8);
      const float4 b1 = *reinterpret_cast<const float4*>(ks + jb * AP + kc + lh * 8 + 4);
      const float af[8] = {a0.x, a0.y, a0.z, a0.w, a1.x, a1.y, a1.z, a1.w};
      const float bf[8] = {b0.x, b0.y, b0.z, b0.w, b1.x, b1.y, b1.z, b1.w};
#pragma unroll
      for (int s = 0; s < 8; ++s) acc = __builtin_amdgcn_mfma_f32_32x32x2f32(af[s], bf[s], acc, 0, 0, 0);
    }
  }
#pragma unroll
  for (int r = 0; r < 16; ++r) {
    const int i = wm * 32 + (r & 3) + 8 * (r >> 2) + 4 * lh;
    ss[i * AP + wn * 32 + li] = acc[r];
  }
  __syncthreads();

  // row softmax over j < T: four lanes per row (16 columns each), quad reductions in DPP
  {
    const int i = tid >> 2, part = tid & 3;
    float* rowp = ss + i * AP + part * 16;
    float e[16];
    float mx = -INFINITY;
#pragma unroll
    for (int q4 = 0; q4 < 4; ++q4) {
      const float4 v4 = *reinterpret_cast<const float4*>(rowp + 4 * q4);
      e[4 * q4] = v4.x; e[4 * q4 + 1] = v4.y; e[4 * q4 + 2] = v4.z; e[4 * q4 + 3] = v4.w;
    }
#pragma unroll
    for (int q = 0; q < 16; ++q) {
      if (part * 16 + q >= T) e[q] = -INFINITY;
      mx = fmaxf(mx, e[q]);
    }
    mx = quad_max(mx);
    float sum = 0.f;
#pragma unroll
    for (int q = 0; q < 16; ++q) {
      e[q] = part * 16 + q < T ? expf(e[q] - mx) : 0.f;
      sum += e[q];
    }
    sum = quad_sum(sum);
    const float inv = 1.f / sum;
#pragma unroll
    for (int q = 0; q < 16; ++q) e[q] = i < T ? e[q] * inv : 0.f;
#pragma unroll
    for (int q4 = 0; q4 < 4; ++q4)
      *reinterpret_cast<float4*>(rowp + 4 * q4) = make_float4(e[4 * q4], e[4 * q4 + 1], e[4 * q4 + 2], e[4 * q4 + 3]);
    if (attn_out && blockIdx.x == 0 && i < T) {
      float* ar = attn_out + ((int64_t)b * T + i) * T;
#pragma unroll
      for (int q = 0; q < 16; ++q)
        if (part * 16 + q < T) ar[part * 16 + q] = e[q];
    }
  }
  __syncthreads();

  // out[c][i] = sum_j V[c][j] A[i][j]: wave (wm, wn) owns channels 32wm.., queries 32wn..
#pragma unroll
  for (int r = 0; r < 16; ++r) acc[r] = 0.f;
  {
    const int ca = wm * 32 + li, ib = wn * 32 + li;
    for (int kc = 0; kc < AT; kc += 16) {
      const float4 a0 = *reinterpret_cast<const float4*>(vs + ca * AP + kc + lh * 8);
      const float4 a1 = *reinterpret_cast<const float4*>(vs + ca * AP + kc + lh * 8 + 4);
      const float4 b0 = *reinterpret_cast<const float4*>(ss + ib * AP + kc + lh * 8);
      const float4 b1 = *reinterpret_cast<const float4*>(ss + ib * AP + kc + lh * 8 + 4);
      const float af[8] = {a0.x, a0.y, a0.z, a0.w, a1.x, a1.y, a1.z, a1.w};
      const float bf[8] = {b0.x, b0.y, b0.z, b0.w, b1.x, b1.y, b1.z, b1.w};
#pragma unroll
      for (int s = 0; s < 8; ++s) acc = __builtin_amdgcn_mfma_f32_32x32x2f32(af[s], bf[s], acc, 0, 0, 0);
    }
  }
  const float g = gamma[0];
  const int i = wn * 32 + li;
  if (i < T) {
#pragma unroll
    for (int r = 0; r < 16; ++r) {
      const int c = c0 + wm * 32 + (r & 3) + 8 * (r >> 2) + 4 * lh;
      if (c >= C) continue;
      const int64_t o = (int64_t)b * x_bs + (int64_t)c * T + i;
      float val = g * acc[r] + x[o];
      if (res) val += res[o];
      y[o] = val;
    }
  }
}

bool attn_core_fits(int C, int T) { return T <= AT && C % 8 == 0 && C / 8 <= AT && (C / 8) % 16 == 0; }

int attn_core(const float* qkv, int64_t qs_b, int B, int C, int T, const float* gamma,
              const float* x, int64_t x_bs, const float* res, float* y, float* attn_out,
              hipStream_t st) {
  dim3 grid((unsigned)cdiv(C, ACH), (unsigned)B);
  hipLaunchKernelGGL(attn_core_kernel, grid, dim3(256), 0, st, qkv, qs_b, C, T, gamma, x, x_bs, res,
                     y, attn_out);
  A2M_LAUNCH_CHECK();
  return A2M_OK;
}

}  // namespace a2m
