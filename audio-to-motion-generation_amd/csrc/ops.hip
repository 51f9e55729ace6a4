// Convolution / linear / attention / normalisation entry points of the C-ABI.
// The GEMM-shaped work goes through the implicit-GEMM MFMA engine (gemm.hip); the small
// row-wise reductions (softmax, LayerNorm, channel pooling) are wave64 kernels here.
#include <algorithm>
#include <cstring>

#include <cstdlib>

#include "a2m_internal.h"

namespace a2m {

static Epilogue epi_bn(float* y, const float* bias, const float* bn_w, const float* bn_b,
                       const float* bn_rm, const float* bn_rv, float eps, int act, float slope) {
  Epilogue e = epi_dense(y, 0);
  e.bias = bias;
  if (bn_w) { e.bn_w = bn_w; e.bn_b = bn_b; e.bn_rm = bn_rm; e.bn_rv = bn_rv; e.bn_eps = eps; }
  e.act = act;
  e.slope = slope;
  return e;
}

static bool fits32(int64_t v) { return v >= 0 && v < (1LL << 31); }

// ---------------------------------------------------------------------------- softmax
// In-place row softmax, one wave64 per row (max-subtracted, like torch.softmax).
__global__ __launch_bounds__(256) void softmax_rows_kernel(float* x, int rows, int n) {
  const int row = blockIdx.x * 4 + (threadIdx.x >> 6);
  const int lane = threadIdx.x & 63;
  if (row >= rows) return;
  float* p = x + (int64_t)row * n;
  float mx = -INFINITY;
  for (int j = lane; j < n; j += 64) mx = fmaxf(mx, p[j]);
  mx = wave64_max(mx);
  float s = 0.f;
  for (int j = lane; j < n; j += 64) {
    const float e = expf(p[j] - mx);
    p[j] = e;
    s += e;
  }
  s = wave64_sum(s);
  const float inv = 1.f / s;
  for (int j = lane; j < n; j += 64) p[j] *= inv;
}

// --------------------------------------------------------------------- time interpolation
// F.interpolate(size=(T,1), mode='bilinear', align_corners=False): source index
// max(0, scale*(dst+0.5)-0.5), scale = in/out computed in fp32 (ATen's
// area_pixel_compute_source_index); zero-weight taps are skipped so never-computed
// (pruned) encoder columns are never read.
__device__ __forceinline__ float interp_time_at(const float* p, int H, int W, int w0, int w1, float lw0,
                                                float lw1, float sh, int t) {
  float src = sh * ((float)t + 0.5f) - 0.5f;
  src = src < 0.f ? 0.f : src;
  const int h0 = (int)src;
  const int h1 = h0 + (h0 < H - 1 ? 1 : 0);
  const float lh1 = src - (float)h0, lh0 = 1.f - lh1;
  auto row = [&](int h) {
    float v = lw0 * p[h * W + w0];
    if (lw1 != 0.f) v += lw1 * p[h * W + w1];
    return v;
  };
  float v = lh0 * row(h0);
  if (lh1 != 0.f) v += lh1 * row(h1);
  return v;
}

// vec: one thread per four consecutive t of a (b, c) row (host: T % 4 == 0, y 16-byte aligned,
// B*C*T < 2^31 for the 32-bit indexing): float4 stores; otherwise one output per thread with
// 64-bit indexing and no alignment requirement.
__global__ void interp_time_kernel(const float* x, int B, int C, int H, int W, float* y, int T, int vec) {
  const float sh = (float)H / (float)T;
  const float sw = (float)W / 1.0f;
  float srcw = sw * 0.5f - 0.5f;
  srcw = srcw < 0.f ? 0.f : srcw;
  const int w0 = (int)srcw;
  const int w1 = w0 + (w0 < W - 1 ? 1 : 0);
  const float lw1 = srcw - (float)w0, lw0 = 1.f - lw1;
  if (vec) {
    const int T4 = T >> 2;
    const int total4 = B * C * T4;
    for (int i = blockIdx.x * blockDim.x + threadIdx.x; i < total4; i += gridDim.x * blockDim.x) {
      const int bc = i / T4, t = (i - bc * T4) * 4;
      const float* p = x + (int64_t)bc * H * W;
      float4 v;
      v.x = interp_time_at(p, H, W, w0, w1, lw0, lw1, sh, t);
      v.y = interp_time_at(p, H, W, w0, w1, lw0, lw1, sh, t + 1);
      v.z = interp_time_at(p, H, W, w0, w1, lw0, lw1, sh, t + 2);
      v.w = interp_time_at(p, H, W, w0, w1, lw0, lw1, sh, t + 3);
      *reinterpret_cast<float4*>(y + (int64_t)i * 4) = v;
    }
    return;
  }
  const int64_t total = (int64_t)B * C * T;
  for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < total;
       i += (int64_t)gridDim.x * blockDim.x) {
    const int t = (int)(i % T);
    const int64_t bc = i / T;
    y[i] = interp_time_at(x + bc * H * W, H, W, w0, w1, lw0, lw1, sh, t);
  }
}

// ---------------------------------------------------------------------- channel attention
// Channel weights, one workgroup per batch element, every global load independent (no
// dependent chains): avg/max pooling one thread per channel over T, the shared MLP's first
// layer as 4-lane partial dot products over C, the second layer one thread per channel;
// att[b][c] = sigmoid(mlp(avg)) + sigmoid(mlp(max)).
__global__ __launch_bounds__(256) void channel_att_weights_kernel(const float* x, int C, int T,
                                                                  const float* w1, const float* b1,
                                                                  int Cr, const float* w2,
                                                                  const float* b2, float* att) {
  extern __shared__ __attribute__((aligned(16))) float sm[];
  float* pavg = sm;
  float* pmax = pavg + C;
  float* hid = pmax + C;  // [2][Cr]
  const int b = blockIdx.x;
  const float* xb = x + (int64_t)b * C * T;
  for (int c = threadIdx.x; c < C; c += blockDim.x) {
    const float* p = xb + (int64_t)c * T;
    float s = 0.f, mx = -INFINITY;
    if ((T & 3) == 0 && ((reinterpret_cast<uintptr_t>(p) & 15) == 0)) {
#pragma unroll 8
      for (int t = 0; t < T; t += 4) {
        const float4 v = *reinterpret_cast<const float4*>(p + t);
        s += v.x + v.y + v.z + v.w;
        mx = fmaxf(fmaxf(mx, fmaxf(v.x, v.y)), fmaxf(v.z, v.w));
      }
    } else {
      for (int t = 0; t < T; ++t) {
        s += p[t];
        mx = fmaxf(mx, p[t]);
      }
    }
    pavg[c] = s / (float)T;
    pmax[c] = mx;
  }
  __syncthreads();
  // layer 1: output j (2*Cr of them) by 4 consecutive lanes, each over a quarter of C
  for (int i = threadIdx.x; i < 8 * Cr; i += blockDim.x) {
    const int j = i >> 2, part = i & 3;
    const int r = j % Cr;
    const float* in = j < Cr ? pavg : pmax;
    const float* wr = w1 + (int64_t)r * C;
    float a = 0.f;
#pragma unroll 8
    for (int c = part; c < C; c += 4) a += wr[c] * in[c];
    a = quad_sum(a);
    if (part == 0) {
      a += b1[r];
      hid[j] = a > 0.f ? a : 0.f;
    }
  }
  __syncthreads();
  for (int c = threadIdx.x; c < C; c += blockDim.x) {
    const float* wr = w2 + (int64_t)c * Cr;
    float a0 = b2[c], a1 = b2[c];
#pragma unroll 8
    for (int r = 0; r < Cr; ++r) {
      const float w = wr[r];
      a0 += w * hid[r];
      a1 += w * hid[Cr + r];
    }
    att[(int64_t)b * C + c] = 1.f / (1.f + expf(-a0)) + 1.f / (1.f + expf(-a1));
  }
}

// The same with the scale fused, for C = 256, Cr = 32 and T = 64 (the model's shape): one
// workgroup per clip keeps the clip's x (64 KB) in registers -- wave w, step k holds rows
// 64w + 4k + (lane >> 4), 16 lanes a row, so every load and store instruction covers 1 KB of
// contiguous rows -- and stores y = x * att from registers without a second pass over x.  The
// MLP weights are loaded at the start alongside x (the layer-by-layer weight loads of the generic
// kernel were its latency chain): layer 1 by (r, eighth of C) threads and an 8-lane sum, layer 2
// one thread per channel.  Every x element is read before any y element of its clip is written
// (the barriers between), so y may alias x.
#ifndef A2M_CA_FUSED
#define A2M_CA_FUSED 1
#endif
__global__ __launch_bounds__(256) void channel_att_fused256_kernel(const float* x, const float* w1,
                                                                   const float* b1, const float* w2,
                                                                   const float* b2, float* att,
                                                                   float* y) {
  constexpr int C = 256, Cr = 32, T = 64, NK = 16;
  __shared__ __attribute__((aligned(16))) float pavg[C];
  __shared__ __attribute__((aligned(16))) float pmax[C];
  __shared__ float hid[2 * Cr];
  __shared__ float satt[C];
  const int b = blockIdx.x, tid = threadIdx.x;
  const int lane = tid & 63, w = tid >> 6, q = lane & 15, sub = lane >> 4;
  const int r = tid >> 3, part = tid & 7;
  float4 w1v[8], w2v[8], xv[NK];
#pragma unroll
  for (int k = 0; k < 8; ++k) {
    w1v[k] = reinterpret_cast<const float4*>(w1 + r * C)[part + 8 * k];
    w2v[k] = reinterpret_cast<const float4*>(w2 + tid * Cr)[k];
  }
  const float bias1 = b1[r], bias2 = b2[tid];
  const float4* xb = reinterpret_cast<const float4*>(x + (int64_t)b * C * T);
#pragma unroll
  for (int k = 0; k < NK; ++k) xv[k] = xb[(64 * w + 4 * k + sub) * (T / 4) + q];
#pragma unroll
  for (int k = 0; k < NK; ++k) {
    float s = xv[k].x + xv[k].y + xv[k].z + xv[k].w;
    float m = fmaxf(fmaxf(xv[k].x, xv[k].y), fmaxf(xv[k].z, xv[k].w));
    s = row16_sum(s);
    m = row16_max(m);
    if (q == 0) {
      pavg[64 * w + 4 * k + sub] = s / (float)T;
      pmax[64 * w + 4 * k + sub] = m;
    }
  }
  __syncthreads();
  float a0 = 0.f, a1 = 0.f;
#pragma unroll
  for (int k = 0; k < 8; ++k) {
    const float4 pa = reinterpret_cast<const float4*>(pavg)[part + 8 * k];
    const float4 pm = reinterpret_cast<const float4*>(pmax)[part + 8 * k];
    a0 += w1v[k].x * pa.x + w1v[k].y * pa.y + w1v[k].z * pa.z + w1v[k].w * pa.w;
    a1 += w1v[k].x * pm.x + w1v[k].y * pm.y + w1v[k].z * pm.z + w1v[k].w * pm.w;
  }
  // sum over the 8 lanes of r (lanes 8r'..8r'+7 of the wave): xor 1, 2 in the quad, then xor 4
  a0 = quad_sum(a0);
  a1 = quad_sum(a1);
  a0 += dpp_f<DPP_HALF_MIRROR>(a0);
  a1 += dpp_f<DPP_HALF_MIRROR>(a1);
  if (part == 0) {
    a0 += bias1;
    a1 += bias1;
    hid[r] = a0 > 0.f ? a0 : 0.f;
    hid[Cr + r] = a1 > 0.f ? a1 : 0.f;
  }
  __syncthreads();
  float o0 = bias2, o1 = bias2;
#pragma unroll
  for (int k = 0; k < 8; ++k) {
    o0 += w2v[k].x * hid[4 * k] + w2v[k].y * hid[4 * k + 1] + w2v[k].z * hid[4 * k + 2] +
          w2v[k].w * hid[4 * k + 3];
    o1 += w2v[k].x * hid[Cr + 4 * k] + w2v[k].y * hid[Cr + 4 * k + 1] +
          w2v[k].z * hid[Cr + 4 * k + 2] + w2v[k].w * hid[Cr + 4 * k + 3];
  }
  const float a = 1.f / (1.f + expf(-o0)) + 1.f / (1.f + expf(-o1));
  att[(int64_t)b * C + tid] = a;
  satt[tid] = a;
  __syncthreads();
  float4* yb = reinterpret_cast<float4*>(y + (int64_t)b * C * T);
#pragma unroll
  for (int k = 0; k < NK; ++k) {
    const int row = 64 * w + 4 * k + sub;
    const float ar = satt[row];
    float4 v = xv[k];
    v.x *= ar; v.y *= ar; v.z *= ar; v.w *= ar;
    yb[row * (T / 4) + q] = v;
  }
}

// y[b][c][t] = x[b][c][t] * att[b][c], float4 along T when T % 4 == 0.
__global__ void channel_scale_kernel(const float* x, const float* att, int T, int64_t n, float* y) {
  if ((T & 3) == 0) {
    const int64_t n4 = n >> 2;
    for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < n4;
         i += (int64_t)gridDim.x * blockDim.x) {
      const float a = att[(i << 2) / T];
      float4 v = reinterpret_cast<const float4*>(x)[i];
      v.x *= a; v.y *= a; v.z *= a; v.w *= a;
      reinterpret_cast<float4*>(y)[i] = v;
    }
  } else {
    for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < n;
         i += (int64_t)gridDim.x * blockDim.x)
      y[i] = x[i] * att[i / T];
  }
}

// ------------------------------------------------------------------------------ LayerNorm
// One wave per row, D <= 64*8.  Biased variance, eps inside the sqrt (torch.layer_norm).
__global__ __launch_bounds__(256) void layernorm_kernel(const float* x, int R, int D,
                                                        const float* w, const float* b, float eps,
                                                        float* y, int T, int64_t ys_b,
                                                        int64_t ys_d, int64_t ys_t, float* mean_out,
                                                        float* rstd_out) {
  const int row = blockIdx.x * 4 + (threadIdx.x >> 6);
  const int lane = threadIdx.x & 63;
  if (row >= R) return;
  const float* p = x + (int64_t)row * D;
  float v[8];
  float s = 0.f;
#pragma unroll
  for (int q = 0; q < 8; ++q) {
    const int d = lane + 64 * q;
    v[q] = d < D ? p[d] : 0.f;
    s += v[q];
  }
  s = wave64_sum(s);
  const float mean = s / (float)D;
  float ss = 0.f;
#pragma unroll
  for (int q = 0; q < 8; ++q) {
    const int d = lane + 64 * q;
    const float c = d < D ? v[q] - mean : 0.f;
    ss += c * c;
  }
  ss = wave64_sum(ss);
  const float rstd = 1.f / sqrtf(ss / (float)D + eps);
  float* yr = y + (int64_t)(row / T) * ys_b + (int64_t)(row % T) * ys_t;
#pragma unroll
  for (int q = 0; q < 8; ++q) {
    const int d = lane + 64 * q;
    if (d < D) yr[d * ys_d] = (v[q] - mean) * rstd * w[d] + b[d];
  }
  if (lane == 0) {
    if (mean_out) mean_out[row] = mean;
    if (rstd_out) rstd_out[row] = rstd;
  }
}

__global__ void mean_time_kernel(const float* x, int64_t xs_b, int64_t xs_c, int C, int T, int BC,
                                 float scale, float* y) {
  const int i = blockIdx.x * 4 + (threadIdx.x >> 6);
  const int lane = threadIdx.x & 63;
  if (i >= BC) return;
  const float* p = x + (int64_t)(i / C) * xs_b + (int64_t)(i % C) * xs_c;
  float s = 0.f;
  for (int t = lane; t < T; t += 64) s += p[t];
  s = wave64_sum(s);
  if (lane == 0) y[i] = scale * (s / (float)T);
}

__global__ void repeat_time_kernel(const float* x, int C, int T, int64_t total, float scale,
                                   float* y, int64_t ys_b, int64_t ys_c) {
  for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < total;
       i += (int64_t)gridDim.x * blockDim.x) {
    const int t = (int)(i % T);
    const int64_t bc = i / T;
    y[(bc / C) * ys_b + (bc % C) * ys_c + t] = scale * x[bc];
  }
}

// ConvTranspose1d weight [Ci][Co][ks] -> per output phase r: P_r[co][tap*Ci + ci] (see
// a2m_convt1d_fwd_f32).  Phase of tap kk: r = (kk - pad) mod s; phases stored in order.
__device__ __forceinline__ int phase_taps(int r, int ks, int s, int pad, int* kk0) {
  int n = 0;
  *kk0 = -1;
  for (int kk = 0; kk < ks; ++kk)
    if ((((r + pad - kk) % s) + s) % s == 0) { if (*kk0 < 0) *kk0 = kk; ++n; }
  return n;
}

__global__ void convt_pack_kernel(const float* w, int Ci, int Co, int ks, int s, int pad, float* out) {
  const int64_t total = (int64_t)Ci * Co * ks;
  for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < total;
       i += (int64_t)gridDim.x * blockDim.x) {
    const int kk = (int)(i % ks);
    const int64_t t = i / ks;
    const int co = (int)(t % Co), ci = (int)(t / Co);
    const int r = (((kk - pad) % s) + s) % s;
    int64_t off = 0;
    int kk0;
    for (int rr = 0; rr < r; ++rr) off += (int64_t)Co * Ci * phase_taps(rr, ks, s, pad, &kk0);
    const int nt = phase_taps(r, ks, s, pad, &kk0);
    const int tap = (kk - kk0) / s;
    out[off + ((int64_t)co * nt + tap) * Ci + ci] = w[i];
  }
}

// ConvTranspose1d weights [Ci][Co][ks] -> per output phase r, tap-chunked for loader mode 5:
// P_r[co][(cc*nt + j')*CH + cl] = W[cc*CH + cl][co][kk0 + (nt - 1 - j')*s].  Taps are reversed
// (j' = nt - 1 - j) so that tap j' reads input u + (off0 - nt + 1) + j', an ascending shift
// like a stride-1 conv1d's; phases back to back as in convt_pack_kernel.
__global__ void convt_tap_pack_kernel(const float* w, int Ci, int Co, int ks, int s, int pad, int ch,
                                      float* out) {
  const int64_t total = (int64_t)Ci * Co * ks;
  for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < total;
       i += (int64_t)gridDim.x * blockDim.x) {
    const int kk = (int)(i % ks);
    const int64_t t = i / ks;
    const int co = (int)(t % Co), ci = (int)(t / Co);
    const int r = (((kk - pad) % s) + s) % s;
    int64_t off = 0;
    int kk0;
    for (int rr = 0; rr < r; ++rr) off += (int64_t)Co * Ci * phase_taps(rr, ks, s, pad, &kk0);
    const int nt = phase_taps(r, ks, s, pad, &kk0);
    const int jr = nt - 1 - (kk - kk0) / s;
    const int cc = ci / ch, cl = ci - cc * ch;
    out[off + (int64_t)co * nt * Ci + ((int64_t)cc * nt + jr) * ch + cl] = w[i];
  }
}

// Conv1d weights [Co][Ci][ks] -> tap-chunked [Co][Ci/CH][ks][CH] (the k order of loader mode 5)
__global__ void conv1d_tap_pack_kernel(const float* w, int Co, int Ci, int ks, int ch, float* out) {
  const int64_t total = (int64_t)Co * Ci * ks;
  for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < total;
       i += (int64_t)gridDim.x * blockDim.x) {
    const int tap = (int)(i % ks);
    const int64_t t = i / ks;
    const int ci = (int)(t % Ci), co = (int)(t / Ci);
    const int cc = ci / ch, cl = ci - cc * ch;
    out[(((int64_t)co * (Ci / ch) + cc) * ks + tap) * ch + cl] = w[i];
  }
}

// [wq; wk; wv] -> wcat [C/4 + C][C], biases -> bcat (zeros where a bias pointer is NULL)
__global__ void stack_qkv_kernel(const float* wq, const float* bq, const float* wk, const float* bk,
                                 const float* wv, const float* bv, int C, float* wcat, float* bcat) {
  const int Cq = C / 8;
  const int64_t total = (int64_t)(2 * Cq + C) * C;
  for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < total;
       i += (int64_t)gridDim.x * blockDim.x) {
    const int row = (int)(i / C);
    const int64_t col = i - (int64_t)row * C;
    const float* src = row < Cq ? wq + (int64_t)row * C : row < 2 * Cq ? wk + (int64_t)(row - Cq) * C
                                                                          : wv + (int64_t)(row - 2 * Cq) * C;
    wcat[i] = src[col];
    if (col == 0) {
      const float* b = row < Cq ? bq : row < 2 * Cq ? bk : bv;
      const int r = row < Cq ? row : row < 2 * Cq ? row - Cq : row - 2 * Cq;
      bcat[row] = b ? b[r] : 0.f;
    }
  }
}

int stack_qkv(const float* wq, const float* bq, const float* wk, const float* bk, const float* wv,
              const float* bv, int C, float* wcat, float* bcat, hipStream_t st) {
  const int64_t total = (int64_t)(C / 4 + C) * C;
  hipLaunchKernelGGL(stack_qkv_kernel, dim3((unsigned)std::min<int64_t>(cdiv(total, 256), 8192)),
                     dim3(256), 0, st, wq, bq, wk, bk, wv, bv, C, wcat, bcat);
  A2M_LAUNCH_CHECK();
  return A2M_OK;
}

// im2col for conv1d over [B][C][T] (t contiguous): col[b*Tout + t][ci*ks + tap] =
// x[b][ci][t*s + tap - pad] (0 outside).  One workgroup per (64 output steps, CC channels,
// clip): the input window is staged through LDS with coalesced row loads, and every output row
// segment (CC*ks contiguous floats) is written by consecutive lanes.  The dense [N][K] result is
// the engine's fastest operand form (mode 0), which the [B][C][T] gather cannot match.
// Blocks are numbered XCD-aware: workgroups are dealt round-robin to the 8 XCDs, so block L
// runs on XCD L % 8; all CC-channel slices of one row tile get the same L % 8, and the row
// segments they write side by side meet in that XCD's L2 as whole 128-byte lines instead of
// being written back as partial lines from different L2s.  With CC = 32 a segment of a
// 3- or 4-tap conv is itself a whole number of lines (384 / 512 B).
constexpr int I2C_T = 64, I2C_SPAN = 2 * (I2C_T - 1) + 8;
template <int CC>
__global__ __launch_bounds__(256) void im2col1d_kernel(const float* __restrict__ x, int64_t xs_b,
                                                       int64_t xs_c, int Ci, int Tin, int Tout,
                                                       int ks, int stride, int pad, int n_rows,
                                                       int n_ctiles, int xcd_map,
                                                       float* __restrict__ col) {
  __shared__ float win[CC][I2C_SPAN + 1];
  int r, ct;
  if (xcd_map) {
    const int L = blockIdx.x, xcd = L & 7, j = L >> 3;
    ct = j % n_ctiles;
    r = (j / n_ctiles) * 8 + xcd;
    if (r >= n_rows) return;
  } else {
    ct = blockIdx.x % n_ctiles;
    r = blockIdx.x / n_ctiles;
  }
  const int n_ttiles = (Tout + I2C_T - 1) / I2C_T;
  const int b = r / n_ttiles, t0 = (r - b * n_ttiles) * I2C_T, ci0 = ct * CC;
  const int span = (I2C_T - 1) * stride + ks;
  const int tin0 = t0 * stride - pad;
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const float* xb = x + (int64_t)b * xs_b;
  // wave w stages channels w, w+4, w+8, ... (lanes along t): all loads issued first
  constexpr int CW = CC / 4;
  float v[CW][3];
#pragma unroll
  for (int j = 0; j < CW; ++j) {
    const int c = wave + 4 * j;
#pragma unroll
    for (int q = 0; q < 3; ++q) {
      const int u = lane + 64 * q, ti = tin0 + u;
      v[j][q] = (u < span && ci0 + c < Ci && ti >= 0 && ti < Tin) ? xb[(int64_t)(ci0 + c) * xs_c + ti] : 0.f;
    }
  }
#pragma unroll
  for (int j = 0; j < CW; ++j)
#pragma unroll
    for (int q = 0; q < 3; ++q)
      if (lane + 64 * q < span) win[wave + 4 * j][lane + 64 * q] = v[j][q];
  __syncthreads();
  // wave w writes rows w, w+4, ...; lane owns the fixed k offsets kk = lane + 64 q
  const int K = Ci * ks, seg = min(CC, Ci - ci0) * ks;
  const int nt = min(I2C_T, Tout - t0);
  constexpr int NQ = CC * 8 / 64;   // ks <= 8
  int src[NQ];
#pragma unroll
  for (int q = 0; q < NQ; ++q) {
    const int kk = lane + 64 * q, c = kk / ks;
    src[q] = c * (I2C_SPAN + 1) + (kk - c * ks);
  }
  const float* w0 = &win[0][0];
  float* base = col + ((int64_t)b * Tout + t0) * K + (int64_t)ci0 * ks;
  for (int tt = wave; tt < nt; tt += 4) {
    float* row = base + (int64_t)tt * K;
#pragma unroll
    for (int q = 0; q < NQ; ++q)
      if (lane + 64 * q < seg) row[lane + 64 * q] = w0[src[q] + tt * stride];
  }
}

int softmax_rows(float* x, int rows, int n, hipStream_t st) {
  if (rows == 0) return A2M_OK;
  hipLaunchKernelGGL(softmax_rows_kernel, dim3((unsigned)cdiv(rows, 4)), dim3(256), 0, st, x,
                     rows, n);
  A2M_LAUNCH_CHECK();
  return A2M_OK;
}

}  // namespace a2m

using namespace a2m;

// [B][C][T] (batch stride xs_b) -> [B*T][C]: the k-contiguous (dense) operand layout of a 1x1
// conv's GEMM.  One workgroup per (clip, 64 channels): the 64 x T tile is read along t and
// written along c through LDS (pitch T + 1).
constexpr int TR_C = 64, TR_MAXT = 64;
__global__ __launch_bounds__(256) void bct_to_btc_kernel(const float* __restrict__ x, int64_t xs_b, int C,
                                                         int T, float* __restrict__ xt) {
  __shared__ float tile[TR_C][TR_MAXT + 1];
  const int b = blockIdx.y, c0 = blockIdx.x * TR_C;
  const float* src = x + b * xs_b + (int64_t)c0 * T;
  const int nc = min(TR_C, C - c0);
  for (int i = threadIdx.x; i < nc * T; i += blockDim.x) tile[i / T][i % T] = src[i];
  __syncthreads();
  float* dst = xt + (int64_t)b * T * C + c0;
  for (int i = threadIdx.x; i < nc * T; i += blockDim.x) {
    const int t = i / nc, c = i % nc;
    dst[(int64_t)t * C + c] = tile[c][t];
  }
}

// The GEMM of a channels-last conv2d over output columns [w_lo, w_lo + Wn) with epilogue E.
static int conv2d_nhwc_gemm(const float* x, int B, int Ci, int H, int W, const float* packed, int Co,
                            int kh, int kw, int stride, int pad_h, int pad_w, int Hout, int w_lo, int Wn,
                            const Epilogue& E, void* ws, size_t ws_bytes, hipStream_t st) {
  Gather A = dense_rk(packed, Ci * kh * kw);
  if (Ci % gemm_k_tile() == 0 && (reinterpret_cast<uintptr_t>(x) & 15) == 0) {
    // every k-tile is one tap's slice of Ci channels: channels-last conv rows (loader mode 6,
    // float4 loads: x 16-byte aligned, and every row's channel run starts at a multiple of Ci
    // floats; a 4-byte-aligned x takes the mode-4 k-run loader below, whose float4u loads need
    // only 4-byte alignment)
    Gather Bc{};
    Bc.base = x; Bc.sr0 = H * W * Ci; Bc.R1 = Hout; Bc.R2 = Wn; Bc.ar1 = stride; Bc.ar2 = stride;
    Bc.ch = -pad_h; Bc.cw = w_lo * stride - pad_w; Bc.Lh = H; Bc.Lw = W; Bc.K1 = kh; Bc.K2 = kw;
    Bc.divh = Bc.divw = 1; Bc.nhwc = Ci; Bc.kcontig = 1;
    return gemm(A, Bc, E, Co, B * Hout * Wn, Ci * kh * kw, 1, ws, ws_bytes, st);
  }
  // rows n = (b, ho, wo - w_lo), k = (i, j, ci): the input element x[b][ho*s - ph + i]
  // [(w_lo + wo)*s - pw + j][ci] sits at w' = win * Ci + ci along the fused (w, c) axis, so the
  // inner k digit (j, ci) is a unit-stride run of kw * Ci floats (loader mode 4, float4 loads)
  Gather Bg{};
  Bg.base = x; Bg.bstride = 0; Bg.sr0 = H * W * Ci;
  Bg.R1 = Hout; Bg.R2 = Wn; Bg.ar1 = stride; Bg.ar2 = stride * Ci;
  Bg.sk0 = 0; Bg.K1 = kh; Bg.K2 = kw * Ci; Bg.bk1 = 1; Bg.bk2 = 1;
  Bg.ch = -pad_h; Bg.cw = (w_lo * stride - pad_w) * Ci; Bg.divh = Bg.divw = 1;
  Bg.Lh = H; Bg.Lw = W * Ci; Bg.sh = W * Ci; Bg.sw = 1; Bg.kcontig = 1;
  return gemm(A, Bg, E, Co, B * Hout * Wn, Ci * kh * kw, 1, ws, ws_bytes, st);
}

extern "C" {

int a2m_conv1d_fwd_f32(const float* x, int64_t xs_b, int64_t xs_c, int64_t xs_t, int32_t B,
                       int32_t Ci, int32_t Tin, const float* w, const float* bias, int32_t Co,
                       int32_t ks, int32_t stride, int32_t pad, const float* bn_w,
                       const float* bn_b, const float* bn_rm, const float* bn_rv, float bn_eps,
                       int32_t act, float slope, float* y, int64_t ys_b, int64_t ys_c,
                       int64_t ys_t, void* ws, size_t ws_bytes, void* stream) {
  A2M_CHECK_ARG(x && w && y, "conv1d: null pointer");
  A2M_CHECK_ARG(B > 0 && Ci > 0 && Tin > 0 && Co > 0 && ks > 0 && stride > 0 && pad >= 0,
                "conv1d: bad shape B=%d Ci=%d T=%d Co=%d k=%d s=%d p=%d", B, Ci, Tin, Co, ks,
                stride, pad);
  const int Tout = (Tin + 2 * pad - ks) / stride + 1;
  A2M_CHECK_ARG(Tout > 0, "conv1d: empty output");
  A2M_CHECK_ARG(fits32(xs_b) && fits32(xs_c) && fits32(xs_t) && fits32(ys_b) && fits32(ys_c) &&
                    fits32(ys_t) && fits32((int64_t)B * xs_b) && fits32((int64_t)B * ys_b),
                "conv1d: tensor too large for 32-bit offsets");
  Gather A = dense_rk(w, Ci * ks);
  Gather Bg{};
  const int64_t K = (int64_t)Ci * ks, N = (int64_t)B * Tout;
  if (ks > 1 && ks <= 8 && stride <= 2 && Co >= 128 && xs_t == 1 && K % 4 == 0 &&
      N * K < (1LL << 31)) {
    // explicit im2col into the workspace head, then a dense x dense GEMM
    const size_t col_bytes = ((size_t)(N * K) * sizeof(float) + 255) & ~size_t(255);
    const size_t need = col_bytes + gemm_ws_bytes(Co, (int)N, (int)K, 1);
    if (!ws || ws_bytes < need) {
      set_error("conv1d: workspace too small (%zu < %zu bytes)", ws_bytes, need);
      return A2M_EWS;
    }
    float* col = static_cast<float*>(ws);
    hipStream_t st = as_stream(stream);
    // 16 channels a block, blocks grouped per XCD (32 channels measured alike, tools/ab_i2c.sh)
    const int n_rows = B * (int)cdiv(Tout, I2C_T), n_ct = (int)cdiv(Ci, 16);
    const unsigned blocks = (unsigned)(8 * n_ct * cdiv(n_rows, 8));
    hipLaunchKernelGGL(im2col1d_kernel<16>, dim3(blocks), dim3(256), 0, st, x, xs_b, xs_c, Ci, Tin,
                       Tout, ks, stride, pad, n_rows, n_ct, 1, col);
    A2M_LAUNCH_CHECK();
    Bg = dense_rk(col, (int)K);
    Epilogue E = epi_bn(y, bias, bn_w, bn_b, bn_rm, bn_rv, bn_eps, act, slope);
    E.N1 = 1; E.N2 = Tout; E.so0 = (int)ys_b; E.so1 = 0; E.so2 = (int)ys_t; E.som = (int)ys_c;
    return gemm(A, Bg, E, Co, (int)N, (int)K, 1, static_cast<char*>(ws) + col_bytes,
                ws_bytes - col_bytes, st);
  }
  if (ks == 1 && pad == 0 && stride == 1 && xs_b == (int64_t)Tin * xs_t) {
    // rows n = b*T + t are uniformly strided: plain [N][Ci] (k-major when xs_c == 1)
    Bg = xs_c == 1 ? dense_rk(x, (int)xs_t) : dense_kr(x, (int)xs_c);
    if (xs_c != 1) Bg.sr0 = (int)xs_t;
  } else {
    Bg.base = x; Bg.bstride = 0;
    Bg.sr0 = (int)xs_b; Bg.R1 = 1; Bg.R2 = Tout; Bg.ar1 = 0; Bg.ar2 = stride;
    Bg.sk0 = (int)xs_c; Bg.K1 = 1; Bg.K2 = ks; Bg.bk1 = 0; Bg.bk2 = 1;
    Bg.ch = 0; Bg.cw = -pad; Bg.divh = Bg.divw = 1; Bg.Lh = 1; Bg.Lw = Tin;
    Bg.sh = 0; Bg.sw = (int)xs_t;
    Bg.kcontig = (ks == 1 && xs_c == 1) ? 1 : 0;
  }
  Epilogue E = epi_bn(y, bias, bn_w, bn_b, bn_rm, bn_rv, bn_eps, act, slope);
  E.N1 = 1; E.N2 = Tout; E.so0 = (int)ys_b; E.so1 = 0; E.so2 = (int)ys_t; E.som = (int)ys_c;
  return gemm(A, Bg, E, Co, B * Tout, Ci * ks, 1, ws, ws_bytes, as_stream(stream));
}

int a2m_convt1d_packed_fwd_f32(const float* x, int64_t xs_b, int64_t xs_c, int32_t B, int32_t Ci,
                        int32_t Tin, const float* packed, const float* bias, int32_t Co, int32_t ks,
                        int32_t stride, int32_t pad, int32_t out_pad, const float* bn_w,
                        const float* bn_b, const float* bn_rm, const float* bn_rv, float bn_eps,
                        int32_t act, float slope, float* y, int64_t ys_b, int64_t ys_c,
                        void* ws, size_t ws_bytes, void* stream) {
  A2M_CHECK_ARG(x && packed && y, "convt1d: null pointer");
  const int Tout = (Tin - 1) * stride - 2 * pad + ks + out_pad;
  A2M_CHECK_ARG(B > 0 && Ci > 0 && Co > 0 && Tout > 0 && stride > 0 && pad >= 0,
                "convt1d: bad shape");
  A2M_CHECK_ARG(fits32((int64_t)B * xs_b) && fits32((int64_t)B * ys_b) &&
                    fits32((int64_t)Ci * Co * ks),
                "convt1d: too large");
  // Output-phase decomposition: out[s*u + r] only sees the taps kk with
  // (r + pad - kk) % s == 0, at input u + (r + pad - kk)/s.  Each phase is a dense GEMM over
  // K = taps_r * Ci (no zero-inserted work); weights packed per phase by a2m_convt1d_pack_f32
  // as P_r[co][tap*Ci + ci] = W[ci][co][kk_tap], phases back to back.
  hipStream_t st = as_stream(stream);
  size_t off = 0;
  for (int r = 0; r < stride; ++r) {
    int kk0 = -1, ntap = 0;
    for (int kk = 0; kk < ks; ++kk)
      if ((((r + pad - kk) % stride) + stride) % stride == 0) { if (kk0 < 0) kk0 = kk; ++ntap; }
    const int nu = (Tout - r + stride - 1) / stride;
    if (nu <= 0) continue;
    float* yr = y + r;
    if (ntap == 0) {  // this phase only gets the bias / BN / act of zero
      Gather Az = dense_rk(packed, 1);
      Gather Bz = dense_rk(x, 1);
      Epilogue E = epi_bn(yr, bias, bn_w, bn_b, bn_rm, bn_rv, bn_eps, act, slope);
      E.N1 = 1; E.N2 = nu; E.so0 = (int)ys_b; E.so2 = stride; E.som = (int)ys_c;
      int rc = gemm(Az, Bz, E, Co, B * nu, 0, 1, nullptr, 0, st);
      if (rc) return rc;
      continue;
    }
    const int off0 = (r + pad - kk0) / stride;  // exact; later taps shift the input by -1 each
    Gather A = dense_rk(packed + off, ntap * Ci);
    Gather Bg{};
    Bg.base = x; Bg.sr0 = (int)xs_b; Bg.R1 = nu; Bg.R2 = 1; Bg.ar1 = 1; Bg.ar2 = 0;
    Bg.K1 = ntap; Bg.K2 = Ci; Bg.sk0 = 0; Bg.bk1 = -1; Bg.bk2 = 1; Bg.ch = off0; Bg.cw = 0;
    Bg.divh = Bg.divw = 1; Bg.Lh = Tin; Bg.Lw = Ci; Bg.sh = 1; Bg.sw = (int)xs_c; Bg.kcontig = 0;
    Epilogue E = epi_bn(yr, bias, bn_w, bn_b, bn_rm, bn_rv, bn_eps, act, slope);
    E.N1 = 1; E.N2 = nu; E.so0 = (int)ys_b; E.so2 = stride; E.som = (int)ys_c;
    int rc = gemm(A, Bg, E, Co, B * nu, ntap * Ci, 1, ws, ws_bytes, st);
    if (rc) return rc;
    off += (size_t)Co * ntap * Ci;
  }
  return A2M_OK;
}

int a2m_conv1d_tap_pack_f32(const float* w, int32_t Co, int32_t Ci, int32_t ks, int32_t chunk,
                            float* packed, void* stream) {
  A2M_CHECK_ARG(w && packed && Co > 0 && Ci > 0 && ks > 0 && (chunk == 32 || chunk == 64) &&
                    Ci % chunk == 0,
                "conv1d_tap_pack: bad args Co=%d Ci=%d k=%d chunk=%d", Co, Ci, ks, chunk);
  A2M_CHECK_ARG(fits32((int64_t)Co * Ci * ks), "conv1d_tap_pack: too large");
  hipLaunchKernelGGL(conv1d_tap_pack_kernel,
                     dim3((unsigned)std::min<int64_t>(cdiv((int64_t)Co * Ci * ks, 256), 8192)),
                     dim3(256), 0, as_stream(stream), w, Co, Ci, ks, chunk, packed);
  A2M_LAUNCH_CHECK();
  return A2M_OK;
}

int32_t a2m_conv1d_tap_chunk(void) { return gemm_k_tile(); }

int a2m_conv1d_tap_fwd_f32(const float* x, int64_t xs_b, int64_t xs_c, int32_t B, int32_t Ci,
                           int32_t T, const float* packed, int32_t chunk, const float* bias,
                           int32_t Co, int32_t ks, int32_t pad, const float* bn_w,
                           const float* bn_b, const float* bn_rm, const float* bn_rv, float bn_eps,
                           int32_t act, float slope, float* y, int64_t ys_b, int64_t ys_c,
                           int64_t ys_t, void* ws, size_t ws_bytes, void* stream) {
  A2M_CHECK_ARG(x && packed && y, "conv1d_tap: null pointer");
  A2M_CHECK_ARG(B > 0 && Ci > 0 && Co > 0 && ks > 1 && 2 * pad == ks - 1,
                "conv1d_tap: bad shape B=%d Ci=%d Co=%d k=%d p=%d (stride 1, same padding)", B, Ci,
                Co, ks, pad);
  A2M_CHECK_ARG(chunk == gemm_k_tile() && Ci % chunk == 0,
                "conv1d_tap: weights packed in %d-channel chunks, the engine's k-tile is %d (Ci=%d)",
                chunk, gemm_k_tile(), Ci);
  A2M_CHECK_ARG(T > 0 && T % 4 == 0 && 64 % T == 0 && pad < T,
                "conv1d_tap: clip length %d must divide the 64-row tile and be a multiple of 4", T);
  A2M_CHECK_ARG(fits32(xs_b) && fits32(xs_c) && fits32((int64_t)B * xs_b) &&
                    fits32((int64_t)B * ys_b) && fits32(ys_c) && fits32(ys_t),
                "conv1d_tap: tensor too large for 32-bit offsets");
  A2M_CHECK_ARG((reinterpret_cast<uintptr_t>(x) % 16) == 0 && xs_b % 4 == 0 && xs_c % 4 == 0,
                "conv1d_tap: x rows must be 16-byte aligned");
  Gather A = dense_rk(packed, Ci * ks);
  Gather Bg{};
  Bg.base = x; Bg.bstride = 0;
  Bg.sr0 = (int)xs_b; Bg.R1 = 1; Bg.R2 = T; Bg.sk0 = (int)xs_c;
  Bg.K1 = Bg.K2 = 1; Bg.divh = Bg.divw = 1; Bg.Lh = Bg.Lw = 1;
  Bg.cw = -pad; Bg.tapconv = ks;
  Epilogue E = epi_bn(y, bias, bn_w, bn_b, bn_rm, bn_rv, bn_eps, act, slope);
  E.N1 = 1; E.N2 = T; E.so0 = (int)ys_b; E.so1 = 0; E.so2 = (int)ys_t; E.som = (int)ys_c;
  return gemm(A, Bg, E, Co, B * T, Ci * ks, 1, ws, ws_bytes, as_stream(stream));
}

int a2m_conv1d_tap_group_fwd_f32(const float* x, int64_t xs_g, int64_t xs_b, int64_t xs_c, int32_t G,
                                 int32_t B, int32_t Ci, int32_t T, const float* packed, int64_t w_gs,
                                 int32_t chunk, const float* bias, int32_t Co, int32_t ks, int32_t pad,
                                 const float* bn_w, const float* bn_b, const float* bn_rm,
                                 const float* bn_rv, float bn_eps, int32_t act, float slope, float* y,
                                 int64_t ys_g, int64_t ys_b, int64_t ys_c, int64_t ys_t, void* ws,
                                 size_t ws_bytes, void* stream) {
  A2M_CHECK_ARG(x && packed && y && G > 0, "conv1d_tap_group: null pointer / G=%d", G);
  A2M_CHECK_ARG(B > 0 && Ci > 0 && Co > 0 && ks > 1 && 2 * pad == ks - 1,
                "conv1d_tap_group: bad shape B=%d Ci=%d Co=%d k=%d p=%d (stride 1, same padding)", B,
                Ci, Co, ks, pad);
  A2M_CHECK_ARG(chunk == gemm_k_tile() && Ci % chunk == 0,
                "conv1d_tap_group: weights packed in %d-channel chunks, the engine's k-tile is %d (Ci=%d)",
                chunk, gemm_k_tile(), Ci);
  A2M_CHECK_ARG(T > 0 && T % 4 == 0 && 64 % T == 0 && pad < T,
                "conv1d_tap_group: clip length %d must divide the 64-row tile and be a multiple of 4", T);
  A2M_CHECK_ARG(fits32(xs_b) && fits32(xs_c) && fits32((int64_t)B * xs_b) && fits32((int64_t)B * ys_b) &&
                    fits32(ys_c) && fits32(ys_t) && ys_g != 0 && w_gs >= (int64_t)Co * Ci * ks,
                "conv1d_tap_group: strides");
  A2M_CHECK_ARG((reinterpret_cast<uintptr_t>(x) % 16) == 0 && xs_b % 4 == 0 && xs_c % 4 == 0 &&
                    xs_g % 4 == 0 && w_gs % 4 == 0 && (reinterpret_cast<uintptr_t>(packed) % 16) == 0,
                "conv1d_tap_group: x rows / packed weights must be 16-byte aligned");
  Gather A = dense_rk(packed, Ci * ks, w_gs);
  Gather Bg{};
  Bg.base = x; Bg.bstride = xs_g;
  Bg.sr0 = (int)xs_b; Bg.R1 = 1; Bg.R2 = T; Bg.sk0 = (int)xs_c;
  Bg.K1 = Bg.K2 = 1; Bg.divh = Bg.divw = 1; Bg.Lh = Bg.Lw = 1;
  Bg.cw = -pad; Bg.tapconv = ks;
  Epilogue E = epi_bn(y, bias, bn_w, bn_b, bn_rm, bn_rv, bn_eps, act, slope);
  E.N1 = 1; E.N2 = T; E.so0 = (int)ys_b; E.so1 = 0; E.so2 = (int)ys_t; E.som = (int)ys_c;
  E.bstride = ys_g; E.pstride = Co;
  return gemm(A, Bg, E, Co, B * T, Ci * ks, G, ws, ws_bytes, as_stream(stream));
}

int a2m_convt1d_pack_f32(const float* w, int32_t Ci, int32_t Co, int32_t ks, int32_t stride,
                         int32_t pad, float* packed, void* stream) {
  A2M_CHECK_ARG(w && packed && Ci > 0 && Co > 0 && ks > 0 && stride > 0 && pad >= 0,
                "convt1d_pack: bad args");
  A2M_CHECK_ARG(fits32((int64_t)Ci * Co * ks), "convt1d_pack: too large");
  hipLaunchKernelGGL(convt_pack_kernel,
                     dim3((unsigned)std::min<int64_t>(cdiv((int64_t)Ci * Co * ks, 256), 8192)),
                     dim3(256), 0, as_stream(stream), w, Ci, Co, ks, stride, pad, packed);
  A2M_LAUNCH_CHECK();
  return A2M_OK;
}

int a2m_convt1d_tap_pack_f32(const float* w, int32_t Ci, int32_t Co, int32_t ks, int32_t stride,
                             int32_t pad, int32_t chunk, float* packed, void* stream) {
  A2M_CHECK_ARG(w && packed && Ci > 0 && Co > 0 && ks > 0 && stride > 0 && pad >= 0 &&
                    (chunk == 32 || chunk == 64) && Ci % chunk == 0,
                "convt1d_tap_pack: bad args Ci=%d Co=%d k=%d s=%d p=%d chunk=%d", Ci, Co, ks, stride,
                pad, chunk);
  A2M_CHECK_ARG(fits32((int64_t)Ci * Co * ks), "convt1d_tap_pack: too large");
  hipLaunchKernelGGL(convt_tap_pack_kernel,
                     dim3((unsigned)std::min<int64_t>(cdiv((int64_t)Ci * Co * ks, 256), 8192)),
                     dim3(256), 0, as_stream(stream), w, Ci, Co, ks, stride, pad, chunk, packed);
  A2M_LAUNCH_CHECK();
  return A2M_OK;
}

int a2m_convt1d_tap_fwd_f32(const float* x, int64_t xs_b, int64_t xs_c, int32_t B, int32_t Ci,
                            int32_t Tin, const float* packed, int32_t chunk, const float* bias,
                            int32_t Co, int32_t ks, int32_t stride, int32_t pad, int32_t out_pad,
                            const float* bn_w, const float* bn_b, const float* bn_rm,
                            const float* bn_rv, float bn_eps, int32_t act, float slope, float* y,
                            int64_t ys_b, int64_t ys_c, void* ws, size_t ws_bytes, void* stream) {
  A2M_CHECK_ARG(x && packed && y, "convt1d_tap: null pointer");
  const int Tout = (Tin - 1) * stride - 2 * pad + ks + out_pad;
  A2M_CHECK_ARG(B > 0 && Ci > 0 && Co > 0 && ks > 0 && stride > 0 && pad >= 0 && Tout == stride * Tin,
                "convt1d_tap: bad shape B=%d Ci=%d T=%d Co=%d k=%d s=%d p=%d op=%d (every output "
                "phase must hold Tin rows)", B, Ci, Tin, Co, ks, stride, pad, out_pad);
  A2M_CHECK_ARG(chunk == gemm_k_tile() && Ci % chunk == 0,
                "convt1d_tap: weights packed in %d-channel chunks, the engine's k-tile is %d (Ci=%d)",
                chunk, gemm_k_tile(), Ci);
  A2M_CHECK_ARG(Tin % 4 == 0 && 64 % Tin == 0,
                "convt1d_tap: clip length %d must divide the 64-row tile and be a multiple of 4", Tin);
  A2M_CHECK_ARG(fits32(xs_b) && fits32(xs_c) && fits32((int64_t)B * xs_b) &&
                    fits32((int64_t)B * ys_b) && fits32(ys_c) && fits32((int64_t)Ci * Co * ks),
                "convt1d_tap: tensor too large for 32-bit offsets");
  A2M_CHECK_ARG((reinterpret_cast<uintptr_t>(x) % 16) == 0 && xs_b % 4 == 0 && xs_c % 4 == 0,
                "convt1d_tap: x rows must be 16-byte aligned");
  // Output phase r = the stride-1 conv1d (loader mode 5) of x with the phase's nt taps at input
  // shifts off0 - nt + 1 .. off0 (a2m_convt1d_tap_pack_f32's reversed tap order), written to
  // y[.., s*u + r]: the same phase decomposition as a2m_convt1d_packed_fwd_f32, with each
  // chunk's x window loaded once for all of the phase's taps instead of gathered per tap.
  hipStream_t st = as_stream(stream);
  size_t off = 0;
  for (int r = 0; r < stride; ++r) {
    int kk0 = -1, ntap = 0;
    for (int kk = 0; kk < ks; ++kk)
      if ((((r + pad - kk) % stride) + stride) % stride == 0) { if (kk0 < 0) kk0 = kk; ++ntap; }
    float* yr = y + r;
    Epilogue E = epi_bn(yr, bias, bn_w, bn_b, bn_rm, bn_rv, bn_eps, act, slope);
    E.N1 = 1; E.N2 = Tin; E.so0 = (int)ys_b; E.so1 = 0; E.so2 = stride; E.som = (int)ys_c;
    if (ntap == 0) {  // this phase only gets the bias / BN / act of zero
      int rc = gemm(dense_rk(packed, 1), dense_rk(x, 1), E, Co, B * Tin, 0, 1, nullptr, 0, st);
      if (rc) return rc;
      continue;
    }
    const int cw = (r + pad - kk0) / stride - ntap + 1;
    A2M_CHECK_ARG(cw > -Tin && cw + ntap - 1 < Tin, "convt1d_tap: tap shift %d..%d outside the clip",
                  cw, cw + ntap - 1);
    Gather Bg{};
    Bg.base = x; Bg.bstride = 0;
    Bg.sr0 = (int)xs_b; Bg.R1 = 1; Bg.R2 = Tin; Bg.sk0 = (int)xs_c;
    Bg.K1 = Bg.K2 = 1; Bg.divh = Bg.divw = 1; Bg.Lh = Bg.Lw = 1;
    Bg.cw = cw; Bg.tapconv = ntap;
    int rc = gemm(dense_rk(packed + off, ntap * Ci), Bg, E, Co, B * Tin, ntap * Ci, 1, ws, ws_bytes, st);
    if (rc) return rc;
    off += (size_t)Co * ntap * Ci;
  }
  return A2M_OK;
}

int a2m_convt1d_fwd_f32(const float* x, int64_t xs_b, int64_t xs_c, int32_t B, int32_t Ci,
                        int32_t Tin, const float* w, const float* bias, int32_t Co, int32_t ks,
                        int32_t stride, int32_t pad, int32_t out_pad, const float* bn_w,
                        const float* bn_b, const float* bn_rm, const float* bn_rv, float bn_eps,
                        int32_t act, float slope, float* y, int64_t ys_b, int64_t ys_c,
                        void* ws, size_t ws_bytes, void* stream) {
  A2M_CHECK_ARG(x && w && y, "convt1d: null pointer");
  // weights packed per output phase into the workspace head, then the packed path
  const size_t pack_bytes = ((size_t)Ci * Co * ks * sizeof(float) + 255) & ~size_t(255);
  if (!ws || ws_bytes < pack_bytes) {
    set_error("convt1d: workspace too small (%zu < %zu bytes)", ws_bytes, pack_bytes);
    return A2M_EWS;
  }
  float* packed = static_cast<float*>(ws);
  int rc = a2m_convt1d_pack_f32(w, Ci, Co, ks, stride, pad, packed, stream);
  if (rc) return rc;
  return a2m_convt1d_packed_fwd_f32(x, xs_b, xs_c, B, Ci, Tin, packed, bias, Co, ks, stride, pad,
                                    out_pad, bn_w, bn_b, bn_rm, bn_rv, bn_eps, act, slope, y, ys_b,
                                    ys_c, static_cast<char*>(ws) + pack_bytes,
                                    ws_bytes - pack_bytes, stream);
}

// im2col for conv2d over a live column range: col[n][k], n = (b, ho, wn) with wn over
// [w_lo, w_hi), k = (ci, i, j) -- the dense [N][K] operand of the encoder convolutions
// (model_layers.py:60-118 at the AudioEncoder shapes).  Rows are written along k, four
// consecutive k per thread (float4 stores); the input reads are L2 hits (each element is read
// kh*kw / stride^2 times).
constexpr int I2C2_QUADS = 256;   // k quads per workgroup (one per thread)
__global__ __launch_bounds__(256) void im2col2d_kernel(const float* __restrict__ x, int Ci, int H, int W,
                                                       int kh, int kw, int stride, int ph, int pw,
                                                       int Hout, int Wn, int w_lo, int K,
                                                       float* __restrict__ col) {
  // workgroup (b, ho) x k-range: each thread decomposes its four k = (ci, i, j) once and then
  // writes them for every live column wn (the k -> input-row arithmetic is amortised over Wn).
  // With one live column the k range is split over blockIdx.y (one quad per thread): conv5's
  // im2col 18.5 -> 14.7 us.  With several columns the split measured slower (27.0 -> 30.4 us at
  // conv3), and so did staging the input patch in LDS (26.3 / 20.6 / 32.4 us at conv3 / 4 / 5):
  // all of these run at 1.5-2 TB/s of columns, like the other copy kernels of the step.
  const int ho = blockIdx.x % Hout, b = blockIdx.x / Hout;
  const int hb = ho * stride - ph;
  const int khw = kh * kw;
  for (int k0 = (blockIdx.y * I2C2_QUADS + threadIdx.x) * 4; k0 < K; k0 += gridDim.y * I2C2_QUADS * 4) {
    float* rows = col + (int64_t)blockIdx.x * Wn * K + k0;
    const float* src[4];
    int jj[4];
    bool hv[4];
#pragma unroll
    for (int q = 0; q < 4; ++q) {
      const int k = k0 + q;
      const int ci = k / khw, r = k - ci * khw;
      const int i = r / kw, j = r - i * kw;
      const int h = hb + i;
      hv[q] = h >= 0 && h < H;
      src[q] = x + ((int64_t)(b * Ci + ci) * H + (hv[q] ? h : 0)) * W;
      jj[q] = j;
    }
#pragma unroll 2
    for (int wn = 0; wn < Wn; ++wn) {
      const int wb = (w_lo + wn) * stride - pw;
      float v[4];
#pragma unroll
      for (int q = 0; q < 4; ++q) {
        const int w = wb + jj[q];
        v[q] = (hv[q] && w >= 0 && w < W) ? src[q][w] : 0.f;
      }
      *reinterpret_cast<float4*>(rows + (int64_t)wn * K) = make_float4(v[0], v[1], v[2], v[3]);
    }
  }
}

// Conv2d weights [Co][Ci][kh][kw] -> [Co][kh][kw][Ci] (the k order of the NHWC operand)
__global__ void conv2d_pack_nhwc_kernel(const float* w, int Co, int Ci, int kh, int kw, float* out) {
  const int64_t total = (int64_t)Co * Ci * kh * kw;
  for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < total;
       i += (int64_t)gridDim.x * blockDim.x) {
    const int j = (int)(i % kw);
    int64_t t = i / kw;
    const int r = (int)(t % kh);
    t /= kh;
    const int ci = (int)(t % Ci), co = (int)(t / Ci);
    out[(((int64_t)co * kh + r) * kw + j) * Ci + ci] = w[i];
  }
}

int a2m_conv2d_fwd_f32(const float* x, int32_t B, int32_t Ci, int32_t H, int32_t W,
                       const float* w, const float* bias, int32_t Co, int32_t kh, int32_t kw,
                       int32_t stride, int32_t pad_h, int32_t pad_w, const float* bn_w,
                       const float* bn_b, const float* bn_rm, const float* bn_rv, float bn_eps,
                       int32_t act, float slope, float* y, int32_t Hout, int32_t Wout,
                       int32_t w_lo, int32_t w_hi, void* ws, size_t ws_bytes, void* stream) {
  A2M_CHECK_ARG(x && w && y, "conv2d: null pointer");
  A2M_CHECK_ARG(Hout == (H + 2 * pad_h - kh) / stride + 1 && Wout == (W + 2 * pad_w - kw) / stride + 1,
                "conv2d: output geometry mismatch");
  A2M_CHECK_ARG(0 <= w_lo && w_lo < w_hi && w_hi <= Wout, "conv2d: bad column range [%d,%d)",
                w_lo, w_hi);
  A2M_CHECK_ARG(fits32((int64_t)B * Ci * H * W) && fits32((int64_t)B * Co * Hout * Wout),
                "conv2d: too large");
  const int Wn = w_hi - w_lo;
  Gather A = dense_rk(w, Ci * kh * kw);
  const int64_t K = (int64_t)Ci * kh * kw, N = (int64_t)B * Hout * Wn;
  // explicit im2col into the workspace head, then a dense x dense GEMM, where the GEMM's gain
  // over the gathered (mode-2) operand outweighs writing the [N][K] matrix: measured on the
  // encoder, K >= 2048 (conv2 / conv3 / conv4: 26 / 22 / 18 us of im2col for 32 / 29 / 32 us
  // of GEMM time saved); conv1 (K = 1024, 92 MB of columns at B = 64) loses.
  if (Co >= 128 && K >= 2048 && K % 4 == 0 && N * K < (1LL << 31)) {
    const size_t col_bytes = ((size_t)(N * K) * sizeof(float) + 255) & ~size_t(255);
    const size_t need = col_bytes + gemm_ws_bytes(Co, (int)N, (int)K, 1);
    if (!ws || ws_bytes < need) {
      set_error("conv2d: workspace too small (%zu < %zu bytes)", ws_bytes, need);
      return A2M_EWS;
    }
    float* col = static_cast<float*>(ws);
    hipStream_t st = as_stream(stream);
    const unsigned ksplit = Wn == 1 ? (unsigned)cdiv(K, 4 * I2C2_QUADS) : 1u;
    hipLaunchKernelGGL(im2col2d_kernel, dim3((unsigned)(B * Hout), ksplit), dim3(256), 0, st, x, Ci, H,
                       W, kh, kw, stride, pad_h, pad_w, Hout, Wn, w_lo, (int)K, col);
    A2M_LAUNCH_CHECK();
    Gather Bd = dense_rk(col, (int)K);
    Epilogue E = epi_bn(y + w_lo, bias, bn_w, bn_b, bn_rm, bn_rv, bn_eps, act, slope);
    E.N1 = Hout; E.N2 = Wn; E.so0 = Co * Hout * Wout; E.so1 = Wout; E.so2 = 1; E.som = Hout * Wout;
    return gemm(A, Bd, E, Co, (int)N, (int)K, 1, static_cast<char*>(ws) + col_bytes,
                ws_bytes - col_bytes, st);
  }
  Gather Bg{};
  Bg.base = x; Bg.sr0 = Ci * H * W; Bg.R1 = Hout; Bg.R2 = Wn; Bg.ar1 = stride; Bg.ar2 = stride;
  Bg.sk0 = H * W; Bg.K1 = kh; Bg.K2 = kw; Bg.bk1 = 1; Bg.bk2 = 1;
  Bg.ch = -pad_h; Bg.cw = w_lo * stride - pad_w; Bg.divh = Bg.divw = 1; Bg.Lh = H; Bg.Lw = W;
  Bg.sh = W; Bg.sw = 1; Bg.kcontig = 0;
  Epilogue E = epi_bn(y + w_lo, bias, bn_w, bn_b, bn_rm, bn_rv, bn_eps, act, slope);
  E.N1 = Hout; E.N2 = Wn; E.so0 = Co * Hout * Wout; E.so1 = Wout; E.so2 = 1; E.som = Hout * Wout;
  return gemm(A, Bg, E, Co, B * Hout * Wn, Ci * kh * kw, 1, ws, ws_bytes, as_stream(stream));
}

int a2m_conv2d_pack_nhwc_f32(const float* w, int32_t Co, int32_t Ci, int32_t kh, int32_t kw,
                             float* packed, void* stream) {
  A2M_CHECK_ARG(w && packed && Co > 0 && Ci > 0 && kh > 0 && kw > 0, "conv2d_pack_nhwc: bad args");
  A2M_CHECK_ARG(fits32((int64_t)Co * Ci * kh * kw), "conv2d_pack_nhwc: too large");
  hipLaunchKernelGGL(conv2d_pack_nhwc_kernel,
                     dim3((unsigned)std::min<int64_t>(cdiv((int64_t)Co * Ci * kh * kw, 256), 8192)),
                     dim3(256), 0, as_stream(stream), w, Co, Ci, kh, kw, packed);
  A2M_LAUNCH_CHECK();
  return A2M_OK;
}

// Single-input-channel conv2d (the encoder's first layer, model_layers.py:262-263: 1 -> 64,
// k 4x4, s 2 over the [B, T, F] mel) as a direct kernel: K = kh*kw = 16 is far too shallow for
// the GEMM engine (its k loop never fills).  One workgroup per C1_ROWS output rows of one clip:
// the input rows they read are staged in LDS once, each thread loads the taps of 4 output
// channels into registers once and sweeps C1_ROWS rows x its output columns, writing float4
// channel groups so a pixel's Co channels leave as one contiguous run (NHWC).  Bias, BN-eval
// affine and the activation are fused as in the GEMM epilogue (gemm_kernel.h epi_value).
constexpr int C1_K = 4, C1_ROWS = 4, C1_MAXW = 512;
constexpr int C1_IN_ROWS = (C1_ROWS - 1) * 2 + C1_K;   // stride <= 2
__global__ __launch_bounds__(256) void conv2d_c1_kernel(
    const float* __restrict__ x, int H, int W, const float* __restrict__ packed, const float* __restrict__ bias,
    int Co, int stride, int ph, int pw, const float* __restrict__ bn_w,
    const float* __restrict__ bn_b, const float* __restrict__ bn_rm, const float* __restrict__ bn_rv,
    float bn_eps, int act, float slope, float* __restrict__ y, int y_nhwc, int Hout, int Wout, int w_lo, int w_hi) {
  constexpr int kh = C1_K, kw = C1_K;
  __shared__ __attribute__((aligned(16))) float rows[C1_IN_ROWS][C1_MAXW];
  const int rb = (Hout + C1_ROWS - 1) / C1_ROWS;
  const int b = blockIdx.x / rb, ho0 = (blockIdx.x % rb) * C1_ROWS;
  const int nr = min(C1_ROWS, Hout - ho0);
  const int tid = threadIdx.x;
  // input rows ho0*s - ph + i and the columns the live outputs read, zero outside the image
  const int c0 = w_lo * stride - pw, nc = (w_hi - 1 - w_lo) * stride + kw;
  const int nin = (nr - 1) * stride + kh;
  // this thread's 4 channels: taps, bias and BN terms requested first, so their round trip
  // overlaps the patch loads below instead of following them
  const int ng = Co / 4;                 // float4 channel groups
  const int wpp = blockDim.x / ng;       // output columns per pass
  const int g = tid % ng, wsub = tid / ng;
  float wt[4][kh * kw];
  float sc[4], sh[4], bo[4], rm[4], rv[4];
#pragma unroll
  for (int j = 0; j < 4; ++j) {
    const int co = 4 * g + j;
    const float4* wp = reinterpret_cast<const float4*>(packed + co * kh * kw);
#pragma unroll
    for (int t = 0; t < kh * kw / 4; ++t) {
      const float4 v = wp[t];
      wt[j][4 * t] = v.x; wt[j][4 * t + 1] = v.y; wt[j][4 * t + 2] = v.z; wt[j][4 * t + 3] = v.w;
    }
    // raw terms only here; the arithmetic on them waits until the patch loads are out
    sh[j] = bias ? bias[co] : 0.f;
    if (bn_w) {
      sc[j] = bn_w[co];
      bo[j] = bn_b[co];
      rm[j] = bn_rm[co];
      rv[j] = bn_rv[co];
    }
  }
  // the input patch: the first C1_PRE elements per thread are loaded all at once (clamped
  // addresses, zeroed after the loads), so their latencies overlap instead of one dependent
  // round trip per element; wider patches finish in the plain loop
  constexpr int C1_PRE = 8;
  {
    float pv[C1_PRE];
    bool ok[C1_PRE];
#pragma unroll
    for (int u = 0; u < C1_PRE; ++u) {
      const int idx = tid + u * 256;
      const int i = idx / nc, c = idx - (idx / nc) * nc;
      const int hi = ho0 * stride - ph + i, wi = c0 + c;
      ok[u] = idx < nin * nc && hi >= 0 && hi < H && wi >= 0 && wi < W;
      pv[u] = x[ok[u] ? ((int64_t)b * H + hi) * W + wi : 0];
    }
#pragma unroll
    for (int u = 0; u < C1_PRE; ++u) {
      const int idx = tid + u * 256;
      if (idx < nin * nc) rows[idx / nc][idx % nc] = ok[u] ? pv[u] : 0.f;
    }
  }
  for (int idx = tid + C1_PRE * 256; idx < nin * nc; idx += blockDim.x) {
    const int i = idx / nc, c = idx % nc;
    const int hi = ho0 * stride - ph + i, wi = c0 + c;
    rows[i][c] = (hi >= 0 && hi < H && wi >= 0 && wi < W) ? x[((int64_t)b * H + hi) * W + wi] : 0.f;
  }
  // epi_value order: + bias, then (v - rm) * (w / sqrt(rv + eps)) + b
#pragma unroll
  for (int j = 0; j < 4; ++j) {
    if (bn_w) {
      sc[j] = sc[j] / sqrtf(rv[j] + bn_eps);
      sh[j] = sh[j] - rm[j];
    } else {
      sc[j] = 1.f;
      bo[j] = 0.f;
    }
  }
  __syncthreads();
  if (wsub >= wpp) return;
  for (int r = 0; r < nr; ++r) {
    const int ho = ho0 + r;
    for (int wo = w_lo + wsub; wo < w_hi; wo += wpp) {
      const int cb = (wo - w_lo) * stride;
      float acc[4] = {0.f, 0.f, 0.f, 0.f};
      if (stride == 2) {   // cb even: each kernel row's 4 inputs as two 8-byte LDS reads
#pragma unroll
        for (int i = 0; i < kh; ++i) {
          const float2 p0 = *reinterpret_cast<const float2*>(&rows[r * 2 + i][cb]);
          const float2 p1 = *reinterpret_cast<const float2*>(&rows[r * 2 + i][cb + 2]);
          const float xr[4] = {p0.x, p0.y, p1.x, p1.y};
#pragma unroll
          for (int j = 0; j < kw; ++j)
#pragma unroll
            for (int c = 0; c < 4; ++c) acc[c] = fmaf(wt[c][i * kw + j], xr[j], acc[c]);
        }
      } else {
#pragma unroll
        for (int i = 0; i < kh; ++i) {
#pragma unroll
          for (int j = 0; j < kw; ++j) {
            const float xv = rows[r * stride + i][cb + j];
#pragma unroll
            for (int c = 0; c < 4; ++c) acc[c] = fmaf(wt[c][i * kw + j], xv, acc[c]);
          }
        }
      }
      float o[4];
#pragma unroll
      for (int c = 0; c < 4; ++c) {
        float v = (acc[c] + sh[c]) * sc[c] + bo[c];
        if (act == ACT_RELU) v = v > 0.f ? v : 0.f;
        else if (act == ACT_LRELU) v = v > 0.f ? v : v * slope;
        else if (act == ACT_SIGMOID) v = 1.f / (1.f + expf(-v));
        o[c] = v;
      }
      if (y_nhwc) {
        *reinterpret_cast<float4*>(y + (((int64_t)b * Hout + ho) * Wout + wo) * Co + 4 * g) =
            make_float4(o[0], o[1], o[2], o[3]);
      } else {
#pragma unroll
        for (int c = 0; c < 4; ++c) y[(((int64_t)b * Co + 4 * g + c) * Hout + ho) * Wout + wo] = o[c];
      }
    }
  }
}

}  // extern "C"

// The same layer on the matrix cores (NHWC output, Co a multiple of 32): the workgroup's
// C1_ROWS x Wn output pixels and Co channels are (32-pixel, 32-channel) jobs of one
// v_mfma_f32_32x32x2_f32 chain each (K = 16 taps = 8 MFMAs): the channel taps are the A operand
// (8 registers per lane, loaded once per channel tile), the pixels' taps the B operand, read
// from the LDS patch (lanes along pixels: stride-2 columns, the two k of a step adjacent, so a
// wave's 64 reads cover 64 consecutive words).  The VALU kernel above spends ~1,800 VALU
// instructions per wave on the same work (PMC, profiles/r03_conv0_pmc.txt); here the per-pixel
// cost is 8 LDS reads and the epilogue.  Lane (li, lh) ends with pixel li and channels
// 8 (q / 4) + 4 lh + q % 4, so each lane stores four float4 channel runs of its pixel.
typedef float c1x16 __attribute__((ext_vector_type(16)));
constexpr int C1_MAXCO = 1024;
__global__ __launch_bounds__(256) void conv2d_c1_mfma_kernel(
    const float* __restrict__ x, int H, int W, const float* __restrict__ packed, const float* __restrict__ bias,
    int Co, int stride, int ph, int pw, const float* __restrict__ bn_w,
    const float* __restrict__ bn_b, const float* __restrict__ bn_rm, const float* __restrict__ bn_rv,
    float bn_eps, int act, float slope, float* __restrict__ y, int Hout, int Wout, int w_lo, int w_hi) {
  constexpr int kh = C1_K, kw = C1_K;
  __shared__ __attribute__((aligned(16))) float rows[C1_IN_ROWS][C1_MAXW];
  __shared__ __attribute__((aligned(16))) float e_sh[C1_MAXCO], e_sc[C1_MAXCO], e_bo[C1_MAXCO];
  const int rb = (Hout + C1_ROWS - 1) / C1_ROWS;
  const int b = blockIdx.x / rb, ho0 = (blockIdx.x % rb) * C1_ROWS;
  const int nr = min(C1_ROWS, Hout - ho0);
  const int tid = threadIdx.x;
  const int c0 = w_lo * stride - pw, nc = (w_hi - 1 - w_lo) * stride + kw;
  const int nin = (nr - 1) * stride + kh;
  constexpr int C1_PRE = 8;
  {
    float pv[C1_PRE];
    bool ok[C1_PRE];
#pragma unroll
    for (int u = 0; u < C1_PRE; ++u) {
      const int idx = tid + u * 256;
      const int i = idx / nc, c = idx - (idx / nc) * nc;
      const int hi = ho0 * stride - ph + i, wi = c0 + c;
      ok[u] = idx < nin * nc && hi >= 0 && hi < H && wi >= 0 && wi < W;
      pv[u] = x[ok[u] ? ((int64_t)b * H + hi) * W + wi : 0];
    }
#pragma unroll
    for (int u = 0; u < C1_PRE; ++u) {
      const int idx = tid + u * 256;
      if (idx < nin * nc) rows[idx / nc][idx % nc] = ok[u] ? pv[u] : 0.f;
    }
  }
  for (int idx = tid + C1_PRE * 256; idx < nin * nc; idx += blockDim.x) {
    const int i = idx / nc, c = idx % nc;
    const int hi = ho0 * stride - ph + i, wi = c0 + c;
    rows[i][c] = (hi >= 0 && hi < H && wi >= 0 && wi < W) ? x[((int64_t)b * H + hi) * W + wi] : 0.f;
  }
  // per-channel epilogue (conv2d_c1_kernel's order): (acc + (bias - rm)) * (w / sqrt(rv + eps)) + b
  for (int co = tid; co < Co; co += blockDim.x) {
    const float bi = bias ? bias[co] : 0.f;
    if (bn_w) {
      e_sh[co] = bi - bn_rm[co];
      e_sc[co] = bn_w[co] / sqrtf(bn_rv[co] + bn_eps);
      e_bo[co] = bn_b[co];
    } else {
      e_sh[co] = bi;
      e_sc[co] = 1.f;
      e_bo[co] = 0.f;
    }
  }
  __syncthreads();
  const int lane = tid & 63, wave = tid >> 6, li = lane & 31, lh = lane >> 5;
  const int Wn = w_hi - w_lo, npix = nr * Wn, npt = (npix + 31) / 32, nct = Co / 32;
  float a[8];
  int cur = -1;
  for (int job = wave; job < npt * nct; job += 4) {
    const int ct = job % nct, pt = job / nct;
    if (ct != cur) {   // wave-uniform: this channel tile's taps, A[m = li][k = 2 s + lh]
      const float* wp = packed + (ct * 32 + li) * (kh * kw) + lh;
#pragma unroll
      for (int st = 0; st < 8; ++st) a[st] = wp[2 * st];
      cur = ct;
    }
    const int p = pt * 32 + li;
    const bool valid = p < npix;
    const int pr = valid ? p / Wn : 0, pc = valid ? p - pr * Wn : 0;
    const float* rp = &rows[pr * stride][pc * stride];
    c1x16 acc;
#pragma unroll
    for (int q = 0; q < 16; ++q) acc[q] = 0.f;
#pragma unroll
    for (int st = 0; st < 8; ++st) {
      const int k = 2 * st + lh;
      acc = __builtin_amdgcn_mfma_f32_32x32x2f32(a[st], rp[(k / kw) * C1_MAXW + (k % kw)], acc, 0, 0, 0);
    }
    if (!valid) continue;
    float* yp = y + (((int64_t)b * Hout + ho0 + pr) * Wout + w_lo + pc) * Co + ct * 32 + 4 * lh;
#pragma unroll
    for (int g = 0; g < 4; ++g) {
      const int ch0 = ct * 32 + 8 * g + 4 * lh;
      const float4 sh4 = *reinterpret_cast<const float4*>(&e_sh[ch0]);
      const float4 sc4 = *reinterpret_cast<const float4*>(&e_sc[ch0]);
      const float4 bo4 = *reinterpret_cast<const float4*>(&e_bo[ch0]);
      const float shq[4] = {sh4.x, sh4.y, sh4.z, sh4.w}, scq[4] = {sc4.x, sc4.y, sc4.z, sc4.w};
      const float boq[4] = {bo4.x, bo4.y, bo4.z, bo4.w};
      float o[4];
#pragma unroll
      for (int q = 0; q < 4; ++q) {
        float v = (acc[4 * g + q] + shq[q]) * scq[q] + boq[q];
        if (act == ACT_RELU) v = v > 0.f ? v : 0.f;
        else if (act == ACT_LRELU) v = v > 0.f ? v : v * slope;
        else if (act == ACT_SIGMOID) v = 1.f / (1.f + expf(-v));
        o[q] = v;
      }
      *reinterpret_cast<float4*>(yp + 8 * g) = make_float4(o[0], o[1], o[2], o[3]);
    }
  }
}

extern "C" {

int a2m_conv2d_nhwc_fwd_f32(const float* x, int32_t B, int32_t Ci, int32_t H, int32_t W,
                            const float* packed, const float* bias, int32_t Co, int32_t kh,
                            int32_t kw, int32_t stride, int32_t pad_h, int32_t pad_w,
                            const float* bn_w, const float* bn_b, const float* bn_rm,
                            const float* bn_rv, float bn_eps, int32_t act, float slope, float* y,
                            int32_t y_nhwc, int32_t Hout, int32_t Wout, int32_t w_lo, int32_t w_hi,
                            void* ws, size_t ws_bytes, void* stream) {
  A2M_CHECK_ARG(x && packed && y, "conv2d_nhwc: null pointer");
  A2M_CHECK_ARG(B > 0 && Ci > 0 && Co > 0 && kh > 0 && kw > 0 && stride > 0,
                "conv2d_nhwc: bad shape");
  A2M_CHECK_ARG(Hout == (H + 2 * pad_h - kh) / stride + 1 && Wout == (W + 2 * pad_w - kw) / stride + 1,
                "conv2d_nhwc: output geometry mismatch");
  A2M_CHECK_ARG(0 <= w_lo && w_lo < w_hi && w_hi <= Wout, "conv2d_nhwc: bad column range [%d,%d)",
                w_lo, w_hi);
  A2M_CHECK_ARG((kw * Ci) % 4 == 0 && (reinterpret_cast<uintptr_t>(x) % 4) == 0,
                "conv2d_nhwc: kw * Ci = %d must be a multiple of 4", kw * Ci);
  A2M_CHECK_ARG(fits32((int64_t)B * Ci * H * W) && fits32((int64_t)B * Co * Hout * Wout),
                "conv2d_nhwc: too large");
  if (Ci == 1 && kh == C1_K && kw == C1_K && stride <= 2 && Co % 4 == 0 && Co <= 1024 &&
      (w_hi - 1 - w_lo) * stride + kw <= C1_MAXW && reinterpret_cast<uintptr_t>(packed) % 16 == 0 &&
      (!y_nhwc || reinterpret_cast<uintptr_t>(y) % 16 == 0)) {
    static const int c1_mfma = std::getenv("A2M_C1_MFMA") ? std::atoi(std::getenv("A2M_C1_MFMA")) : 1;
    if (c1_mfma && y_nhwc && Co % 32 == 0 && Co <= C1_MAXCO) {
      hipLaunchKernelGGL(conv2d_c1_mfma_kernel, dim3((unsigned)(B * cdiv(Hout, C1_ROWS))), dim3(256), 0,
                         as_stream(stream), x, H, W, packed, bias, Co, stride, pad_h, pad_w, bn_w, bn_b,
                         bn_rm, bn_rv, bn_eps, act, slope, y, Hout, Wout, w_lo, w_hi);
      A2M_LAUNCH_CHECK();
      return A2M_OK;
    }
    hipLaunchKernelGGL(conv2d_c1_kernel, dim3((unsigned)(B * cdiv(Hout, C1_ROWS))), dim3(256), 0,
                       as_stream(stream), x, H, W,
                       packed, bias, Co, stride, pad_h, pad_w, bn_w, bn_b, bn_rm, bn_rv, bn_eps, act,
                       slope, y, y_nhwc, Hout, Wout, w_lo, w_hi);
    A2M_LAUNCH_CHECK();
    return A2M_OK;
  }
  const int Wn = w_hi - w_lo;
  Epilogue E{};
  if (y_nhwc) {
    E = epi_bn(y + (int64_t)w_lo * Co, bias, bn_w, bn_b, bn_rm, bn_rv, bn_eps, act, slope);
    E.N1 = Hout; E.N2 = Wn; E.so0 = Hout * Wout * Co; E.so1 = Wout * Co; E.so2 = Co; E.som = 1;
  } else {
    E = epi_bn(y + w_lo, bias, bn_w, bn_b, bn_rm, bn_rv, bn_eps, act, slope);
    E.N1 = Hout; E.N2 = Wn; E.so0 = Co * Hout * Wout; E.so1 = Wout; E.so2 = 1; E.som = Hout * Wout;
  }
  return conv2d_nhwc_gemm(x, B, Ci, H, W, packed, Co, kh, kw, stride, pad_h, pad_w, Hout, w_lo, Wn, E,
                          ws, ws_bytes, as_stream(stream));
}

// The encoder's last ConvNormRelu (one live output column w_col) with the bilinear time
// resample fused into the GEMM's reduce (gemm.hip splitk_reduce_interp_kernel): y [B][Co][T] is
// a2m_conv2d_nhwc_fwd_f32 (y_nhwc = 0, columns [w_col, w_col + 1)) followed by
// a2m_interp_time_f32, bit for bit, in one GEMM launch and one reduce launch.
int a2m_conv2d_nhwc_interp_fwd_f32(const float* x, int32_t B, int32_t Ci, int32_t H, int32_t W,
                                   const float* packed, const float* bias, int32_t Co, int32_t kh,
                                   int32_t kw, int32_t stride, int32_t pad_h, int32_t pad_w,
                                   const float* bn_w, const float* bn_b, const float* bn_rm,
                                   const float* bn_rv, float bn_eps, int32_t act, float slope,
                                   float* y, int32_t T, int32_t Hout, int32_t Wout, int32_t w_col,
                                   void* ws, size_t ws_bytes, void* stream) {
  A2M_CHECK_ARG(x && packed && y, "conv2d_nhwc_interp: null pointer");
  A2M_CHECK_ARG(B > 0 && Ci > 0 && Co > 0 && kh > 0 && kw > 0 && stride > 0 && T > 0,
                "conv2d_nhwc_interp: bad shape");
  A2M_CHECK_ARG(Hout == (H + 2 * pad_h - kh) / stride + 1 && Wout == (W + 2 * pad_w - kw) / stride + 1,
                "conv2d_nhwc_interp: output geometry mismatch");
  A2M_CHECK_ARG((kw * Ci) % 4 == 0 && (reinterpret_cast<uintptr_t>(x) % 4) == 0,
                "conv2d_nhwc_interp: kw * Ci = %d must be a multiple of 4", kw * Ci);
  A2M_CHECK_ARG(fits32((int64_t)B * Ci * H * W) && fits32((int64_t)B * Co * T) && fits32((int64_t)B * Co * Hout),
                "conv2d_nhwc_interp: too large");
  // the resample's column weights (interp_time_kernel): w_col must be its only live column
  float srcw = (float)Wout * 0.5f - 0.5f;
  srcw = srcw < 0.f ? 0.f : srcw;
  const int w0 = (int)srcw;
  const float lw1 = srcw - (float)w0;
  A2M_CHECK_ARG(w0 == w_col && lw1 == 0.f,
                "conv2d_nhwc_interp: column %d is not the resample's only live column (Wout %d)", w_col, Wout);
  Epilogue E = epi_bn(y, bias, bn_w, bn_b, bn_rm, bn_rv, bn_eps, act, slope);
  E.N1 = Hout; E.N2 = 1; E.so0 = 0; E.so1 = 0; E.so2 = 0; E.som = 0;
  E.interp_T = T;
  E.interp_H = Hout;
  E.interp_lw0 = 1.f - lw1;
  return conv2d_nhwc_gemm(x, B, Ci, H, W, packed, Co, kh, kw, stride, pad_h, pad_w, Hout, w_col, 1, E,
                          ws, ws_bytes, as_stream(stream));
}

int a2m_mean_time_f32(const float* x, int64_t xs_b, int64_t xs_c, int32_t B, int32_t C,
                      int32_t T, float scale, float* y, void* stream) {
  A2M_CHECK_ARG(x && y && B > 0 && C > 0 && T > 0, "mean_time: bad args");
  const int BC = B * C;
  hipLaunchKernelGGL(mean_time_kernel, dim3((unsigned)cdiv(BC, 4)), dim3(256), 0,
                     as_stream(stream), x, xs_b, xs_c, C, T, BC, scale, y);
  A2M_LAUNCH_CHECK();
  return A2M_OK;
}

int a2m_repeat_time_f32(const float* x, int32_t B, int32_t C, int32_t T, float scale, float* y,
                        int64_t ys_b, int64_t ys_c, void* stream) {
  A2M_CHECK_ARG(x && y && B > 0 && C > 0 && T > 0, "repeat_time: bad args");
  const int64_t total = (int64_t)B * C * T;
  const int blocks = (int)std::min<int64_t>(cdiv(total, 256), 4096);
  hipLaunchKernelGGL(repeat_time_kernel, dim3(blocks), dim3(256), 0, as_stream(stream), x, C, T,
                     total, scale, y, ys_b, ys_c);
  A2M_LAUNCH_CHECK();
  return A2M_OK;
}

int a2m_interp_time_f32(const float* x, int32_t B, int32_t C, int32_t H, int32_t W, float* y,
                        int32_t T, void* stream) {
  A2M_CHECK_ARG(x && y && B > 0 && C > 0 && H > 0 && W > 0 && T > 0, "interp: bad args");
  const int vec = (T & 3) == 0 && (reinterpret_cast<uintptr_t>(y) & 15) == 0 &&
                  (int64_t)B * C * T < (1LL << 31);
  const int64_t total = (int64_t)B * C * T / (vec ? 4 : 1);
  const int blocks = (int)std::min<int64_t>(cdiv(total, 256), 8192);
  hipLaunchKernelGGL(interp_time_kernel, dim3(blocks), dim3(256), 0, as_stream(stream), x, B, C,
                     H, W, y, T, vec);
  A2M_LAUNCH_CHECK();
  return A2M_OK;
}

size_t a2m_self_attention_ws_bytes(int32_t B, int32_t C, int32_t T) {
  const int Cq = C / 8;
  size_t s = 0;
  s = std::max(s, gemm_ws_bytes(Cq, B * T, C, 1));
  s = std::max(s, gemm_ws_bytes(C, B * T, C, 1));
  s = std::max(s, gemm_ws_bytes(T, T, Cq, B));
  s = std::max(s, gemm_ws_bytes(C, T, T, B));
  return s;
}

int a2m_stack_qkv_f32(const float* wq, const float* bq, const float* wk, const float* bk,
                      const float* wv, const float* bv, int32_t C, float* wqkv, float* bqkv,
                      void* stream) {
  A2M_CHECK_ARG(wq && wk && wv && wqkv && bqkv && C >= 8 && C % 8 == 0, "stack_qkv: bad args");
  return stack_qkv(wq, bq, wk, bk, wv, bv, C, wqkv, bqkv, as_stream(stream));
}

int a2m_self_attention_packed_fwd_f32(const float* x, int64_t x_bs, int32_t B, int32_t C,
                                      int32_t T, const float* wqkv, const float* bqkv,
                                      const float* gamma, const float* res, float* y, int64_t y_bs,
                                      float* qkv, float* attn, void* ws, size_t ws_bytes,
                                      void* stream) {
  A2M_CHECK_ARG(x && wqkv && bqkv && gamma && y && qkv && attn, "self_attention: null pointer");
  A2M_CHECK_ARG(B > 0 && C >= 8 && C % 8 == 0 && T > 0, "self_attention: bad shape C=%d T=%d", C, T);
  A2M_CHECK_ARG(x_bs == y_bs, "self_attention: x and y must share a layout");
  A2M_CHECK_ARG(fits32((int64_t)B * x_bs) && fits32((int64_t)B * (C + C / 4) * T) &&
                    fits32((int64_t)B * T * T),
                "self_attention: too large");
  hipStream_t st = as_stream(stream);
  const int Cq = C / 8, Cqkv = C / 4 + C;
  const int64_t qs_b = (int64_t)Cqkv * T;
  // q, k, v as ONE 1x1 convolution with the stacked weights: qkv[b][0:Cq | Cq:2Cq | 2Cq:][t]
  int rc;
#ifndef A2M_WIDE_BTC
#define A2M_WIDE_BTC 2   // 0 never, 1 always, 2 in the bf16 operand mode only
#endif
  if ((A2M_WIDE_BTC == 1 || (A2M_WIDE_BTC == 2 && a2m_get_gemm_precision() != 0)) && C >= 1024 &&
      T <= TR_MAXT) {
    // wide channels (the UNet's SelfAttention(2048)) in bf16 mode: x is first copied to [B*T][C]
    // so the projection GEMM reads both operands as dense k-contiguous rows instead of gathering
    // x's t-runs (mode 3).  Round 6, with the pipelined tiles: the bf16 step 1.293 vs 1.494 ms
    // without the copy, the fp32 step 2.257 vs 2.242 ms (the fp32 pipelined tile gathers the
    // t-runs well), so fp32 skips it (profiles/r06_q_wide_btc_ab.txt).  Same k order either way,
    // so the same result bit for bit.
    const size_t xt_bytes = (((size_t)B * T * C * sizeof(float)) + 255) & ~size_t(255);
    const size_t need = xt_bytes + gemm_ws_bytes(Cqkv, B * T, C, 1);
    if (!ws || ws_bytes < need) {
      set_error("self_attention: workspace too small (%zu < %zu bytes)", ws_bytes, need);
      return A2M_EWS;
    }
    float* xt = static_cast<float*>(ws);
    hipLaunchKernelGGL(bct_to_btc_kernel, dim3((unsigned)cdiv(C, TR_C), (unsigned)B), dim3(256), 0, st,
                       x, x_bs, C, T, xt);
    A2M_LAUNCH_CHECK();
    Gather A = dense_rk(wqkv, C);
    Gather Bx = dense_rk(xt, C);
    Epilogue E = epi_bn(qkv, bqkv, nullptr, nullptr, nullptr, nullptr, 1e-5f, A2M_ACT_NONE, 0.f);
    E.N1 = 1; E.N2 = T; E.so0 = (int)qs_b; E.so1 = 0; E.so2 = 1; E.som = T;
    rc = gemm(A, Bx, E, Cqkv, B * T, C, 1, static_cast<char*>(ws) + xt_bytes, ws_bytes - xt_bytes, st);
  } else {
    rc = a2m_conv1d_fwd_f32(x, x_bs, T, 1, B, C, T, wqkv, bqkv, Cqkv, 1, 1, 0, nullptr, nullptr,
                            nullptr, nullptr, 0.f, A2M_ACT_NONE, 0.f, qkv, qs_b, T, 1, ws,
                            ws_bytes, stream);
  }
  if (rc) return rc;
  if (attn_core_fits(C, T))
    return attn_core(qkv, qs_b, B, C, T, gamma, x, x_bs, res, y, attn, st);
  if (attn_core_wide_fits(C, T))   // the UNet's / D's SelfAttention(2048), T <= 32
    return attn_core_wide(qkv, qs_b, B, C, T, gamma, x, x_bs, res, y, attn, st);
  // scores[b][i][j] = sum_c q[b][c][i] k[b][c][j]
  Gather Aq = dense_kr(qkv, T, qs_b);
  Gather Bk = dense_kr(qkv + (int64_t)Cq * T, T, qs_b);
  Epilogue Es = epi_dense(attn, T, (int64_t)T * T);
  rc = gemm(Aq, Bk, Es, T, T, Cq, B, ws, ws_bytes, st);
  if (rc) return rc;
  rc = softmax_rows(attn, B * T, T, st);
  if (rc) return rc;
  // y[b][c][i] = gamma * sum_j v[b][c][j] attn[b][i][j] + x[b][c][i] (+ res)
  Gather Av = dense_rk(qkv + (int64_t)2 * Cq * T, T, qs_b);
  Gather Ba = dense_rk(attn, T, (int64_t)T * T);
  Epilogue Eo = epi_dense(y, T, y_bs);
  Eo.gamma = gamma;
  Eo.res1 = x;
  Eo.res2 = res;
  return gemm(Av, Ba, Eo, C, T, T, B, ws, ws_bytes, st);
}

int a2m_bct_to_btc_f32(const float* x, int64_t xs_b, int32_t B, int32_t C, int32_t T, float* y,
                       void* stream) {
  A2M_CHECK_ARG(x && y && B > 0 && C > 0 && T > 0 && T <= TR_MAXT && xs_b >= (int64_t)C * T,
                "bct_to_btc: bad shape (T <= %d)", TR_MAXT);
  A2M_CHECK_ARG(fits32((int64_t)B * xs_b) && fits32((int64_t)B * T * C), "bct_to_btc: too large");
  hipLaunchKernelGGL(bct_to_btc_kernel, dim3((unsigned)cdiv(C, TR_C), (unsigned)B), dim3(256), 0,
                     as_stream(stream), x, xs_b, C, T, y);
  A2M_LAUNCH_CHECK();
  return A2M_OK;
}

int32_t a2m_self_attention_eval_fits(int32_t C, int32_t T) { return attn_fused_eval_fits(C, T) ? 1 : 0; }

int a2m_self_attention_eval_group_f32(const float* x, int64_t x_gs, int64_t x_bs, int32_t G, int32_t B,
                                      int32_t C, int32_t T, const float* wqkv, const float* bqkv,
                                      const float* gamma, const float* res, int64_t res_gs, float* y,
                                      int64_t y_gs, void* stream) {
  A2M_CHECK_ARG(x && wqkv && bqkv && gamma && y && B > 0 && G > 0, "self_attention_eval_group: null pointer");
  A2M_CHECK_ARG(attn_fused_eval_fits(C, T), "self_attention_eval_group: C=%d T=%d not supported", C, T);
  A2M_CHECK_ARG(x_bs % 4 == 0 && x_gs % 4 == 0 && y_gs % 4 == 0 && res_gs % 4 == 0 &&
                    (reinterpret_cast<uintptr_t>(x) & 15) == 0,
                "self_attention_eval_group: x / y layout");
  A2M_CHECK_ARG(fits32((int64_t)B * x_bs), "self_attention_eval_group: too large");
  return attn_fused_eval(x, x_bs, B, C, T, wqkv, bqkv, gamma, res, y, as_stream(stream), G, x_gs,
                         res_gs, y_gs);
}

int a2m_self_attention_eval_f32(const float* x, int64_t x_bs, int32_t B, int32_t C, int32_t T,
                                const float* wqkv, const float* bqkv, const float* gamma,
                                const float* res, float* y, int64_t y_bs, void* stream) {
  A2M_CHECK_ARG(x && wqkv && bqkv && gamma && y && B > 0, "self_attention_eval: null pointer");
  A2M_CHECK_ARG(attn_fused_eval_fits(C, T), "self_attention_eval: C=%d T=%d not supported (C in {128, 256}, T <= 64, T %% 4 == 0)", C, T);
  A2M_CHECK_ARG(x_bs == y_bs && x_bs % 4 == 0 && (reinterpret_cast<uintptr_t>(x) & 15) == 0,
                "self_attention_eval: x / y layout (batch stride %lld)", (long long)x_bs);
  A2M_CHECK_ARG(fits32((int64_t)B * x_bs), "self_attention_eval: too large");
  return attn_fused_eval(x, x_bs, B, C, T, wqkv, bqkv, gamma, res, y, as_stream(stream));
}

int a2m_self_attention_eval_ex_f32(const float* x, int64_t x_bs, int32_t B, int32_t C, int32_t T,
                                   const float* wqkv, const float* bqkv, const float* gamma,
                                   const float* res, float* y, int64_t y_bs, const void* wqkv_h,
                                   void* stream) {
  A2M_CHECK_ARG(x && wqkv && bqkv && gamma && y && B > 0, "self_attention_eval: null pointer");
  A2M_CHECK_ARG(attn_fused_eval_fits(C, T), "self_attention_eval: C=%d T=%d not supported (C in {128, 256}, T <= 64, T %% 4 == 0)", C, T);
  A2M_CHECK_ARG(x_bs == y_bs && x_bs % 4 == 0 && (reinterpret_cast<uintptr_t>(x) & 15) == 0,
                "self_attention_eval: x / y layout (batch stride %lld)", (long long)x_bs);
  A2M_CHECK_ARG(fits32((int64_t)B * x_bs), "self_attention_eval: too large");
  return attn_fused_eval(x, x_bs, B, C, T, wqkv, bqkv, gamma, res, y, as_stream(stream), 1, 0, 0, 0, wqkv_h);
}

int a2m_self_attention_fwd_f32(const float* x, int64_t x_bs, int32_t B, int32_t C, int32_t T,
                               const float* wq, const float* bq, const float* wk, const float* bk,
                               const float* wv, const float* bv, const float* gamma,
                               const float* res, float* y, int64_t y_bs, float* qkv,
                               float* attn, void* ws, size_t ws_bytes, void* stream) {
  A2M_CHECK_ARG(x && wq && wk && wv && gamma && y && qkv && attn, "self_attention: null pointer");
  A2M_CHECK_ARG(C >= 8 && C % 8 == 0, "self_attention: bad shape C=%d T=%d", C, T);
  // the three weights stacked in the workspace head, then the packed path
  const int Cqkv = C / 4 + C;
  const size_t wcat_bytes = (((size_t)Cqkv * C + Cqkv) * sizeof(float) + 255) & ~size_t(255);
  if (!ws || ws_bytes < wcat_bytes) {
    set_error("self_attention: workspace too small (%zu < %zu bytes)", ws_bytes, wcat_bytes);
    return A2M_EWS;
  }
  float* wcat = static_cast<float*>(ws);
  float* bcat = wcat + (size_t)Cqkv * C;
  int rc = stack_qkv(wq, bq, wk, bk, wv, bv, C, wcat, bcat, as_stream(stream));
  if (rc) return rc;
  return a2m_self_attention_packed_fwd_f32(x, x_bs, B, C, T, wcat, bcat, gamma, res, y, y_bs, qkv,
                                           attn, static_cast<char*>(ws) + wcat_bytes,
                                           ws_bytes - wcat_bytes, stream);
}

int a2m_channel_attention_fwd_f32(const float* x, int32_t B, int32_t C, int32_t T,
                                  const float* w1, const float* b1, int32_t Cr, const float* w2,
                                  const float* b2, float* y, float* att_out, void* stream) {
  A2M_CHECK_ARG(x && w1 && b1 && w2 && b2 && y && att_out && B > 0 && C > 0 && Cr > 0 && T > 0,
                "channel_attention: bad args");
  const size_t lds = sizeof(float) * (2 * (size_t)C + 2 * Cr);
  A2M_CHECK_ARG(lds <= 64 * 1024, "channel_attention: C too large");
  hipStream_t st = as_stream(stream);
  const bool al16 = ((reinterpret_cast<uintptr_t>(x) | reinterpret_cast<uintptr_t>(y) |
                      reinterpret_cast<uintptr_t>(w1) | reinterpret_cast<uintptr_t>(w2)) & 15) == 0;
  if (A2M_CA_FUSED && C == 256 && Cr == 32 && T == 64 && al16) {
    hipLaunchKernelGGL(channel_att_fused256_kernel, dim3(B), dim3(256), 0, st, x, w1, b1, w2, b2,
                       att_out, y);
    A2M_LAUNCH_CHECK();
    return A2M_OK;
  }
  hipLaunchKernelGGL(channel_att_weights_kernel, dim3(B), dim3(256), lds, st, x, C, T, w1, b1, Cr,
                     w2, b2, att_out);
  A2M_LAUNCH_CHECK();
  const int64_t n = (int64_t)B * C * T;
  const int blocks = (int)std::min<int64_t>(cdiv(n / 4 + 1, 256), 2048);
  hipLaunchKernelGGL(channel_scale_kernel, dim3(blocks), dim3(256), 0, st, x, att_out, T, n, y);
  A2M_LAUNCH_CHECK();
  return A2M_OK;
}

int a2m_layernorm_fwd_f32(const float* x, int32_t R, int32_t D, const float* w, const float* b,
                          float eps, float* y, int32_t T, int64_t ys_b, int64_t ys_d,
                          int64_t ys_t, float* mean_out, float* rstd_out, void* stream) {
  A2M_CHECK_ARG(x && w && b && y && R >= 0 && D > 0 && D <= 512 && T > 0, "layernorm: bad args");
  if (R == 0) return A2M_OK;
  hipLaunchKernelGGL(layernorm_kernel, dim3((unsigned)cdiv(R, 4)), dim3(256), 0,
                     as_stream(stream), x, R, D, w, b, eps, y, T, ys_b, ys_d, ys_t, mean_out,
                     rstd_out);
  A2M_LAUNCH_CHECK();
  return A2M_OK;
}

}  // extern "C"
