// Backward of SelfAttention (model_layers.py:121-146) and ChannelAttention (:149-174).
//
// SelfAttention: y = gamma*O + x (+res), O = V A^T, A = softmax(Q^T K).  With
// G = dy^T V (per batch, [T][T]):
//   dgamma = sum A (.) G,   dS = gamma * A (.) (G - rowsum(A (.) G))   (softmax backward)
//   dV = gamma * dy A,      dQ = K dS^T,      dK = Q dS,     dx = dy + [Wq;Wk;Wv]^T [dQ;dK;dV]
//   d[Wq;Wk;Wv] = [dQ;dK;dV] x^T (sum over b,t),  d[bq;bk;bv] = sum_{b,t} [dQ;dK;dV]
// All products run on the MFMA implicit-GEMM engine; the softmax backward and the row
// reductions are wave64 kernels.
#include <algorithm>

#include "a2m_internal.h"

namespace a2m {

// in place: G -> dS, rowdot[b*T+i] = sum_j A_ij G_ij
__global__ __launch_bounds__(256) void attn_softmax_bwd_kernel(const float* attn, float* g, int rows,
                                                               int T, const float* gamma,
                                                               float* rowdot) {
  const int row = blockIdx.x * 4 + (threadIdx.x >> 6);
  const int lane = threadIdx.x & 63;
  if (row >= rows) return;
  const float* a = attn + (int64_t)row * T;
  float* gr = g + (int64_t)row * T;
  float s = 0.f;
  for (int j = lane; j < T; j += 64) s += a[j] * gr[j];
  s = wave64_sum(s);
  const float gm = gamma[0];
  for (int j = lane; j < T; j += 64) gr[j] = gm * a[j] * (gr[j] - s);
  if (lane == 0) rowdot[row] = s;
}

__global__ __launch_bounds__(256) void sum_vector_kernel(const float* x, int n, float* out,
                                                         int accumulate) {
  __shared__ double red[4];
  double s = 0.0;
  for (int i = threadIdx.x; i < n; i += blockDim.x) s += x[i];
  for (int o = 32; o > 0; o >>= 1) s += __shfl_xor(s, o);
  if ((threadIdx.x & 63) == 0) red[threadIdx.x >> 6] = s;
  __syncthreads();
  if (threadIdx.x == 0) {
    const double t = red[0] + red[1] + red[2] + red[3];
    out[0] = (float)(accumulate ? out[0] + t : t);
  }
}

// ChannelAttention backward, one workgroup of 512 threads per batch element; weight-gradient
// partials per batch element go to part[b][W1 (Cr*C) | b1 (Cr) | W2 (C*Cr) | b2 (C)].
// The reductions over channels / time run on groups of 8 lanes (strided partial sums, then
// three xor shuffles), so every phase keeps all waves busy instead of one thread per output.
constexpr int CAB_NT = 512, CAB_G = 8;
__device__ __forceinline__ float group8_sum(float v) {
  v += __shfl_xor(v, 1);
  v += __shfl_xor(v, 2);
  return v + __shfl_xor(v, 4);
}
__global__ __launch_bounds__(CAB_NT) void channel_attention_bwd_kernel(
    const float* dy, const float* x, int C, int T, const float* w1, const float* b1, int Cr,
    const float* w2, const float* b2, float* dx, float* part) {
  extern __shared__ __attribute__((aligned(16))) float sm[];
  float* pavg = sm;              // C
  float* pmax = pavg + C;        // C
  int* amax = reinterpret_cast<int*>(pmax + C);  // C
  float* h = reinterpret_cast<float*>(amax + C); // 2*Cr
  float* s = h + 2 * Cr;         // 2*C (sigmoids)
  float* dz = s + 2 * C;         // 2*C
  float* dh = dz + 2 * C;        // 2*Cr
  float* dpool = dh + 2 * Cr;    // 2*C (davg, dmax)
  float* att = dpool + 2 * C;    // C
  const int b = blockIdx.x;
  const float* xb = x + (int64_t)b * C * T;
  const float* gb = dy + (int64_t)b * C * T;
  const int tid = threadIdx.x, gl = tid & (CAB_G - 1), grp = tid / CAB_G;
  constexpr int NGRP = CAB_NT / CAB_G;
  const int P = 2 * Cr * C + Cr + C;
  float* pb = part + (int64_t)b * P;
  // pooled stats (first-occurrence argmax, like ATen's adaptive max pool) and da = sum dy*x:
  // one 8-lane group per channel, lane g over t = g, g + 8, ...
  for (int c = grp; c < C; c += NGRP) {
    const float* p = xb + (int64_t)c * T;
    const float* q = gb + (int64_t)c * T;
    float sm_ = 0.f, mx = -INFINITY, da = 0.f;
    int ai = T;
    for (int t = gl; t < T; t += CAB_G) {
      const float v = p[t];
      sm_ += v;
      da += v * q[t];
      if (v > mx) { mx = v; ai = t; }
    }
#pragma unroll
    for (int o = 1; o < CAB_G; o <<= 1) {
      sm_ += __shfl_xor(sm_, o);
      da += __shfl_xor(da, o);
      const float om = __shfl_xor(mx, o);
      const int oi = __shfl_xor(ai, o);
      if (om > mx || (om == mx && oi < ai)) { mx = om; ai = oi; }
    }
    if (gl == 0) {
      pavg[c] = sm_ / (float)T;
      pmax[c] = mx;
      amax[c] = ai;
      dpool[c] = da;  // temporarily holds da
    }
  }
  __syncthreads();
  // h = relu(W1 pooled + b1) for both pools: one 8-lane group per output
  for (int j = grp; j < 2 * Cr; j += NGRP) {
    const int r = j % Cr;
    const float* in = j < Cr ? pavg : pmax;
    float a = 0.f;
    for (int c = gl; c < C; c += CAB_G) a += w1[(int64_t)r * C + c] * in[c];
    a = group8_sum(a) + b1[r];
    if (gl == 0) h[j] = a > 0.f ? a : 0.f;
  }
  __syncthreads();
  for (int c = tid; c < C; c += CAB_NT) {
    float a0 = b2[c], a1 = b2[c];
    for (int r = 0; r < Cr; ++r) {
      a0 += w2[(int64_t)c * Cr + r] * h[r];
      a1 += w2[(int64_t)c * Cr + r] * h[Cr + r];
    }
    const float s0 = 1.f / (1.f + expf(-a0)), s1 = 1.f / (1.f + expf(-a1));
    s[c] = s0;
    s[C + c] = s1;
    att[c] = s0 + s1;
    const float da = dpool[c];
    dz[c] = da * s0 * (1.f - s0);
    dz[C + c] = da * s1 * (1.f - s1);
  }
  __syncthreads();
  // dW2[c][r] = dz1[c] h1[r] + dz2[c] h2[r]; db2[c] = dz1 + dz2
  for (int i = tid; i < C * Cr; i += CAB_NT) {
    const int c = i / Cr, r = i - c * Cr;
    pb[Cr * C + Cr + i] = dz[c] * h[r] + dz[C + c] * h[Cr + r];
  }
  for (int c = tid; c < C; c += CAB_NT) pb[2 * Cr * C + Cr + c] = dz[c] + dz[C + c];
  // dh = W2^T dz * relu'
  for (int j = grp; j < 2 * Cr; j += NGRP) {
    const int r = j % Cr;
    const float* d = j < Cr ? dz : dz + C;
    float a = 0.f;
    for (int c = gl; c < C; c += CAB_G) a += w2[(int64_t)c * Cr + r] * d[c];
    a = group8_sum(a);
    if (gl == 0) dh[j] = h[j] > 0.f ? a : 0.f;
  }
  __syncthreads();
  // dW1[r][c] = dh1[r] avg[c] + dh2[r] max[c]; db1[r] = dh1 + dh2; dpool = W1^T dh
  for (int i = tid; i < Cr * C; i += CAB_NT) {
    const int r = i / C, c = i - r * C;
    pb[i] = dh[r] * pavg[c] + dh[Cr + r] * pmax[c];
  }
  for (int r = tid; r < Cr; r += CAB_NT) pb[Cr * C + r] = dh[r] + dh[Cr + r];
  for (int c = tid; c < C; c += CAB_NT) {
    float a0 = 0.f, a1 = 0.f;
    for (int r = 0; r < Cr; ++r) {
      a0 += w1[(int64_t)r * C + c] * dh[r];
      a1 += w1[(int64_t)r * C + c] * dh[Cr + r];
    }
    dpool[c] = a0 / (float)T;
    dpool[C + c] = a1;
  }
  __syncthreads();
  float* db_ = dx + (int64_t)b * C * T;
  if ((T & 3) == 0) {   // float4 runs along t (rows start 16-byte aligned: C*T and T multiples of 4)
    const int n4 = C * T / 4;
    for (int i = tid; i < n4; i += CAB_NT) {
      const int c = (4 * i) / T, t = 4 * i - c * T;
      const float4 g = *reinterpret_cast<const float4*>(gb + 4 * (int64_t)i);
      const float at = att[c], dp = dpool[c], dm = dpool[C + c];
      const int am = amax[c] - t;
      float4 v;
      v.x = g.x * at + dp + (am == 0 ? dm : 0.f);
      v.y = g.y * at + dp + (am == 1 ? dm : 0.f);
      v.z = g.z * at + dp + (am == 2 ? dm : 0.f);
      v.w = g.w * at + dp + (am == 3 ? dm : 0.f);
      *reinterpret_cast<float4*>(db_ + 4 * (int64_t)i) = v;
    }
  } else {
    for (int i = tid; i < C * T; i += CAB_NT) {
      const int c = i / T, t = i - c * T;
      float v = gb[i] * att[c] + dpool[c];
      if (t == amax[c]) v += dpool[C + c];
      db_[i] = v;
    }
  }
}

}  // namespace a2m

using namespace a2m;

extern "C" {

size_t a2m_self_attention_bwd_ws_bytes(int32_t B, int32_t C, int32_t T) {
  const int Cqkv = C / 4 + C;
  size_t s = (((size_t)Cqkv * C + Cqkv) * 4 + 255) & ~size_t(255);       // stacked weights
  s += (((size_t)B * Cqkv * T) * 4 + 255) & ~size_t(255);                 // dqkv
  s += (((size_t)B * T * T + (size_t)B * T) * 4 + 255) & ~size_t(255);    // dS, rowdot
  size_t g = 0;
  g = std::max(g, gemm_ws_bytes(T, T, C, B));
  g = std::max(g, gemm_ws_bytes(C, T, T, B));
  g = std::max(g, gemm_ws_bytes(C / 8, T, T, B));
  g = std::max(g, gemm_ws_bytes(C, B * T, Cqkv, 1));
  g = std::max(g, gemm_ws_bytes(C, C, B * T, 1));
  g = std::max(g, gemm_ws_bytes(Cqkv, C, B * T, 1));
  g = std::max(g, gemm_ws_bytes(C / 8, C, B * T, 1));
  return s + g;
}

int a2m_self_attention_bwd_f32(const float* dy, const float* x, int64_t bs, int32_t B, int32_t C,
                               int32_t T, const float* wq, const float* bq, const float* wk,
                               const float* bk, const float* wv, const float* bv,
                               const float* gamma, const float* qkv, const float* attn, float* dx,
                               float* dwq, float* dbq, float* dwk, float* dbk, float* dwv,
                               float* dbv, float* dgamma, void* ws, size_t ws_bytes, void* stream) {
  A2M_CHECK_ARG(dy && x && wq && wk && wv && gamma && qkv && attn && dx && dwq && dwk && dwv && dgamma,
                "self_attention_bwd: null pointer");
  A2M_CHECK_ARG(B > 0 && C >= 8 && C % 8 == 0 && T > 0, "self_attention_bwd: bad shape");
  const size_t need = a2m_self_attention_bwd_ws_bytes(B, C, T);
  if (!ws || ws_bytes < need) {
    set_error("self_attention_bwd: workspace too small (%zu < %zu bytes)", ws_bytes, need);
    return A2M_EWS;
  }
  hipStream_t st = as_stream(stream);
  const int Cq = C / 8, Cqkv = C / 4 + C;
  const int64_t qs_b = (int64_t)Cqkv * T, TT = (int64_t)T * T;
  char* p = static_cast<char*>(ws);
  float* wcat = reinterpret_cast<float*>(p);
  float* bcat = wcat + (size_t)Cqkv * C;
  p += (((size_t)Cqkv * C + Cqkv) * 4 + 255) & ~size_t(255);
  float* dqkv = reinterpret_cast<float*>(p);
  p += (((size_t)B * Cqkv * T) * 4 + 255) & ~size_t(255);
  float* dS = reinterpret_cast<float*>(p);
  float* rowdot = dS + (size_t)B * TT;
  p += (((size_t)B * T * T + (size_t)B * T) * 4 + 255) & ~size_t(255);
  void* gws = p;
  const size_t gbytes = ws_bytes - (size_t)(p - static_cast<char*>(ws));
  int rc;
  // G[b][i][j] = sum_c dy[b][c][i] v[b][c][j]
  rc = gemm(dense_kr(dy, T, bs), dense_kr(qkv + 2 * Cq * T, T, qs_b), epi_dense(dS, T, TT), T, T, C, B,
            gws, gbytes, st);
  if (rc) return rc;
  hipLaunchKernelGGL(attn_softmax_bwd_kernel, dim3((unsigned)cdiv(B * T, 4)), dim3(256), 0, st, attn,
                     dS, B * T, T, gamma, rowdot);
  A2M_LAUNCH_CHECK();
  hipLaunchKernelGGL(sum_vector_kernel, dim3(1), dim3(256), 0, st, rowdot, B * T, dgamma, 0);
  A2M_LAUNCH_CHECK();
  // dV[b][c][j] = gamma * sum_i dy[b][c][i] A[b][i][j]
  Epilogue Ev = epi_dense(dqkv + 2 * Cq * T, T, qs_b);
  Ev.gamma = gamma;
  rc = gemm(dense_rk(dy, T, bs), dense_kr(attn, T, TT), Ev, C, T, T, B, gws, gbytes, st);
  if (rc) return rc;
  // dQ[b][c][i] = sum_j dS[i][j] k[b][c][j];  dK[b][c][j] = sum_i dS[i][j] q[b][c][i]
  rc = gemm(dense_rk(qkv + Cq * T, T, qs_b), dense_rk(dS, T, TT), epi_dense(dqkv, T, qs_b), Cq, T, T, B,
            gws, gbytes, st);
  if (rc) return rc;
  rc = gemm(dense_rk(qkv, T, qs_b), dense_kr(dS, T, TT), epi_dense(dqkv + Cq * T, T, qs_b), Cq, T, T, B,
            gws, gbytes, st);
  if (rc) return rc;
  // dx = dy + Wcat^T dqkv
  rc = stack_qkv(wq, bq, wk, bk, wv, bv, C, wcat, bcat, st);
  if (rc) return rc;
  Gather Aw = dense_kr(wcat, C);
  Epilogue Ex = epi_dense(dx, 0);
  Ex.N1 = 1; Ex.N2 = T; Ex.so0 = (int)bs; Ex.so2 = 1; Ex.som = T; Ex.res1 = dy;
  rc = gemm(Aw, gather_bct(dqkv, qs_b, T, T), Ex, C, B * T, Cqkv, 1, gws, gbytes, st);
  if (rc) return rc;
  // dW = dqkv x^T over (b, t), per segment
  Gather Bx{};
  Bx.base = x; Bx.sr0 = T; Bx.R1 = Bx.R2 = 1; Bx.sk0 = (int)bs; Bx.K1 = 1; Bx.K2 = T; Bx.bk2 = 1;
  Bx.sw = 1; Bx.Lw = T; Bx.Lh = 1; Bx.divh = Bx.divw = 1; Bx.kcontig = 1;
  float* dws[3] = {dwq, dwk, dwv};
  float* dbs[3] = {dbq, dbk, dbv};
  const int rows[3] = {Cq, Cq, C}, offs[3] = {0, Cq, 2 * Cq};
  // dwq|dwk|dwv (and dbq|dbk|dbv) laid out back to back, as the Python layer allocates them:
  // one [Cqkv x C] GEMM and one bias reduction instead of three each
  const bool packed_w = dwk == dwq + (size_t)Cq * C && dwv == dwk + (size_t)Cq * C;
  const bool packed_b = dbq && dbk && dbv && dbk == dbq + Cq && dbv == dbk + Cq;
  if (packed_w) {
    Gather Ad = Bx;
    Ad.base = dqkv;
    Ad.sk0 = (int)qs_b;
    rc = gemm(Ad, Bx, epi_dense(dwq, C), Cqkv, C, B * T, 1, gws, gbytes, st);
    if (rc) return rc;
  }
  if (packed_b) {
    rc = a2m_sum_bt_f32(dqkv, qs_b, T, 1, B, Cqkv, T, dbq, 0, stream);
    if (rc) return rc;
  }
  for (int i = 0; i < 3; ++i) {
    if (packed_w && (packed_b || !dbs[i])) continue;
    Gather Ad = Bx;
    Ad.base = dqkv + (int64_t)offs[i] * T;
    Ad.sk0 = (int)qs_b;
    if (!packed_w) {
      rc = gemm(Ad, Bx, epi_dense(dws[i], C), rows[i], C, B * T, 1, gws, gbytes, st);
      if (rc) return rc;
    }
    if (dbs[i] && !packed_b) {
      rc = a2m_sum_bt_f32(dqkv + (int64_t)offs[i] * T, qs_b, T, 1, B, rows[i], T, dbs[i], 0, stream);
      if (rc) return rc;
    }
  }
  return A2M_OK;
}

int a2m_channel_attention_bwd_f32(const float* dy, const float* x, int32_t B, int32_t C, int32_t T,
                                  const float* w1, const float* b1, int32_t Cr, const float* w2,
                                  const float* b2, float* dx, float* dw1, float* db1, float* dw2,
                                  float* db2, void* ws, size_t ws_bytes, void* stream) {
  A2M_CHECK_ARG(dy && x && w1 && b1 && w2 && b2 && dx && dw1 && db1 && dw2 && db2 && B > 0 && C > 0 &&
                    Cr > 0 && T > 0, "channel_attention_bwd: bad args");
  const int P = 2 * Cr * C + Cr + C;
  const size_t need = sizeof(float) * (size_t)B * P;
  if (!ws || ws_bytes < need) {
    set_error("channel_attention_bwd: workspace too small (%zu < %zu bytes)", ws_bytes, need);
    return A2M_EWS;
  }
  const size_t lds = sizeof(float) * (10 * (size_t)C + 4 * Cr);
  A2M_CHECK_ARG(lds <= 64 * 1024, "channel_attention_bwd: C too large");
  hipStream_t st = as_stream(stream);
  float* part = static_cast<float*>(ws);
  A2M_CHECK_ARG((int64_t)C * T < (1LL << 31) && (T % 4 != 0 || ((reinterpret_cast<uintptr_t>(dy) |
                                                                    reinterpret_cast<uintptr_t>(dx)) & 15) == 0),
                "channel_attention_bwd: too large, or dy / dx not 16-byte aligned");
  hipLaunchKernelGGL(channel_attention_bwd_kernel, dim3(B), dim3(CAB_NT), lds, st, dy, x, C, T, w1, b1, Cr,
                     w2, b2, dx, part);
  A2M_LAUNCH_CHECK();
  ColOuts outs{};
  outs.out[0] = dw1; outs.start[0] = 0;
  outs.out[1] = db1; outs.start[1] = Cr * C;
  outs.out[2] = dw2; outs.start[2] = Cr * C + Cr;
  outs.out[3] = db2; outs.start[3] = 2 * Cr * C + Cr;
  outs.n = 4;
  int rc = reduce_cols(part, B, P, P, outs, 0, st);
  return rc;
}

}  // extern "C"
