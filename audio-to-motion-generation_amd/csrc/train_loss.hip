// Training-step losses, small adjoints and the Adam update.
//   pose losses backward   real_motion_model.py:307-461
//   motion terms           version5_model_train.py:208-248 (L1 on motion, smoothness, jerk)
//   MSE (adversarial)      version5_model_train.py:367, 400-403
//   pos_to_motion          version5_model_train.py:208-213
//   interpolate backward   model_layers.py:277
//   Adam                   torch.optim.Adam defaults (version5_model_train.py:285-286)
#include <algorithm>

#include "a2m_internal.h"

namespace a2m {

__constant__ int kPar[52] = {-1, 0, 1, 2, 0, 4, 5, 0, 7, 7, 6,
                             10, 11, 12, 13, 10, 15, 16, 17, 10, 19, 20, 21, 10, 23, 24, 25,
                             10, 27, 28, 29, 3, 31, 32, 33, 34, 31, 36, 37, 38, 31, 40, 41,
                             42, 31, 44, 45, 46, 31, 48, 49, 50};
__constant__ int kHT[30][3] = {
    {0, 1, 2}, {1, 2, 3}, {2, 3, 4}, {0, 5, 6}, {5, 6, 7}, {6, 7, 8}, {0, 9, 10}, {9, 10, 11},
    {10, 11, 12}, {0, 13, 14}, {13, 14, 15}, {14, 15, 16}, {0, 17, 18}, {17, 18, 19}, {18, 19, 20},
    {21, 22, 23}, {22, 23, 24}, {23, 24, 25}, {21, 26, 27}, {26, 27, 28}, {27, 28, 29},
    {21, 30, 31}, {30, 31, 32}, {31, 32, 33}, {21, 34, 35}, {34, 35, 36}, {35, 36, 37},
    {21, 38, 39}, {38, 39, 40}, {39, 40, 41}};
__constant__ int kBT[5][3] = {{0, 1, 2}, {1, 2, 3}, {0, 4, 5}, {4, 5, 6}, {0, 7, 8}};

constexpr float kPi = 3.14159265358979f;
constexpr int kTC = 16;  // time steps per workgroup in the pose-loss backward

__device__ __forceinline__ double bsum(double v, double* red) {
  for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o);
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  __syncthreads();
  if (lane == 0) red[w] = v;
  __syncthreads();
  double s = 0.0;
  for (int i = 0; i < (int)(blockDim.x >> 6); ++i) s += red[i];
  __syncthreads();
  return s;
}

// angle a = atan2(cross(u,v), dot(u,v)), u = p_j - p_a, v = p_c - p_j; dL/da = g.  Returns the
// adjoints of u and v (gux, guy, gvx, gvy): joint j receives (gux - gvx, guy - gvy), joint a
// (-gux, -guy), joint c (gvx, gvy).
__device__ __forceinline__ float4 angle_grad(const float* p, int a, int j, int c, float g) {
  const float ux = p[2 * j] - p[2 * a], uy = p[2 * j + 1] - p[2 * a + 1];
  const float vx = p[2 * c] - p[2 * j], vy = p[2 * c + 1] - p[2 * j + 1];
  const float cr = ux * vy - uy * vx, dt = ux * vx + uy * vy;
  const float den = cr * cr + dt * dt;
  if (den == 0.f || g == 0.f) return make_float4(0.f, 0.f, 0.f, 0.f);
  const float gcr = g * dt / den, gdt = -g * cr / den;  // d atan2(y,x)/dy = x/r^2, /dx = -y/r^2
  // cross = ux vy - uy vx ; dot = ux vx + uy vy
  return make_float4(gcr * vy + gdt * vx, -gcr * vx + gdt * vy, -gcr * uy + gdt * ux, gcr * ux + gdt * uy);
}

// One workgroup per (clip, kTC time steps): the clip's mean bone lengths (over all T, as in the
// forward) are recomputed by each of its workgroups, then phase 1 writes every bone's and every
// angle triple's adjoint into its own LDS slot, and phase 2 has one thread per (time step, joint)
// add the slots that touch its joint in a fixed order -- its own bone, its children's bones
// ascending, then the triples ascending (middle, first, last joint roles) -- from a per-joint
// adjacency list the workgroup builds once.  No atomics: the gradient is bitwise reproducible.
// (Round 6: one workgroup per clip scanning all 86 bones / triples per output element took
// ~150 us a call at B = 8 / 32, latency-bound on a handful of CUs.)
constexpr int kAdjMax = 16;   // entries per joint (the hand roots: 5 child bones + 6 triples)
__global__ __launch_bounds__(256) void pose_loss_bwd_kernel(const float* gen, int64_t gs_b,
                                                            int64_t gs_t, const float* real,
                                                            int64_t rs_b, int64_t rs_t, int B, int T,
                                                            float hand_w, float body_w,
                                                            const float* grad_out, float* dgen) {
  __shared__ float lg[51], lr[51], coef[51];
  __shared__ float2 bone_g[kTC][51];    // (s dx, s dy) of bone k (joint k+1 from its parent)
  __shared__ float4 tri_g[kTC][35];     // angle adjoints: 30 hand triples, then 5 body triples
  __shared__ short adj[52][kAdjMax];    // per joint: 0x1000 | k own bone k, 0x2000 | k a child's
  __shared__ unsigned char nadj[52];    //   bone k, 0x3000 | q << 2 | role  triple q (role 0/1/2)
  const int b = blockIdx.x, t0 = blockIdx.y * kTC;
  const int nt = min(kTC, T - t0);
  if (threadIdx.x < 52) {
    const int jn = threadIdx.x;
    int n = 0;
    if (jn >= 1) adj[jn][n++] = (short)(0x1000 | (jn - 1));
    for (int c = 1; c < 52; ++c)
      if (kPar[c] == jn) adj[jn][n++] = (short)(0x2000 | (c - 1));
    for (int q = 0; q < 35; ++q) {
      const int* tr = q < 30 ? kHT[q] : kBT[q - 30];
      const int off = q < 30 ? 10 : 0;   // the hand triples index joints from 10 (p + 20)
      if (tr[1] + off == jn) adj[jn][n++] = (short)(0x3000 | (q << 2) | 1);
      if (tr[0] + off == jn) adj[jn][n++] = (short)(0x3000 | (q << 2) | 0);
      if (tr[2] + off == jn) adj[jn][n++] = (short)(0x3000 | (q << 2) | 2);
    }
    nadj[jn] = (unsigned char)n;
  }
  const float gbone = real ? grad_out[0] : 0.f, gang = grad_out[1];
  // mean bone lengths over time (as in the forward: one wave per series, lanes along t); only
  // the bone loss needs them, and it exists only with a real pose
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  for (int i = wave; real != nullptr && i < 102; i += (int)(blockDim.x >> 6)) {
    const bool isr = i >= 51;
    const int jb = (i % 51) + 1, pj = kPar[jb];
    const float* base = isr ? real + b * rs_b : gen + b * gs_b;
    const int64_t st = isr ? rs_t : gs_t;
    float s = 0.f;
    for (int t = lane; t < T; t += 64) {
      const float* p = base + t * st;
      const float dx = p[2 * jb] - p[2 * pj], dy = p[2 * jb + 1] - p[2 * pj + 1];
      s += sqrtf(dx * dx + dy * dy);
    }
    s = wave64_sum(s);
    if (lane == 0) (isr ? lr : lg)[i % 51] = s / (float)T;
  }
  __syncthreads();
  for (int k = threadIdx.x; k < 51; k += blockDim.x)
    coef[k] = real ? gbone * 2.f * (lg[k] - lr[k]) / (float)(B * 51) / (float)T : 0.f;
  __syncthreads();
  const float gh = gang * hand_w / (float)(B * T * 30), gb = gang * body_w / (float)(B * T * 5);
  for (int i = threadIdx.x; i < nt * 51; i += blockDim.x) {  // bones
    const int tt = i / 51, k = i % 51, jb = k + 1, pj = kPar[jb];
    const float* p = gen + b * gs_b + (t0 + tt) * gs_t;
    const float dx = p[2 * jb] - p[2 * pj], dy = p[2 * jb + 1] - p[2 * pj + 1];
    const float n = sqrtf(dx * dx + dy * dy);
    const float s = (n == 0.f || coef[k] == 0.f) ? 0.f : coef[k] / n;
    bone_g[tt][k] = make_float2(s * dx, s * dy);
  }
  for (int i = threadIdx.x; i < nt * 35; i += blockDim.x) {  // angle triples
    const int tt = i / 35, q = i % 35;
    const float* p = gen + b * gs_b + (t0 + tt) * gs_t;
    if (q < 30) {
      const int* tr = kHT[q];
      const float* ph = p + 20;
      const float ux = ph[2 * tr[1]] - ph[2 * tr[0]], uy = ph[2 * tr[1] + 1] - ph[2 * tr[0] + 1];
      const float vx = ph[2 * tr[2]] - ph[2 * tr[1]], vy = ph[2 * tr[2] + 1] - ph[2 * tr[1] + 1];
      const float ang = atan2f(ux * vy - uy * vx, ux * vx + uy * vy);
      const float g = (ang < 0.f ? -gh : 0.f) + (ang > kPi ? gh : 0.f);
      tri_g[tt][q] = angle_grad(ph, tr[0], tr[1], tr[2], g);
    } else {
      const int* tr = kBT[q - 30];
      const float ux = p[2 * tr[1]] - p[2 * tr[0]], uy = p[2 * tr[1] + 1] - p[2 * tr[0] + 1];
      const float vx = p[2 * tr[2]] - p[2 * tr[1]], vy = p[2 * tr[2] + 1] - p[2 * tr[1] + 1];
      const float ang = atan2f(ux * vy - uy * vx, ux * vx + uy * vy);
      const float g = (ang < -0.5f * kPi ? -gb : 0.f) + (ang > kPi ? gb : 0.f);
      tri_g[tt][q] = angle_grad(p, tr[0], tr[1], tr[2], g);
    }
  }
  __syncthreads();
  for (int i = threadIdx.x; i < nt * 52; i += blockDim.x) {
    const int tt = i / 52, jn = i % 52;
    float sx = 0.f, sy = 0.f;
    for (int e = 0; e < nadj[jn]; ++e) {
      const int code = adj[jn][e], kind = code >> 12, idx = code & 0xfff;
      if (kind == 1) { sx += bone_g[tt][idx].x; sy += bone_g[tt][idx].y; }
      else if (kind == 2) { sx -= bone_g[tt][idx].x; sy -= bone_g[tt][idx].y; }
      else {
        const float4 v = tri_g[tt][idx >> 2];
        const int role = idx & 3;
        if (role == 1) { sx += v.x - v.z; sy += v.y - v.w; }
        else if (role == 0) { sx -= v.x; sy -= v.y; }
        else { sx += v.z; sy += v.w; }
      }
    }
    float* d = dgen + ((int64_t)b * T + t0 + tt) * 104 + 2 * jn;
    d[0] += sx;
    d[1] += sy;
  }
}

// motion terms on [B][T][F]; one workgroup per clip, partials to part[b][3]; dfake written
__global__ __launch_bounds__(256) void motion_terms_kernel(const float* fake, const float* real, int B,
                                                           int T, int Fd, const float* gterms,
                                                           float* part, float* dfake) {
  __shared__ double red[4];
  __shared__ float nacc[512], njerk[512];  // per-time norms (T <= 512)
  const int b = blockIdx.x;
  const float* fp = fake + (int64_t)b * T * Fd;
  const float* rp = real ? real + (int64_t)b * T * Fd : nullptr;
  auto m = [&](const float* p, int t, int f) { return p[(t + 1) * Fd + f] - p[t * Fd + f]; };
  // L1 over motion
  double l1 = 0.0;
  if (rp)
    for (int i = threadIdx.x; i < (T - 1) * Fd; i += blockDim.x) {
      const int t = i / Fd, f = i % Fd;
      l1 += fabsf(m(fp, t, f) - m(rp, t, f));
    }
  // norms of acceleration (T-2) and jerk (T-3): four lanes per time step (a DPP quad), each
  // summing every fourth feature, so the block's 256 threads all take part (one thread per t
  // walking all Fd features was the kernel's latency-bound half)
  for (int t0 = 0; t0 < T; t0 += 64) {
    const int t = t0 + (threadIdx.x >> 2), q = threadIdx.x & 3;
    float sa = 0.f, sj = 0.f;
    if (t < T - 2)
      for (int f = q; f < Fd; f += 4) {
        const float a = m(fp, t + 1, f) - m(fp, t, f);
        sa += a * a;
      }
    if (t < T - 3)
      for (int f = q; f < Fd; f += 4) {
        const float j = (m(fp, t + 2, f) - m(fp, t + 1, f)) - (m(fp, t + 1, f) - m(fp, t, f));
        sj += j * j;
      }
    sa = quad_sum(sa);
    sj = quad_sum(sj);
    if (q == 0 && t < T) {
      nacc[t] = sqrtf(sa);
      njerk[t] = sqrtf(sj);
    }
  }
  __syncthreads();
  double sa = 0.0, sj = 0.0;
  for (int t = threadIdx.x; t < T; t += blockDim.x) {
    if (t < T - 2) sa += nacc[t];
    if (t < T - 3) sj += njerk[t];
  }
  l1 = bsum(l1, red);
  sa = bsum(sa, red);
  sj = bsum(sj, red);
  if (threadIdx.x == 0) {
    part[3 * b] = (float)l1;
    part[3 * b + 1] = (float)sa;
    part[3 * b + 2] = (float)sj;
  }
  if (!dfake || !gterms) return;
  // gradient w.r.t. motion m[t][f] (t < T-1), then the diff adjoint
  const float w1 = gterms[0], ws_ = gterms[1], wj = gterms[2];
  const float cl1 = rp ? w1 / (float)(B * (T - 1) * Fd) : 0.f;
  const float cs = T > 2 ? ws_ / (float)(B * (T - 2)) : 0.f, cj = T > 3 ? wj / (float)(B * (T - 3)) : 0.f;
  auto gm = [&](int t, int f) -> float {  // dL/dm[t][f]
    float g = 0.f;
    if (rp) {
      const float d = m(fp, t, f) - m(rp, t, f);
      g += cl1 * (d > 0.f ? 1.f : (d < 0.f ? -1.f : 0.f));
    }
    // acc[s] = m[s+1] - m[s]  (s < T-2)
    if (t - 1 >= 0 && t - 1 < T - 2 && nacc[t - 1] > 0.f) g += cs * (m(fp, t, f) - m(fp, t - 1, f)) / nacc[t - 1];
    if (t < T - 2 && nacc[t] > 0.f) g -= cs * (m(fp, t + 1, f) - m(fp, t, f)) / nacc[t];
    // jerk[s] = m[s+2] - 2 m[s+1] + m[s]  (s < T-3)
    for (int s = t - 2; s <= t; ++s) {
      if (s < 0 || s >= T - 3 || njerk[s] == 0.f) continue;
      const float js = m(fp, s + 2, f) - 2.f * m(fp, s + 1, f) + m(fp, s, f);
      const float coef = (s == t) ? 1.f : (s == t - 1 ? -2.f : 1.f);
      g += cj * coef * js / njerk[s];
    }
    return g;
  };
  for (int i = threadIdx.x; i < T * Fd; i += blockDim.x) {
    const int t = i / Fd, f = i % Fd;
    float g = 0.f;
    if (t - 1 >= 0) g += gm(t - 1, f);  // pose[t] enters m[t-1] with +
    if (t < T - 1) g -= gm(t, f);       // and m[t] with -
    dfake[(int64_t)b * T * Fd + i] = g;
  }
}

__global__ void terms_final_kernel(const float* part, int B, int T, int Fd, int has_real, float* terms) {
  if (threadIdx.x != 0) return;
  double a = 0.0, s = 0.0, j = 0.0;
  for (int b = 0; b < B; ++b) {
    a += part[3 * b];
    s += part[3 * b + 1];
    j += part[3 * b + 2];
  }
  terms[0] = has_real ? (float)(a / ((double)B * (T - 1) * Fd)) : 0.f;
  terms[1] = T > 2 ? (float)(s / ((double)B * (T - 2))) : 0.f;
  terms[2] = T > 3 ? (float)(j / ((double)B * (T - 3))) : 0.f;
}

__global__ __launch_bounds__(256) void mse_partial_kernel(const float* p, const float* t, int64_t n,
                                                          const float* gl, float* part, float* dpred) {
  __shared__ double red[4];
  double s = 0.0;
  const float g = gl ? gl[0] : 1.f;
  for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < n;
       i += (int64_t)gridDim.x * blockDim.x) {
    const float d = p[i] - t[i];
    s += (double)d * d;
    if (dpred) dpred[i] = g * (2.f * d / (float)n);
  }
  s = bsum(s, red);
  if (threadIdx.x == 0) part[blockIdx.x] = (float)s;
}

__global__ void mse_final_kernel(const float* part, int nb, int64_t n, float* loss) {
  if (threadIdx.x != 0) return;
  double s = 0.0;
  for (int i = 0; i < nb; ++i) s += part[i];
  loss[0] = (float)(s / (double)n);
}

__global__ void diff_time_kernel(const float* x, int T, int Fd, int64_t total, float* y) {
  for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < total;
       i += (int64_t)gridDim.x * blockDim.x) {
    const int64_t b = i / ((int64_t)(T - 1) * Fd);
    const int64_t r = i - b * (T - 1) * Fd;
    const float* xb = x + b * T * Fd;
    y[i] = xb[r + Fd] - xb[r];
  }
}

__global__ void diff_time_bwd_kernel(const float* dy, int T, int Fd, int64_t total, float* dx, int accumulate) {
  for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < total;
       i += (int64_t)gridDim.x * blockDim.x) {
    const int64_t b = i / ((int64_t)T * Fd);
    const int t = (int)((i / Fd) % T), f = (int)(i % Fd);
    const float* g = dy + b * (T - 1) * Fd;
    float v = 0.f;
    if (t >= 1) v += g[(t - 1) * Fd + f];
    if (t < T - 1) v -= g[t * Fd + f];
    dx[i] = accumulate ? dx[i] + v : v;
  }
}

// adjoint of interp_time_kernel (ops.hip): dx[b][c][h][w] = sum_t weight(t -> h, w) dy[b][c][t]
__global__ void interp_time_bwd_kernel(const float* dy, int C, int H, int W, int T, int64_t total, float* dx) {
  const float sh = (float)H / (float)T;
  float srcw = (float)W * 0.5f - 0.5f;
  srcw = srcw < 0.f ? 0.f : srcw;
  const int w0 = (int)srcw;
  const int w1 = w0 + (w0 < W - 1 ? 1 : 0);
  const float lw1 = srcw - (float)w0, lw0 = 1.f - lw1;
  for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < total;
       i += (int64_t)gridDim.x * blockDim.x) {
    const int w = (int)(i % W);
    const int h = (int)((i / W) % H);
    const int64_t bc = i / ((int64_t)H * W);
    float wcoef = 0.f;
    if (w == w0) wcoef += lw0;
    if (w == w1 && lw1 != 0.f) wcoef += lw1;
    float v = 0.f;
    if (wcoef != 0.f) {
      const float* g = dy + bc * T;
      for (int t = 0; t < T; ++t) {
        float src = sh * ((float)t + 0.5f) - 0.5f;
        src = src < 0.f ? 0.f : src;
        const int h0 = (int)src;
        const int h1 = h0 + (h0 < H - 1 ? 1 : 0);
        const float l1 = src - (float)h0, l0 = 1.f - l1;
        float c = 0.f;
        if (h0 == h) c += l0;
        if (h1 == h && l1 != 0.f) c += l1;
        v += c * g[t];
      }
    }
    dx[i] = v * wcoef;
  }
}

__global__ void adam_kernel(float* p, const float* g, float* m, float* v, int64_t n, float lr, float b1,
                            float b2, float eps, float wd, float bc1, float bc2_sqrt) {
  for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < n;
       i += (int64_t)gridDim.x * blockDim.x) {
    float gi = g[i];
    if (wd != 0.f) gi += wd * p[i];
    const float mi = b1 * m[i] + (1.f - b1) * gi;
    const float vi = b2 * v[i] + (1.f - b2) * gi * gi;
    m[i] = mi;
    v[i] = vi;
    const float denom = sqrtf(vi) / bc2_sqrt + eps;
    p[i] -= (lr / bc1) * (mi / denom);
  }
}

// The same update with its step-dependent hyperparameters in device memory, for a step captured
// in a HIP graph (a replay re-runs the launch with its baked arguments): adam_tick_kernel advances
// the step counter, then every thread derives the bias corrections from it exactly as the host
// entry point does (double pow / sqrt, rounded to float) and reads the learning rate, which the
// host rewrites only when it changes (DynamicGANTraining.adjust_learning_rates).
__global__ void adam_tick_kernel(int32_t* step) {
  if (threadIdx.x == 0) step[0] += 1;
}

__global__ void adam_dev_kernel(float* p, const float* g, float* m, float* v, int64_t n, const float* lr_p,
                                float b1, float b2, float eps, float wd, const int32_t* step_p) {
  const int32_t step = step_p[0];
  const float lr = lr_p[0];
  const float bc1 = (float)(1.0 - pow((double)b1, (double)step));
  const float bc2_sqrt = (float)sqrt(1.0 - pow((double)b2, (double)step));
  for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < n;
       i += (int64_t)gridDim.x * blockDim.x) {
    float gi = g[i];
    if (wd != 0.f) gi += wd * p[i];
    const float mi = b1 * m[i] + (1.f - b1) * gi;
    const float vi = b2 * v[i] + (1.f - b2) * gi * gi;
    m[i] = mi;
    v[i] = vi;
    const float denom = sqrtf(vi) / bc2_sqrt + eps;
    p[i] -= (lr / bc1) * (mi / denom);
  }
}

// Segment gather: dst[off_i .. off_i + n_i) = src_i[0 .. n_i) for up to GS_MAX segments per
// launch (FlatAdam: the step's per-parameter gradients, which autograd hands over as fresh
// tensors, land in the flat gradient buffer in one launch instead of one add or copy per
// parameter).  Block row y = segment; float4 when the segment is 16-byte aligned at both ends.
constexpr int GS_MAX = 48;
struct GatherSegs {
  const float* src[GS_MAX];
  int64_t off[GS_MAX];
  int64_t n[GS_MAX];
};

__global__ void gather_segments_kernel(GatherSegs segs, float* __restrict__ dst) {
  const int s = blockIdx.y;
  const float* src = segs.src[s];
  float* d = dst + segs.off[s];
  const int64_t n = segs.n[s];
  const int64_t stride = (int64_t)gridDim.x * blockDim.x;
  const int64_t i0 = blockIdx.x * (int64_t)blockDim.x + threadIdx.x;
  if (((reinterpret_cast<uintptr_t>(src) | reinterpret_cast<uintptr_t>(d)) & 15) == 0) {
    const int64_t n4 = n / 4;
    for (int64_t i = i0; i < n4; i += stride)
      reinterpret_cast<float4*>(d)[i] = reinterpret_cast<const float4*>(src)[i];
    for (int64_t i = n4 * 4 + i0; i < n; i += stride) d[i] = src[i];
  } else {
    for (int64_t i = i0; i < n; i += stride) d[i] = src[i];
  }
}

}  // namespace a2m

using namespace a2m;

extern "C" {

int a2m_pose_losses_w_bwd_f32(const float* gen, int64_t gs_b, int64_t gs_t, const float* real,
                              int64_t rs_b, int64_t rs_t, int32_t B, int32_t T, float hand_w,
                              float body_w, const float* grad_out, float* dgen, void* ws,
                              size_t ws_bytes, void* stream) {
  (void)ws; (void)ws_bytes;
  A2M_CHECK_ARG(gen && grad_out && dgen && B > 0 && T > 0, "pose_losses_bwd: bad args");
  hipLaunchKernelGGL(pose_loss_bwd_kernel, dim3(B, (unsigned)cdiv(T, kTC)), dim3(256), 0, as_stream(stream), gen,
                     gs_b, gs_t,
                     real, rs_b, rs_t, B, T, hand_w, body_w, grad_out, dgen);
  A2M_LAUNCH_CHECK();
  return A2M_OK;
}

int a2m_pose_losses_bwd_f32(const float* gen, int64_t gs_b, int64_t gs_t, const float* real,
                            int64_t rs_b, int64_t rs_t, int32_t B, int32_t T, const float* grad_out,
                            float* dgen, void* ws, size_t ws_bytes, void* stream) {
  return a2m_pose_losses_w_bwd_f32(gen, gs_b, gs_t, real, rs_b, rs_t, B, T, 0.7f, 0.3f, grad_out,
                                   dgen, ws, ws_bytes, stream);
}

int a2m_motion_losses_f32(const float* fake, const float* real, int32_t B, int32_t T, int32_t Fd,
                          float* terms, const float* grad_terms, float* dfake, void* ws,
                          size_t ws_bytes, void* stream) {
  A2M_CHECK_ARG(fake && terms && B > 0 && T > 1 && T <= 512 && Fd > 0, "motion_losses: bad args");
  const size_t need = sizeof(float) * 3 * (size_t)B;
  if (!ws || ws_bytes < need) { set_error("motion_losses: workspace too small (%zu < %zu bytes)", ws_bytes, need); return A2M_EWS; }
  hipStream_t st = as_stream(stream);
  float* part = static_cast<float*>(ws);
  hipLaunchKernelGGL(motion_terms_kernel, dim3(B), dim3(256), 0, st, fake, real, B, T, Fd, grad_terms,
                     part, dfake);
  A2M_LAUNCH_CHECK();
  hipLaunchKernelGGL(terms_final_kernel, dim3(1), dim3(64), 0, st, part, B, T, Fd, real != nullptr ? 1 : 0,
                     terms);
  A2M_LAUNCH_CHECK();
  return A2M_OK;
}

int a2m_mse_loss_f32(const float* pred, const float* target, int64_t n, float* loss,
                     const float* grad_loss, float* dpred, void* ws, size_t ws_bytes, void* stream) {
  A2M_CHECK_ARG(pred && target && loss && n > 0, "mse_loss: bad args");
  const int nb = (int)std::min<int64_t>(cdiv(n, 256), 256);
  if (!ws || ws_bytes < sizeof(float) * nb) { set_error("mse_loss: workspace too small (%zu < %zu bytes)", ws_bytes, sizeof(float) * nb); return A2M_EWS; }
  hipStream_t st = as_stream(stream);
  float* part = static_cast<float*>(ws);
  hipLaunchKernelGGL(mse_partial_kernel, dim3(nb), dim3(256), 0, st, pred, target, n, grad_loss, part, dpred);
  A2M_LAUNCH_CHECK();
  hipLaunchKernelGGL(mse_final_kernel, dim3(1), dim3(64), 0, st, part, nb, n, loss);
  A2M_LAUNCH_CHECK();
  return A2M_OK;
}

int a2m_diff_time_f32(const float* x, int32_t B, int32_t T, int32_t Fd, float* y, void* stream) {
  A2M_CHECK_ARG(x && y && B > 0 && T > 1 && Fd > 0, "diff_time: bad args");
  const int64_t total = (int64_t)B * (T - 1) * Fd;
  hipLaunchKernelGGL(diff_time_kernel, dim3((unsigned)std::min<int64_t>(cdiv(total, 256), 4096)), dim3(256), 0,
                     as_stream(stream), x, T, Fd, total, y);
  A2M_LAUNCH_CHECK();
  return A2M_OK;
}

int a2m_diff_time_bwd_f32(const float* dy, int32_t B, int32_t T, int32_t Fd, float* dx, int32_t accumulate,
                          void* stream) {
  A2M_CHECK_ARG(dy && dx && B > 0 && T > 1 && Fd > 0, "diff_time_bwd: bad args");
  const int64_t total = (int64_t)B * T * Fd;
  hipLaunchKernelGGL(diff_time_bwd_kernel, dim3((unsigned)std::min<int64_t>(cdiv(total, 256), 4096)), dim3(256),
                     0, as_stream(stream), dy, T, Fd, total, dx, accumulate);
  A2M_LAUNCH_CHECK();
  return A2M_OK;
}

int a2m_interp_time_bwd_f32(const float* dy, int32_t B, int32_t C, int32_t H, int32_t W, float* dx, int32_t T,
                            void* stream) {
  A2M_CHECK_ARG(dy && dx && B > 0 && C > 0 && H > 0 && W > 0 && T > 0, "interp_time_bwd: bad args");
  const int64_t total = (int64_t)B * C * H * W;
  hipLaunchKernelGGL(interp_time_bwd_kernel, dim3((unsigned)std::min<int64_t>(cdiv(total, 256), 8192)),
                     dim3(256), 0, as_stream(stream), dy, C, H, W, T, total, dx);
  A2M_LAUNCH_CHECK();
  return A2M_OK;
}

int a2m_adam_f32(float* param, const float* grad, float* exp_avg, float* exp_avg_sq, int64_t n, float lr,
                 float beta1, float beta2, float eps, float weight_decay, int32_t step, void* stream) {
  A2M_CHECK_ARG(param && grad && exp_avg && exp_avg_sq && n >= 0 && step >= 1, "adam: bad args");
  if (n == 0) return A2M_OK;
  const double bc1 = 1.0 - std::pow((double)beta1, step);
  const double bc2 = 1.0 - std::pow((double)beta2, step);
  hipLaunchKernelGGL(adam_kernel, dim3((unsigned)std::min<int64_t>(cdiv(n, 256), 8192)), dim3(256), 0,
                     as_stream(stream), param, grad, exp_avg, exp_avg_sq, n, lr, beta1, beta2, eps,
                     weight_decay, (float)bc1, (float)std::sqrt(bc2));
  A2M_LAUNCH_CHECK();
  return A2M_OK;
}

int a2m_adam_dev_f32(float* param, const float* grad, float* exp_avg, float* exp_avg_sq, int64_t n,
                     const float* lr, float beta1, float beta2, float eps, float weight_decay,
                     int32_t* step, void* stream) {
  A2M_CHECK_ARG(param && grad && exp_avg && exp_avg_sq && lr && step && n >= 0, "adam_dev: bad args");
  hipStream_t st = as_stream(stream);
  hipLaunchKernelGGL(adam_tick_kernel, dim3(1), dim3(64), 0, st, step);
  A2M_LAUNCH_CHECK();
  if (n == 0) return A2M_OK;
  hipLaunchKernelGGL(adam_dev_kernel, dim3((unsigned)std::min<int64_t>(cdiv(n, 256), 8192)), dim3(256), 0,
                     st, param, grad, exp_avg, exp_avg_sq, n, lr, beta1, beta2, eps, weight_decay, step);
  A2M_LAUNCH_CHECK();
  return A2M_OK;
}

int a2m_gather_segments_f32(const float* const* src, const int64_t* dst_off, const int64_t* n,
                            int32_t count, float* dst, void* stream) {
  A2M_CHECK_ARG(count >= 0 && (count == 0 || (src && dst_off && n && dst)), "gather_segments: bad args");
  hipStream_t st = as_stream(stream);
  for (int c0 = 0; c0 < count; c0 += GS_MAX) {
    GatherSegs segs{};
    const int m = std::min(GS_MAX, count - c0);
    int64_t maxn = 0;
    for (int i = 0; i < m; ++i) {
      A2M_CHECK_ARG(src[c0 + i] && n[c0 + i] >= 0 && dst_off[c0 + i] >= 0, "gather_segments: segment %d",
                    c0 + i);
      segs.src[i] = src[c0 + i];
      segs.off[i] = dst_off[c0 + i];
      segs.n[i] = n[c0 + i];
      maxn = std::max(maxn, n[c0 + i]);
    }
    if (maxn == 0) continue;
    const unsigned gx = (unsigned)std::min<int64_t>(cdiv(maxn, 4 * 256), 64);
    hipLaunchKernelGGL(gather_segments_kernel, dim3(gx, (unsigned)m), dim3(256), 0, st, segs, dst);
    A2M_LAUNCH_CHECK();
  }
  return A2M_OK;
}

}  // extern "C"
