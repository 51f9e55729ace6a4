// Training-mode normalisation, dropout and reduction kernels.
//
// BatchNorm (train): ConvNormRelu applies conv -> dropout -> BN -> act (model_layers.py:118);
// the discriminator applies conv -> BN -> LeakyReLU -> dropout (real_motion_model.py:504-551).
// Statistics are per channel over (batch, spatial) exactly as nn.BatchNorm*d in training
// mode: biased variance normalises, the running variance gets the unbiased one, momentum
// 0.1.  Per-channel sums are reduced in float64 over (channel, slice) partials, so any
// B*L fits (encoder layer 0: 131,072 elements per channel) with deterministic order.
// Dropout masks come from a counter-based hash of (seed, logical element index) and are
// regenerated in the backward pass rather than stored.
#include "a2m_internal.h"

namespace a2m {

// elements of one channel per workgroup: four per thread, issued together (a [64, 256, 64]
// activation is 1,024 workgroups instead of 256 at one latency-bound round trip per element)
constexpr int kSlice = 1024;

__device__ __forceinline__ uint32_t hash_u32(uint64_t seed, uint64_t idx) {
  uint64_t z = seed + idx * 0x9E3779B97F4A7C15ull;
  z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
  z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
  z ^= z >> 31;
  return (uint32_t)(z >> 32);
}

// keep-scale of element: 0 (dropped) or 1/(1-p)
__device__ __forceinline__ float drop_scale(uint64_t seed, uint64_t idx, float p) {
  if (p <= 0.f) return 1.f;
  const float u = (float)(hash_u32(seed, idx) >> 8) * (1.0f / 16777216.0f);
  return u >= p ? 1.f / (1.f - p) : 0.f;
}

enum DropMode { DROP_NONE = 0, DROP_BEFORE = 1, DROP_BEFORE_CH = 2, DROP_AFTER = 3 };

struct BNArgs {
  const float* x; int64_t xs_b, xs_c;
  int B, C, L, slices;
  float p; int mode; uint64_t seed;
  const uint64_t* seed_off;  // device step counter (a2m_set_dropout_seed_offset) or null
};

// Dropout seed offset for captured training steps: a HIP graph bakes every launch's seed, so a
// replayed step would redraw the same masks.  With a device counter registered (the trainer
// bumps it once per replayed step, inside the graph) each launch hashes seed + counter * K,
// read when the kernel runs.  Null: the seed as passed (eager steps, unchanged bits).
static const uint64_t* g_seed_off = nullptr;

__device__ __forceinline__ uint64_t eff_seed(uint64_t seed, const uint64_t* off, float p) {
  return (off && p > 0.f) ? seed + off[0] * 0xA0761D6478BD642Full : seed;
}
// kernels take their arguments as `a_in` and work on a copy whose seed has the offset applied
#define A2M_BN_RESOLVE(T, a_in) T a = a_in; a.seed = eff_seed(a_in.seed, a_in.seed_off, a_in.p)
#define A2M_BNB_RESOLVE(a_in) BNBwdArgs a = a_in; a.f.seed = eff_seed(a_in.f.seed, a_in.f.seed_off, a_in.f.p)

__device__ __forceinline__ float pre_drop(const BNArgs& a, int b, int c, int l) {
  if (a.mode == DROP_BEFORE) return drop_scale(a.seed, ((uint64_t)b * a.C + c) * a.L + l, a.p);
  if (a.mode == DROP_BEFORE_CH) return drop_scale(a.seed, (uint64_t)b * a.C + c, a.p);
  return 1.f;
}

__device__ __forceinline__ double block_sum_d(double v, double* red) {
  for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o);
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  __syncthreads();
  if (lane == 0) red[w] = v;
  __syncthreads();
  double s = 0.0;
  for (int i = 0; i < (int)(blockDim.x >> 6); ++i) s += red[i];
  return s;
}

// partial (sum z, sum z^2) per (channel, slice)
__global__ __launch_bounds__(256) void bn_stats_kernel(BNArgs a_in, double* part) {
  A2M_BN_RESOLVE(BNArgs, a_in);
  __shared__ double red[4];
  const int c = blockIdx.x / a.slices, s = blockIdx.x % a.slices;
  const int64_t N = (int64_t)a.B * a.L;
  const int64_t i0 = (int64_t)s * kSlice, i1 = min<int64_t>(N, i0 + kSlice);
  double s1 = 0.0, s2 = 0.0;
  #pragma unroll 4
  for (int i = (int)i0 + threadIdx.x; i < (int)i1; i += blockDim.x) {
    const int b = i / a.L, l = i - (i / a.L) * a.L;
    const float z = a.x[b * a.xs_b + c * a.xs_c + l] * pre_drop(a, b, c, l);
    s1 += z;
    s2 += (double)z * z;
  }
  s1 = block_sum_d(s1, red);
  s2 = block_sum_d(s2, red);
  if (threadIdx.x == 0) {
    part[2 * ((int64_t)c * a.slices + s)] = s1;
    part[2 * ((int64_t)c * a.slices + s) + 1] = s2;
  }
}

__device__ __forceinline__ float act_fwd(float v, int act, float slope) {
  if (act == ACT_RELU) return v > 0.f ? v : 0.f;
  if (act == ACT_LRELU) return v > 0.f ? v : v * slope;
  return v;
}

__device__ __forceinline__ float act_grad(float pre, int act, float slope) {
  if (act == ACT_RELU) return pre > 0.f ? 1.f : 0.f;
  if (act == ACT_LRELU) return pre > 0.f ? 1.f : slope;
  return 1.f;
}

// The per-channel finalize (mean, rstd, running statistics) folded into the apply pass (one
// launch fewer per BatchNorm layer): every workgroup of channel c reduces the channel's slice
// partials in the same fixed order (so every workgroup gets the same mean / rstd bits), and the
// slice-0 workgroup publishes them and updates the running statistics.
__global__ __launch_bounds__(256) void bn_apply_fused_kernel(BNArgs a_in, const double* part, float eps,
                                                             float momentum, float* rmean,
                                                             float* rvar, float* mean_out,
                                                             float* rstd_out, const float* gamma,
                                                             const float* beta, int act, float slope,
                                                             float* y, int64_t ys_b, int64_t ys_c) {
  A2M_BN_RESOLVE(BNArgs, a_in);
  __shared__ float stat[2];
  const int c = blockIdx.x / a.slices, s = blockIdx.x % a.slices;
  const int64_t N = (int64_t)a.B * a.L;
  if (threadIdx.x == 0) {
    double s1 = 0.0, s2 = 0.0;
    for (int q = 0; q < a.slices; ++q) {
      s1 += part[2 * ((int64_t)c * a.slices + q)];
      s2 += part[2 * ((int64_t)c * a.slices + q) + 1];
    }
    const double mean = s1 / (double)N;
    double var = s2 / (double)N - mean * mean;
    var = var > 0.0 ? var : 0.0;
    stat[0] = (float)mean;
    stat[1] = (float)(1.0 / sqrt(var + (double)eps));
    if (s == 0) {
      mean_out[c] = stat[0];
      rstd_out[c] = stat[1];
      if (rmean) {
        const double unb = N > 1 ? var * (double)N / (double)(N - 1) : var;
        rmean[c] = (float)((1.0 - momentum) * rmean[c] + momentum * mean);
        rvar[c] = (float)((1.0 - momentum) * rvar[c] + momentum * unb);
      }
    }
  }
  __syncthreads();
  const int64_t i0 = (int64_t)s * kSlice, i1 = min<int64_t>(N, i0 + kSlice);
  const float mu = stat[0], rs = stat[1], g = gamma ? gamma[c] : 1.f, bt = beta ? beta[c] : 0.f;
  #pragma unroll 4
  for (int i = (int)i0 + threadIdx.x; i < (int)i1; i += blockDim.x) {
    const int b = i / a.L, l = i - (i / a.L) * a.L;
    const float z = a.x[b * a.xs_b + c * a.xs_c + l] * pre_drop(a, b, c, l);
    float v = act_fwd((z - mu) * rs * g + bt, act, slope);
    if (a.mode == DROP_AFTER) v *= drop_scale(a.seed, ((uint64_t)b * a.C + c) * a.L + l, a.p);
    y[b * ys_b + c * ys_c + l] = v;
  }
}

__global__ __launch_bounds__(256) void bn_apply_kernel(BNArgs a_in, const float* mean, const float* rstd,
                                                       const float* gamma, const float* beta,
                                                       int act, float slope, float* y,
                                                       int64_t ys_b, int64_t ys_c) {
  A2M_BN_RESOLVE(BNArgs, a_in);
  const int c = blockIdx.x / a.slices, s = blockIdx.x % a.slices;
  const int64_t N = (int64_t)a.B * a.L;
  const int64_t i0 = (int64_t)s * kSlice, i1 = min<int64_t>(N, i0 + kSlice);
  const float mu = mean[c], rs = rstd[c], g = gamma ? gamma[c] : 1.f, bt = beta ? beta[c] : 0.f;
  #pragma unroll 4
  for (int i = (int)i0 + threadIdx.x; i < (int)i1; i += blockDim.x) {
    const int b = i / a.L, l = i - (i / a.L) * a.L;
    const float z = a.x[b * a.xs_b + c * a.xs_c + l] * pre_drop(a, b, c, l);
    float v = act_fwd((z - mu) * rs * g + bt, act, slope);
    if (a.mode == DROP_AFTER) v *= drop_scale(a.seed, ((uint64_t)b * a.C + c) * a.L + l, a.p);
    y[b * ys_b + c * ys_c + l] = v;
  }
}

struct BNBwdArgs {
  BNArgs f;
  const float* dy; int64_t dys_b, dys_c;
  const float* mean; const float* rstd; const float* gamma; const float* beta;
  int act; float slope;
  float n_div;  // element count the means divide by: B*L here, the all-rank total under SyncBN
};

// g = dL/d(bn output before act): dy * act' (* drop-after scale)
__device__ __forceinline__ float bn_g(const BNBwdArgs& a, int b, int c, int l, float xhat) {
  const float gm = a.gamma ? a.gamma[c] : 1.f, bt = a.beta ? a.beta[c] : 0.f;
  float g = a.dy[b * a.dys_b + c * a.dys_c + l] * act_grad(xhat * gm + bt, a.act, a.slope);
  if (a.f.mode == DROP_AFTER) g *= drop_scale(a.f.seed, ((uint64_t)b * a.f.C + c) * a.f.L + l, a.f.p);
  return g;
}

__global__ __launch_bounds__(256) void bn_bwd_stats_kernel(BNBwdArgs a_in, double* part) {
  A2M_BNB_RESOLVE(a_in);
  __shared__ double red[4];
  const BNArgs& f = a.f;
  const int c = blockIdx.x / f.slices, s = blockIdx.x % f.slices;
  const int64_t N = (int64_t)f.B * f.L;
  const int64_t i0 = (int64_t)s * kSlice, i1 = min<int64_t>(N, i0 + kSlice);
  const float mu = a.mean[c], rs = a.rstd[c];
  double sg = 0.0, sgx = 0.0;
  #pragma unroll 4
  for (int i = (int)i0 + threadIdx.x; i < (int)i1; i += blockDim.x) {
    const int b = i / f.L, l = i - (i / f.L) * f.L;
    const float xhat = (f.x[b * f.xs_b + c * f.xs_c + l] * pre_drop(f, b, c, l) - mu) * rs;
    const float g = bn_g(a, b, c, l, xhat);
    sg += g;
    sgx += (double)g * xhat;
  }
  sg = block_sum_d(sg, red);
  sgx = block_sum_d(sgx, red);
  if (threadIdx.x == 0) {
    part[2 * ((int64_t)c * f.slices + s)] = sg;
    part[2 * ((int64_t)c * f.slices + s) + 1] = sgx;
  }
}

// dz = gamma*rstd*(g - mean(g) - xhat*mean(g*xhat)); dx_raw = dz * drop-before scale;
// partial sums of dx_raw (the conv bias gradient) per (channel, slice)
__global__ __launch_bounds__(256) void bn_bwd_apply_kernel(BNBwdArgs a_in, const float* sums, float* dx,
                                                           double* part) {
  A2M_BNB_RESOLVE(a_in);
  __shared__ double red[4];
  const BNArgs& f = a.f;
  const int c = blockIdx.x / f.slices, s = blockIdx.x % f.slices;
  const int64_t N = (int64_t)f.B * f.L;
  const int64_t i0 = (int64_t)s * kSlice, i1 = min<int64_t>(N, i0 + kSlice);
  const float mu = a.mean[c], rs = a.rstd[c], gm = a.gamma ? a.gamma[c] : 1.f;
  const float mg = sums[2 * c] / a.n_div, mgx = sums[2 * c + 1] / a.n_div;
  double sd = 0.0;
  #pragma unroll 4
  for (int i = (int)i0 + threadIdx.x; i < (int)i1; i += blockDim.x) {
    const int b = i / f.L, l = i - (i / f.L) * f.L;
    const float ds = pre_drop(f, b, c, l);
    const float xhat = (f.x[b * f.xs_b + c * f.xs_c + l] * ds - mu) * rs;
    const float g = bn_g(a, b, c, l, xhat);
    const float v = gm * rs * (g - mg - xhat * mgx) * ds;
    dx[((int64_t)b * f.C + c) * f.L + l] = v;
    sd += v;
  }
  sd = block_sum_d(sd, red);
  if (threadIdx.x == 0) part[(int64_t)c * f.slices + s] = sd;
}

// The backward's per-channel finalize folded into the apply pass, as in the forward: each workgroup reduces
// its channel's (sum g, sum g xhat) partials in the fixed slice order, the slice-0 workgroup
// writes dgamma / dbeta; the dbias partials go to their own region (dpart) because other
// workgroups may still be reading `part`.
__global__ __launch_bounds__(256) void bn_bwd_apply_fused_kernel(BNBwdArgs a_in, const double* part,
                                                                 float* dgamma, float* dbeta,
                                                                 float* dx, double* dpart) {
  A2M_BNB_RESOLVE(a_in);
  __shared__ double red[4];
  __shared__ float sums[2];
  const BNArgs& f = a.f;
  const int c = blockIdx.x / f.slices, s = blockIdx.x % f.slices;
  if (threadIdx.x == 0) {
    double sg = 0.0, sgx = 0.0;
    for (int q = 0; q < f.slices; ++q) {
      sg += part[2 * ((int64_t)c * f.slices + q)];
      sgx += part[2 * ((int64_t)c * f.slices + q) + 1];
    }
    sums[0] = (float)sg;
    sums[1] = (float)sgx;
    if (s == 0) {
      if (dgamma) dgamma[c] = sums[1];
      if (dbeta) dbeta[c] = sums[0];
    }
  }
  __syncthreads();
  const int64_t N = (int64_t)f.B * f.L;
  const int64_t i0 = (int64_t)s * kSlice, i1 = min<int64_t>(N, i0 + kSlice);
  const float mu = a.mean[c], rs = a.rstd[c], gm = a.gamma ? a.gamma[c] : 1.f;
  const float mg = sums[0] / a.n_div, mgx = sums[1] / a.n_div;
  double sd = 0.0;
  #pragma unroll 4
  for (int i = (int)i0 + threadIdx.x; i < (int)i1; i += blockDim.x) {
    const int b = i / f.L, l = i - (i / f.L) * f.L;
    const float ds = pre_drop(f, b, c, l);
    const float xhat = (f.x[b * f.xs_b + c * f.xs_c + l] * ds - mu) * rs;
    const float g = bn_g(a, b, c, l, xhat);
    const float v = gm * rs * (g - mg - xhat * mgx) * ds;
    dx[((int64_t)b * f.C + c) * f.L + l] = v;
    sd += v;
  }
  sd = block_sum_d(sd, red);
  if (threadIdx.x == 0) dpart[(int64_t)c * f.slices + s] = sd;
}

// Eval-mode BatchNorm with gradients (nn.BatchNorm*d in .eval(), model_layers.py:51-118): the
// running statistics normalise and are not updated; the kernels above run with mean = running
// mean and rstd = 1 / sqrt(running var + eps), and the backward drops the batch-statistics terms
// (the apply divides the (sum g, sum g xhat) pair by n_div = +inf: exactly 0, so dz = gamma rstd g).
// Dropout follows the caller's Dropout module, which may still be in training mode when only the
// norms are frozen (bn.eval()): the masks are applied exactly as in the training kernels.
__global__ void bn_eval_consts_kernel(const float* rmean, const float* rvar, int C, float eps,
                                      float* mean, float* rstd) {
  const int c = blockIdx.x * blockDim.x + threadIdx.x;
  if (c < C) {
    mean[c] = rmean[c];
    rstd[c] = (float)(1.0 / sqrt((double)rvar[c] + (double)eps));
  }
}

// Whole-channel BatchNorm (round 6): one workgroup per channel when a channel's B * L elements fit
// the workgroup's registers (kChanMax): the forward reads x once, reduces (sum z, sum z^2) in the
// workgroup (float64, fixed order), finalises mean / rstd / the running statistics and applies, in
// ONE launch (the sliced path: stats + apply, x read twice); the backward reads dy and x once and
// writes dgamma / dbeta, dx and the conv-bias gradient in ONE launch (the sliced path: three).  At
// the training step's sizes most BatchNorms are latency- and launch-bound (decoder 256 x 4096,
// UNet 512..2048 x 1024..4096, D), so the launch count and the second read are the cost.
constexpr int kChanMax = 16384;

// Workgroup sums in fp64 for the whole-channel kernels, as the sliced kernels accumulate (the
// B = 2 train step is chaotic enough to amplify fp32 statistics into its gradients): wave sums
// with the DPP / permlane exchanges on the two 32-bit halves of each double (no LDS round trip
// per step, unlike __shfl_xor), one LDS slot per wave, every thread adding the slots in the same
// fixed order.
template <int CTRL>
__device__ __forceinline__ double dpp_d(double v) {
  const int64_t u = __double_as_longlong(v);
  const int lo = __builtin_amdgcn_mov_dpp((int)(u & 0xffffffff), CTRL, 0xF, 0xF, true);
  const int hi = __builtin_amdgcn_mov_dpp((int)(u >> 32), CTRL, 0xF, 0xF, true);
  return __longlong_as_double(((int64_t)hi << 32) | (uint32_t)lo);
}
__device__ __forceinline__ double wave64_sum_d(double v) {
  v += dpp_d<DPP_XOR1>(v);
  v += dpp_d<DPP_XOR2>(v);
  v += dpp_d<DPP_HALF_MIRROR>(v);
  v += dpp_d<DPP_MIRROR>(v);
  {
    const int64_t u = __double_as_longlong(v);
    const auto rl = __builtin_amdgcn_permlane16_swap((uint32_t)(u & 0xffffffff), (uint32_t)(u & 0xffffffff), false, false);
    const auto rh = __builtin_amdgcn_permlane16_swap((uint32_t)(u >> 32), (uint32_t)(u >> 32), false, false);
    v = __longlong_as_double(((int64_t)rh[0] << 32) | rl[0]) + __longlong_as_double(((int64_t)rh[1] << 32) | rl[1]);
  }
  {
    const int64_t u = __double_as_longlong(v);
    const auto rl = __builtin_amdgcn_permlane32_swap((uint32_t)(u & 0xffffffff), (uint32_t)(u & 0xffffffff), false, false);
    const auto rh = __builtin_amdgcn_permlane32_swap((uint32_t)(u >> 32), (uint32_t)(u >> 32), false, false);
    v = __longlong_as_double(((int64_t)rh[0] << 32) | rl[0]) + __longlong_as_double(((int64_t)rh[1] << 32) | rl[1]);
  }
  return v;
}
template <int NT, int NV>
__device__ __forceinline__ void chan_sum(double (&v)[NV], double* red) {
#pragma unroll
  for (int q = 0; q < NV; ++q) v[q] = wave64_sum_d(v[q]);
  __syncthreads();   // the slots' previous values have been read
  if ((threadIdx.x & 63) == 0)
#pragma unroll
    for (int q = 0; q < NV; ++q) red[q * (NT / 64) + (threadIdx.x >> 6)] = v[q];
  __syncthreads();
#pragma unroll
  for (int q = 0; q < NV; ++q) {
    double s = 0.0;
#pragma unroll
    for (int w = 0; w < NT / 64; ++w) s += red[q * (NT / 64) + w];
    v[q] = s;
  }
}

template <int NT, int EPT>
__global__ __launch_bounds__(NT) void bn_train_chan_kernel(BNArgs a_in, float eps, float momentum,
                                                            float* rmean, float* rvar, float* mean_out,
                                                            float* rstd_out, const float* gamma,
                                                            const float* beta, int act, float slope,
                                                            float* y, int64_t ys_b, int64_t ys_c) {
  A2M_BN_RESOLVE(BNArgs, a_in);
  __shared__ double red[2 * (NT / 64)];
  const int c = blockIdx.x;
  const int N = a.B * a.L;
  // the per-channel operands first: their round trips overlap the channel's loads instead of
  // following the reductions (the running-statistics update ends the kernel)
  const float g = gamma ? gamma[c] : 1.f, bt = beta ? beta[c] : 0.f;
  const float rm0 = rmean ? rmean[c] : 0.f, rv0 = rmean ? rvar[c] : 0.f;
  float z[EPT];
  double sums[2] = {0.0, 0.0};
#pragma unroll
  for (int j = 0; j < EPT; ++j) {
    const int i = threadIdx.x + NT * j;
    z[j] = 0.f;
    if (i < N) {
      const int b = i / a.L, l = i - b * a.L;
      z[j] = a.x[b * a.xs_b + c * a.xs_c + l] * pre_drop(a, b, c, l);
    }
  }
#pragma unroll
  for (int j = 0; j < EPT; ++j) {
    sums[0] += z[j];
    sums[1] += (double)z[j] * z[j];
  }
  chan_sum<NT, 2>(sums, red);
  const double mean = sums[0] / (double)N;
  double var = sums[1] / (double)N - mean * mean;
  var = var > 0.0 ? var : 0.0;
  const float mu = (float)mean, rs = (float)(1.0 / sqrt(var + (double)eps));
  if (threadIdx.x == 0) {
    mean_out[c] = mu;
    rstd_out[c] = rs;
    if (rmean) {
      const double unb = N > 1 ? var * (double)N / (double)(N - 1) : var;
      rmean[c] = (float)((1.0 - momentum) * rm0 + momentum * mean);
      rvar[c] = (float)((1.0 - momentum) * rv0 + momentum * unb);
    }
  }
#pragma unroll
  for (int j = 0; j < EPT; ++j) {
    const int i = threadIdx.x + NT * j;
    if (i < N) {
      const int b = i / a.L, l = i - b * a.L;
      float v = act_fwd((z[j] - mu) * rs * g + bt, act, slope);
      if (a.mode == DROP_AFTER) v *= drop_scale(a.seed, ((uint64_t)b * a.C + c) * a.L + l, a.p);
      y[b * ys_b + c * ys_c + l] = v;
    }
  }
}

template <int NT, int EPT>
__global__ __launch_bounds__(NT) void bn_bwd_chan_kernel(BNBwdArgs a_in, float* dgamma, float* dbeta,
                                                          float* dx, float* dbias) {
  A2M_BNB_RESOLVE(a_in);
  __shared__ double red[2 * (NT / 64)];
  const BNArgs& f = a.f;
  const int c = blockIdx.x;
  const int N = f.B * f.L;
  const float mu = a.mean[c], rs = a.rstd[c], gm = a.gamma ? a.gamma[c] : 1.f;
  float xh[EPT], gg[EPT], ds[EPT];
#pragma unroll
  for (int j = 0; j < EPT; ++j) {
    const int i = threadIdx.x + NT * j;
    xh[j] = gg[j] = ds[j] = 0.f;
    if (i < N) {
      const int b = i / f.L, l = i - b * f.L;
      ds[j] = pre_drop(f, b, c, l);
      xh[j] = (f.x[b * f.xs_b + c * f.xs_c + l] * ds[j] - mu) * rs;
      gg[j] = bn_g(a, b, c, l, xh[j]);
    }
  }
  double sums[2] = {0.0, 0.0};
#pragma unroll
  for (int j = 0; j < EPT; ++j) {
    sums[0] += gg[j];
    sums[1] += (double)gg[j] * xh[j];
  }
  chan_sum<NT, 2>(sums, red);
  const float fsg = (float)sums[0], fsgx = (float)sums[1];
  if (threadIdx.x == 0) {
    if (dgamma) dgamma[c] = fsgx;
    if (dbeta) dbeta[c] = fsg;
  }
  const float mg = fsg / a.n_div, mgx = fsgx / a.n_div;
  double sd[1] = {0.0};
#pragma unroll
  for (int j = 0; j < EPT; ++j) {
    const int i = threadIdx.x + NT * j;
    if (i < N) {
      const int b = i / f.L, l = i - b * f.L;
      const float v = gm * rs * (gg[j] - mg - xh[j] * mgx) * ds[j];
      dx[((int64_t)b * f.C + c) * f.L + l] = v;
      sd[0] += v;
    }
  }
  chan_sum<NT, 1>(sd, red);
  if (threadIdx.x == 0 && dbias) dbias[c] = (float)sd[0];
}

// the whole-channel launches, EPT = elements per thread (a power of two >= N / 256); false when the
// channel does not fit (the sliced kernels run instead)
static bool bn_chan_fwd(const BNArgs& a, float eps, float momentum, float* rmean, float* rvar, float* mean_out,
                        float* rstd_out, const float* gamma, const float* beta, int act, float slope, float* y,
                        int64_t ys_b, int64_t ys_c, hipStream_t st) {
  const int64_t N = (int64_t)a.B * a.L;
  if (N > kChanMax) return false;
#define A2M_CHAN_FWD(T, E) hipLaunchKernelGGL((bn_train_chan_kernel<T, E>), dim3(a.C), dim3(T), 0, st, a, eps, \
                                              momentum, rmean, rvar, mean_out, rstd_out, gamma, beta, act, slope, y, \
                                              ys_b, ys_c)
  // 1,024 threads (16 waves) for channels of >= 4,096 elements: every load of the channel in flight
  // at once (256 threads took 14.6 us a call at 4,096 elements, latency-bound)
  if (N <= 256) A2M_CHAN_FWD(256, 1);
  else if (N <= 512) A2M_CHAN_FWD(256, 2);
  else if (N <= 1024) A2M_CHAN_FWD(256, 4);
  else if (N <= 2048) A2M_CHAN_FWD(512, 4);
  else if (N <= 4096) A2M_CHAN_FWD(1024, 4);
  else if (N <= 8192) A2M_CHAN_FWD(1024, 8);
  else A2M_CHAN_FWD(1024, 16);
#undef A2M_CHAN_FWD
  return true;
}

static bool bn_chan_bwd(const BNBwdArgs& a, float* dgamma, float* dbeta, float* dx, float* dbias, hipStream_t st) {
  const int64_t N = (int64_t)a.f.B * a.f.L;
  if (N > kChanMax) return false;
#define A2M_CHAN_BWD(T, E) hipLaunchKernelGGL((bn_bwd_chan_kernel<T, E>), dim3(a.f.C), dim3(T), 0, st, a, dgamma, \
                                              dbeta, dx, dbias)
  if (N <= 256) A2M_CHAN_BWD(256, 1);
  else if (N <= 512) A2M_CHAN_BWD(256, 2);
  else if (N <= 1024) A2M_CHAN_BWD(256, 4);
  else if (N <= 2048) A2M_CHAN_BWD(512, 4);
  else if (N <= 4096) A2M_CHAN_BWD(1024, 4);
  else if (N <= 8192) A2M_CHAN_BWD(1024, 8);
  else A2M_CHAN_BWD(1024, 16);
#undef A2M_CHAN_BWD
  return true;
}

// SyncBN helpers: per-channel float64 (sum, sum2) pairs over the slices (all-reduced by the
// host between the stats and apply phases), and the finalize / conversion steps on them.
__global__ void reduce_pairs_kernel(const double* part, int C, int slices, double* sums,
                                    float* lo_out, float* hi_out) {
  const int c = blockIdx.x * blockDim.x + threadIdx.x;
  if (c >= C) return;
  double s1 = 0.0, s2 = 0.0;
  for (int s = 0; s < slices; ++s) {
    s1 += part[2 * ((int64_t)c * slices + s)];
    s2 += part[2 * ((int64_t)c * slices + s) + 1];
  }
  sums[2 * c] = s1;
  sums[2 * c + 1] = s2;
  if (lo_out) lo_out[c] = (float)s1;  // backward: local dbeta = sum g
  if (hi_out) hi_out[c] = (float)s2;  //           local dgamma = sum g xhat
}

__global__ void bn_finalize_sums_kernel(const double* sums, int C, int64_t N, float eps,
                                        float momentum, float* rmean, float* rvar, float* mean_out,
                                        float* rstd_out) {
  const int c = blockIdx.x * blockDim.x + threadIdx.x;
  if (c >= C) return;
  const double mean = sums[2 * c] / (double)N;
  double var = sums[2 * c + 1] / (double)N - mean * mean;
  var = var > 0.0 ? var : 0.0;
  mean_out[c] = (float)mean;
  rstd_out[c] = (float)(1.0 / sqrt(var + (double)eps));
  if (rmean) {
    const double unb = N > 1 ? var * (double)N / (double)(N - 1) : var;
    rmean[c] = (float)((1.0 - momentum) * rmean[c] + momentum * mean);
    rvar[c] = (float)((1.0 - momentum) * rvar[c] + momentum * unb);
  }
}

__global__ void sums_to_float_kernel(const double* sums, int n, float* out) {
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i < n) out[i] = (float)sums[i];
}

__global__ void reduce_slices_kernel(const double* part, int C, int slices, float* out) {
  const int c = blockIdx.x * blockDim.x + threadIdx.x;
  if (c >= C) return;
  double s = 0.0;
  for (int k = 0; k < slices; ++k) s += part[(int64_t)c * slices + k];
  out[c] = (float)s;
}

__global__ void dropout_kernel(const float* x, int64_t n, float p, uint64_t seed_in,
                               const uint64_t* seed_off, float* y) {
  const uint64_t seed = eff_seed(seed_in, seed_off, p);
  for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < n;
       i += (int64_t)gridDim.x * blockDim.x)
    y[i] = x[i] * drop_scale(seed, (uint64_t)i, p);
}

// y[c] (+)= scale * sum_{b,t} x[b][c][t]; one workgroup per channel, fixed order
__global__ __launch_bounds__(256) void sum_bt_kernel(const float* x, int64_t xs_b, int64_t xs_c,
                                                     int64_t xs_t, int B, int T, float* y,
                                                     int accumulate) {
  __shared__ double red[4];
  const int c = blockIdx.x;
  double s = 0.0;
  for (int64_t i = threadIdx.x; i < (int64_t)B * T; i += blockDim.x) {
    const int b = (int)(i / T), t = (int)(i % T);
    s += x[b * xs_b + c * xs_c + t * xs_t];
  }
  s = block_sum_d(s, red);
  if (threadIdx.x == 0) y[c] = (float)(accumulate ? y[c] + s : s);
}

// LayerNorm backward over rows [R][D]; dy element (r, d) at dy + (r/T)*s_b + d*s_d + (r%T)*s_t.
// dx = rstd*(g - mean(g) - xhat*mean(g*xhat)), g = dy*w; per-workgroup partials of
// sum(dy*xhat) and sum(dy) (dw, db) reduced by reduce_cols_kernel.
__global__ __launch_bounds__(256) void layernorm_bwd_kernel(const float* dy, int64_t s_b, int64_t s_d,
                                                            int64_t s_t, int T, const float* x, int R,
                                                            int D, const float* w, const float* mean,
                                                            const float* rstd, float* dx, float* part) {
  extern __shared__ float lsm[];  // [4 waves][2][D] partials
  const int wv = threadIdx.x >> 6, lane = threadIdx.x & 63;
  float* pw = lsm + wv * 2 * D;
  for (int d = lane; d < 2 * D; d += 64) pw[d] = 0.f;
  const int rows_per_block = (R + gridDim.x - 1) / gridDim.x;
  const int r0 = blockIdx.x * rows_per_block, r1 = min(R, r0 + rows_per_block);
  for (int r = r0 + wv; r < r1; r += 4) {
    const float mu = mean[r], rs = rstd[r];
    const float* dyr = dy + (int64_t)(r / T) * s_b + (int64_t)(r % T) * s_t;
    float g[8], xh[8];
    float sg = 0.f, sgx = 0.f;
#pragma unroll
    for (int q = 0; q < 8; ++q) {
      const int d = lane + 64 * q;
      if (d < D) {
        const float dv = dyr[d * s_d];
        xh[q] = (x[(int64_t)r * D + d] - mu) * rs;
        g[q] = dv * w[d];
        sg += g[q];
        sgx += g[q] * xh[q];
        pw[d] += dv * xh[q];
        pw[D + d] += dv;
      } else {
        g[q] = xh[q] = 0.f;
      }
    }
    sg = wave64_sum(sg);
    sgx = wave64_sum(sgx);
    const float mg = sg / (float)D, mgx = sgx / (float)D;
#pragma unroll
    for (int q = 0; q < 8; ++q) {
      const int d = lane + 64 * q;
      if (d < D) dx[(int64_t)r * D + d] = rs * (g[q] - mg - xh[q] * mgx);
    }
  }
  __syncthreads();
  for (int d = threadIdx.x; d < 2 * D; d += blockDim.x)
    part[(int64_t)blockIdx.x * 2 * D + d] = lsm[d] + lsm[2 * D + d] + lsm[4 * D + d] + lsm[6 * D + d];
}

// out[j] (+)= sum_i part[i*stride + j], i < rows, j < cols (fixed order)
// out[j] (+)= sum_i part[i*stride + j] in double.  One 1024-thread workgroup per 64 columns:
// 16 row groups per column, each summing rows g, g+16, ... with 8 loads in flight, then the 16
// partials combined in a fixed order (bitwise reproducible).
// Column j lands in the output segment i with start[i] <= j < start[i + 1] (up to 4 segments:
// one launch for several gradient vectors that share a partials row, e.g. dbias | dln_w | dln_b).
__global__ __launch_bounds__(1024) void reduce_cols_kernel(const float* part, int rows, int stride,
                                                           int cols, ColOuts outs, int accumulate) {
  __shared__ double red[16][64];
  const int c = threadIdx.x & 63, g = threadIdx.x >> 6;
  const int j = blockIdx.x * 64 + c;
  double s = 0.0;
  if (j < cols) {
#pragma unroll 8
    for (int i = g; i < rows; i += 16) s += part[(int64_t)i * stride + j];
  }
  red[g][c] = s;
  __syncthreads();
  if (g == 0 && j < cols) {
    double t = 0.0;
#pragma unroll
    for (int q = 0; q < 16; ++q) t += red[q][c];
    int seg = 0;
    while (seg + 1 < outs.n && j >= outs.start[seg + 1]) ++seg;
    float* o = outs.out[seg] + (j - outs.start[seg]);
    *o = (float)(accumulate ? *o + t : t);
  }
}

// the kernels index a channel's B * L elements in 32 bits
static int bn_slices(int64_t N) { return N < (1LL << 31) ? (int)cdiv(N, kSlice) : -1; }

int reduce_cols(const float* part, int rows, int stride, int cols, float* out, int accumulate,
                hipStream_t st) {
  ColOuts o{};
  o.out[0] = out;
  o.n = 1;
  return reduce_cols(part, rows, stride, cols, o, accumulate, st);
}

int reduce_cols(const float* part, int rows, int stride, int cols, const ColOuts& outs,
                int accumulate, hipStream_t st) {
  A2M_CHECK_ARG(outs.n >= 1 && outs.n <= 4 && outs.start[0] == 0, "reduce_cols: bad segments");
  hipLaunchKernelGGL(reduce_cols_kernel, dim3((unsigned)cdiv(cols, 64)), dim3(1024), 0, st, part,
                     rows, stride, cols, outs, accumulate);
  A2M_LAUNCH_CHECK();
  return A2M_OK;
}

}  // namespace a2m

using namespace a2m;

extern "C" {

int a2m_bn_train_fwd_f32(const float* x, int64_t xs_b, int64_t xs_c, int32_t B, int32_t C,
                         int32_t L, const float* gamma, const float* beta, float* running_mean,
                         float* running_var, float momentum, float eps, float drop_p,
                         int32_t drop_mode, uint64_t seed, int32_t act, float slope, float* y,
                         int64_t ys_b, int64_t ys_c, float* save_mean, float* save_rstd,
                         void* ws, size_t ws_bytes, void* stream) {
  A2M_CHECK_ARG(x && y && save_mean && save_rstd && B > 0 && C > 0 && L > 0, "bn_train_fwd: bad args");
  const int64_t N = (int64_t)B * L;
  const int S = bn_slices(N);
  A2M_CHECK_ARG(S > 0, "batchnorm: %lld elements per channel (at most 2^31 - 1)", (long long)N);
  const size_t need = sizeof(double) * 2 * (size_t)C * S;
  if (!ws || ws_bytes < need) { set_error("bn_train_fwd: workspace too small (%zu < %zu bytes)", ws_bytes, need); return A2M_EWS; }
  BNArgs a{x, xs_b, xs_c, B, C, L, S, drop_p, drop_mode, seed, g_seed_off};
  hipStream_t st = as_stream(stream);
  if (bn_chan_fwd(a, eps, momentum, running_mean, running_var, save_mean, save_rstd, gamma, beta, act, slope, y,
                  ys_b, ys_c, st)) {
    A2M_LAUNCH_CHECK();
    return A2M_OK;
  }
  double* part = static_cast<double*>(ws);
  hipLaunchKernelGGL(bn_stats_kernel, dim3(C * S), dim3(256), 0, st, a, part);
  A2M_LAUNCH_CHECK();
  hipLaunchKernelGGL(bn_apply_fused_kernel, dim3(C * S), dim3(256), 0, st, a, part, eps, momentum,
                     running_mean, running_var, save_mean, save_rstd, gamma, beta, act, slope, y,
                     ys_b, ys_c);
  A2M_LAUNCH_CHECK();
  return A2M_OK;
}

int a2m_bn_train_bwd_f32(const float* dy, int64_t dys_b, int64_t dys_c, const float* x,
                         int64_t xs_b, int64_t xs_c, int32_t B, int32_t C, int32_t L,
                         const float* gamma, const float* beta, const float* save_mean,
                         const float* save_rstd, float drop_p, int32_t drop_mode, uint64_t seed,
                         int32_t act, float slope, float* dx, float* dgamma, float* dbeta,
                         float* dbias, void* ws, size_t ws_bytes, void* stream) {
  A2M_CHECK_ARG(dy && x && dx && save_mean && save_rstd && B > 0 && C > 0 && L > 0, "bn_train_bwd: bad args");
  const int64_t N = (int64_t)B * L;
  const int S = bn_slices(N);
  A2M_CHECK_ARG(S > 0, "batchnorm: %lld elements per channel (at most 2^31 - 1)", (long long)N);
  const size_t need = sizeof(double) * 3 * (size_t)C * S;
  if (!ws || ws_bytes < need) { set_error("bn_train_bwd: workspace too small (%zu < %zu bytes)", ws_bytes, need); return A2M_EWS; }
  BNBwdArgs a;
  a.f = BNArgs{x, xs_b, xs_c, B, C, L, S, drop_p, drop_mode, seed, g_seed_off};
  a.dy = dy; a.dys_b = dys_b; a.dys_c = dys_c;
  a.mean = save_mean; a.rstd = save_rstd; a.gamma = gamma; a.beta = beta; a.act = act; a.slope = slope;
  a.n_div = (float)N;
  hipStream_t st = as_stream(stream);
  if (bn_chan_bwd(a, dgamma, dbeta, dx, dbias, st)) {
    A2M_LAUNCH_CHECK();
    return A2M_OK;
  }
  double* part = static_cast<double*>(ws);
  double* dpart = part + 2 * (size_t)C * S;
  hipLaunchKernelGGL(bn_bwd_stats_kernel, dim3(C * S), dim3(256), 0, st, a, part);
  A2M_LAUNCH_CHECK();
  hipLaunchKernelGGL(bn_bwd_apply_fused_kernel, dim3(C * S), dim3(256), 0, st, a, part, dgamma, dbeta,
                     dx, dpart);
  A2M_LAUNCH_CHECK();
  if (dbias) {
    hipLaunchKernelGGL(reduce_slices_kernel, dim3((unsigned)cdiv(C, 256)), dim3(256), 0, st, dpart, C,
                       S, dbias);
    A2M_LAUNCH_CHECK();
  }
  return A2M_OK;
}

int a2m_bn_eval_fwd_f32(const float* x, int64_t xs_b, int64_t xs_c, int32_t B, int32_t C, int32_t L,
                        const float* gamma, const float* beta, const float* running_mean,
                        const float* running_var, float eps, float drop_p, int32_t drop_mode,
                        uint64_t seed, int32_t act, float slope, float* y, int64_t ys_b, int64_t ys_c,
                        float* save_mean, float* save_rstd, void* stream) {
  A2M_CHECK_ARG(x && y && running_mean && running_var && save_mean && save_rstd && B > 0 && C > 0 && L > 0,
                "bn_eval_fwd: bad args");
  A2M_CHECK_ARG(drop_p >= 0.f && drop_p < 1.f && drop_mode >= DROP_NONE && drop_mode <= DROP_AFTER,
                "bn_eval_fwd: bad dropout (p %g, mode %d)", (double)drop_p, drop_mode);
  const int S = bn_slices((int64_t)B * L);
  A2M_CHECK_ARG(S > 0, "batchnorm: %lld elements per channel (at most 2^31 - 1)", (long long)B * L);
  BNArgs a{x, xs_b, xs_c, B, C, L, S, drop_p, drop_mode, seed, g_seed_off};
  hipStream_t st = as_stream(stream);
  hipLaunchKernelGGL(bn_eval_consts_kernel, dim3((unsigned)cdiv(C, 256)), dim3(256), 0, st, running_mean,
                     running_var, C, eps, save_mean, save_rstd);
  A2M_LAUNCH_CHECK();
  hipLaunchKernelGGL(bn_apply_kernel, dim3(C * S), dim3(256), 0, st, a, save_mean, save_rstd, gamma, beta,
                     act, slope, y, ys_b, ys_c);
  A2M_LAUNCH_CHECK();
  return A2M_OK;
}

int a2m_bn_eval_bwd_f32(const float* dy, int64_t dys_b, int64_t dys_c, const float* x, int64_t xs_b,
                        int64_t xs_c, int32_t B, int32_t C, int32_t L, const float* gamma,
                        const float* beta, const float* save_mean, const float* save_rstd, float drop_p,
                        int32_t drop_mode, uint64_t seed, int32_t act, float slope, float* dx,
                        float* dgamma, float* dbeta, float* dbias, void* ws, size_t ws_bytes,
                        void* stream) {
  A2M_CHECK_ARG(dy && x && dx && save_mean && save_rstd && B > 0 && C > 0 && L > 0, "bn_eval_bwd: bad args");
  A2M_CHECK_ARG(drop_p >= 0.f && drop_p < 1.f && drop_mode >= DROP_NONE && drop_mode <= DROP_AFTER,
                "bn_eval_bwd: bad dropout (p %g, mode %d)", (double)drop_p, drop_mode);
  const int64_t N = (int64_t)B * L;
  const int S = bn_slices(N);
  A2M_CHECK_ARG(S > 0, "batchnorm: %lld elements per channel (at most 2^31 - 1)", (long long)N);
  const size_t need = sizeof(double) * 3 * (size_t)C * S;
  if (!ws || ws_bytes < need) { set_error("bn_eval_bwd: workspace too small (%zu < %zu bytes)", ws_bytes, need); return A2M_EWS; }
  BNBwdArgs a;
  a.f = BNArgs{x, xs_b, xs_c, B, C, L, S, drop_p, drop_mode, seed, g_seed_off};
  a.dy = dy; a.dys_b = dys_b; a.dys_c = dys_c;
  a.mean = save_mean; a.rstd = save_rstd; a.gamma = gamma; a.beta = beta; a.act = act; a.slope = slope;
  a.n_div = __builtin_inff();   // fixed statistics: no mean(g) / mean(g xhat) terms
  hipStream_t st = as_stream(stream);
  if (bn_chan_bwd(a, dgamma, dbeta, dx, dbias, st)) {
    A2M_LAUNCH_CHECK();
    return A2M_OK;
  }
  double* part = static_cast<double*>(ws);
  double* dpart = part + 2 * (size_t)C * S;
  hipLaunchKernelGGL(bn_bwd_stats_kernel, dim3(C * S), dim3(256), 0, st, a, part);
  A2M_LAUNCH_CHECK();
  hipLaunchKernelGGL(bn_bwd_apply_fused_kernel, dim3(C * S), dim3(256), 0, st, a, part, dgamma, dbeta,
                     dx, dpart);
  A2M_LAUNCH_CHECK();
  if (dbias) {
    hipLaunchKernelGGL(reduce_slices_kernel, dim3((unsigned)cdiv(C, 256)), dim3(256), 0, st, dpart, C,
                       S, dbias);
    A2M_LAUNCH_CHECK();
  }
  return A2M_OK;
}

// ---- SyncBN phases (the fused entry points above split at their reductions)
int a2m_bn_sync_stats_f32(const float* x, int64_t xs_b, int64_t xs_c, int32_t B, int32_t C,
                          int32_t L, float drop_p, int32_t drop_mode, uint64_t seed, double* sums,
                          void* ws, size_t ws_bytes, void* stream) {
  A2M_CHECK_ARG(x && sums && B > 0 && C > 0 && L > 0, "bn_sync_stats: bad args");
  const int64_t N = (int64_t)B * L;
  const int S = bn_slices(N);
  A2M_CHECK_ARG(S > 0, "batchnorm: %lld elements per channel (at most 2^31 - 1)", (long long)N);
  const size_t need = sizeof(double) * 2 * (size_t)C * S;
  if (!ws || ws_bytes < need) { set_error("bn_sync_stats: workspace too small (%zu < %zu bytes)", ws_bytes, need); return A2M_EWS; }
  BNArgs a{x, xs_b, xs_c, B, C, L, S, drop_p, drop_mode, seed, g_seed_off};
  hipStream_t st = as_stream(stream);
  double* part = static_cast<double*>(ws);
  hipLaunchKernelGGL(bn_stats_kernel, dim3(C * S), dim3(256), 0, st, a, part);
  A2M_LAUNCH_CHECK();
  hipLaunchKernelGGL(reduce_pairs_kernel, dim3((unsigned)cdiv(C, 256)), dim3(256), 0, st, part, C, S,
                     sums, nullptr, nullptr);
  A2M_LAUNCH_CHECK();
  return A2M_OK;
}

int a2m_bn_sync_apply_f32(const float* x, int64_t xs_b, int64_t xs_c, int32_t B, int32_t C,
                          int32_t L, const double* sums, int64_t n_total, const float* gamma,
                          const float* beta, float* running_mean, float* running_var,
                          float momentum, float eps, float drop_p, int32_t drop_mode,
                          uint64_t seed, int32_t act, float slope, float* y, int64_t ys_b,
                          int64_t ys_c, float* save_mean, float* save_rstd, void* stream) {
  A2M_CHECK_ARG(x && y && sums && save_mean && save_rstd && B > 0 && C > 0 && L > 0 && n_total > 0,
                "bn_sync_apply: bad args");
  const int S = bn_slices((int64_t)B * L);
  BNArgs a{x, xs_b, xs_c, B, C, L, S, drop_p, drop_mode, seed, g_seed_off};
  hipStream_t st = as_stream(stream);
  hipLaunchKernelGGL(bn_finalize_sums_kernel, dim3((unsigned)cdiv(C, 256)), dim3(256), 0, st, sums, C,
                     n_total, eps, momentum, running_mean, running_var, save_mean, save_rstd);
  A2M_LAUNCH_CHECK();
  hipLaunchKernelGGL(bn_apply_kernel, dim3(C * S), dim3(256), 0, st, a, save_mean, save_rstd, gamma,
                     beta, act, slope, y, ys_b, ys_c);
  A2M_LAUNCH_CHECK();
  return A2M_OK;
}

int a2m_bn_sync_bwd_stats_f32(const float* dy, int64_t dys_b, int64_t dys_c, const float* x,
                              int64_t xs_b, int64_t xs_c, int32_t B, int32_t C, int32_t L,
                              const float* gamma, const float* beta, const float* save_mean,
                              const float* save_rstd, float drop_p, int32_t drop_mode,
                              uint64_t seed, int32_t act, float slope, double* sums,
                              float* dgamma, float* dbeta, void* ws, size_t ws_bytes, void* stream) {
  A2M_CHECK_ARG(dy && x && sums && save_mean && save_rstd && B > 0 && C > 0 && L > 0,
                "bn_sync_bwd_stats: bad args");
  const int64_t N = (int64_t)B * L;
  const int S = bn_slices(N);
  A2M_CHECK_ARG(S > 0, "batchnorm: %lld elements per channel (at most 2^31 - 1)", (long long)N);
  const size_t need = sizeof(double) * 2 * (size_t)C * S;
  if (!ws || ws_bytes < need) { set_error("bn_sync_bwd_stats: workspace too small (%zu < %zu bytes)", ws_bytes, need); return A2M_EWS; }
  BNBwdArgs a;
  a.f = BNArgs{x, xs_b, xs_c, B, C, L, S, drop_p, drop_mode, seed, g_seed_off};
  a.dy = dy; a.dys_b = dys_b; a.dys_c = dys_c;
  a.mean = save_mean; a.rstd = save_rstd; a.gamma = gamma; a.beta = beta; a.act = act; a.slope = slope;
  a.n_div = (float)N;
  hipStream_t st = as_stream(stream);
  double* part = static_cast<double*>(ws);
  hipLaunchKernelGGL(bn_bwd_stats_kernel, dim3(C * S), dim3(256), 0, st, a, part);
  A2M_LAUNCH_CHECK();
  hipLaunchKernelGGL(reduce_pairs_kernel, dim3((unsigned)cdiv(C, 256)), dim3(256), 0, st, part, C, S,
                     sums, dbeta, dgamma);
  A2M_LAUNCH_CHECK();
  return A2M_OK;
}

int a2m_bn_sync_bwd_apply_f32(const float* dy, int64_t dys_b, int64_t dys_c, const float* x,
                              int64_t xs_b, int64_t xs_c, int32_t B, int32_t C, int32_t L,
                              const float* gamma, const float* beta, const float* save_mean,
                              const float* save_rstd, float drop_p, int32_t drop_mode,
                              uint64_t seed, int32_t act, float slope, const double* sums,
                              int64_t n_total, float* dx, float* dbias, void* ws, size_t ws_bytes,
                              void* stream) {
  A2M_CHECK_ARG(dy && x && dx && sums && save_mean && save_rstd && B > 0 && C > 0 && L > 0 &&
                n_total > 0, "bn_sync_bwd_apply: bad args");
  const int64_t N = (int64_t)B * L;
  const int S = bn_slices(N);
  A2M_CHECK_ARG(S > 0, "batchnorm: %lld elements per channel (at most 2^31 - 1)", (long long)N);
  const size_t need = sizeof(double) * (size_t)C * S + sizeof(float) * 2 * (size_t)C + 16;
  if (!ws || ws_bytes < need) { set_error("bn_sync_bwd_apply: workspace too small (%zu < %zu bytes)", ws_bytes, need); return A2M_EWS; }
  BNBwdArgs a;
  a.f = BNArgs{x, xs_b, xs_c, B, C, L, S, drop_p, drop_mode, seed, g_seed_off};
  a.dy = dy; a.dys_b = dys_b; a.dys_c = dys_c;
  a.mean = save_mean; a.rstd = save_rstd; a.gamma = gamma; a.beta = beta; a.act = act; a.slope = slope;
  a.n_div = (float)n_total;
  hipStream_t st = as_stream(stream);
  double* part = static_cast<double*>(ws);
  float* fsums = reinterpret_cast<float*>(part + (size_t)C * S);
  hipLaunchKernelGGL(sums_to_float_kernel, dim3((unsigned)cdiv(2 * C, 256)), dim3(256), 0, st, sums,
                     2 * C, fsums);
  A2M_LAUNCH_CHECK();
  hipLaunchKernelGGL(bn_bwd_apply_kernel, dim3(C * S), dim3(256), 0, st, a, fsums, dx, part);
  A2M_LAUNCH_CHECK();
  if (dbias) {
    hipLaunchKernelGGL(reduce_slices_kernel, dim3((unsigned)cdiv(C, 256)), dim3(256), 0, st, part, C,
                       S, dbias);
    A2M_LAUNCH_CHECK();
  }
  return A2M_OK;
}

int a2m_set_dropout_seed_offset(const uint64_t* counter) {
  g_seed_off = counter;
  return A2M_OK;
}

int a2m_dropout_f32(const float* x, int64_t n, float p, uint64_t seed, float* y, void* stream) {
  A2M_CHECK_ARG(x && y && n >= 0 && p >= 0.f && p < 1.f, "dropout: bad args");
  if (n == 0) return A2M_OK;
  const int blocks = (int)std::min<int64_t>(cdiv(n, 256), 8192);
  hipLaunchKernelGGL(dropout_kernel, dim3(blocks), dim3(256), 0, as_stream(stream), x, n, p, seed,
                     g_seed_off, y);
  A2M_LAUNCH_CHECK();
  return A2M_OK;
}

int a2m_sum_bt_f32(const float* x, int64_t xs_b, int64_t xs_c, int64_t xs_t, int32_t B, int32_t C,
                   int32_t T, float* y, int32_t accumulate, void* stream) {
  A2M_CHECK_ARG(x && y && B > 0 && C > 0 && T > 0, "sum_bt: bad args");
  hipLaunchKernelGGL(sum_bt_kernel, dim3(C), dim3(256), 0, as_stream(stream), x, xs_b, xs_c, xs_t, B,
                     T, y, accumulate);
  A2M_LAUNCH_CHECK();
  return A2M_OK;
}

int a2m_layernorm_bwd_f32(const float* dy, int64_t dys_b, int64_t dys_d, int64_t dys_t, int32_t T,
                          const float* x, int32_t R, int32_t D, const float* w, const float* mean,
                          const float* rstd, float* dx, float* dw, float* db, void* ws,
                          size_t ws_bytes, void* stream) {
  A2M_CHECK_ARG(dy && x && w && mean && rstd && dx && dw && db && R > 0 && D > 0 && D <= 512,
                "layernorm_bwd: bad args");
  const int blocks = (int)std::min<int64_t>(cdiv(R, 16), 1024);
  const size_t need = sizeof(float) * (size_t)blocks * 2 * D;
  if (!ws || ws_bytes < need) { set_error("layernorm_bwd: workspace too small (%zu < %zu bytes)", ws_bytes, need); return A2M_EWS; }
  float* part = static_cast<float*>(ws);
  hipStream_t st = as_stream(stream);
  hipLaunchKernelGGL(layernorm_bwd_kernel, dim3(blocks), dim3(256), sizeof(float) * 8 * D, st, dy,
                     dys_b, dys_d, dys_t, T, x, R, D, w, mean, rstd, dx, part);
  A2M_LAUNCH_CHECK();
  ColOuts outs{};
  outs.out[0] = dw; outs.start[0] = 0;
  outs.out[1] = db; outs.start[1] = D;
  outs.n = 2;
  return reduce_cols(part, blocks, 2 * D, 2 * D, outs, 0, st);
}

}  // extern "C"
