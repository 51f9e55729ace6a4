// Fused skeleton-graph layer of the body / hand decoders
// (real_motion_model.py:173-201 body, :225-253 hand; PyG layer semantics restated in
// oracle/pyg_restatement.py):
//     y = LeakyReLU(LayerNorm64(L(x))) + x,   L = GATConv(64,64,heads=4,concat=False) | GraphConv
// Every frame is an independent J-node tree (J = 10 body, 42 hand) with the same in-neighbour
// CSR, so a workgroup owns FPB = 128 / J whole frames: the node tile x [NB][64] is loaded
// into LDS once (coalesced float4), the 64x64 per-head projections run as register-tiled
// fp32 FMAs against an LDS copy of the (transposed) weight, the edge softmax / neighbour
// aggregation read LDS only, and LayerNorm(64) is a 16-lane shuffle reduction over the
// threads that hold one node's 64 features.  HBM traffic per layer = x in + y out
// (2 x 256 B per node); the weights stay in L2.
#include "a2m_internal.h"

namespace a2m {

constexpr int GF = 64;         // joint feature dim
constexpr int GHEADS = 4;
constexpr int GMAXN = 128;     // nodes per workgroup
constexpr int GR = GMAXN / 16; // node rows per thread
constexpr int ZP = GF + 4;     // LDS pitch of node rows (floats), 16-B aligned, staggers banks

__device__ __forceinline__ void load_wt(float* wt, const float* w, int row0, int ld) {
  // wt[k][c] = w[(row0 + c) * ld + k], c, k in [0, 64)
  for (int i = threadIdx.x; i < GF * GF; i += blockDim.x) {
    const int c = i / GF, k = i % GF;
    wt[k * GF + c] = w[(int64_t)(row0 + c) * ld + k];
  }
}

// acc[r][0..3] (+)= sum_k src[n_r][k] * wt[k][cg*4 .. cg*4+3]
__device__ __forceinline__ void tile_matmul(float (&acc)[GR][4], const float* src, const float* wt,
                                            int nrow0, int cg, int NB) {
#pragma unroll 4
  for (int k = 0; k < GF; k += 4) {
    float4 w4[4];
#pragma unroll
    for (int q = 0; q < 4; ++q) w4[q] = *reinterpret_cast<const float4*>(wt + (k + q) * GF + cg * 4);
#pragma unroll
    for (int r = 0; r < GR; ++r) {
      const int n = nrow0 + 16 * r;
      if (n >= NB) break;
      const float4 xv = *reinterpret_cast<const float4*>(src + n * ZP + k);
      const float xa[4] = {xv.x, xv.y, xv.z, xv.w};
#pragma unroll
      for (int q = 0; q < 4; ++q) {
        acc[r][0] += xa[q] * w4[q].x;
        acc[r][1] += xa[q] * w4[q].y;
        acc[r][2] += xa[q] * w4[q].z;
        acc[r][3] += xa[q] * w4[q].w;
      }
    }
  }
}

__global__ __launch_bounds__(256) void graph_layer_kernel(
    const float* __restrict__ x, int F, int J, int kind, int norm_res, const int* __restrict__ nbr_ptr,
    const int* __restrict__ nbr_idx, const float* __restrict__ w0, const float* __restrict__ w1,
    const float* __restrict__ att_src, const float* __restrict__ att_dst,
    const float* __restrict__ bias, const float* __restrict__ ln_w, const float* __restrict__ ln_b,
    float slope, float* __restrict__ y, float* __restrict__ pre_ln) {
  __shared__ __attribute__((aligned(16))) float xs[GMAXN * ZP];
  __shared__ __attribute__((aligned(16))) float zs[GMAXN * ZP];
  __shared__ __attribute__((aligned(16))) float wt[GF * GF];
  __shared__ float asrc[GMAXN], adst[GMAXN];

  const int fpb = GMAXN / J;
  const int NBmax = fpb * J;
  const int64_t node0 = (int64_t)blockIdx.x * NBmax;
  const int64_t nodes_total = (int64_t)F * J;
  const int NB = (int)min<int64_t>(NBmax, nodes_total - node0);
  const int tid = threadIdx.x;
  const int cg = tid & 15, nrow0 = tid >> 4;

  // load x tile (float4 per thread-step)
  for (int i = tid; i < NB * (GF / 4); i += blockDim.x) {
    const int n = i / (GF / 4), q = i % (GF / 4);
    *reinterpret_cast<float4*>(xs + n * ZP + q * 4) =
        *reinterpret_cast<const float4*>(x + (node0 + n) * GF + q * 4);
  }

  float out[GR][4];
#pragma unroll
  for (int r = 0; r < GR; ++r) out[r][0] = out[r][1] = out[r][2] = out[r][3] = 0.f;

  if (kind == 0) {
    for (int h = 0; h < GHEADS; ++h) {
      __syncthreads();  // previous head done with zs / wt
      load_wt(wt, w0, h * GF, GF);
      __syncthreads();
      float z[GR][4];
#pragma unroll
      for (int r = 0; r < GR; ++r) z[r][0] = z[r][1] = z[r][2] = z[r][3] = 0.f;
      tile_matmul(z, xs, wt, nrow0, cg, NB);
#pragma unroll
      for (int r = 0; r < GR; ++r) {
        const int n = nrow0 + 16 * r;
        if (n < NB)
          *reinterpret_cast<float4*>(zs + n * ZP + cg * 4) = make_float4(z[r][0], z[r][1], z[r][2], z[r][3]);
      }
      __syncthreads();
      for (int i = tid; i < 2 * NB; i += blockDim.x) {
        const int n = i % NB;
        const float* a = (i < NB ? att_src : att_dst) + h * GF;
        const float* zr = zs + n * ZP;
        float s = 0.f;
        for (int c = 0; c < GF; ++c) s += zr[c] * a[c];
        (i < NB ? asrc : adst)[n] = s;
      }
      __syncthreads();
#pragma unroll
      for (int r = 0; r < GR; ++r) {
        const int n = nrow0 + 16 * r;
        if (n >= NB) break;
        const int f0 = (n / J) * J, li = n % J;
        const int e0 = nbr_ptr[li], e1 = nbr_ptr[li + 1];
        const float ad = adst[n];
        // PyG: edges (in edge order) then the appended self loop
        float mx = -INFINITY;
        for (int e = e0; e <= e1; ++e) {
          const int j = e < e1 ? f0 + nbr_idx[e] : n;
          float s = asrc[j] + ad;
          s = s > 0.f ? s : s * 0.2f;
          mx = fmaxf(mx, s);
        }
        float den = 0.f;
        for (int e = e0; e <= e1; ++e) {
          const int j = e < e1 ? f0 + nbr_idx[e] : n;
          float s = asrc[j] + ad;
          s = s > 0.f ? s : s * 0.2f;
          den += expf(s - mx);
        }
        const float inv = 1.f / (den + 1e-16f);
        float agg[4] = {0.f, 0.f, 0.f, 0.f};
        for (int e = e0; e <= e1; ++e) {
          const int j = e < e1 ? f0 + nbr_idx[e] : n;
          float s = asrc[j] + ad;
          s = s > 0.f ? s : s * 0.2f;
          const float al = expf(s - mx) * inv;
          const float4 zj = *reinterpret_cast<const float4*>(zs + j * ZP + cg * 4);
          agg[0] += zj.x * al; agg[1] += zj.y * al; agg[2] += zj.z * al; agg[3] += zj.w * al;
        }
#pragma unroll
        for (int q = 0; q < 4; ++q) out[r][q] += agg[q];
      }
    }
#pragma unroll
    for (int r = 0; r < GR; ++r)
#pragma unroll
      for (int q = 0; q < 4; ++q) out[r][q] = out[r][q] * 0.25f + bias[cg * 4 + q];
  } else {
    __syncthreads();
    // aggregated neighbours (sum over in-edges) into zs
    for (int i = tid; i < NB * (GF / 4); i += blockDim.x) {
      const int n = i / (GF / 4), q = i % (GF / 4);
      const int f0 = (n / J) * J, li = n % J;
      float4 a = make_float4(0.f, 0.f, 0.f, 0.f);
      for (int e = nbr_ptr[li]; e < nbr_ptr[li + 1]; ++e) {
        const float4 v = *reinterpret_cast<const float4*>(xs + (f0 + nbr_idx[e]) * ZP + q * 4);
        a.x += v.x; a.y += v.y; a.z += v.z; a.w += v.w;
      }
      *reinterpret_cast<float4*>(zs + n * ZP + q * 4) = a;
    }
    load_wt(wt, w0, 0, GF);  // lin_rel
    __syncthreads();
    float rel[GR][4];
#pragma unroll
    for (int r = 0; r < GR; ++r) rel[r][0] = rel[r][1] = rel[r][2] = rel[r][3] = 0.f;
    tile_matmul(rel, zs, wt, nrow0, cg, NB);
    __syncthreads();
    load_wt(wt, w1, 0, GF);  // lin_root
    __syncthreads();
    tile_matmul(out, xs, wt, nrow0, cg, NB);
#pragma unroll
    for (int r = 0; r < GR; ++r)
#pragma unroll
      for (int q = 0; q < 4; ++q) out[r][q] = (rel[r][q] + bias[cg * 4 + q]) + out[r][q];
  }

  if (!norm_res) {
#pragma unroll
    for (int r = 0; r < GR; ++r) {
      const int n = nrow0 + 16 * r;
      if (n < NB)
        *reinterpret_cast<float4*>(y + (node0 + n) * GF + cg * 4) =
            make_float4(out[r][0], out[r][1], out[r][2], out[r][3]);
    }
    return;
  }
  // LayerNorm(64) over the 16 lanes that hold one node, LeakyReLU, residual, store.
#pragma unroll
  for (int r = 0; r < GR; ++r) {
    const int n = nrow0 + 16 * r;   // uniform across the 16-lane group
    float s = out[r][0] + out[r][1] + out[r][2] + out[r][3];
    for (int o = 1; o < 16; o <<= 1) s += __shfl_xor(s, o);
    const float mean = s * (1.f / GF);
    float ss = 0.f;
#pragma unroll
    for (int q = 0; q < 4; ++q) {
      const float c = out[r][q] - mean;
      ss += c * c;
    }
    for (int o = 1; o < 16; o <<= 1) ss += __shfl_xor(ss, o);
    const float rstd = 1.f / sqrtf(ss * (1.f / GF) + 1e-5f);
    if (n >= NB) continue;
    float v[4];
#pragma unroll
    for (int q = 0; q < 4; ++q) {
      const int c = cg * 4 + q;
      float t = (out[r][q] - mean) * rstd * ln_w[c] + ln_b[c];
      t = t > 0.f ? t : t * slope;
      v[q] = t + xs[n * ZP + c];
    }
    *reinterpret_cast<float4*>(y + (node0 + n) * GF + cg * 4) = make_float4(v[0], v[1], v[2], v[3]);
    if (pre_ln)
      *reinterpret_cast<float4*>(pre_ln + (node0 + n) * GF + cg * 4) =
          make_float4(out[r][0], out[r][1], out[r][2], out[r][3]);
  }
}

}  // namespace a2m

using namespace a2m;

extern "C" int a2m_graph_layer_fwd_f32(const float* x, int32_t F, int32_t J, int32_t kind,
                                       int32_t norm_res, const int32_t* nbr_ptr, const int32_t* nbr_idx,
                                       const float* w0, const float* w1, const float* att_src,
                                       const float* att_dst, const float* bias,
                                       const float* ln_w, const float* ln_b, float slope, float* y,
                                       float* lin_out, float* pre_ln, void* ws, size_t ws_bytes,
                                       void* stream) {
  (void)lin_out; (void)ws; (void)ws_bytes;
  A2M_CHECK_ARG(x && y && nbr_ptr && nbr_idx && w0 && bias && (!norm_res || (ln_w && ln_b)),
                "graph_layer: null pointer");
  A2M_CHECK_ARG(J > 0 && J <= GMAXN && F >= 0, "graph_layer: bad J=%d", J);
  A2M_CHECK_ARG(kind == 0 ? (att_src && att_dst) : (kind == 1 && w1), "graph_layer: bad kind/params");
  A2M_CHECK_ARG(x != y, "graph_layer: in-place not supported");
  if (F == 0) return A2M_OK;
  const int fpb = GMAXN / J;
  const int64_t blocks = cdiv(F, fpb);
  hipLaunchKernelGGL(graph_layer_kernel, dim3((unsigned)blocks), dim3(256), 0, as_stream(stream),
                     x, F, J, kind, norm_res, nbr_ptr, nbr_idx, w0, w1, att_src, att_dst, bias, ln_w, ln_b,
                     slope, y, pre_ln);
  A2M_LAUNCH_CHECK();
  return A2M_OK;
}
