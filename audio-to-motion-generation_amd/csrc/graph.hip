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

constexpr int GF = 64;          // joint feature dim
constexpr int GHEADS = 4;
constexpr int GMAXN = 128;      // node rows per workgroup (4 waves x 32 MFMA rows)
constexpr int ZP = GF + 4;      // LDS row pitch (floats): 16-B aligned, conflict-free b128 reads
constexpr int GMAXDEG = 8;      // max in-degree (+ self loop) of a skeleton node (hand roots: 5 + 1)

typedef float floatx16 __attribute__((ext_vector_type(16)));

// Layer math, restructured "aggregate, then transform" so the 256-wide GAT projection is
// never materialised:
//   GAT:  a_src[n,h] = x_n . (W_h^T att_src_h),  a_dst likewise      (8 dot products / node)
//         alpha = edge softmax_h(leaky(a_src[j,h] + a_dst[i,h]))      (in-edges + self loop)
//         out_i = 1/4 sum_h (sum_j alpha_ijh x_j) W_h^T + bias         (K = 4 x 64 MFMA GEMM)
//   GraphConv: out_i = (sum_{j->i} x_j) W_rel^T + x_i W_root^T + b_rel (K = 2 x 64)
// The per-segment A tile [128 rows][64] is built in LDS by VALU, then 4 waves run
// v_mfma_f32_32x32x2_f32 with B fragments (64 output channels) read straight from L2.
// U[q][k] = sum_c W_h[c][k] att_h[c], q = h (source) or 4 + h (target): the attention logits
// a_{src,dst}[n,h] = x_n . U[q] without projecting x (one 512-thread block per layer).
__global__ __launch_bounds__(512) void graph_att_proj_kernel(const float* __restrict__ w0,
                                                             const float* __restrict__ att_src,
                                                             const float* __restrict__ att_dst,
                                                             float* __restrict__ Ug) {
  const int q = threadIdx.x / GF, k = threadIdx.x % GF, h = q & 3;
  const float* att = (q < GHEADS ? att_src : att_dst) + h * GF;
  const float* wk = w0 + (int64_t)h * GF * GF + k;
  float s = 0.f;
  for (int c = 0; c < GF; ++c) s += wk[c * GF] * att[c];
  Ug[threadIdx.x] = s;
}

__global__ __launch_bounds__(256, 2) void graph_layer_kernel(
    const float* __restrict__ x, int F, int J, int kind, int norm_res, const int* __restrict__ nbr_ptr,
    const int* __restrict__ nbr_idx, const float* __restrict__ w0, const float* __restrict__ w1,
    const float* __restrict__ att_src, const float* __restrict__ att_dst,
    const float* __restrict__ bias, const float* __restrict__ ln_w, const float* __restrict__ ln_b,
    float slope, const float* __restrict__ Ug, float* __restrict__ y, float* __restrict__ pre_ln) {
  __shared__ __attribute__((aligned(16))) float xs[GMAXN * ZP];
  __shared__ __attribute__((aligned(16))) float ys[GMAXN * ZP];
  // U (attention projections) is only needed before the segment loop, the per-head edge
  // weights ew only inside it: they share one 4 KB array so two workgroups fit per CU.
  __shared__ __attribute__((aligned(16))) float u_ew[GMAXN * GMAXDEG];
  float (*U)[GF] = reinterpret_cast<float (*)[GF]>(u_ew);
  float (*ew)[GMAXDEG] = reinterpret_cast<float (*)[GMAXDEG]>(u_ew);
  __shared__ float al[GMAXN][2 * GHEADS];
  __shared__ unsigned char nbl[GMAXN][GMAXDEG];
  __shared__ unsigned char ndeg[GMAXN];

  const int fpb = GMAXN / J;
  const int NBmax = fpb * J;
  const int64_t node0 = (int64_t)blockIdx.x * NBmax;
  const int NB = (int)min<int64_t>(NBmax, (int64_t)F * J - node0);
  const int tid = threadIdx.x;
  const int lane = tid & 63, wave = tid >> 6;
  const int li = lane & 31, lh = lane >> 5;

  for (int i = tid; i < GMAXN * (GF / 4); i += blockDim.x) {
    const int n = i / (GF / 4), q = i % (GF / 4);
    float4 v = make_float4(0.f, 0.f, 0.f, 0.f);
    if (n < NB) v = *reinterpret_cast<const float4*>(x + (node0 + n) * GF + q * 4);
    *reinterpret_cast<float4*>(xs + n * ZP + q * 4) = v;
  }
  if (kind == 0)
    for (int i = tid; i < 2 * GHEADS * GF; i += blockDim.x) (&U[0][0])[i] = Ug[i];
  // block-local neighbour lists: in-edges in edge order, then (GAT) the PyG self loop
  for (int n = tid; n < NB; n += blockDim.x) {
    const int f0 = (n / J) * J, ln = n % J;
    const int e0 = nbr_ptr[ln], e1 = nbr_ptr[ln + 1];
    int d = 0;
    for (int e = e0; e < e1 && d < GMAXDEG; ++e) nbl[n][d++] = f0 + nbr_idx[e];
    if (kind == 0 && d < GMAXDEG) nbl[n][d++] = n;
    ndeg[n] = d;
  }
  __syncthreads();
  if (kind == 0) {
    for (int i = tid; i < NB * 2 * GHEADS; i += blockDim.x) {
      const int n = i >> 3, q = i & 7;
      const float* xr = xs + n * ZP;
      float s = 0.f;
      for (int k = 0; k < GF; ++k) s += xr[k] * U[q][k];
      al[n][q] = s;
    }
    __syncthreads();
  }

  floatx16 acc[2];
#pragma unroll
  for (int t = 0; t < 2; ++t)
#pragma unroll
    for (int q = 0; q < 16; ++q) acc[t][q] = 0.f;

  const int nseg = kind == 0 ? GHEADS : 2;
  const int arow = wave * 32 + li;
  for (int seg = 0; seg < nseg; ++seg) {
    const float* W = kind == 0 ? w0 + (int64_t)seg * GF * GF : (seg == 0 ? w0 : w1);
    // B fragments: lane (li, lh) needs W[t*32 + li][kc*16 + 8*lh .. +8]; issue before the build
    float4 bw[2][4][2];
#pragma unroll
    for (int t = 0; t < 2; ++t)
#pragma unroll
      for (int kc = 0; kc < 4; ++kc) {
        const float* p = W + (t * 32 + li) * GF + kc * 16 + lh * 8;
        bw[t][kc][0] = *reinterpret_cast<const float4*>(p);
        bw[t][kc][1] = *reinterpret_cast<const float4*>(p + 4);
      }
    const float* A = ys;
    if (kind == 0 || seg == 0) {
      if (kind == 0) {  // edge softmax of head `seg`, one thread per target node
        for (int n = tid; n < NB; n += blockDim.x) {
          const int d = ndeg[n];
          const float ad = al[n][GHEADS + seg];
          float e[GMAXDEG];
          float mx = -INFINITY;
#pragma unroll
          for (int q = 0; q < GMAXDEG; ++q) {
            if (q < d) {
              float s = al[nbl[n][q]][seg] + ad;
              e[q] = s > 0.f ? s : s * 0.2f;
              mx = fmaxf(mx, e[q]);
            }
          }
          float den = 0.f;
#pragma unroll
          for (int q = 0; q < GMAXDEG; ++q)
            if (q < d) { e[q] = expf(e[q] - mx); den += e[q]; }
          const float inv = 1.f / (den + 1e-16f);
#pragma unroll
          for (int q = 0; q < GMAXDEG; ++q) ew[n][q] = q < d ? e[q] * inv : 0.f;
        }
        __syncthreads();
      }
      // 16 threads per node row, 4 features each: ys[n] = sum_q w_q x[nbl[n][q]]
      for (int i = tid; i < GMAXN * 16; i += blockDim.x) {
        const int n = i >> 4, cg = i & 15;
        float4 a = make_float4(0.f, 0.f, 0.f, 0.f);
        const int d = n < NB ? ndeg[n] : 0;
        for (int q = 0; q < d; ++q) {
          const float w = kind == 0 ? ew[n][q] : 1.f;
          const float4 v = *reinterpret_cast<const float4*>(xs + nbl[n][q] * ZP + cg * 4);
          a.x += w * v.x; a.y += w * v.y; a.z += w * v.z; a.w += w * v.w;
        }
        *reinterpret_cast<float4*>(ys + n * ZP + cg * 4) = a;
      }
      __syncthreads();
    } else {
      A = xs;  // GraphConv root term
    }
#pragma unroll
    for (int kc = 0; kc < 4; ++kc) {
      const float* p = A + arow * ZP + kc * 16 + lh * 8;
      const float4 a0 = *reinterpret_cast<const float4*>(p);
      const float4 a1 = *reinterpret_cast<const float4*>(p + 4);
      const float af[8] = {a0.x, a0.y, a0.z, a0.w, a1.x, a1.y, a1.z, a1.w};
#pragma unroll
      for (int t = 0; t < 2; ++t) {
        const float bf[8] = {bw[t][kc][0].x, bw[t][kc][0].y, bw[t][kc][0].z, bw[t][kc][0].w,
                             bw[t][kc][1].x, bw[t][kc][1].y, bw[t][kc][1].z, bw[t][kc][1].w};
#pragma unroll
        for (int s = 0; s < 8; ++s)
          acc[t] = __builtin_amdgcn_mfma_f32_32x32x2f32(af[s], bf[s], acc[t], 0, 0, 0);
      }
    }
    __syncthreads();  // ys is rebuilt by the next segment
  }

  // accumulators -> ys (pre-LayerNorm layer output)
  const float scale = kind == 0 ? 1.f / GHEADS : 1.f;
#pragma unroll
  for (int t = 0; t < 2; ++t)
#pragma unroll
    for (int q = 0; q < 16; ++q) {
      const int r = wave * 32 + (q & 3) + 8 * (q >> 2) + 4 * lh;
      const int c = t * 32 + li;
      ys[r * ZP + c] = kind == 0 ? acc[t][q] * scale + bias[c] : acc[t][q] + bias[c];
    }
  __syncthreads();

  // 16 lanes per node row: LayerNorm(64) by shuffles, LeakyReLU, residual, float4 stores
  const int cg = tid & 15;
  for (int n = tid >> 4; n < GMAXN; n += 16) {
    const float4 o4 = *reinterpret_cast<const float4*>(ys + n * ZP + cg * 4);
    const float o[4] = {o4.x, o4.y, o4.z, o4.w};
    if (!norm_res) {
      if (n < NB) *reinterpret_cast<float4*>(y + (node0 + n) * GF + cg * 4) = o4;
      continue;
    }
    float s = o[0] + o[1] + o[2] + o[3];
    for (int m = 1; m < 16; m <<= 1) s += __shfl_xor(s, m);
    const float mean = s * (1.f / GF);
    float ss = 0.f;
#pragma unroll
    for (int q = 0; q < 4; ++q) ss += (o[q] - mean) * (o[q] - mean);
    for (int m = 1; m < 16; m <<= 1) ss += __shfl_xor(ss, m);
    const float rstd = 1.f / sqrtf(ss * (1.f / GF) + 1e-5f);
    if (n >= NB) continue;
    float v[4];
#pragma unroll
    for (int q = 0; q < 4; ++q) {
      const int c = cg * 4 + q;
      float t = (o[q] - mean) * rstd * ln_w[c] + ln_b[c];
      t = t > 0.f ? t : t * slope;
      v[q] = t + xs[n * ZP + c];
    }
    *reinterpret_cast<float4*>(y + (node0 + n) * GF + cg * 4) = make_float4(v[0], v[1], v[2], v[3]);
    if (pre_ln) *reinterpret_cast<float4*>(pre_ln + (node0 + n) * GF + cg * 4) = o4;
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
  (void)lin_out;
  A2M_CHECK_ARG(x && y && nbr_ptr && nbr_idx && w0 && bias && (!norm_res || (ln_w && ln_b)),
                "graph_layer: null pointer");
  A2M_CHECK_ARG(J > 0 && J <= GMAXN && F >= 0, "graph_layer: bad J=%d", J);
  A2M_CHECK_ARG(kind == 0 ? (att_src && att_dst) : (kind == 1 && w1), "graph_layer: bad kind/params");
  A2M_CHECK_ARG(x != y, "graph_layer: in-place not supported");
  if (F == 0) return A2M_OK;
  const int fpb = GMAXN / J;
  const int64_t blocks = cdiv(F, fpb);
  hipStream_t st = as_stream(stream);
  float* Ug = nullptr;
  if (kind == 0) {
    if (!ws || ws_bytes < 2 * GHEADS * GF * sizeof(float)) {
      set_error("graph_layer: workspace too small (%zu < %zu bytes)", ws_bytes,
                (size_t)(2 * GHEADS * GF * sizeof(float)));
      return A2M_EWS;
    }
    Ug = static_cast<float*>(ws);
    hipLaunchKernelGGL(graph_att_proj_kernel, dim3(1), dim3(2 * GHEADS * GF), 0, st, w0, att_src,
                       att_dst, Ug);
    A2M_LAUNCH_CHECK();
  }
  hipLaunchKernelGGL(graph_layer_kernel, dim3((unsigned)blocks), dim3(256), 0, st,
                     x, F, J, kind, norm_res, nbr_ptr, nbr_idx, w0, w1, att_src, att_dst, bias, ln_w, ln_b,
                     slope, Ug, y, pre_ln);
  A2M_LAUNCH_CHECK();
  return A2M_OK;
}
