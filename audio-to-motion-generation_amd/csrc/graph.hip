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
// Diagnostic builds only (never the shipped library): STACK_ABL = 1 drops the stack's MFMAs,
// 2 its neighbour gathers, 4 the weight-fragment loads (tools/stack_bench.py times them).
#ifndef STACK_ABL
#define STACK_ABL 0
#endif
#ifndef STACK_PINGPONG
#define STACK_PINGPONG 0
#endif
#ifndef STACK_IGLP   // the backend's MFMA / VALU interleaving hint for the k steps (-1: none)
#define STACK_IGLP 2
#endif
#ifndef STACK_WG_PER_CU
#define STACK_WG_PER_CU 3
#endif
// 1: the stack's layer products computed transposed (MFMA rows = output features, columns = the
// wave's 32 nodes), so each lane ends a layer holding 32 of its node's 64 features and the
// partner lane (l ^ 32) the other 32: the LayerNorm statistics are register sums plus one
// v_permlane32_swap, with no per-wave LDS scratch and no wave barriers (0: the round-2 epilogue
// through an 8-row LDS scratch)
#ifndef STACK_TEPI
#define STACK_TEPI 1
#endif
constexpr int GHEADS = 4;
constexpr int GMAXN = 128;      // node rows per workgroup (4 waves x 32 MFMA rows)
constexpr int ZP = GF + 4;      // LDS row pitch (floats): 16-B aligned, conflict-free b128 reads
constexpr int GMAXDEG = 8;      // max in-degree (+ self loop) of a skeleton node (hand roots: 5 + 1)

typedef float floatx16 __attribute__((ext_vector_type(16)));

// LDS ordering between the lanes of ONE wave (its private scratch): a wavefront-scope fence pair
// around a wave barrier.
__device__ __forceinline__ void stack_wave_sync() {
  __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
  __builtin_amdgcn_wave_barrier();
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
}

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

// One workgroup = whole frames (<= 128 node rows), 4 waves; wave w owns rows 32w..32w+31 of
// the layer GEMM out[128 x 64] = sum_seg A_seg[128 x 64] . W_seg^T.  The A fragments are built
// straight in registers by the lane that feeds them to the MFMA (lane (li, lh) holds row 32w+li,
// k = 16kc + 8lh + s), so the aggregation needs no LDS tile and no barrier: per segment each lane
// computes its row's edge softmax (GAT head `seg`) from the block's logits, gathers its
// neighbours' 8-float k-slices from the LDS node tile and issues the MFMAs.  LayerNorm(64),
// LeakyReLU and the residual run on the accumulators (row reductions = 32-lane shuffles).
// LDS = node tile + logits + lists (~40 KB): several workgroups per CU hide the HBM latency.
#ifndef GL_WG_PER_CU
#define GL_WG_PER_CU 3
#endif
__global__ __launch_bounds__(256, GL_WG_PER_CU) void graph_layer_kernel(
    const float* __restrict__ x, int F, int J, int kind, int norm_res, const int* __restrict__ nbr_ptr,
    const int* __restrict__ nbr_idx, const float* __restrict__ w0, const float* __restrict__ w1,
    const float* __restrict__ att_src, const float* __restrict__ att_dst,
    const float* __restrict__ bias, const float* __restrict__ ln_w, const float* __restrict__ ln_b,
    float slope, const float* __restrict__ Ug, float* __restrict__ y, float* __restrict__ pre_ln) {
  __shared__ __attribute__((aligned(16))) float xs[GMAXN * ZP];
  __shared__ __attribute__((aligned(16))) float Uk[GF][2 * GHEADS];   // k-major attention projections
  __shared__ float al[2 * GHEADS][GMAXN];                              // logits, q-major
  __shared__ __attribute__((aligned(8))) unsigned char nbl[GMAXN][GMAXDEG];
  __shared__ unsigned char ndeg[GMAXN];
  __shared__ int csr[2 * GMAXN];

  const int fpb = GMAXN / J;
  const int NBmax = fpb * J;
  const int64_t node0 = (int64_t)blockIdx.x * NBmax;
  const int NB = (int)min<int64_t>(NBmax, (int64_t)F * J - node0);
  const int tid = threadIdx.x;
  const int lane = tid & 63, wave = tid >> 6;
  const int li = lane & 31, lh = lane >> 5;

  // ---- prologue: node tile, U, CSR (independent loads, one barrier)
  const int ne = min(nbr_ptr[J], 2 * GMAXN - (J + 1));
  {  // node tile: all 8 float4 loads of this thread in flight before the LDS writes
    constexpr int NL = GMAXN * (GF / 4) / 256;
    float4 v[NL];
#pragma unroll
    for (int j = 0; j < NL; ++j) {
      const int i = tid + j * 256, n = i / (GF / 4), q = i % (GF / 4);
      v[j] = n < NB ? *reinterpret_cast<const float4*>(x + (node0 + n) * GF + q * 4)
                    : make_float4(0.f, 0.f, 0.f, 0.f);
    }
#pragma unroll
    for (int j = 0; j < NL; ++j) {
      const int i = tid + j * 256, n = i / (GF / 4), q = i % (GF / 4);
      *reinterpret_cast<float4*>(xs + n * ZP + q * 4) = v[j];
    }
  }
  if (kind == 0)
    for (int i = tid; i < 2 * GHEADS * GF; i += blockDim.x) Uk[i % GF][i / GF] = Ug[i];
  for (int i = tid; i < J + 1 + ne; i += blockDim.x) csr[i] = i <= J ? nbr_ptr[i] : nbr_idx[i - (J + 1)];
  __syncthreads();
  // block-local neighbour lists (in-edges in edge order, then the GAT self loop) and logits
  for (int n = tid; n < GMAXN; n += blockDim.x) {
    int d = 0;
    if (n < NB) {
      const int f0 = (n / J) * J, ln = n % J;
      for (int e = csr[ln]; e < csr[ln + 1] && d < GMAXDEG; ++e) nbl[n][d++] = f0 + csr[J + 1 + e];
      if (kind == 0 && d < GMAXDEG) nbl[n][d++] = n;
    }
    for (int q = d; q < GMAXDEG; ++q) nbl[n][q] = 0;
    ndeg[n] = d;
  }
  if (kind == 0) {
    for (int n = tid; n < NB; n += blockDim.x) {
      const float* xr = xs + n * ZP;
      float sacc[2 * GHEADS];
#pragma unroll
      for (int q = 0; q < 2 * GHEADS; ++q) sacc[q] = 0.f;
#pragma unroll 4
      for (int k = 0; k < GF; k += 4) {
        const float4 xv = *reinterpret_cast<const float4*>(xr + k);
        const float xk[4] = {xv.x, xv.y, xv.z, xv.w};
#pragma unroll
        for (int j = 0; j < 4; ++j) {
          const float4 u0 = *reinterpret_cast<const float4*>(&Uk[k + j][0]);
          const float4 u1 = *reinterpret_cast<const float4*>(&Uk[k + j][4]);
          sacc[0] += xk[j] * u0.x; sacc[1] += xk[j] * u0.y; sacc[2] += xk[j] * u0.z; sacc[3] += xk[j] * u0.w;
          sacc[4] += xk[j] * u1.x; sacc[5] += xk[j] * u1.y; sacc[6] += xk[j] * u1.z; sacc[7] += xk[j] * u1.w;
        }
      }
#pragma unroll
      for (int q = 0; q < 2 * GHEADS; ++q) al[q][n] = sacc[q];
    }
  }
  __syncthreads();

  // ---- segments: register-built A fragments -> MFMA
  const int row = wave * 32 + li;
  const int d = ndeg[row];
  int ids[GMAXDEG];
  {
    const uint2 nb = *reinterpret_cast<const uint2*>(&nbl[row][0]);
#pragma unroll
    for (int q = 0; q < GMAXDEG; ++q) ids[q] = ((q < 4 ? nb.x : nb.y) >> (8 * (q & 3))) & 0xff;
  }
  floatx16 acc[2];
#pragma unroll
  for (int t = 0; t < 2; ++t)
#pragma unroll
    for (int q = 0; q < 16; ++q) acc[t][q] = 0.f;

  // B fragments (L2-resident weights) run one k-chunk ahead of the MFMAs; the neighbour gather
  // is unpredicated (rows past the degree read node 0 with weight 0), so its 16 LDS reads issue
  // back to back and wait once per k-chunk.
  const int nseg = kind == 0 ? GHEADS : 2;
  auto wseg = [&](int sg) { return kind == 0 ? w0 + (int64_t)sg * GF * GF : (sg == 0 ? w0 : w1); };
  auto load_b = [&](int sg, int kc, float4 (&bw)[2][2]) {
    const float* W = wseg(sg);
#pragma unroll
    for (int t = 0; t < 2; ++t) {
      const float* p = W + (t * 32 + li) * GF + kc * 16 + lh * 8;
      bw[t][0] = *reinterpret_cast<const float4*>(p);
      bw[t][1] = *reinterpret_cast<const float4*>(p + 4);
    }
  };
  float4 bcur[2][2], bnxt[2][2];
  load_b(0, 0, bcur);
  for (int seg = 0; seg < nseg; ++seg) {
    const bool agg = kind == 0 || seg == 0;
    float wq[GMAXDEG];
    if (kind == 0) {  // edge softmax of head `seg` for this lane's row (PyG: LeakyReLU 0.2)
      const float ad = al[GHEADS + seg][row];
      float mx = -INFINITY;
#pragma unroll
      for (int q = 0; q < GMAXDEG; ++q) {
        const float sv = al[seg][ids[q]] + ad;
        wq[q] = sv > 0.f ? sv : sv * 0.2f;
        if (q < d) mx = fmaxf(mx, wq[q]);
      }
      float den = 0.f;
#pragma unroll
      for (int q = 0; q < GMAXDEG; ++q) {
        wq[q] = q < d ? expf(wq[q] - mx) : 0.f;
        den += wq[q];
      }
      const float inv = 1.f / (den + 1e-16f);
#pragma unroll
      for (int q = 0; q < GMAXDEG; ++q) wq[q] *= inv;
    } else {
#pragma unroll
      for (int q = 0; q < GMAXDEG; ++q) wq[q] = q < d ? 1.f : 0.f;
    }
#pragma unroll
    for (int kc = 0; kc < 4; ++kc) {
      if (kc < 3) load_b(seg, kc + 1, bnxt);
      else if (seg + 1 < nseg) load_b(seg + 1, 0, bnxt);
      float af[8];
      if (agg) {
        float4 v[GMAXDEG][2];
#pragma unroll
        for (int q = 0; q < GMAXDEG; ++q) {
          const float* p = xs + ids[q] * ZP + kc * 16 + lh * 8;
          v[q][0] = *reinterpret_cast<const float4*>(p);
          v[q][1] = *reinterpret_cast<const float4*>(p + 4);
        }
#pragma unroll
        for (int s8 = 0; s8 < 8; ++s8) af[s8] = 0.f;
#pragma unroll
        for (int q = 0; q < GMAXDEG; ++q) {
          const float w = wq[q];
          af[0] += w * v[q][0].x; af[1] += w * v[q][0].y; af[2] += w * v[q][0].z; af[3] += w * v[q][0].w;
          af[4] += w * v[q][1].x; af[5] += w * v[q][1].y; af[6] += w * v[q][1].z; af[7] += w * v[q][1].w;
        }
      } else {  // GraphConv root term
        const float* p = xs + row * ZP + kc * 16 + lh * 8;
        const float4 v0 = *reinterpret_cast<const float4*>(p);
        const float4 v1 = *reinterpret_cast<const float4*>(p + 4);
        af[0] = v0.x; af[1] = v0.y; af[2] = v0.z; af[3] = v0.w;
        af[4] = v1.x; af[5] = v1.y; af[6] = v1.z; af[7] = v1.w;
      }
#pragma unroll
      for (int t = 0; t < 2; ++t) {
        const float bf[8] = {bcur[t][0].x, bcur[t][0].y, bcur[t][0].z, bcur[t][0].w,
                             bcur[t][1].x, bcur[t][1].y, bcur[t][1].z, bcur[t][1].w};
#pragma unroll
        for (int s = 0; s < 8; ++s)
          acc[t] = __builtin_amdgcn_mfma_f32_32x32x2f32(af[s], bf[s], acc[t], 0, 0, 0);
      }
#pragma unroll
      for (int t = 0; t < 2; ++t) {
        bcur[t][0] = bnxt[t][0];
        bcur[t][1] = bnxt[t][1];
      }
    }
  }

  // ---- epilogue on the accumulators: acc[t][q] = out[r][t*32 + li],
  //      r = 32*wave + (q & 3) + 8*(q >> 2) + 4*lh
  const float scale = kind == 0 ? 1.f / GHEADS : 1.f;
  const float b0 = bias[li], b1 = bias[32 + li];
  float lw0 = 1.f, lw1 = 1.f, lb0 = 0.f, lb1 = 0.f;
  if (norm_res) {
    lw0 = ln_w[li]; lw1 = ln_w[32 + li];
    lb0 = ln_b[li]; lb1 = ln_b[32 + li];
  }
#pragma unroll
  for (int q = 0; q < 16; ++q) {
    const int r = wave * 32 + (q & 3) + 8 * (q >> 2) + 4 * lh;
    const float o0 = acc[0][q] * scale + b0, o1 = acc[1][q] * scale + b1;
    float* yr = y + (node0 + r) * GF;
    if (!norm_res) {
      if (r < NB) { yr[li] = o0; yr[32 + li] = o1; }
      continue;
    }
    const float mean = half32_sum(o0 + o1) * (1.f / GF);
    const float sv = half32_sum((o0 - mean) * (o0 - mean) + (o1 - mean) * (o1 - mean));
    const float rstd = 1.f / sqrtf(sv * (1.f / GF) + 1e-5f);
    if (r >= NB) continue;
    float u0 = (o0 - mean) * rstd * lw0 + lb0, u1 = (o1 - mean) * rstd * lw1 + lb1;
    u0 = u0 > 0.f ? u0 : u0 * slope;
    u1 = u1 > 0.f ? u1 : u1 * slope;
    yr[li] = u0 + xs[r * ZP + li];
    yr[32 + li] = u1 + xs[r * ZP + 32 + li];
    if (pre_ln) {
      float* pr = pre_ln + (node0 + r) * GF;
      pr[li] = o0;
      pr[32 + li] = o1;
    }
  }
}

// ---------------------------------------------------------------------------------------------
// Fused eval graph stack: the decoders' five {GAT | GraphConv} + LN64 + LeakyReLU + residual
// layers (real_motion_model.py:173-201 body, :225-253 hand; eval: dropout = identity) in ONE
// launch.  A workgroup keeps its frames' node tile in LDS for the whole stack -- each layer's
// output overwrites it in place (every lane rewrites only the elements it alone reads) -- so
// HBM sees the stack input once and its output once instead of five times each, the neighbour
// lists are built once, and the per-layer launches / attention-projection launches disappear
// (the GAT projections U = W_h^T att come precomputed, cached per weight version).
//
// Work layout (differs from graph_layer_kernel):
//  * MFMA rows are the block's nodes sorted by in-degree, the 32 heaviest (hand wrists: 5 in-edges
//    + self loop) in one wave, rotated over the four waves by block so each SIMD gets its share;
//    every wave gathers only up to its own rows' maximum degree (wave-uniform bound), not the
//    GMAXDEG slots of the skeleton-wide maximum (hand: 2.9 gathers a row on average, not 8);
//  * one gather of a neighbour's k-slice feeds all heads: the four GAT heads' edge softmaxes
//    are held in registers and each gathered float4 is weighted four times, so the LDS gather
//    traffic of a GAT layer is a quarter of the per-head loop's;
//  * the logits x . U are computed by all 256 threads (two per node, four logits each).
constexpr int GMAXL = 8;
struct GraphStack {
  int nlayers;
  int kind[GMAXL];
  const float* w0[GMAXL];
  const float* w1[GMAXL];
  const float* U[GMAXL];
  const float* bias[GMAXL];
  const float* ln_w[GMAXL];
  const float* ln_b[GMAXL];
  // bf16 mode: the layer weights as bf16 copies in the fp32 weights' [row][64] layout (made once
  // per weight version, a2m_to_bf16_f32); null: rounded from the fp32 weights in the k loop
  const __bf16* w0h[GMAXL];
  const __bf16* w1h[GMAXL];
  float slope;
  int bf16;   // 1: layer products with bf16 operands (precision 1)
};

// The k loop of one layer for a wave whose rows have at most DL gather slots (compile-time, so
// the gathered slices and edge weights stay in registers): 8 steps of k = 8 (4 per lane half);
// each gathered float4 is weighted for every segment, then 8 MFMAs per segment.  B fragments
// (64 output channels) come from L2 one step ahead.
__device__ __forceinline__ void stack_mfma4(const float (&af)[4], const float4 (&b)[2], floatx16 (&acc)[2]) {
#pragma unroll
  for (int t = 0; t < 2; ++t) {
    const float bf[4] = {b[t].x, b[t].y, b[t].z, b[t].w};
#pragma unroll
    for (int s = 0; s < 4; ++s) {
      if (STACK_ABL == 1) acc[t][s] += af[s] * bf[s];
      else if (STACK_TEPI) acc[t] = __builtin_amdgcn_mfma_f32_32x32x2f32(bf[s], af[s], acc[t], 0, 0, 0);
      else acc[t] = __builtin_amdgcn_mfma_f32_32x32x2f32(af[s], bf[s], acc[t], 0, 0, 0);
    }
  }
}

// edge weights of a row's DL gather slots: GAT, the edge softmax per head over the in-edges + self
// loop (slot d0; PyG: LeakyReLU 0.2); GraphConv, 1 for the in-edges
template <int DL, bool GAT>
__device__ __forceinline__ void stack_edge_weights(const float (*al)[GMAXN], const int (&id)[GMAXDEG], int node,
                                                   int d0, float (&wq)[GAT ? GHEADS : 1][DL]) {
  constexpr int NS = GAT ? GHEADS : 1;
  if (GAT) {  // edge softmax per head over the in-edges + self loop (slot d0; PyG: LeakyReLU 0.2)
    const int d = d0 + 1;
#pragma unroll
    for (int h = 0; h < NS; ++h) {
      const float ad = al[GHEADS + h][node];
      float mx = -INFINITY;
#pragma unroll
      for (int q = 0; q < DL; ++q) {
        const float sv = al[h][id[q]] + ad;
        wq[h][q] = sv > 0.f ? sv : sv * 0.2f;
        if (q < d) mx = fmaxf(mx, wq[h][q]);
      }
      float den = 0.f;
#pragma unroll
      for (int q = 0; q < DL; ++q) {
        wq[h][q] = q < d ? expf(wq[h][q] - mx) : 0.f;
        den += wq[h][q];
      }
      const float inv = 1.f / (den + 1e-16f);
#pragma unroll
      for (int q = 0; q < DL; ++q) wq[h][q] *= inv;
    }
  } else {
#pragma unroll
    for (int q = 0; q < DL; ++q) wq[0][q] = q < d0 ? 1.f : 0.f;
  }
}

template <int DL, bool GAT>
__device__ __forceinline__ void stack_layer_k(const float* xs, const float (*al)[GMAXN], const int (&id)[GMAXDEG],
                                              int node, int d0, const float* W0, const float* W1, int li,
                                              int lh, floatx16 (&acc)[2]) {
  typedef float f2 __attribute__((ext_vector_type(2)));
  constexpr int NS = GAT ? GHEADS : 1;   // aggregated segments (GraphConv: + the root term)
  float wq[NS][DL];
  stack_edge_weights<DL, GAT>(al, id, node, d0, wq);
  // per-lane 32-bit offsets of the B rows (t*32 + li) at this lane half's k; segment h adds h*GF*GF
  const uint32_t boff = (uint32_t)(li * GF + lh * 8);
  auto load_b = [&](int st, float4 (&bw)[GHEADS][2]) {
    const uint32_t off = boff + (st >> 1) * 16 + (st & 1) * 4;
#pragma unroll
    for (int h = 0; h < (GAT ? GHEADS : 2); ++h) {
      const float* W = GAT ? W0 + h * GF * GF : (h == 0 ? W0 : W1);
#pragma unroll
      for (int t = 0; t < 2; ++t)
        bw[h][t] = STACK_ABL == 4 ? make_float4(W0[0] * st, 1.f, 0.5f, (float)h) : *reinterpret_cast<const float4*>(W + off + t * 32 * GF);
    }
  };
  auto step = [&](int st, const float4 (&bc)[GHEADS][2]) {
#if STACK_IGLP >= 0
    __builtin_amdgcn_iglp_opt(STACK_IGLP);
#endif
    const int off = (st >> 1) * 16 + lh * 8 + (st & 1) * 4;
    f2 a01[NS], a23[NS];
#pragma unroll
    for (int h = 0; h < NS; ++h) a01[h] = a23[h] = f2{0.f, 0.f};
#pragma unroll
    for (int q = 0; q < DL; ++q) {
      const float4 v = *reinterpret_cast<const float4*>(xs + (STACK_ABL == 2 ? node : id[q]) * ZP + off);
#pragma unroll
      for (int h = 0; h < NS; ++h) {
        a01[h].x += wq[h][q] * v.x; a01[h].y += wq[h][q] * v.y; a23[h].x += wq[h][q] * v.z; a23[h].y += wq[h][q] * v.w;
      }
    }
#pragma unroll
    for (int h = 0; h < NS; ++h) {
      const float af[4] = {a01[h].x, a01[h].y, a23[h].x, a23[h].y};
      stack_mfma4(af, bc[h], acc);
    }
    if (!GAT) {
      const float4 o = *reinterpret_cast<const float4*>(xs + node * ZP + off);   // root term
      const float ao[4] = {o.x, o.y, o.z, o.w};
      stack_mfma4(ao, bc[1], acc);
    }
  };
#if STACK_PINGPONG
  // ping-pong B buffers: each step's fragments are loaded one step ahead, no register copies
  float4 ba[GHEADS][2], bb[GHEADS][2];
  load_b(0, ba);
#pragma unroll 1
  for (int st = 0; st < 8; st += 2) {
    load_b(st + 1, bb);
    step(st, ba);
    if (st + 2 < 8) load_b(st + 2, ba);
    step(st + 1, bb);
  }
#else
  // single-buffered B (registers for three workgroups per CU): a step's fragments are requested
  // before its gathers and FMAs, which cover part of the L2 latency; co-resident waves the rest
#pragma unroll 1
  for (int st = 0; st < 8; ++st) {
    float4 bc[GHEADS][2];
    load_b(st, bc);
    step(st, bc);
  }
#endif
}

// bf16 operand mode (a2m_set_gemm_precision(1), configs[4]): the layer products on
// v_mfma_f32_32x32x16_bf16 -- the aggregated rows and the weights rounded to bf16 (RNE) in
// registers, fp32 accumulation -- as torch.autocast runs the reference's GATConv / GraphConv
// linears in bf16.  Per 16-k chunk each lane aggregates its row's 8 consecutive features (two
// float4 gathers per neighbour, all heads at once) and issues one MFMA per (segment, t): 1/16 of
// the fp32 k loop's matrix-pipe time.
typedef __bf16 sbf16x8 __attribute__((ext_vector_type(8)));
__device__ __forceinline__ sbf16x8 stack_pack8(const float (&v)[8]) {
  typedef float f2 __attribute__((ext_vector_type(2)));
  typedef __bf16 h2 __attribute__((ext_vector_type(2)));
  uint32_t u[4];
#pragma unroll
  for (int j = 0; j < 4; ++j) {
    const f2 p = {v[2 * j], v[2 * j + 1]};
    u[j] = __builtin_bit_cast(uint32_t, __builtin_convertvector(p, h2));
  }
  typedef uint32_t u4 __attribute__((ext_vector_type(4)));
  return __builtin_bit_cast(sbf16x8, u4{u[0], u[1], u[2], u[3]});
}

template <int DL, bool GAT>
__device__ __forceinline__ void stack_layer_kh(const float* xs, const float (*al)[GMAXN], const int (&id)[GMAXDEG],
                                               int node, int d0, const float* W0, const float* W1,
                                               const __bf16* H0, const __bf16* H1, int li, int lh,
                                               floatx16 (&acc)[2]) {
  constexpr int NS = GAT ? GHEADS : 1;
  constexpr int NSEG = GAT ? GHEADS : 2;
  float wq[NS][DL];
  stack_edge_weights<DL, GAT>(al, id, node, d0, wq);
#pragma unroll 1
  for (int kc = 0; kc < GF / 16; ++kc) {
    const int off = 16 * kc + 8 * lh;   // this lane's 8 consecutive k of the chunk
    float a[NSEG][8];
#pragma unroll
    for (int h = 0; h < NSEG; ++h)
#pragma unroll
      for (int e = 0; e < 8; ++e) a[h][e] = 0.f;
#pragma unroll
    for (int q = 0; q < DL; ++q) {
      const float4 v0 = *reinterpret_cast<const float4*>(xs + id[q] * ZP + off);
      const float4 v1 = *reinterpret_cast<const float4*>(xs + id[q] * ZP + off + 4);
      const float v[8] = {v0.x, v0.y, v0.z, v0.w, v1.x, v1.y, v1.z, v1.w};
#pragma unroll
      for (int h = 0; h < NS; ++h)
#pragma unroll
        for (int e = 0; e < 8; ++e) a[h][e] += wq[h][q] * v[e];
    }
    if (!GAT) {   // GraphConv's root term: the node's own features
      const float4 o0 = *reinterpret_cast<const float4*>(xs + node * ZP + off);
      const float4 o1 = *reinterpret_cast<const float4*>(xs + node * ZP + off + 4);
      const float o[8] = {o0.x, o0.y, o0.z, o0.w, o1.x, o1.y, o1.z, o1.w};
#pragma unroll
      for (int e = 0; e < 8; ++e) a[1][e] = o[e];
    }
#pragma unroll
    for (int h = 0; h < NSEG; ++h) {
      const sbf16x8 af = stack_pack8(a[h]);
      const float* W = GAT ? W0 + h * GF * GF : (h == 0 ? W0 : W1);
#pragma unroll
      for (int t = 0; t < 2; ++t) {
        sbf16x8 wb;
        if (H0) {   // the cached bf16 copy: one 16-byte load, no rounding in the loop
          const __bf16* H = GAT ? H0 + h * GF * GF : (h == 0 ? H0 : H1);
          wb = *reinterpret_cast<const sbf16x8*>(H + (t * 32 + li) * GF + off);
        } else {
          const float* wr = W + (t * 32 + li) * GF + off;
          const float4 b0 = *reinterpret_cast<const float4*>(wr);
          const float4 b1 = *reinterpret_cast<const float4*>(wr + 4);
          const float bv[8] = {b0.x, b0.y, b0.z, b0.w, b1.x, b1.y, b1.z, b1.w};
          wb = stack_pack8(bv);
        }
        if (STACK_TEPI) acc[t] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(wb, af, acc[t], 0, 0, 0);
        else acc[t] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(af, wb, acc[t], 0, 0, 0);
      }
    }
  }
}

template <bool GAT>
__device__ __forceinline__ void stack_layer_dispatch_h(int dl, const float* xs, const float (*al)[GMAXN],
                                                       const int (&id)[GMAXDEG], int node, int d0, const float* W0,
                                                       const float* W1, const __bf16* H0, const __bf16* H1, int li,
                                                       int lh, floatx16 (&acc)[2]) {
  switch (dl) {
    case 1: stack_layer_kh<1, GAT>(xs, al, id, node, d0, W0, W1, H0, H1, li, lh, acc); break;
    case 2: stack_layer_kh<2, GAT>(xs, al, id, node, d0, W0, W1, H0, H1, li, lh, acc); break;
    case 3: stack_layer_kh<3, GAT>(xs, al, id, node, d0, W0, W1, H0, H1, li, lh, acc); break;
    case 4: stack_layer_kh<4, GAT>(xs, al, id, node, d0, W0, W1, H0, H1, li, lh, acc); break;
    case 5: stack_layer_kh<5, GAT>(xs, al, id, node, d0, W0, W1, H0, H1, li, lh, acc); break;
    case 6: stack_layer_kh<6, GAT>(xs, al, id, node, d0, W0, W1, H0, H1, li, lh, acc); break;
    case 7: stack_layer_kh<7, GAT>(xs, al, id, node, d0, W0, W1, H0, H1, li, lh, acc); break;
    default: stack_layer_kh<8, GAT>(xs, al, id, node, d0, W0, W1, H0, H1, li, lh, acc); break;
  }
}

template <bool GAT>
__device__ __forceinline__ void stack_layer_dispatch(int dl, const float* xs, const float (*al)[GMAXN],
                                                     const int (&id)[GMAXDEG], int node, int d0, const float* W0,
                                                     const float* W1, int li, int lh, floatx16 (&acc)[2]) {
  switch (dl) {
    case 1: stack_layer_k<1, GAT>(xs, al, id, node, d0, W0, W1, li, lh, acc); break;
    case 2: stack_layer_k<2, GAT>(xs, al, id, node, d0, W0, W1, li, lh, acc); break;
    case 3: stack_layer_k<3, GAT>(xs, al, id, node, d0, W0, W1, li, lh, acc); break;
    case 4: stack_layer_k<4, GAT>(xs, al, id, node, d0, W0, W1, li, lh, acc); break;
    case 5: stack_layer_k<5, GAT>(xs, al, id, node, d0, W0, W1, li, lh, acc); break;
    case 6: stack_layer_k<6, GAT>(xs, al, id, node, d0, W0, W1, li, lh, acc); break;
    case 7: stack_layer_k<7, GAT>(xs, al, id, node, d0, W0, W1, li, lh, acc); break;
    default: stack_layer_k<8, GAT>(xs, al, id, node, d0, W0, W1, li, lh, acc); break;
  }
}

// bf16 stack: two workgroups per CU (256 VGPRs, no spills).  Three (168 VGPRs, 114 spilled) won
// while every wave rounded its fp32 weights in the k loop (hand 228.7 vs 250 us alone); with the
// cached bf16 weights two is faster in the step -- hand 164 vs 159 us alone but body 53 vs 58.5 us,
// and the other branch's kernels fit beside it: bf16 B = 64 1.354 -> 1.346 ms, B = 32 0.977 ->
// 0.959 ms (profiles/r06_v_stack_wg_ab.txt)
#ifndef STACK_WG_PER_CU_BF16
#define STACK_WG_PER_CU_BF16 2
#endif
#ifndef STACK_WG_PER_CU_BF16_WIDE   // diagnostic: the bf16 stack's occupancy for J > 32 (the hand)
#define STACK_WG_PER_CU_BF16_WIDE STACK_WG_PER_CU_BF16
#endif
#ifndef STACK_WG_PER_CU_WIDE        // diagnostic: the fp32 stack's occupancy for J > 32 (the hand)
#define STACK_WG_PER_CU_WIDE STACK_WG_PER_CU
#endif
template <bool BF16, int WG = (BF16 ? STACK_WG_PER_CU_BF16 : STACK_WG_PER_CU)>
__global__ __launch_bounds__(256, WG) void graph_stack_kernel(
    const float* __restrict__ x, int F, int J, const int* __restrict__ nbr_ptr,
    const int* __restrict__ nbr_idx, GraphStack S, float* __restrict__ y) {
  __shared__ __attribute__((aligned(16))) float xs[GMAXN * ZP];        // node-indexed tile
  __shared__ __attribute__((aligned(16))) float Uk[GF][2 * GHEADS];
  __shared__ float al[2 * GHEADS][GMAXN];                              // node-indexed logits
  __shared__ __attribute__((aligned(8))) unsigned char nbl[GMAXN][GMAXDEG];
  __shared__ unsigned char ndeg[GMAXN];
  __shared__ unsigned char rown[GMAXN];                                // MFMA row -> node (0xff: none)
  __shared__ int csr[2 * GMAXN];
#if !STACK_TEPI
  __shared__ __attribute__((aligned(16))) float osc[4][8 * ZP];         // per-wave epilogue scratch (8 rows)
#endif
  __shared__ __attribute__((aligned(16))) float lnp[3 * GF];            // this layer's LN weight | bias | layer bias

  const int fpb = GMAXN / J;
  const int NBmax = fpb * J;
  const int64_t node0 = (int64_t)blockIdx.x * NBmax;
  const int NB = (int)min<int64_t>(NBmax, (int64_t)F * J - node0);
  const int tid = threadIdx.x;
  const int lane = tid & 63, wave = tid >> 6;
  const int li = lane & 31, lh = lane >> 5;

  const int ne = min(nbr_ptr[J], 2 * GMAXN - (J + 1));
  {
    constexpr int NL = GMAXN * (GF / 4) / 256;
    float4 v[NL];
#pragma unroll
    for (int j = 0; j < NL; ++j) {
      const int i = tid + j * 256, n = i / (GF / 4), q = i % (GF / 4);
      v[j] = n < NB ? *reinterpret_cast<const float4*>(x + (node0 + n) * GF + q * 4)
                    : make_float4(0.f, 0.f, 0.f, 0.f);
    }
#pragma unroll
    for (int j = 0; j < NL; ++j) {
      const int i = tid + j * 256, n = i / (GF / 4), q = i % (GF / 4);
      *reinterpret_cast<float4*>(xs + n * ZP + q * 4) = v[j];
    }
  }
  for (int i = tid; i < J + 1 + ne; i += blockDim.x) csr[i] = i <= J ? nbr_ptr[i] : nbr_idx[i - (J + 1)];
  __syncthreads();
  // block-local in-neighbour lists (edge order; the GAT self loop is added per layer)
  for (int n = tid; n < GMAXN; n += blockDim.x) {
    int d = 0;
    if (n < NB) {
      const int f0 = (n / J) * J, ln = n % J;
      for (int e = csr[ln]; e < csr[ln + 1] && d < GMAXDEG - 1; ++e) nbl[n][d++] = f0 + csr[J + 1 + e];
    }
    for (int q = d; q < GMAXDEG; ++q) nbl[n][q] = 0;
    ndeg[n] = d;
    rown[n] = 0xff;
  }
  __syncthreads();
  // rows sorted by degree (descending; stable), the heaviest 32 in wave blockIdx & 3
  for (int n = tid; n < NB; n += blockDim.x) {
    const int d = ndeg[n];
    int pos = 0;
    for (int m = 0; m < NB; ++m) {
      const int dm = ndeg[m];
      pos += (dm > d) || (dm == d && m < n);
    }
    rown[((((pos >> 5) + blockIdx.x) & 3) << 5) | (pos & 31)] = (unsigned char)n;
  }
  __syncthreads();
  const int rn = rown[wave * 32 + li];
  const bool live = rn != 0xff;
  const int node = live ? rn : 0;
  const int d0 = live ? ndeg[node] : 0;
  int ids[GMAXDEG];
  {
    const uint2 nb = *reinterpret_cast<const uint2*>(&nbl[node][0]);
#pragma unroll
    for (int q = 0; q < GMAXDEG; ++q) ids[q] = live ? ((q < 4 ? nb.x : nb.y) >> (8 * (q & 3))) & 0xff : 0;
  }
  int idg[GMAXDEG];   // in-neighbours, then the GAT self loop at slot d0 (weight 0 in GraphConv)
#pragma unroll
  for (int q = 0; q < GMAXDEG; ++q) idg[q] = q < d0 ? ids[q] : (q == d0 ? node : 0);
  // wave-uniform gather bound: the largest in-degree among this wave's rows
  int dw = d0;
#pragma unroll
  for (int o = 1; o < 64; o <<= 1) dw = max(dw, __shfl_xor(dw, o));
  dw = __builtin_amdgcn_readfirstlane(dw);
  for (int L = 0; L < S.nlayers; ++L) {
    const int kind = S.kind[L];
    const bool gat = kind == 0;
    int dl;                      // wave-uniform number of gather slots this layer
    if (gat) {
      const float* U = S.U[L];
      for (int i = tid; i < 2 * GHEADS * GF; i += blockDim.x) Uk[i % GF][i / GF] = U[i];
      __syncthreads();
      {  // logits al[q][n] = x_n . U[q]: two threads per node, four logits each
        const int n = tid >> 1, qh = (tid & 1) * 4;
        if (n < NB) {
          const float* xr = xs + n * ZP;
          typedef float f2 __attribute__((ext_vector_type(2)));
          f2 s01 = {0.f, 0.f}, s23 = {0.f, 0.f};
#pragma unroll 4
          for (int k = 0; k < GF; k += 4) {
            const float4 xv = *reinterpret_cast<const float4*>(xr + k);
            const float xk[4] = {xv.x, xv.y, xv.z, xv.w};
#pragma unroll
            for (int j = 0; j < 4; ++j) {
              const float4 u = *reinterpret_cast<const float4*>(&Uk[k + j][qh]);
              const f2 x2 = {xk[j], xk[j]};
              s01 = __builtin_elementwise_fma(x2, f2{u.x, u.y}, s01);
              s23 = __builtin_elementwise_fma(x2, f2{u.z, u.w}, s23);
            }
          }
          al[qh][n] = s01.x; al[qh + 1][n] = s01.y; al[qh + 2][n] = s23.x; al[qh + 3][n] = s23.y;
        }
      }
      __syncthreads();
      dl = dw + 1;
    } else {
      dl = dw;
    }

    floatx16 acc[2];
#pragma unroll
    for (int t = 0; t < 2; ++t)
#pragma unroll
      for (int q = 0; q < 16; ++q) acc[t][q] = 0.f;
    dl = __builtin_amdgcn_readfirstlane(dl);
    if constexpr (BF16) {
      if (gat) stack_layer_dispatch_h<true>(dl, xs, al, idg, node, d0, S.w0[L], S.w1[L], S.w0h[L], S.w1h[L], li, lh, acc);
      else stack_layer_dispatch_h<false>(max(dl, 1), xs, al, idg, node, d0, S.w0[L], S.w1[L], S.w0h[L], S.w1h[L],
                                         li, lh, acc);
    } else if (gat) {
      stack_layer_dispatch<true>(dl, xs, al, idg, node, d0, S.w0[L], S.w1[L], li, lh, acc);
    } else {
      stack_layer_dispatch<false>(max(dl, 1), xs, al, idg, node, d0, S.w0[L], S.w1[L], li, lh, acc);
    }
    // epilogue: out = LReLU(LN(acc * scale + bias)) + x, in place (or to y after the last layer).
    // The wave's 32 x 64 result goes through its private LDS scratch, 8 rows at a time (rows
    // 8p..8p+7 are exactly accumulator entries q = 4p..4p+3), so that each lane then owns 8
    // contiguous features of a row: the LayerNorm sums are 8-element register sums plus two
    // DPP adds over the row's 8 lanes, instead of cross-lane reductions in the MFMA layout.
    const float scale = gat ? 1.f / GHEADS : 1.f;
    if (tid < 3 * GF) lnp[tid] = tid < GF ? S.ln_w[L][tid] : tid < 2 * GF ? S.ln_b[L][tid - GF] : S.bias[L][tid - 2 * GF];
    __syncthreads();   // every gather of this layer has read the tile; LN params visible
#if STACK_TEPI
    {
      // lane (li, lh) holds features 32 t + 8 g + 4 lh + j (j < 4) of node `node` (MFMA column li)
      // in acc[t][4 g + j]; lane li ^ 32 holds the others
      const bool last_l = L + 1 == S.nlayers;
      float v[2][16];
      float sm = 0.f;
#pragma unroll
      for (int t = 0; t < 2; ++t)
#pragma unroll
        for (int g = 0; g < 4; ++g) {
          const float4 bb = *reinterpret_cast<const float4*>(lnp + 2 * GF + 32 * t + 8 * g + 4 * lh);
          const float bv[4] = {bb.x, bb.y, bb.z, bb.w};
#pragma unroll
          for (int j = 0; j < 4; ++j) {
            v[t][4 * g + j] = acc[t][4 * g + j] * scale + bv[j];
            sm += v[t][4 * g + j];
          }
        }
      {
        const auto r = __builtin_amdgcn_permlane32_swap(__float_as_uint(sm), __float_as_uint(sm), false, false);
        sm = __uint_as_float(r[0]) + __uint_as_float(r[1]);
      }
      const float mean = sm * (1.f / GF);
      float sq = 0.f;
#pragma unroll
      for (int t = 0; t < 2; ++t)
#pragma unroll
        for (int e = 0; e < 16; ++e) sq += (v[t][e] - mean) * (v[t][e] - mean);
      {
        const auto r = __builtin_amdgcn_permlane32_swap(__float_as_uint(sq), __float_as_uint(sq), false, false);
        sq = __uint_as_float(r[0]) + __uint_as_float(r[1]);
      }
      const float rstd = 1.f / sqrtf(sq * (1.f / GF) + 1e-5f);
      if (live) {
        float* xr = xs + node * ZP;
        float* yr = y + (node0 + node) * GF;
#pragma unroll
        for (int t = 0; t < 2; ++t)
#pragma unroll
          for (int g = 0; g < 4; ++g) {
            const int f = 32 * t + 8 * g + 4 * lh;
            const float4 xv = *reinterpret_cast<const float4*>(xr + f);
            const float4 w = *reinterpret_cast<const float4*>(lnp + f);
            const float4 bb = *reinterpret_cast<const float4*>(lnp + GF + f);
            const float* q = &v[t][4 * g];
            float4 u;
            u.x = (q[0] - mean) * rstd * w.x + bb.x;
            u.y = (q[1] - mean) * rstd * w.y + bb.y;
            u.z = (q[2] - mean) * rstd * w.z + bb.z;
            u.w = (q[3] - mean) * rstd * w.w + bb.w;
            u.x = (u.x > 0.f ? u.x : u.x * S.slope) + xv.x;
            u.y = (u.y > 0.f ? u.y : u.y * S.slope) + xv.y;
            u.z = (u.z > 0.f ? u.z : u.z * S.slope) + xv.z;
            u.w = (u.w > 0.f ? u.w : u.w * S.slope) + xv.w;
            if (last_l) *reinterpret_cast<float4*>(yr + f) = u;
            else *reinterpret_cast<float4*>(xr + f) = u;
          }
      }
    }
#else
    {
      const float* bias = S.bias[L];
      const float b0 = bias[li], b1 = bias[32 + li];
      const bool last_l = L + 1 == S.nlayers;
      float* o = osc[wave];
      const int r8 = lane >> 3, seg = (lane & 7) * 8;
#pragma unroll
      for (int p = 0; p < 4; ++p) {
        if (p > 0) stack_wave_sync();   // the previous pass's scratch reads of this wave
#pragma unroll
        for (int qq = 0; qq < 4; ++qq) {
          const int q = 4 * p + qq;
          const int rr = (q & 3) + 4 * lh;
          o[rr * ZP + li] = acc[0][q] * scale + b0;
          o[rr * ZP + 32 + li] = acc[1][q] * scale + b1;
        }
        stack_wave_sync();
        const int nd = rown[wave * 32 + 8 * p + r8];
        const float4 v0 = *reinterpret_cast<const float4*>(o + r8 * ZP + seg);
        const float4 v1 = *reinterpret_cast<const float4*>(o + r8 * ZP + seg + 4);
        const float v[8] = {v0.x, v0.y, v0.z, v0.w, v1.x, v1.y, v1.z, v1.w};
        float sm = 0.f;
#pragma unroll
        for (int j = 0; j < 8; ++j) sm += v[j];
        sm = quad_sum(sm);
        sm += dpp_f<DPP_HALF_MIRROR>(sm);
        const float mean = sm * (1.f / GF);
        float sq = 0.f;
#pragma unroll
        for (int j = 0; j < 8; ++j) sq += (v[j] - mean) * (v[j] - mean);
        sq = quad_sum(sq);
        sq += dpp_f<DPP_HALF_MIRROR>(sq);
        const float rstd = 1.f / sqrtf(sq * (1.f / GF) + 1e-5f);
        if (nd != 0xff) {
          float* xr = xs + nd * ZP + seg;
          float* yr = y + (node0 + nd) * GF + seg;
#pragma unroll
          for (int j = 0; j < 2; ++j) {
            const float4 xv = *reinterpret_cast<const float4*>(xr + 4 * j);
            const float4 w = *reinterpret_cast<const float4*>(lnp + seg + 4 * j);
            const float4 bb = *reinterpret_cast<const float4*>(lnp + GF + seg + 4 * j);
            float4 u;
            u.x = (v[4 * j] - mean) * rstd * w.x + bb.x;
            u.y = (v[4 * j + 1] - mean) * rstd * w.y + bb.y;
            u.z = (v[4 * j + 2] - mean) * rstd * w.z + bb.z;
            u.w = (v[4 * j + 3] - mean) * rstd * w.w + bb.w;
            u.x = (u.x > 0.f ? u.x : u.x * S.slope) + xv.x;
            u.y = (u.y > 0.f ? u.y : u.y * S.slope) + xv.y;
            u.z = (u.z > 0.f ? u.z : u.z * S.slope) + xv.z;
            u.w = (u.w > 0.f ? u.w : u.w * S.slope) + xv.w;
            if (last_l) *reinterpret_cast<float4*>(yr + 4 * j) = u;
            else *reinterpret_cast<float4*>(xr + 4 * j) = u;
          }
        }
      }
    }
#endif
    const bool last = L + 1 == S.nlayers;
    if (!last) __syncthreads();   // the layer's output is the next layer's tile
  }
}

}  // namespace a2m

using namespace a2m;

extern "C" int a2m_graph_att_proj_f32(const float* w0, const float* att_src, const float* att_dst,
                                      float* U, void* stream) {
  A2M_CHECK_ARG(w0 && att_src && att_dst && U, "graph_att_proj: null pointer");
  hipLaunchKernelGGL(graph_att_proj_kernel, dim3(1), dim3(2 * GHEADS * GF), 0, as_stream(stream),
                     w0, att_src, att_dst, U);
  A2M_LAUNCH_CHECK();
  return A2M_OK;
}

// RNE fp32 -> bf16 with the k loop's conversion (stack_pack8), so a cached copy holds exactly the
// values the loop would round to
__global__ void to_bf16_kernel(const float* __restrict__ x, __bf16* __restrict__ y, int64_t n) {
  typedef float f2 __attribute__((ext_vector_type(2)));
  typedef __bf16 h2 __attribute__((ext_vector_type(2)));
  for (int64_t i = 2 * (blockIdx.x * (int64_t)blockDim.x + threadIdx.x); i < n;
       i += 2 * (int64_t)gridDim.x * blockDim.x) {
    if (i + 1 < n) {
      *reinterpret_cast<h2*>(y + i) = __builtin_convertvector((f2{x[i], x[i + 1]}), h2);
    } else {
      y[i] = __builtin_convertvector((f2{x[i], 0.f}), h2)[0];
    }
  }
}

extern "C" int a2m_to_bf16_f32(const float* x, void* y, int64_t n, void* stream) {
  A2M_CHECK_ARG(x && y && n >= 0, "to_bf16: bad args");
  A2M_CHECK_ARG((reinterpret_cast<uintptr_t>(y) & 3) == 0, "to_bf16: y not 4-byte aligned");
  if (n == 0) return A2M_OK;
  const int blocks = (int)std::min<int64_t>(cdiv(cdiv(n, 2), 256), 1024);
  hipLaunchKernelGGL(to_bf16_kernel, dim3(blocks), dim3(256), 0, as_stream(stream), x,
                     static_cast<__bf16*>(y), n);
  A2M_LAUNCH_CHECK();
  return A2M_OK;
}

extern "C" int a2m_graph_stack_fwd_ex_f32(const float* x, int32_t F, int32_t J, const int32_t* nbr_ptr,
                                          const int32_t* nbr_idx, int32_t nlayers, const int32_t* kinds,
                                          const float* const* w0, const float* const* w1,
                                          const float* const* U, const float* const* bias,
                                          const float* const* ln_w, const float* const* ln_b,
                                          const void* const* w0h, const void* const* w1h, float slope,
                                          float* y, void* stream);

extern "C" int a2m_graph_stack_fwd_f32(const float* x, int32_t F, int32_t J, const int32_t* nbr_ptr,
                                       const int32_t* nbr_idx, int32_t nlayers, const int32_t* kinds,
                                       const float* const* w0, const float* const* w1,
                                       const float* const* U, const float* const* bias,
                                       const float* const* ln_w, const float* const* ln_b,
                                       float slope, float* y, void* stream) {
  return a2m_graph_stack_fwd_ex_f32(x, F, J, nbr_ptr, nbr_idx, nlayers, kinds, w0, w1, U, bias, ln_w, ln_b,
                                    nullptr, nullptr, slope, y, stream);
}

extern "C" int a2m_graph_stack_fwd_ex_f32(const float* x, int32_t F, int32_t J, const int32_t* nbr_ptr,
                                          const int32_t* nbr_idx, int32_t nlayers, const int32_t* kinds,
                                          const float* const* w0, const float* const* w1,
                                          const float* const* U, const float* const* bias,
                                          const float* const* ln_w, const float* const* ln_b,
                                          const void* const* w0h, const void* const* w1h, float slope,
                                          float* y, void* stream) {
  A2M_CHECK_ARG(w0 && w1, "graph_stack: null pointer");
  A2M_CHECK_ARG(x && y && nbr_ptr && nbr_idx && kinds && U && bias && ln_w && ln_b,
                "graph_stack: null pointer");
  A2M_CHECK_ARG(J > 0 && J <= GMAXN && F >= 0, "graph_stack: bad J=%d", J);
  A2M_CHECK_ARG(nlayers > 0 && nlayers <= GMAXL, "graph_stack: %d layers (1..%d)", nlayers, GMAXL);
  A2M_CHECK_ARG(x != y, "graph_stack: in-place not supported");
  GraphStack S{};
  S.nlayers = nlayers;
  S.slope = slope;
  // bf16 operand mode: the layer products on the bf16 MFMA
  S.bf16 = a2m_get_gemm_precision() == 1;
  for (int L = 0; L < nlayers; ++L) {
    A2M_CHECK_ARG(kinds[L] == 0 || kinds[L] == 1, "graph_stack: layer %d kind %d", L, kinds[L]);
    const bool has_w = w0[L] && (kinds[L] == 0 || w1[L]);
    A2M_CHECK_ARG(has_w && bias[L] && ln_w[L] && ln_b[L] && (kinds[L] != 0 || U[L] != nullptr),
                  "graph_stack: layer %d parameters missing", L);
    S.kind[L] = kinds[L];
    S.w0[L] = w0[L]; S.w1[L] = w1[L];
    S.U[L] = U[L];
    S.bias[L] = bias[L]; S.ln_w[L] = ln_w[L]; S.ln_b[L] = ln_b[L];
    // the cached bf16 copies count only when every weight of the layer has one (16-byte aligned)
    const void* h0 = w0h ? w0h[L] : nullptr;
    const void* h1 = w1h && kinds[L] == 1 ? w1h[L] : nullptr;
    const bool cached = S.bf16 && h0 && (kinds[L] == 0 || h1) &&
                        ((reinterpret_cast<uintptr_t>(h0) | reinterpret_cast<uintptr_t>(h1)) & 15) == 0;
    S.w0h[L] = cached ? static_cast<const __bf16*>(h0) : nullptr;
    S.w1h[L] = cached ? static_cast<const __bf16*>(h1) : nullptr;
  }
  if (F == 0) return A2M_OK;
  const int fpb = GMAXN / J;
  if (S.bf16 && J > 32 && STACK_WG_PER_CU_BF16_WIDE != STACK_WG_PER_CU_BF16)
    hipLaunchKernelGGL((graph_stack_kernel<true, STACK_WG_PER_CU_BF16_WIDE>), dim3((unsigned)cdiv(F, fpb)), dim3(256),
                       0, as_stream(stream), x, F, J, nbr_ptr, nbr_idx, S, y);
  else if (S.bf16)
    hipLaunchKernelGGL(graph_stack_kernel<true>, dim3((unsigned)cdiv(F, fpb)), dim3(256), 0, as_stream(stream),
                       x, F, J, nbr_ptr, nbr_idx, S, y);
  else if (J > 32 && STACK_WG_PER_CU_WIDE != STACK_WG_PER_CU)
    hipLaunchKernelGGL((graph_stack_kernel<false, STACK_WG_PER_CU_WIDE>), dim3((unsigned)cdiv(F, fpb)), dim3(256),
                       0, as_stream(stream), x, F, J, nbr_ptr, nbr_idx, S, y);
  else
    hipLaunchKernelGGL(graph_stack_kernel<false>, dim3((unsigned)cdiv(F, fpb)), dim3(256), 0, as_stream(stream),
                       x, F, J, nbr_ptr, nbr_idx, S, y);
  A2M_LAUNCH_CHECK();
  return A2M_OK;
}

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
