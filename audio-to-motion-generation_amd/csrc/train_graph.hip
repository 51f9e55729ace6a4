// Backward of the fused skeleton-graph layer (forward: graph.hip).
//
// Per workgroup of whole frames (<= 128 nodes) the forward is recomputed from x (attention
// logits, per-head edge softmax, aggregated inputs Y_h, pre-LayerNorm output o), then:
//   LN/LeakyReLU/residual:  du = dy * leaky'(u),  do = rstd (g - mean g - ohat mean(g ohat)),
//                           g = du * ln_w;  dln_w += du ohat, dln_b += du, dbias += do
//   GAT (4 heads, mean):    dY_h = do W_h / 4                         (MFMA)
//                           dalpha_ijh = dY_h,i . x_j;  softmax + LeakyReLU backward -> ds
//                           da_dst[i,h] = sum_j ds_ijh,  da_src[j,h] = sum_i ds_ijh
//                           dx_j += sum_i alpha_ijh dY_h,i + da_src[j,h] U_h + da_dst[j,h] U_4+h
//                           dU_q += sum_n da_q[n] x_n   (U_h = W_h^T att_h, chained on the host)
//   GraphConv:              dagg = do W_rel, dx = do W_root + sum_{i ~ j} dagg_i
// Gathers over the (symmetric) skeleton graph replace scatters, so every sum has a fixed
// order.  Weight gradients need sums over all nodes: the kernel writes Y_h (GAT) / agg
// (GraphConv) and do (x 1/4 for GAT) to global memory and the host reduces them with
// engine GEMMs; bias / LayerNorm / U partials are reduced per workgroup.
#include <algorithm>

#include "a2m_internal.h"

namespace a2m {

constexpr int BF = 64;
constexpr int BH = 4;
constexpr int BMAXN = 128;
constexpr int BZP = BF + 4;
constexpr int BDEG = 8;
constexpr int BPART = 3 * BF + 2 * BH * BF;  // dbias | dln_w | dln_b | dU[8][64]
// 512 threads = 8 waves (two per SIMD, so one wave's LDS / barrier waits overlap the other's
// work at one workgroup per CU): MFMA wave w owns rows 32 (w & 3).. and columns 32 (w >> 2)..;
// the row-wise phases use 16 lanes per node row, BRG = 32 row groups of BRPT rows each.
constexpr int BNT = 512, BRG = BNT / 16, BRPT = BMAXN / BRG;
static_assert(BNT == 2 * BH * BF, "one thread per GAT projection element in the prologue");
static_assert(BNT >= 2 * BMAXN, "one thread per CSR entry in the prologue");

typedef float floatx16 __attribute__((ext_vector_type(16)));

// A2M_GBWD_STAMPS (diagnostic build, tools/build_variant.sh): thread 0 of every workgroup stamps
// the wall clock after each phase's barrier (tools/graph_bwd_phases.py reads them back)
#ifdef A2M_GBWD_STAMPS
constexpr int kGbStamps = 32, kGbBlocks = 4096;
__device__ unsigned long long g_gb_stamps[kGbBlocks * kGbStamps];
#define GB_STAMP(i)                                                              \
  do {                                                                           \
    if (threadIdx.x == 0 && blockIdx.x < kGbBlocks)                              \
      g_gb_stamps[blockIdx.x * kGbStamps + (i)] = (unsigned long long)wall_clock64(); \
  } while (0)
#else
#define GB_STAMP(i) do {} while (0)
#endif

// acc += A[rows][64] (LDS, pitch BZP) . W^T over output columns c0 + (0..31), where
// B(n=j, k=c) = Wt(j, c) given by functor
template <class WF>
__device__ __forceinline__ void mfma_rows64(floatx16& acc, const float* A, int arow, int c0, int lh,
                                            int li, WF wf) {
#pragma unroll
  for (int kc = 0; kc < 4; ++kc) {
    const float* p = A + arow * BZP + kc * 16 + lh * 8;
    const float4 a0 = *reinterpret_cast<const float4*>(p);
    const float4 a1 = *reinterpret_cast<const float4*>(p + 4);
    const float af[8] = {a0.x, a0.y, a0.z, a0.w, a1.x, a1.y, a1.z, a1.w};
    float bf[8];
#pragma unroll
    for (int s = 0; s < 8; ++s) bf[s] = wf(c0 + li, kc * 16 + lh * 8 + s);
#pragma unroll
    for (int s = 0; s < 8; ++s) acc = __builtin_amdgcn_mfma_f32_32x32x2f32(af[s], bf[s], acc, 0, 0, 0);
  }
}

// the same product with the B fragments preloaded: w[8 kc + s] = W^T(c0 + li, 16 kc + 8 lh + s)
// (load_wt: W row-major [64][64], B(n = j, k = c) = W[c][j])
__device__ __forceinline__ void load_wt(float (&w)[32], const float* __restrict__ W, int c0, int lh, int li) {
#pragma unroll
  for (int kc = 0; kc < 4; ++kc)
#pragma unroll
    for (int s = 0; s < 8; ++s) w[kc * 8 + s] = W[(kc * 16 + lh * 8 + s) * BF + c0 + li];
}

__device__ __forceinline__ void mfma_rows64_w(floatx16& acc, const float* A, int arow, int lh, const float (&w)[32]) {
#pragma unroll
  for (int kc = 0; kc < 4; ++kc) {
    const float* p = A + arow * BZP + kc * 16 + lh * 8;
    const float4 a0 = *reinterpret_cast<const float4*>(p);
    const float4 a1 = *reinterpret_cast<const float4*>(p + 4);
    const float af[8] = {a0.x, a0.y, a0.z, a0.w, a1.x, a1.y, a1.z, a1.w};
#pragma unroll
    for (int s = 0; s < 8; ++s) acc = __builtin_amdgcn_mfma_f32_32x32x2f32(af[s], w[kc * 8 + s], acc, 0, 0, 0);
  }
}

__device__ __forceinline__ void acc_to_lds(const floatx16& acc, float* dst, int rblk, int c0, int lh,
                                           int li, float scale) {
#pragma unroll
  for (int q = 0; q < 16; ++q) {
    const int r = rblk * 32 + (q & 3) + 8 * (q >> 2) + 4 * lh;
    dst[r * BZP + c0 + li] = acc[q] * scale;
  }
}

__device__ __forceinline__ void zero_acc(floatx16& acc) {
#pragma unroll
  for (int q = 0; q < 16; ++q) acc[q] = 0.f;
}

__global__ __launch_bounds__(BNT) void graph_layer_bwd_kernel(
    const float* __restrict__ x, const float* __restrict__ dy, const float* __restrict__ pre_ln, int F,
    int J, int kind, int norm_res, const int* __restrict__ nbr_ptr, const int* __restrict__ nbr_idx, const float* __restrict__ w0,
    const float* __restrict__ w1, const float* __restrict__ Ug, const float* __restrict__ bias,
    const float* __restrict__ ln_w, const float* __restrict__ ln_b, float slope,
    float* __restrict__ dx, float* __restrict__ ybuf, float* __restrict__ dout,
    float* __restrict__ part) {
  __shared__ __attribute__((aligned(16))) float xs[BMAXN * BZP];
  __shared__ __attribute__((aligned(16))) float bufA[BMAXN * BZP];
  __shared__ __attribute__((aligned(16))) float bufB[BMAXN * BZP];
  __shared__ float U[2 * BH][BF];
  __shared__ float al[BMAXN][2 * BH];
  __shared__ float ew[BMAXN][BDEG];
  __shared__ float dsb[BMAXN][BDEG];
  __shared__ float dal[BMAXN][2];
  __shared__ float dalh[BH][2][BMAXN];  // every head's (da_src, da_dst), for the dU pass
  __shared__ __attribute__((aligned(8))) unsigned char nbl[BMAXN][BDEG];
  __shared__ __attribute__((aligned(8))) unsigned char rev[BMAXN][BDEG];  // GAT: slot of n in nbl[nbl[n][q]] (0xff: none)
  __shared__ unsigned char ndeg[BMAXN];
  __shared__ float red[BRG][3 * BF];
  __shared__ int csr[2 * BMAXN];   // the in-neighbour CSR (row pointers, then sources)

  const int fpb = BMAXN / J;
  const int NBmax = fpb * J;
  const int64_t node0 = (int64_t)blockIdx.x * NBmax;
  const int NB = (int)min<int64_t>(NBmax, (int64_t)F * J - node0);
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int li = lane & 31, lh = lane >> 5, cg = tid & 15, nr0 = tid >> 4;
  const int rblk = wave & 3, c0 = (wave >> 2) * 32;   // MFMA rows / columns of this wave
  const int arow = rblk * 32 + li;
  const int ywidth = kind == 0 ? BH * BF : BF;
  GB_STAMP(0);

  // the forward's saved pre-LayerNorm output o (bias included) replaces the recompute
  const bool saved = pre_ln != nullptr;
  const bool load_o = saved && norm_res;
  // ---- prologue: every global load of the block issued before the first LDS write (oldest
  // first: what the first barrier needs, then the weight fragments and dy rows that stay in flight)
  const int ne = min(nbr_ptr[J], 2 * BMAXN - (J + 1));
  constexpr int NL = BMAXN * (BF / 4) / BNT;
  float4 v[NL], u[NL];
#pragma unroll
  for (int j = 0; j < NL; ++j) {
    const int i = tid + j * BNT, n = i / (BF / 4), q = i % (BF / 4);
    v[j] = n < NB ? *reinterpret_cast<const float4*>(x + (node0 + n) * BF + q * 4)
                  : make_float4(0.f, 0.f, 0.f, 0.f);
    u[j] = load_o && n < NB ? *reinterpret_cast<const float4*>(pre_ln + (node0 + n) * BF + q * 4)
                            : make_float4(0.f, 0.f, 0.f, 0.f);
  }
  const float uval = kind == 0 ? Ug[tid] : 0.f;   // 512 threads = the [8][64] projections
  const int csr_v = tid <= J ? nbr_ptr[tid] : (tid < J + 1 + ne ? nbr_idx[tid - (J + 1)] : 0);
  // B fragments of the backward MFMAs (GAT: head 0, the next head's one head ahead; GraphConv:
  // W_rel and W_root)
  float wcur[32], wnxt[32];
  load_wt(wcur, w0, c0, lh, li);
  if (kind != 0) load_wt(wnxt, w1, c0, lh, li);
  // this thread's columns of the bias / LayerNorm parameters and its rows of dy, in flight across
  // the prologue / recompute
  const float4 bias4 = saved ? make_float4(0.f, 0.f, 0.f, 0.f) : *reinterpret_cast<const float4*>(bias + cg * 4);
  const float4 lnw4 = norm_res ? *reinterpret_cast<const float4*>(ln_w + cg * 4) : make_float4(1.f, 1.f, 1.f, 1.f);
  const float4 lnb4 = norm_res ? *reinterpret_cast<const float4*>(ln_b + cg * 4) : make_float4(0.f, 0.f, 0.f, 0.f);
  const float biasv[4] = {bias4.x, bias4.y, bias4.z, bias4.w};
  const float lnwv[4] = {lnw4.x, lnw4.y, lnw4.z, lnw4.w};
  const float lnbv[4] = {lnb4.x, lnb4.y, lnb4.z, lnb4.w};
  float4 dyr[BRPT];
#pragma unroll
  for (int r = 0; r < BRPT; ++r) {
    const int n = nr0 + BRG * r;
    dyr[r] = n < NB ? *reinterpret_cast<const float4*>(dy + (node0 + n) * BF + cg * 4)
                    : make_float4(0.f, 0.f, 0.f, 0.f);
  }
#pragma unroll
  for (int j = 0; j < NL; ++j) {
    const int i = tid + j * BNT, n = i / (BF / 4), q = i % (BF / 4);
    *reinterpret_cast<float4*>(xs + n * BZP + q * 4) = v[j];
    if (load_o) *reinterpret_cast<float4*>(bufA + n * BZP + q * 4) = u[j];
  }
  if (kind == 0) (&U[0][0])[tid] = uval;
  if (tid < J + 1 + ne) csr[tid] = csr_v;
  __syncthreads();
  for (int n = tid; n < BMAXN; n += blockDim.x) {
    int d = 0;
    if (n < NB) {
      const int f0 = (n / J) * J, ln = n % J;
      for (int e = csr[ln]; e < csr[ln + 1] && d < BDEG; ++e) nbl[n][d++] = f0 + csr[J + 1 + e];
      if (kind == 0 && d < BDEG) nbl[n][d++] = n;
    }
    for (int q = d; q < BDEG; ++q) nbl[n][q] = 0;  // unpredicated gathers read row 0, weight 0
    ndeg[n] = d;
  }
  __syncthreads();
  GB_STAMP(1);
  if (kind == 0) {
    // reverse-edge slots, once per block (the per-head adjoint loops index them directly
    // instead of searching the neighbour list of every neighbour)
    // (one thread per (n, q); neighbour i's list read as one 8-byte word)
    for (int it = tid; it < NB * BDEG; it += blockDim.x) {
      const int n = it / BDEG, q = it % BDEG;
      unsigned char r = 0xff;
      if (q < ndeg[n]) {
        const int i = nbl[n][q], di = ndeg[i];
        const uint2 nb = *reinterpret_cast<const uint2*>(&nbl[i][0]);
#pragma unroll
        for (int p = BDEG - 1; p >= 0; --p)
          if (p < di && (((p < 4 ? nb.x : nb.y) >> (8 * (p & 3))) & 0xff) == (unsigned)n)
            r = (unsigned char)p;  // first match, as the search did
      }
      rev[n][q] = r;
    }
    for (int i = tid; i < NB * 2 * BH; i += blockDim.x) {
      const int n = i >> 3, q = i & 7;
      float s = 0.f;   // k in order, as the forward's logits (graph.hip)
#pragma unroll 4
      for (int k = 0; k < BF; k += 4) {
        const float4 xv = *reinterpret_cast<const float4*>(xs + n * BZP + k);
        const float4 uv = *reinterpret_cast<const float4*>(&U[q][k]);
        s += xv.x * uv.x; s += xv.y * uv.y; s += xv.z * uv.z; s += xv.w * uv.w;
      }
      al[n][q] = s;
    }
    __syncthreads();
    GB_STAMP(2);
  }

  auto edge_softmax = [&](int h) {
    for (int n = tid; n < NB; n += blockDim.x) {
      const int d = ndeg[n];
      const float ad = al[n][BH + h];
      float e[BDEG];
      float mx = -INFINITY;
#pragma unroll
      for (int q = 0; q < BDEG; ++q)
        if (q < d) {
          const float s = al[nbl[n][q]][h] + ad;
          e[q] = s > 0.f ? s : s * 0.2f;
          mx = fmaxf(mx, e[q]);
        }
      float den = 0.f;
#pragma unroll
      for (int q = 0; q < BDEG; ++q)
        if (q < d) { e[q] = expf(e[q] - mx); den += e[q]; }
      const float inv = 1.f / (den + 1e-16f);
#pragma unroll
      for (int q = 0; q < BDEG; ++q) ew[n][q] = q < d ? e[q] * inv : 0.f;
    }
  };

  // ---------------------------------------------------------------- forward recompute
  // (without the saved o: Y_h / agg -> ybuf for the weight gradients, o -> bufA)
  floatx16 acc;
  zero_acc(acc);
  const int nseg = saved ? 0 : (kind == 0 ? BH : 2);
  for (int seg = 0; seg < nseg; ++seg) {
    const float* Wseg = kind == 0 ? w0 + (int64_t)seg * BF * BF : (seg == 0 ? w0 : w1);
    const float* A = bufA;
    if (kind == 0 || seg == 0) {
      if (kind == 0) {
        edge_softmax(seg);
        __syncthreads();
      }
      for (int i = tid; i < BMAXN * 16; i += blockDim.x) {
        const int n = i >> 4, c4 = i & 15;
        float4 a = make_float4(0.f, 0.f, 0.f, 0.f);
        const int d = n < NB ? ndeg[n] : 0;
        float4 v[BDEG];
#pragma unroll
        for (int q = 0; q < BDEG; ++q)
          v[q] = *reinterpret_cast<const float4*>(xs + nbl[n][q] * BZP + c4 * 4);
#pragma unroll
        for (int q = 0; q < BDEG; ++q) {
          const float w = q < d ? (kind == 0 ? ew[n][q] : 1.f) : 0.f;
          a.x += w * v[q].x; a.y += w * v[q].y; a.z += w * v[q].z; a.w += w * v[q].w;
        }
        *reinterpret_cast<float4*>(bufA + n * BZP + c4 * 4) = a;
        if (n < NB) *reinterpret_cast<float4*>(ybuf + (node0 + n) * ywidth + seg * BF + c4 * 4) = a;
      }
      __syncthreads();
    } else {
      A = xs;
    }
    mfma_rows64(acc, A, arow, c0, lh, li, [&](int j, int c) { return Wseg[j * BF + c]; });
    __syncthreads();
  }
  if (!saved) {
    acc_to_lds(acc, bufA, rblk, c0, lh, li, kind == 0 ? 1.f / BH : 1.f);  // o (bias added below)
    __syncthreads();
  }
  GB_STAMP(3);

  // ---------------------------------------------------------------- LN / act / residual bwd
  float dxa[BRPT][4];
  float pb[4] = {0.f, 0.f, 0.f, 0.f}, plw[4] = {0.f, 0.f, 0.f, 0.f}, plb[4] = {0.f, 0.f, 0.f, 0.f};
  const float oscale = kind == 0 ? 1.f / BH : 1.f;
#pragma unroll
  for (int r = 0; r < BRPT; ++r) {
    const int n = nr0 + BRG * r;
    float o[4], g4[4];
    const float dyv[4] = {dyr[r].x, dyr[r].y, dyr[r].z, dyr[r].w};
#pragma unroll
    for (int q = 0; q < 4; ++q) o[q] = saved ? bufA[n * BZP + cg * 4 + q] : bufA[n * BZP + cg * 4 + q] + biasv[q];
    float dov[4];
    if (norm_res) {
      float s = o[0] + o[1] + o[2] + o[3];
      s = row16_sum(s);
      const float mean = s * (1.f / BF);
      float ss = 0.f;
#pragma unroll
      for (int q = 0; q < 4; ++q) ss += (o[q] - mean) * (o[q] - mean);
      ss = row16_sum(ss);
      const float rstd = 1.f / sqrtf(ss * (1.f / BF) + 1e-5f);
      float sg = 0.f, sgx = 0.f, oh[4];
#pragma unroll
      for (int q = 0; q < 4; ++q) {
        oh[q] = (o[q] - mean) * rstd;
        const float u = oh[q] * lnwv[q] + lnbv[q];
        const float du = n < NB ? dyv[q] * (u > 0.f ? 1.f : slope) : 0.f;
        plw[q] += du * oh[q];
        plb[q] += du;
        g4[q] = du * lnwv[q];
        sg += g4[q];
        sgx += g4[q] * oh[q];
      }
      sg = row16_sum(sg);
      sgx = row16_sum(sgx);
      const float mg = sg * (1.f / BF), mgx = sgx * (1.f / BF);
#pragma unroll
      for (int q = 0; q < 4; ++q) {
        dov[q] = n < NB ? rstd * (g4[q] - mg - oh[q] * mgx) : 0.f;
        dxa[r][q] = n < NB ? dyv[q] : 0.f;
      }
    } else {
#pragma unroll
      for (int q = 0; q < 4; ++q) {
        dov[q] = dyv[q];
        dxa[r][q] = 0.f;
      }
    }
#pragma unroll
    for (int q = 0; q < 4; ++q) pb[q] += dov[q];
    *reinterpret_cast<float4*>(bufB + n * BZP + cg * 4) = make_float4(dov[0], dov[1], dov[2], dov[3]);
    if (n < NB && dout)
      *reinterpret_cast<float4*>(dout + (node0 + n) * BF + cg * 4) =
          make_float4(dov[0] * oscale, dov[1] * oscale, dov[2] * oscale, dov[3] * oscale);
  }
  __syncthreads();
  GB_STAMP(4);

  float dU = 0.f;  // per-thread item tid of the dU partial [8][64]
  if (kind == 0) {
    for (int h = 0; h < BH; ++h) {
      edge_softmax(h);
      // dY_h = do W_h / 4  -> bufA
      zero_acc(acc);
      if (h + 1 < BH) load_wt(wnxt, w0 + (int64_t)(h + 1) * BF * BF, c0, lh, li);
      mfma_rows64_w(acc, bufB, arow, lh, wcur);
      acc_to_lds(acc, bufA, rblk, c0, lh, li, 1.f / BH);
#pragma unroll
      for (int s = 0; s < 32; ++s) wcur[s] = wnxt[s];
      __syncthreads();
      GB_STAMP(5 + 5 * h + 0);
      // dalpha[n][q] = dY_h[n] . x[nbl[n][q]]  (16 lanes per node), then on every lane of the
      // node's group (identical row sums) the softmax + LeakyReLU backward: ds (pre-activation
      // logit grads, -> dsb) and da_dst
      for (int i = tid; i < BMAXN * 16; i += blockDim.x) {
        const int n = i >> 4, c4 = i & 15;
        const int d = ndeg[n];
        const float4 g = *reinterpret_cast<const float4*>(bufA + n * BZP + c4 * 4);
        const uint2 nb = *reinterpret_cast<const uint2*>(&nbl[n][0]);
        int ids[BDEG];
#pragma unroll
        for (int q = 0; q < BDEG; ++q) ids[q] = ((q < 4 ? nb.x : nb.y) >> (8 * (q & 3))) & 0xff;
        float4 xv[BDEG];
#pragma unroll
        for (int q = 0; q < BDEG; ++q)
          xv[q] = *reinterpret_cast<const float4*>(xs + ids[q] * BZP + c4 * 4);
        float v[BDEG];
#pragma unroll
        for (int q = 0; q < BDEG; ++q)
          v[q] = q < d ? g.x * xv[q].x + g.y * xv[q].y + g.z * xv[q].z + g.w * xv[q].w : 0.f;
#pragma unroll
        for (int q = 0; q < BDEG; ++q) v[q] = row16_sum(v[q]);
        if (n < NB) {
          const float ad = al[n][BH + h];
          float e[BDEG], sv[BDEG];
#pragma unroll
          for (int q = 0; q < BDEG; ++q) {
            e[q] = ew[n][q];
            sv[q] = al[ids[q]][h] + ad;
          }
          float sdot = 0.f;
#pragma unroll
          for (int q = 0; q < BDEG; ++q)
            if (q < d) sdot += e[q] * v[q];
          float sum = 0.f;
#pragma unroll
          for (int q = 0; q < BDEG; ++q)
            if (q < d) {
              const float de = e[q] * (v[q] - sdot);
              v[q] = de * (sv[q] > 0.f ? 1.f : 0.2f);
              sum += v[q];
            }
          if (c4 == 0) {
#pragma unroll
            for (int q = 0; q < BDEG; ++q)
              if (q < d) dsb[n][q] = v[q];
            dal[n][1] = sum;
            dalh[h][1][n] = sum;
          }
        }
      }
      __syncthreads();
      GB_STAMP(5 + 5 * h + 1);
      // dx += aggregation adjoint + logit adjoint (with da_src);  dU partials
#pragma unroll
      for (int r = 0; r < BRPT; ++r) {
        const int n = nr0 + BRG * r;
        if (n >= NB) continue;
        float a[4] = {0.f, 0.f, 0.f, 0.f};
        float4 gv[BDEG];
        float al4[BDEG];
        const uint2 nb = *reinterpret_cast<const uint2*>(&nbl[n][0]);
        const uint2 rv = *reinterpret_cast<const uint2*>(&rev[n][0]);
        int ids[BDEG], ps[BDEG];
#pragma unroll
        for (int q = 0; q < BDEG; ++q) {
          ids[q] = ((q < 4 ? nb.x : nb.y) >> (8 * (q & 3))) & 0xff;
          ps[q] = ((q < 4 ? rv.x : rv.y) >> (8 * (q & 3))) & 0xff;
        }
        // da_src[n] = sum of ds over the edges out of n (j = n's targets, symmetric graph)
        const int dn = ndeg[n];
        float das = 0.f;
#pragma unroll
        for (int q = 0; q < BDEG; ++q) {
          gv[q] = *reinterpret_cast<const float4*>(bufA + ids[q] * BZP + cg * 4);
          const bool e = ps[q] != 0xff;   // 0xff past the degree
          al4[q] = e ? ew[ids[q]][ps[q] & 7] : 0.f;
          const float dsv = e ? dsb[ids[q]][ps[q] & 7] : 0.f;
          if (q < dn && e) das += dsv;
        }
        if (cg == 0) dalh[h][0][n] = das;
#pragma unroll
        for (int q = 0; q < BDEG; ++q) {
          a[0] += al4[q] * gv[q].x; a[1] += al4[q] * gv[q].y; a[2] += al4[q] * gv[q].z;
          a[3] += al4[q] * gv[q].w;
        }
#pragma unroll
        for (int q = 0; q < 4; ++q)
          dxa[r][q] += a[q] + das * U[h][cg * 4 + q] + dal[n][1] * U[BH + h][cg * 4 + q];
        if (saved) {
          // Z_h[n] = sum_i alpha_inh dout_i (the aggregation adjoint of dout): dW_h = sum_n Z_h[n] x_n^T
          float4 z = make_float4(0.f, 0.f, 0.f, 0.f);
#pragma unroll
          for (int q = 0; q < BDEG; ++q) {
            const float4 dv = *reinterpret_cast<const float4*>(bufB + ids[q] * BZP + cg * 4);
            z.x += al4[q] * dv.x; z.y += al4[q] * dv.y; z.z += al4[q] * dv.z; z.w += al4[q] * dv.w;
          }
          *reinterpret_cast<float4*>(ybuf + (node0 + n) * ywidth + h * BF + cg * 4) =
              make_float4(z.x * oscale, z.y * oscale, z.z * oscale, z.w * oscale);
        }
      }
      __syncthreads();
      GB_STAMP(5 + 5 * h + 4);
    }
    // dU partials, all heads in one pass over the block's nodes (thread tid: item tid of
    // [8][64], q = which * 4 + h)
    {
      const int qq = tid / BF, k = tid % BF;
      const float* dl = dalh[qq & 3][qq >> 2];
      float s = 0.f;
      for (int n = 0; n < NB; ++n) s += dl[n] * xs[n * BZP + k];
      dU = s;
    }
  } else {
    // dagg = do W_rel -> bufA ; dx_root = do W_root -> xs (x no longer needed)
    zero_acc(acc);
    mfma_rows64_w(acc, bufB, arow, lh, wcur);
    acc_to_lds(acc, bufA, rblk, c0, lh, li, 1.f);
    zero_acc(acc);
    mfma_rows64_w(acc, bufB, arow, lh, wnxt);
    __syncthreads();
    GB_STAMP(5);
    acc_to_lds(acc, xs, rblk, c0, lh, li, 1.f);
    __syncthreads();
    GB_STAMP(6);
#pragma unroll
    for (int r = 0; r < BRPT; ++r) {
      const int n = nr0 + BRG * r;
      if (n >= NB) continue;
      float a[4];
#pragma unroll
      for (int q = 0; q < 4; ++q) a[q] = xs[n * BZP + cg * 4 + q];
      const int dn = ndeg[n];
      float4 gv[BDEG];
#pragma unroll
      for (int q = 0; q < BDEG; ++q)
        gv[q] = *reinterpret_cast<const float4*>(bufA + nbl[n][q] * BZP + cg * 4);
#pragma unroll
      for (int q = 0; q < BDEG; ++q)
        if (q < dn) { a[0] += gv[q].x; a[1] += gv[q].y; a[2] += gv[q].z; a[3] += gv[q].w; }
#pragma unroll
      for (int q = 0; q < 4; ++q) dxa[r][q] += a[q];
      if (saved) {  // Z[n] = sum_{i ~ n} do_i: dW_rel = sum_n Z[n] x_n^T
        float4 z = make_float4(0.f, 0.f, 0.f, 0.f);
#pragma unroll
        for (int q = 0; q < BDEG; ++q)
          if (q < dn) {
            const float4 dv = *reinterpret_cast<const float4*>(bufB + nbl[n][q] * BZP + cg * 4);
            z.x += dv.x; z.y += dv.y; z.z += dv.z; z.w += dv.w;
          }
        *reinterpret_cast<float4*>(ybuf + (node0 + n) * BF + cg * 4) = z;
      }
    }
  }

#pragma unroll
  for (int r = 0; r < BRPT; ++r) {
    const int n = nr0 + BRG * r;
    if (n < NB)
      *reinterpret_cast<float4*>(dx + (node0 + n) * BF + cg * 4) =
          make_float4(dxa[r][0], dxa[r][1], dxa[r][2], dxa[r][3]);
  }
  // per-workgroup partials: reduce the BRG row groups through LDS
#pragma unroll
  for (int q = 0; q < 4; ++q) {
    red[nr0][cg * 4 + q] = pb[q];
    red[nr0][BF + cg * 4 + q] = plw[q];
    red[nr0][2 * BF + cg * 4 + q] = plb[q];
  }
  __syncthreads();
  GB_STAMP(25);
  float* pp = part + (int64_t)blockIdx.x * BPART;
  for (int c = tid; c < 3 * BF; c += blockDim.x) {
    float s = 0.f;
    for (int g = 0; g < BRG; ++g) s += red[g][c];
    pp[c] = s;
  }
  if (kind == 0) pp[3 * BF + tid] = dU;
  GB_STAMP(26);
}

// dU -> att gradients and the extra dW terms: U_q[k] = sum_c W_h[c][k] att_q[c]
//   datt_q[c] = sum_k W_h[c][k] dU_q[k];   dW_h[c][k] += att_src_h[c] dU_h[k] + att_dst_h[c] dU_4+h[k]
__global__ void graph_att_bwd_kernel(const float* w0, const float* att_src, const float* att_dst,
                                     const float* dU, float* dw0, float* datt_src, float* datt_dst) {
  const int i = blockIdx.x * blockDim.x + threadIdx.x;  // [4][64][64] (h, c, k)
  if (i < BH * BF * BF) {
    const int h = i / (BF * BF), c = (i / BF) % BF, k = i % BF;
    dw0[i] += att_src[h * BF + c] * dU[h * BF + k] + att_dst[h * BF + c] * dU[(BH + h) * BF + k];
  }
  if (i < 2 * BH * BF) {
    const int q = i / BF, c = i % BF, h = q & 3;
    float s = 0.f;
    for (int k = 0; k < BF; ++k) s += w0[((int64_t)h * BF + c) * BF + k] * dU[q * BF + k];
    (q < BH ? datt_src : datt_dst)[h * BF + c] = s;
  }
}

__global__ void graph_att_proj_kernel2(const float* w0, const float* att_src, const float* att_dst,
                                       float* Ug) {
  const int q = threadIdx.x / BF, k = threadIdx.x % BF, h = q & 3;
  const float* att = (q < BH ? att_src : att_dst) + h * BF;
  float s = 0.f;
  for (int c = 0; c < BF; ++c) s += w0[((int64_t)h * BF + c) * BF + k] * att[c];
  Ug[threadIdx.x] = s;
}

}  // namespace a2m

using namespace a2m;

#ifdef A2M_GBWD_STAMPS
extern "C" int a2m_debug_gbwd_stamps(unsigned long long* host, size_t n) {
  const size_t cap = (size_t)kGbBlocks * kGbStamps;
  return hipMemcpyFromSymbol(host, HIP_SYMBOL(g_gb_stamps), sizeof(unsigned long long) * (n < cap ? n : cap)) ==
         hipSuccess ? A2M_OK : A2M_EHIP;
}
#endif

// pre_ln (nullable): the forward's saved pre-LayerNorm output (a2m_graph_layer_fwd_f32's pre_ln,
// written when norm_res).  With it the kernel skips the forward recompute and the weight
// gradients contract the aggregation adjoint of dout with x instead of dout with the aggregated
// inputs (same sums, another order); without it, the recompute path.
extern "C" int a2m_graph_layer_bwd_saved_f32(const float* x, const float* dy, const float* pre_ln, int32_t F,
                                             int32_t J, int32_t kind, int32_t norm_res, const int32_t* nbr_ptr,
                                             const int32_t* nbr_idx, const float* w0, const float* w1,
                                             const float* att_src, const float* att_dst, const float* bias,
                                             const float* ln_w, const float* ln_b, float slope, float* dx,
                                             float* dw0, float* dw1, float* datt_src, float* datt_dst,
                                             float* dbias, float* dln_w, float* dln_b, void* ws, size_t ws_bytes,
                                             void* stream) {
  A2M_CHECK_ARG(x && dy && dx && nbr_ptr && nbr_idx && w0 && bias && dw0 && dbias,
                "graph_layer_bwd: null pointer");
  A2M_CHECK_ARG(J > 0 && J <= BMAXN && F > 0, "graph_layer_bwd: bad shape");
  A2M_CHECK_ARG(kind == 0 ? (att_src && att_dst && datt_src && datt_dst) : (kind == 1 && w1 && dw1),
                "graph_layer_bwd: bad kind / params");
  A2M_CHECK_ARG(!norm_res || (ln_w && ln_b && dln_w && dln_b), "graph_layer_bwd: LN params");
  auto al16 = [](const void* q) { return q == nullptr || (reinterpret_cast<uintptr_t>(q) & 15) == 0; };
  A2M_CHECK_ARG(al16(bias) && al16(ln_w) && al16(ln_b), "graph_layer_bwd: bias / LayerNorm vectors must be 16-byte aligned");
  const int fpb = BMAXN / J;
  const int blocks = (int)cdiv(F, fpb);
  const int64_t Nn = (int64_t)F * J;
  const int yw = kind == 0 ? BH * BF : BF;
  auto al256 = [](size_t b) { return (b + 255) & ~size_t(255); };
  const size_t b_u = al256(sizeof(float) * 2 * BH * BF);
  const size_t b_y = al256(sizeof(float) * Nn * yw);
  const size_t b_do = al256(sizeof(float) * Nn * BF);
  const size_t b_part = al256(sizeof(float) * (size_t)blocks * BPART);
  const size_t b_red = al256(sizeof(float) * BPART);
  const size_t fixed = b_u + b_y + b_do + b_part + b_red;
  const size_t need = fixed + std::max(gemm_ws_bytes(BF, BF, (int)Nn, BH), gemm_ws_bytes(BF, BF, (int)Nn, 1));
  if (!ws || ws_bytes < need) {
    set_error("graph_layer_bwd: workspace too small (%zu < %zu bytes)", ws_bytes, need);
    return A2M_EWS;
  }
  char* p = static_cast<char*>(ws);
  float* Ug = reinterpret_cast<float*>(p); p += b_u;
  float* ybuf = reinterpret_cast<float*>(p); p += b_y;
  float* dob = reinterpret_cast<float*>(p); p += b_do;
  float* part = reinterpret_cast<float*>(p); p += b_part;
  float* redv = reinterpret_cast<float*>(p); p += b_red;
  void* gws = p;
  const size_t gbytes = ws_bytes - fixed;
  hipStream_t st = as_stream(stream);
  if (kind == 0) {
    hipLaunchKernelGGL(graph_att_proj_kernel2, dim3(1), dim3(2 * BH * BF), 0, st, w0, att_src, att_dst, Ug);
    A2M_LAUNCH_CHECK();
  }
  // the saved path of the GAT needs no dout rows (its weight gradient contracts Z with x)
  const bool saved = pre_ln != nullptr;
  hipLaunchKernelGGL(graph_layer_bwd_kernel, dim3(blocks), dim3(BNT), 0, st, x, dy, pre_ln, F, J, kind, norm_res,
                     nbr_ptr, nbr_idx, w0, w1, Ug, bias, ln_w, ln_b, slope, dx, ybuf,
                     saved && kind == 0 ? nullptr : dob, part);
  A2M_LAUNCH_CHECK();
  const int cols = kind == 0 ? BPART : 3 * BF;
  // dbias | dln_w | dln_b straight into the caller's vectors, the attention partials into redv
  ColOuts outs{};
  outs.out[0] = dbias; outs.start[0] = 0;
  outs.out[1] = norm_res ? dln_w : redv + BF; outs.start[1] = BF;
  outs.out[2] = norm_res ? dln_b : redv + 2 * BF; outs.start[2] = 2 * BF;
  outs.out[3] = redv + 3 * BF; outs.start[3] = 3 * BF;
  outs.n = cols > 3 * BF ? 4 : 3;
  int rc = reduce_cols(part, blocks, BPART, cols, outs, 0, st);
  if (rc) return rc;
  // weight gradients: sum over all nodes of do (x) Y  (saved path: of Z (x) x)
  if (kind == 0) {
    // dW_h[c][k] = sum_n dout[n][c] Y[n][h*64 + k] = sum_n Z[n][h*64 + c] x[n][k]  (batch over heads)
    rc = saved ? gemm(dense_kr(ybuf, yw, BF), dense_kr(x, BF, 0), epi_dense(dw0, BF, (int64_t)BF * BF), BF, BF,
                      (int)Nn, BH, gws, gbytes, st)
               : gemm(dense_kr(dob, BF, 0), dense_kr(ybuf, yw, BF), epi_dense(dw0, BF, (int64_t)BF * BF), BF, BF,
                      (int)Nn, BH, gws, gbytes, st);
    if (rc) return rc;
    hipLaunchKernelGGL(graph_att_bwd_kernel, dim3((unsigned)cdiv(BH * BF * BF, 256)), dim3(256), 0, st, w0,
                       att_src, att_dst, redv + 3 * BF, dw0, datt_src, datt_dst);
    A2M_LAUNCH_CHECK();
  } else {
    rc = saved ? gemm(dense_kr(ybuf, BF), dense_kr(x, BF), epi_dense(dw0, BF), BF, BF, (int)Nn, 1, gws, gbytes, st)
               : gemm(dense_kr(dob, BF), dense_kr(ybuf, BF), epi_dense(dw0, BF), BF, BF, (int)Nn, 1, gws, gbytes, st);
    if (rc) return rc;
    rc = gemm(dense_kr(dob, BF), dense_kr(x, BF), epi_dense(dw1, BF), BF, BF, (int)Nn, 1, gws, gbytes, st);
    if (rc) return rc;
  }
  return A2M_OK;
}

extern "C" int a2m_graph_layer_bwd_f32(const float* x, const float* dy, int32_t F, int32_t J,
                                       int32_t kind, int32_t norm_res, const int32_t* nbr_ptr,
                                       const int32_t* nbr_idx, const float* w0, const float* w1,
                                       const float* att_src, const float* att_dst,
                                       const float* bias, const float* ln_w, const float* ln_b,
                                       float slope, float* dx, float* dw0, float* dw1,
                                       float* datt_src, float* datt_dst, float* dbias,
                                       float* dln_w, float* dln_b, void* ws, size_t ws_bytes,
                                       void* stream) {
  return a2m_graph_layer_bwd_saved_f32(x, dy, nullptr, F, J, kind, norm_res, nbr_ptr, nbr_idx, w0, w1, att_src,
                                       att_dst, bias, ln_w, ln_b, slope, dx, dw0, dw1, datt_src, datt_dst, dbias,
                                       dln_w, dln_b, ws, ws_bytes, stream);
}
