// Fused attention core for short sequences (T <= 64) and narrow queries (C/8 <= 64): the
// decoders' SelfAttention(256) at T = 64 (model_layers.py:121-146):
//     S = Q^T K  (no 1/sqrt(d) scaling, :140),  A = softmax_j(S),
//     y[c][i] = gamma * sum_j V[c][j] A[i][j] + x[c][i] (+ res[c][i])
// One workgroup per (clip, 64-channel chunk of V): the 64 x 64 score tile is recomputed per
// chunk (K = C/8 <= 64, a few MFMAs) instead of making a round trip through HBM, the softmax
// runs on the LDS tile, and the PV product + epilogue follow without leaving the workgroup.
// The normalised attention matrix is also written out when the backward pass needs it.
// Replaces three launches (score GEMM, softmax, PV GEMM) of the general path.
#include "gemm_pipe.h"

namespace a2m {

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

// ---------------------------------------------------------------------------------------
// Eval-only fusion of the q/k/v 1x1 convolutions into the core (no qkv / attention outputs
// are kept for a backward pass): one workgroup per (clip, 64-channel chunk of V), C in
// {128, 256}, T <= 64.  Step 1 is a pipelined GEMM P[t][col] = sum_c x[c][t] W[col][c] over
// 128 columns = Q (C/8, zero-padded to 32) | K (same) | this chunk's 64 V rows: k-tiles of 32
// channels of x ([t][c], transposed on the way in) and of the stacked weight rows are staged
// through double-buffered LDS shared by eight waves (two per SIMD), one barrier per k-step,
// global loads of the next tile in flight behind the current tile's MFMAs; each wave owns one
// 32 x 32 block of P.  Then Q^T, K^T and the V chunk move to LDS and the score (waves 0-3) /
// softmax / PV + epilogue (waves 4-7) steps of attn_core_kernel follow.  Q and K are
// recomputed by each of the C/64 chunks of a clip (C/4 of the 5C/4 projection rows), which
// costs less than a second launch and a round trip of qkv through memory.
// ---------------------------------------------------------------------------------------
constexpr int QP = 36;        // Q^T / K^T pitch (32 columns): conflict-free b128 rows
constexpr int FK = 32;        // projection k-tile (channels)
constexpr int FKP = FK + 4;   // staged tile pitch
constexpr int kHWP = FK + 8;  // bf16 weight tile pitch (halves): conflict-free b128 fragment rows
// V channels per workgroup at C % 128 == 0.  128 computes a C = 256 clip's Q / K twice instead of
// four times: the kernel's time drops 358.5 -> 305.8 us a step, but the step got 0.5-0.7 % slower
// (fp32 2.520 vs 2.503 ms, bf16 1.439 vs 1.432, three interleaved pairs,
// profiles/r06_j_attn_chunk_ab.txt): half the workgroups, each longer, on the decoder's critical
// path.  64 stays the default; 128 is reachable through a2m_set_attn_eval_chunk (tests).
#ifndef A2M_ATTN_NV
#define A2M_ATTN_NV 64
#endif
static int g_attn_nv = A2M_ATTN_NV;   // a2m_set_attn_eval_chunk (test hook)

// bf16 operand mode (precision 1): the projection's products on v_mfma_f32_32x32x16_bf16 --
// each lane's 8 staged k of a 16-k half rounded to bf16 in registers (the fp32 fragment layout is
// the bf16 MFMA's), one MFMA per half instead of eight -- as the engine's bf16 QKV GEMM rounds
// them; scores, softmax and PV stay fp32 as in every mode.
__device__ __forceinline__ bf16x8 attn_pack8(const float (&v)[8]) {
  typedef float f2 __attribute__((ext_vector_type(2)));
  typedef __bf16 h2 __attribute__((ext_vector_type(2)));
  typedef uint32_t u4 __attribute__((ext_vector_type(4)));
  uint32_t u[4];
#pragma unroll
  for (int j = 0; j < 4; ++j) {
    const f2 p = {v[2 * j], v[2 * j + 1]};
    u[j] = __builtin_bit_cast(uint32_t, __builtin_convertvector(p, h2));
  }
  return __builtin_bit_cast(bf16x8, u4{u[0], u[1], u[2], u[3]});
}

// NV = V channels per workgroup (64 or 128): the projection has FC = 64 + NV columns (Q 32 | K 32 |
// V NV), FC / 32 column tiles by 2 t tiles = one 32 x 32 tile per wave (8 waves at NV = 64, 12 at
// 128).  At NV = 128 a C = 256 clip's Q and K are computed twice instead of four times (the
// projection 1.33x the non-redundant 5C/4 rows instead of 1.6x); every output element sees the
// same operations in the same order at either NV, so the two are bitwise equal (NV = 64 is the
// default, A2M_ATTN_NV below).
// WH (bf16 mode): the stacked weights come as a bf16 copy (wqkv_h, made once per weight version)
// and are staged as bf16 -- one 16-byte load and store per thread a k-tile instead of two, and the
// fragments read ready for the MFMA instead of rounded at every read; the same values, so bitwise
// the same result.
template <bool BF16, int NV, bool WH = false>
__global__ __launch_bounds__(NV == 64 ? 512 : 768, NV == 64 ? 2 : 1) void attn_fused_eval_kernel(
    const float* __restrict__ x, int64_t x_bs, int C, int T, const float* __restrict__ wqkv,
    const float* __restrict__ bqkv, const float* __restrict__ gamma, const float* __restrict__ res,
    float* __restrict__ y, int B, int64_t x_gs, int64_t res_gs, int64_t y_gs,
    const __bf16* __restrict__ wqkv_h) {
  static_assert(BF16 || !WH, "bf16 weights only in bf16 mode");
  {  // grouped launches: blockIdx.y = g * B + b, problem g with its own weights
    const int g = blockIdx.y / B;
    x += g * x_gs;
    y += g * y_gs;
    if (res) res += g * res_gs;
    wqkv += (int64_t)g * (C / 4 + C) * C;
    if (WH) wqkv_h += (int64_t)g * (C / 4 + C) * C;
    bqkv += (int64_t)g * (C / 4 + C);
    gamma += g;
  }
  constexpr int FC = 64 + NV, NCT = FC / 32, NT = 64 * 2 * NCT;
  constexpr int XT = AT * FKP, WTL = FC * FKP, STG = XT + WTL;
  // stages (2 x (x tile + w tile)) early; Q^T, K^T, V, scores overlay them afterwards
  __shared__ __attribute__((aligned(16))) float lds[2 * STG];
  float* qs = lds;                     // [i][c'] pitch QP
  float* ks = qs + AT * QP;            // [j][c']
  float* vs = ks + AT * QP;            // [c][j]  pitch AP
  float* ss = vs + NV * AP;            // [i][j]  pitch AP
  static_assert(2 * AT * QP + (NV + AT) * AP <= 2 * STG, "overlay must fit the stages");
  static_assert(FC * 8 == 2 * NT, "two float4 of weight rows per thread");
  const int b = blockIdx.y % B, c0 = blockIdx.x * NV;
  const int Cq = C / 8;
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int li = lane & 31, lh = lane >> 5;
  // projection: wave (pt, pc) = (wave / NCT, wave % NCT) owns t rows 32 pt.. and columns 32 pc..
  // (one accumulator; two or three waves per SIMD hide each other's LDS and barrier waits);
  // attention steps: the score product on waves 0-3 as (wt, wc) = (wave >> 1, wave & 1), PV on
  // waves 4.. as (channel tile, query tile) = ((wave - 4) >> 1, (wave - 4) & 1)
  const int pt = wave / NCT, pc = wave % NCT;
  const int wt = wave < 4 ? wave >> 1 : (wave - 4) >> 1, wc = wave & 1;
  const float* xb = x + (int64_t)b * x_bs;

  // Staging maps.  x tile [t][c] from x[c][t]: thread -> (c = tid % 32, t quad = tid / 32), one
  // float4 per thread of the first 512, transposed writes conflict-free (32 lanes = 32
  // consecutive c).
  // w tile [col][c]: stacked rows Q 0..Cq-1 -> cols 0.., K Cq.. -> 32.., V 2Cq + c0.. -> 64..;
  // two float4 per thread along c.  All loads are raw buffer loads (rows past Cq / t past T read
  // 0), so the k-step below is branch-free and its operand work is placed between the MFMAs
  // (pipe_step, gemm_pipe.h: tile i + 1 stored and tile i + 3 loaded behind the first half's
  // MFMAs, one barrier, the next fragments read behind the second half's first MFMAs).
  const __amdgpu_buffer_rsrc_t xrs = pipe_rsrc(xb),
                               wrs = pipe_rsrc(WH ? reinterpret_cast<const float*>(wqkv_h) : wqkv);
  const int xc = tid & 31, xq = tid >> 5;
  const bool xst = xq < AT / 4;   // this thread stages a piece of the x tile
  uint32_t xoff = 4 * xq < T ? (uint32_t)(xc * T + 4 * xq) * 4u : kPipeOOB;   // advanced 32 channels a tile
  uint32_t woff[2];
  if constexpr (WH) {   // one 16-byte piece (8 bf16 of k) per thread: row tid / 4, k 8 (tid % 4)
    const int col = tid >> 2;
    const int wrow = col < 32 ? (col < Cq ? col : -1)
                              : col < 64 ? (col - 32 < Cq ? Cq + col - 32 : -1) : 2 * Cq + c0 + col - 64;
    woff[0] = wrow >= 0 && col < FC ? (uint32_t)(wrow * C + (tid & 3) * 8) * 2u : kPipeOOB;
    woff[1] = kPipeOOB;
  } else {
#pragma unroll
    for (int u = 0; u < 2; ++u) {
      const int col = (tid + u * NT) >> 3;
      const int wrow = col < 32 ? (col < Cq ? col : -1)
                                : col < 64 ? (col - 32 < Cq ? Cq + col - 32 : -1) : 2 * Cq + c0 + col - 64;
      woff[u] = wrow >= 0 ? (uint32_t)(wrow * C + ((tid + u * NT) & 7) * 4) * 4u : kPipeOOB;
    }
  }
  struct Regs { float4 x, w[2]; };
  Regs rg[2];
  // the straight-line prefetch also issues the loads of the (unused) tiles past the last one:
  // those must read 0 (kPipeOOB), not channels past C -- for the last clip and the last weight
  // rows that would be memory past the tensors
  int cnext = 0;   // first channel of the next tile to load
  auto load_piece = [&](Regs& r, int piece) {   // piece 0: x, 1-2: w rows
    const bool ok = cnext < C;
    if (piece == 0) { r.x = pipe_load(xrs, ok ? xoff : kPipeOOB); xoff += 4u * FK * T; }
    else if (WH) { if (piece == 1) { r.w[0] = pipe_load(wrs, ok ? woff[0] : kPipeOOB); woff[0] += 2u * FK; } }
    else { r.w[piece - 1] = pipe_load(wrs, ok ? woff[piece - 1] : kPipeOOB); woff[piece - 1] += 4u * FK; }
    if (piece == 2) cnext += FK;
  };
  auto store_piece = [&](float* st, const Regs& r, int piece) {   // 0-1: x halves, 2-3: w rows
    if (piece < 2) {
      if (!xst) return;
      float* xs = st + (4 * xq + 2 * piece) * FKP + xc;
      xs[0] = piece == 0 ? r.x.x : r.x.z;
      xs[FKP] = piece == 0 ? r.x.y : r.x.w;
    } else if (WH) {   // the bf16 w tile: [col][k] rows of kHWP halves
      if (piece == 2 && tid < 4 * FC)
        *reinterpret_cast<float4*>(reinterpret_cast<__bf16*>(st + XT) + (tid >> 2) * kHWP + (tid & 3) * 8) = r.w[0];
    } else {
      const int e = tid + (piece - 2) * NT;
      *reinterpret_cast<float4*>(st + XT + (e >> 3) * FKP + (e & 7) * 4) = r.w[piece - 2];
    }
  };

  floatx16 acc;
#pragma unroll
  for (int r = 0; r < 16; ++r) acc[r] = 0.f;
  const int nk = C / FK;   // even (C in {128, 256})
  const int arow = (pt * 32 + li) * FKP + lh * 8, brow = XT + (pc * 32 + li) * FKP + lh * 8;
  const int bhrow = (pc * 32 + li) * kHWP + lh * 8;   // WH: in halves from the w tile's start
  auto hfrag = [&](const float* stage, int k) {
    return *reinterpret_cast<const bf16x8*>(reinterpret_cast<const __bf16*>(stage + XT) + bhrow + k);
  };
  float fa0[8], fb0[8];
  bf16x8 hb0;
  for (int pc2 = 0; pc2 < 3; ++pc2) load_piece(rg[0], pc2);   // tile 0
  for (int pc2 = 0; pc2 < 3; ++pc2) load_piece(rg[1], pc2);   // tile 1
  for (int pc2 = 0; pc2 < 4; ++pc2) store_piece(lds, rg[0], pc2);
  for (int pc2 = 0; pc2 < 3; ++pc2) load_piece(rg[0], pc2);   // tile 2
  __syncthreads();
  pipe_frag(lds + arow, fa0);
  if constexpr (WH) hb0 = hfrag(lds, 0);
  else pipe_frag(lds + brow, fb0);
  // step i: tile i in stage i & 1; stores tile i + 1 from set (i + 1) & 1, then loads tile
  // i + 3 into that set (tiles past nk read channels past C: harmless, never stored as used)
  auto step = [&](auto par, int i) {
    constexpr int Q = (decltype(par)::value + 1) & 1;
    float* const cur = lds + (i & 1) * STG;
    float* const nxt = lds + ((i + 1) & 1) * STG;
    if constexpr (BF16) {
      // pipe_step's LDS protocol with one bf16 MFMA per half: tile i's second-half fragments,
      // the first half's MFMA, tile i + 1's stores and tile i + 3's loads, the barrier, the second
      // half's MFMA, tile i + 1's first-half fragments
      float fa1[8], fb1[8];
      bf16x8 hb1;
      pipe_frag(cur + arow + 16, fa1);
      if constexpr (WH) hb1 = hfrag(cur, 16);
      else pipe_frag(cur + brow + 16, fb1);
      acc = __builtin_amdgcn_mfma_f32_32x32x16_bf16(attn_pack8(fa0), WH ? hb0 : attn_pack8(fb0), acc, 0, 0, 0);
#pragma unroll
      for (int s = 0; s < 4; ++s) store_piece(nxt, rg[Q], s);
#pragma unroll
      for (int s = 0; s < 3; ++s) load_piece(rg[Q], s);
      __builtin_amdgcn_s_waitcnt(0xC07F);   // lgkmcnt(0)
      __builtin_amdgcn_s_barrier();
      acc = __builtin_amdgcn_mfma_f32_32x32x16_bf16(attn_pack8(fa1), WH ? hb1 : attn_pack8(fb1), acc, 0, 0, 0);
      pipe_frag(nxt + arow, fa0);
      if constexpr (WH) hb0 = hfrag(nxt, 0);
      else pipe_frag(nxt + brow, fb0);
    } else {
      pipe_step(acc, fa0, fb0, cur + arow, cur + brow, nxt + arow, nxt + brow, [&](int s) {
        if (s < 4) store_piece(nxt, rg[Q], s);
        else if (s < 7) load_piece(rg[Q], s - 4);
      });
    }
  };
  for (int kt = 0; kt < nk; kt += 2) {
    step(std::integral_constant<int, 0>(), kt);
    step(std::integral_constant<int, 1>(), kt + 1);
  }
  __syncthreads();   // the stages are overlaid by Q^T / K^T / V below

  // projection outputs (+ bias) to LDS: acc[r] = P[t][col], t = 32 pt + (r&3) + 8 (r>>2) + 4 lh,
  // col = 32 pc + li.  Q^T / K^T rows t (zero past Cq), V chunk rows c (zero past T)
  {
    const int col = pc * 32 + li;
    float bias;
    if (col < 64) {
      const int cq = col & 31;
      bias = cq < Cq ? bqkv[(col < 32 ? 0 : Cq) + cq] : 0.f;
    } else {
      bias = bqkv[2 * Cq + c0 + col - 64];
    }
#pragma unroll
    for (int r = 0; r < 16; ++r) {
      const int t = pt * 32 + (r & 3) + 8 * (r >> 2) + 4 * lh;
      if (col < 64) {
        const int cq = col & 31;
        (col < 32 ? qs : ks)[t * QP + cq] = cq < Cq ? acc[r] + bias : 0.f;
      } else {
        vs[(col - 64) * AP + t] = t < T ? acc[r] + bias : 0.f;
      }
    }
  }
  __syncthreads();

  // waves 4.. (PV + epilogue) fetch their x / residual values now, while waves 0-3 run the
  // score product and the softmax, instead of after their PV MFMAs
  float xv[16], rv[16];
  if (wave >= 4 && wc * 32 + li < T) {
#pragma unroll
    for (int r = 0; r < 16; ++r) {
      const int c = c0 + wt * 32 + (r & 3) + 8 * (r >> 2) + 4 * lh;
      const int64_t o = (int64_t)b * x_bs + (int64_t)c * T + wc * 32 + li;
      xv[r] = x[o];
      rv[r] = res ? res[o] : 0.f;
    }
  }

  // S[i][j] = sum_c' Q^T[i][c'] K^T[j][c']: waves 0-3, wave (wt, wc) owns the 32 x 32 tile
  floatx16 sacc;
#pragma unroll
  for (int r = 0; r < 16; ++r) sacc[r] = 0.f;
  if (wave < 4) {
    const int ia = wt * 32 + li, jb = wc * 32 + li;
#pragma unroll
    for (int kc = 0; kc < 32; kc += 16) {
      const float4 a0 = *reinterpret_cast<const float4*>(qs + ia * QP + kc + lh * 8);
      const float4 a1 = *reinterpret_cast<const float4*>(qs + ia * QP + kc + lh * 8 + 4);
      const float4 b0 = *reinterpret_cast<const float4*>(ks + jb * QP + kc + lh * 8);
      const float4 b1 = *reinterpret_cast<const float4*>(ks + jb * QP + kc + lh * 8 + 4);
      const float af[8] = {a0.x, a0.y, a0.z, a0.w, a1.x, a1.y, a1.z, a1.w};
      const float bf[8] = {b0.x, b0.y, b0.z, b0.w, b1.x, b1.y, b1.z, b1.w};
#pragma unroll
      for (int s = 0; s < 8; ++s) sacc = __builtin_amdgcn_mfma_f32_32x32x2f32(af[s], bf[s], sacc, 0, 0, 0);
    }
  }
  if (wave < 4) {
#pragma unroll
    for (int r = 0; r < 16; ++r) {
      const int i = wt * 32 + (r & 3) + 8 * (r >> 2) + 4 * lh;
      ss[i * AP + wc * 32 + li] = sacc[r];
    }
  }
  __syncthreads();

  if (tid < 256) {  // row softmax over j < T: four lanes per row, quad reductions in DPP
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
  }
  __syncthreads();

  // out[c][i] = sum_j V[c][j] A[i][j]: waves 4.., wave (wt, wc) owns channels 32 wt.., queries 32 wc..
  if (wave < 4) return;
#pragma unroll
  for (int r = 0; r < 16; ++r) sacc[r] = 0.f;
  {
    const int ca = wt * 32 + li, ib = wc * 32 + li;
    for (int kc = 0; kc < AT; kc += 16) {
      if (kc >= T) break;
      const float4 a0 = *reinterpret_cast<const float4*>(vs + ca * AP + kc + lh * 8);
      const float4 a1 = *reinterpret_cast<const float4*>(vs + ca * AP + kc + lh * 8 + 4);
      const float4 b0 = *reinterpret_cast<const float4*>(ss + ib * AP + kc + lh * 8);
      const float4 b1 = *reinterpret_cast<const float4*>(ss + ib * AP + kc + lh * 8 + 4);
      const float af[8] = {a0.x, a0.y, a0.z, a0.w, a1.x, a1.y, a1.z, a1.w};
      const float bf[8] = {b0.x, b0.y, b0.z, b0.w, b1.x, b1.y, b1.z, b1.w};
#pragma unroll
      for (int s = 0; s < 8; ++s) sacc = __builtin_amdgcn_mfma_f32_32x32x2f32(af[s], bf[s], sacc, 0, 0, 0);
    }
  }
  const float g = gamma[0];
  const int i = wc * 32 + li;
  if (i < T) {
#pragma unroll
    for (int r = 0; r < 16; ++r) {
      const int c = c0 + wt * 32 + (r & 3) + 8 * (r >> 2) + 4 * lh;
      const int64_t o = (int64_t)b * x_bs + (int64_t)c * T + i;
      float val = g * sacc[r] + xv[r];
      if (res) val += rv[r];
      y[o] = val;
    }
  }
}

bool attn_fused_eval_fits(int C, int T) { return T <= AT && T % 4 == 0 && (C == 128 || C == 256); }

// ---------------------------------------------------------------------------------------
// Wide queries, short sequences: the UNet's SelfAttention(2048) at T = 16 / 32 (bottleneck and
// up_attention, model_layers.py:336-339) and the discriminator's at T = 4: C/8 = 256 query
// channels, T <= 32.  One workgroup per (clip, 256-channel chunk of V); the four waves split
// the score product's K = C/8 in quarters (32 MFMAs each) and sum the partial 32 x 32 tiles
// through LDS, one softmax, then each wave multiplies 64 V channels (fragments straight from
// L2 into registers, issued first) by the attention tile.  Replaces the score GEMM, the
// softmax launch and the PV GEMM of the general path (three tiny-batched launches).
// ---------------------------------------------------------------------------------------
constexpr int WT = 32;            // max T
constexpr int WQ = 256;           // max C/8
constexpr int WQP = WQ + 4;       // Q^T / K^T pitch
constexpr int WAP = WT + 4;       // attention-tile pitch
constexpr int WCH = 256;          // V channels per workgroup

__global__ __launch_bounds__(256, 2) void attn_core_wide_kernel(
    const float* __restrict__ qkv, int64_t qs_b, int C, int T, const float* __restrict__ gamma,
    const float* __restrict__ x, int64_t x_bs, const float* __restrict__ res,
    float* __restrict__ y, float* __restrict__ attn_out) {
  __shared__ __attribute__((aligned(16))) float qs[WT * WQP];   // Q^T [i][c'], later partials
  __shared__ __attribute__((aligned(16))) float ks[WT * WQP];   // K^T [j][c']
  __shared__ __attribute__((aligned(16))) float as[WT * WAP];   // attention [i][j]
  const int b = blockIdx.y, c0 = blockIdx.x * WCH;
  const int Cq = C / 8;
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int li = lane & 31, lh = lane >> 5;
  const float* q = qkv + (int64_t)b * qs_b;
  const float* k = q + (int64_t)Cq * T;
  const float* v = q + (int64_t)2 * Cq * T;

  // V fragments of this wave's 64 channels (two 32-row tiles), k = j = 16 kc + 8 lh + s
  float4 vf[2][2][2];
#pragma unroll
  for (int m = 0; m < 2; ++m) {
    const float* vr = v + (int64_t)(c0 + wave * 64 + m * 32 + li) * T;
#pragma unroll
    for (int kc = 0; kc < 2; ++kc) {
      const int j = kc * 16 + lh * 8;
      vf[m][kc][0] = j < T ? *reinterpret_cast<const float4*>(vr + j) : make_float4(0.f, 0.f, 0.f, 0.f);
      vf[m][kc][1] = j + 4 < T ? *reinterpret_cast<const float4*>(vr + j + 4) : make_float4(0.f, 0.f, 0.f, 0.f);
    }
  }
  // the epilogue's x (and residual) values, fetched now so their latency hides behind the
  // score / softmax phases instead of following the PV MFMAs
  float xv[2][16], rv[2][16];
  if (li < T) {
#pragma unroll
    for (int m = 0; m < 2; ++m)
#pragma unroll
      for (int r = 0; r < 16; ++r) {
        const int c = c0 + wave * 64 + m * 32 + (r & 3) + 8 * (r >> 2) + 4 * lh;
        const int64_t o = (int64_t)blockIdx.y * x_bs + (int64_t)c * T + li;
        xv[m][r] = x[o];
        rv[m][r] = res ? res[o] : 0.f;
      }
  }
  // Q^T, K^T into LDS (float4 along t, written transposed); rows t >= T are zero
  {
    const int nq = Cq * (T / 4);
    for (int e0 = 0; e0 < Cq * (WT / 4); e0 += 256 * 4) {
      float4 qv[4], kv[4];
#pragma unroll
      for (int u = 0; u < 4; ++u) {
        const int e = e0 + tid + u * 256;
        const int c = e / (T / 4), tq = e % (T / 4);
        const bool ok = e < nq;
        qv[u] = ok ? *reinterpret_cast<const float4*>(q + (int64_t)c * T + 4 * tq) : make_float4(0.f, 0.f, 0.f, 0.f);
        kv[u] = ok ? *reinterpret_cast<const float4*>(k + (int64_t)c * T + 4 * tq) : make_float4(0.f, 0.f, 0.f, 0.f);
      }
#pragma unroll
      for (int u = 0; u < 4; ++u) {
        const int e = e0 + tid + u * 256;
        if (e >= nq) continue;
        const int c = e / (T / 4), t = 4 * (e % (T / 4));
        qs[(t + 0) * WQP + c] = qv[u].x; qs[(t + 1) * WQP + c] = qv[u].y;
        qs[(t + 2) * WQP + c] = qv[u].z; qs[(t + 3) * WQP + c] = qv[u].w;
        ks[(t + 0) * WQP + c] = kv[u].x; ks[(t + 1) * WQP + c] = kv[u].y;
        ks[(t + 2) * WQP + c] = kv[u].z; ks[(t + 3) * WQP + c] = kv[u].w;
      }
    }
    for (int e = tid; e < (WT - T) * Cq; e += 256) {   // zero rows T..31
      const int t = T + e / Cq, c = e % Cq;
      qs[t * WQP + c] = 0.f;
      ks[t * WQP + c] = 0.f;
    }
  }
  __syncthreads();

  // partial scores over this wave's quarter of c': S_w[i][j], i = query row, j = key
  floatx16 acc;
#pragma unroll
  for (int r = 0; r < 16; ++r) acc[r] = 0.f;
  {
    const int cq4 = Cq / 4, cb = wave * cq4;
    for (int kc = 0; kc < cq4; kc += 16) {
      const float* qa = qs + li * WQP + cb + kc + lh * 8;
      const float* kb = ks + li * WQP + cb + kc + lh * 8;
      const float4 a0 = *reinterpret_cast<const float4*>(qa), a1 = *reinterpret_cast<const float4*>(qa + 4);
      const float4 b0 = *reinterpret_cast<const float4*>(kb), b1 = *reinterpret_cast<const float4*>(kb + 4);
      const float af[8] = {a0.x, a0.y, a0.z, a0.w, a1.x, a1.y, a1.z, a1.w};
      const float bf[8] = {b0.x, b0.y, b0.z, b0.w, b1.x, b1.y, b1.z, b1.w};
#pragma unroll
      for (int s = 0; s < 8; ++s) acc = __builtin_amdgcn_mfma_f32_32x32x2f32(af[s], bf[s], acc, 0, 0, 0);
    }
  }
  __syncthreads();   // every Q^T / K^T read done: the partials overlay qs
  float* part = qs;  // [wave][i][j], pitch WAP
#pragma unroll
  for (int r = 0; r < 16; ++r) {
    const int i = (r & 3) + 8 * (r >> 2) + 4 * lh;
    part[(wave * WT + i) * WAP + li] = acc[r];
  }
  __syncthreads();

  // softmax over j < T: 8 threads per row (4 columns each), the four partials summed in a
  // fixed order; rows / columns >= T are zero
  {
    const int i = tid >> 3, p8 = tid & 7;
    float e[4];
    float mx = -INFINITY;
#pragma unroll
    for (int u = 0; u < 4; ++u) {
      const int j = p8 * 4 + u;
      float sv = part[(0 * WT + i) * WAP + j] + part[(1 * WT + i) * WAP + j];
      sv += part[(2 * WT + i) * WAP + j];
      sv += part[(3 * WT + i) * WAP + j];
      e[u] = j < T ? sv : -INFINITY;
      mx = fmaxf(mx, e[u]);
    }
    mx = fmaxf(mx, dpp_f<DPP_XOR1>(mx));
    mx = fmaxf(mx, dpp_f<DPP_XOR2>(mx));
    mx = fmaxf(mx, __shfl_xor(mx, 4));
    float sum = 0.f;
#pragma unroll
    for (int u = 0; u < 4; ++u) {
      e[u] = p8 * 4 + u < T ? expf(e[u] - mx) : 0.f;
      sum += e[u];
    }
    sum += dpp_f<DPP_XOR1>(sum);
    sum += dpp_f<DPP_XOR2>(sum);
    sum += __shfl_xor(sum, 4);
    const float inv = 1.f / sum;
#pragma unroll
    for (int u = 0; u < 4; ++u) e[u] = i < T ? e[u] * inv : 0.f;
    *reinterpret_cast<float4*>(as + i * WAP + p8 * 4) = make_float4(e[0], e[1], e[2], e[3]);
    if (attn_out && blockIdx.x == 0 && i < T) {
      float* ar = attn_out + ((int64_t)b * T + i) * T;
#pragma unroll
      for (int u = 0; u < 4; ++u)
        if (p8 * 4 + u < T) ar[p8 * 4 + u] = e[u];
    }
  }
  __syncthreads();

  // out[c][i] = gamma * sum_j V[c][j] A[i][j] + x[c][i] (+ res): this wave's 64 channels
  const float g = gamma[0];
#pragma unroll
  for (int m = 0; m < 2; ++m) {
#pragma unroll
    for (int r = 0; r < 16; ++r) acc[r] = 0.f;
#pragma unroll
    for (int kc = 0; kc < 2; ++kc) {
      if (kc * 16 >= T) break;
      const float* ar = as + li * WAP + kc * 16 + lh * 8;
      const float4 b0 = *reinterpret_cast<const float4*>(ar), b1 = *reinterpret_cast<const float4*>(ar + 4);
      const float af[8] = {vf[m][kc][0].x, vf[m][kc][0].y, vf[m][kc][0].z, vf[m][kc][0].w,
                           vf[m][kc][1].x, vf[m][kc][1].y, vf[m][kc][1].z, vf[m][kc][1].w};
      const float bf[8] = {b0.x, b0.y, b0.z, b0.w, b1.x, b1.y, b1.z, b1.w};
#pragma unroll
      for (int s = 0; s < 8; ++s) acc = __builtin_amdgcn_mfma_f32_32x32x2f32(af[s], bf[s], acc, 0, 0, 0);
    }
    if (li < T) {
#pragma unroll
      for (int r = 0; r < 16; ++r) {
        const int c = c0 + wave * 64 + m * 32 + (r & 3) + 8 * (r >> 2) + 4 * lh;
        const int64_t o = (int64_t)b * x_bs + (int64_t)c * T + li;
        float val = g * acc[r] + xv[m][r];
        if (res) val += rv[m][r];
        y[o] = val;
      }
    }
  }
}

bool attn_core_wide_fits(int C, int T) {
  return T >= 4 && T <= WT && T % 4 == 0 && C % 8 == 0 && C % WCH == 0 && C / 8 <= WQ && (C / 8) % 64 == 0;
}

int attn_core_wide(const float* qkv, int64_t qs_b, int B, int C, int T, const float* gamma,
                   const float* x, int64_t x_bs, const float* res, float* y, float* attn_out,
                   hipStream_t st) {
  dim3 grid((unsigned)(C / WCH), (unsigned)B);
  hipLaunchKernelGGL(attn_core_wide_kernel, grid, dim3(256), 0, st, qkv, qs_b, C, T, gamma, x, x_bs,
                     res, y, attn_out);
  A2M_LAUNCH_CHECK();
  return A2M_OK;
}

template <int NV>
static void attn_fused_eval_launch(bool bf16, bool wh, dim3 grid, hipStream_t st, const float* x, int64_t x_bs,
                                   int C, int T, const float* wqkv, const float* bqkv, const float* gamma,
                                   const float* res, float* y, int B, int64_t x_gs, int64_t res_gs,
                                   int64_t y_gs, const __bf16* wqkv_h) {
  const dim3 blk(NV == 64 ? 512 : 768);
  if (bf16 && wh)
    hipLaunchKernelGGL((attn_fused_eval_kernel<true, NV, true>), grid, blk, 0, st, x, x_bs, C, T, wqkv, bqkv,
                       gamma, res, y, B, x_gs, res_gs, y_gs, wqkv_h);
  else if (bf16)
    hipLaunchKernelGGL((attn_fused_eval_kernel<true, NV>), grid, blk, 0, st, x, x_bs, C, T, wqkv, bqkv, gamma,
                       res, y, B, x_gs, res_gs, y_gs, wqkv_h);
  else
    hipLaunchKernelGGL((attn_fused_eval_kernel<false, NV>), grid, blk, 0, st, x, x_bs, C, T, wqkv, bqkv, gamma,
                       res, y, B, x_gs, res_gs, y_gs, wqkv_h);
}

int attn_fused_eval(const float* x, int64_t x_bs, int B, int C, int T, const float* wqkv,
                    const float* bqkv, const float* gamma, const float* res, float* y,
                    hipStream_t st, int G, int64_t x_gs, int64_t res_gs, int64_t y_gs, const void* wqkv_h) {
  const bool bf16 = a2m_get_gemm_precision() == 1;
  // the bf16 copy counts when 16-byte aligned (rows of C halves are then 16-byte aligned too)
  const bool wh = wqkv_h != nullptr && (reinterpret_cast<uintptr_t>(wqkv_h) & 15) == 0;
  const __bf16* h = static_cast<const __bf16*>(wqkv_h);
  if (g_attn_nv == 128 && C % 128 == 0)
    attn_fused_eval_launch<128>(bf16, wh, dim3((unsigned)(C / 128), (unsigned)(B * G)), st, x, x_bs, C, T, wqkv,
                                bqkv, gamma, res, y, B, x_gs, res_gs, y_gs, h);
  else
    attn_fused_eval_launch<64>(bf16, wh, dim3((unsigned)cdiv(C, 64), (unsigned)(B * G)), st, x, x_bs, C, T, wqkv,
                               bqkv, gamma, res, y, B, x_gs, res_gs, y_gs, h);
  A2M_LAUNCH_CHECK();
  return A2M_OK;
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

extern "C" int a2m_set_attn_eval_chunk(int32_t nv) {
  if (nv != 64 && nv != 128) {
    a2m::set_error("set_attn_eval_chunk: %d (64 or 128)", (int)nv);
    return A2M_EINVAL;
  }
  a2m::g_attn_nv = nv;
  return A2M_OK;
}
