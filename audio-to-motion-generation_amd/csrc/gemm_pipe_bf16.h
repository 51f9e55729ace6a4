// Software-pipelined 64x64 tile of the implicit-GEMM engine in bf16 operand mode (precision 1,
// configs[4]): the fp32 operands are rounded to bf16 (RNE) on their way into LDS and multiplied by
// v_mfma_f32_32x32x16_bf16 with fp32 accumulation over 64-k steps -- gemm_tile<64, 64, 64, 0, MB,
// 1>'s numerics (the same rounded operands, the same products in the same order: bitwise equal),
// on gemm_pipe.h's schedule.
//
// A 64-k step of a wave is only four 32-cycle MFMAs (32 x 32 outputs, four K16 chunks) against
// eight float4 loads, their bf16 packing and four to eight LDS stores per thread, so the bf16
// tile is held by its operand staging and its load latency, not by the matrix pipe: gemm_tile
// issued that work as one block ahead of the MFMAs and waited on each k-step's loads one step
// later.  Here, as in the fp32 pipelined tile,
//   * every operand load is a raw buffer load (out-of-range rows / k / channels read 0), so the
//     k-step has no branches;
//   * a k-step is explicit slices (sched_barrier): the next tile's stores behind the first two
//     MFMAs, the barrier, the next tile's first fragments behind the third MFMA, the loads of
//     the tile two steps ahead behind the fourth;
//   * two operand register sets: a tile is loaded two k-steps before it is stored.
// LDS: per operand two [64][72-half] stages (a 16-byte multiple pitch of 36 dwords, conflict-free
// ds_read_b128 fragments), 36 KB a block.
//
// B operand modes: 0 dense k-contiguous rows, 6 channels-last conv rows (Ci % 64 == 0), 3
// row-contiguous [B][C][T] / [K][R] operands (k-pair map: each thread packs the same row of two
// adjacent k into one 32-bit LDS store), 5 the tap-chunked conv1d / ConvTranspose phases with 1-3
// taps (64-channel chunks loaded once, stored once per tap, shifted).  A is dense rows (mode 0).
#pragma once
#include "gemm_pipe.h"

namespace a2m {

// Diagnostic builds only: A2M_PIPE_HALF_A = 1 skips half of the A (weight) loads (results
// wrong; times what a bf16 weight copy would save)
#ifndef A2M_PIPE_HALF_A
#define A2M_PIPE_HALF_A 0
#endif

// operand register sets of the dense / channels-last / row-contiguous loops: a tile is loaded
// A2M_PIPE_H_DEPTH k-steps before it is stored
#ifndef A2M_PIPE_H_DEPTH
#define A2M_PIPE_H_DEPTH 2
#endif

constexpr int kHK = 72;                 // [row][k] pitch of a 64-k bf16 stage, in halves
constexpr int kHStage = 64 * kHK / 2;   // one operand stage, in floats

__device__ __forceinline__ uint32_t hpack2(float a, float b) {
  typedef float f2 __attribute__((ext_vector_type(2)));
  typedef __bf16 h2 __attribute__((ext_vector_type(2)));
  const f2 v = {a, b};
  return __builtin_bit_cast(uint32_t, __builtin_convertvector(v, h2));
}
__device__ __forceinline__ bf16x8 hld(const __bf16* p) { return *reinterpret_cast<const bf16x8*>(p); }
__device__ __forceinline__ void hmfma(floatx16& acc, const bf16x8& a, const bf16x8& b) {
  if (A2M_PIPE_ABL == 3) acc[0] += (float)a[0] * (float)b[0];
  else acc = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a, b, acc, 0, 0, 0);
}

template <int S>
using HS = std::integral_constant<int, S>;

// k-contiguous rows (mode 0): 64 rows x 64 k, four float4 per thread (rows tid / 16 + 16 p at k
// offset 4 (tid % 16)), stored as one ds_write_b64 of four bf16 each
struct PipeRowsH {
  static constexpr int NST = 4;   // store items per tile
  __amdgpu_buffer_rsrc_t rs;
  uint32_t off[4];
  int kq, lrow, knext, K;
  __device__ __forceinline__ void init(const Gather& g, int z, int row0, int R, int KK, int tid, int kbeg) {
    rs = pipe_rsrc(g.base + (int64_t)z * g.bstride);
    kq = (tid & 15) * 4;
    lrow = tid >> 4;
    K = KK;
    knext = kbeg;
#pragma unroll
    for (int p = 0; p < 4; ++p) {
      const int row = row0 + lrow + 16 * p;
      off[p] = row < R ? (uint32_t)(row * g.sr0 + kbeg + kq) * 4u : kPipeOOB;
    }
  }
  __device__ __forceinline__ void load(float4 (&r)[4], int p) {
    r[p] = pipe_load(rs, knext + kq < K ? off[p] : kPipeOOB);
    off[p] += 4u * 64;
    if (p == 3) knext += 64;
  }
  __device__ __forceinline__ void store(float* st, const float4 (&r)[4], int s) const {
    *reinterpret_cast<uint2*>(reinterpret_cast<__bf16*>(st) + (lrow + 16 * s) * kHK + kq) =
        make_uint2(hpack2(r[s].x, r[s].y), hpack2(r[s].z, r[s].w));
  }
};

// k-contiguous runs (mode 4, the 1-D conv weight gradients; PipeRuns' addressing and per-lane run
// position with 64-k tiles, K2 % 4 == 0): PipeRowsH's map, a quad across a run's edge loaded
// element by element (S = 2: stride-2 runs, as PipeRuns<2>)
template <int S = 1>
struct PipeRunsH {
  static constexpr int NST = 4;
  __amdgpu_buffer_rsrc_t rs;
  int rbase[4], w0[4];
  bool rv[4];
  int kq, lrow, knext, K, k0, k2, K2, sk0, Lw;
  __device__ __forceinline__ void init(const Gather& g, int z, int row0, int R, int KK, int tid, int kbeg) {
    rs = pipe_rsrc(g.base + (int64_t)z * g.bstride);
    kq = (tid & 15) * 4;
    lrow = tid >> 4;
    K = KK;
    knext = kbeg;
    K2 = g.K2; sk0 = g.sk0; Lw = g.Lw;
    k0 = (kbeg + kq) / K2;
    k2 = kbeg + kq - k0 * K2;
#pragma unroll
    for (int p = 0; p < 4; ++p) {
      const RowInfo ri = row_info(g, row0 + lrow + 16 * p, R);
      rv[p] = ri.valid && ri.h >= 0 && ri.h < g.Lh;
      rbase[p] = ri.base + ri.h * g.sh + ri.w;
      w0[p] = ri.w;
    }
  }
  __device__ __forceinline__ void load(float4 (&r)[4], int p) {
    const int w = w0[p] + S * k2;
    const int e0 = rbase[p] + k0 * sk0 + S * k2;
    const bool inb = rv[p] && knext + kq < K;
    const bool full = inb && w >= 0 && w + 4 * S - 1 < Lw;
    if constexpr (S == 1) {
      r[p] = pipe_load(rs, full ? (uint32_t)e0 * 4u : kPipeOOB);
    } else {
      const float4 lo = pipe_load(rs, full ? (uint32_t)e0 * 4u : kPipeOOB);
      const float4 hi = pipe_load(rs, full ? (uint32_t)(e0 + 4) * 4u : kPipeOOB);
      r[p] = make_float4(lo.x, lo.z, hi.x, hi.z);
    }
    if (inb && !full) {
      float e[4];
#pragma unroll
      for (int j = 0; j < 4; ++j)
        e[j] = __builtin_bit_cast(float, __builtin_amdgcn_raw_buffer_load_b32(
                   rs, (unsigned)(w + S * j) < (unsigned)Lw ? (uint32_t)(e0 + S * j) * 4u : kPipeOOB, 0, 0));
      r[p] = make_float4(e[0], e[1], e[2], e[3]);
    }
    if (p == 3) {
      knext += 64;
      k2 += 64;
      while (k2 >= K2) { k2 -= K2; ++k0; }
    }
  }
  __device__ __forceinline__ void store(float* st, const float4 (&r)[4], int s) const {
    *reinterpret_cast<uint2*>(reinterpret_cast<__bf16*>(st) + (lrow + 16 * s) * kHK + kq) =
        make_uint2(hpack2(r[s].x, r[s].y), hpack2(r[s].z, r[s].w));
  }
};

// channels-last conv rows (mode 6): a k-tile is 64 channels of one tap (i, j); each row reads its
// pixel (h + i, w + j) if it lies in the image
struct PipeNhwcH {
  static constexpr int NST = 4;
  __amdgpu_buffer_rsrc_t rs;
  int rbase[4], rh[4], rw[4];
  bool rv[4];
  int kq, lrow;
  int i6, j6, c6;   // tap and channel offset of the next load's k-tile (uniform)
  int Ci, K2, Lh, Lw;
  __device__ __forceinline__ void init(const Gather& g, int z, int row0, int R, int KK, int tid, int kbeg) {
    (void)KK;
    rs = pipe_rsrc(g.base + (int64_t)z * g.bstride);
    kq = (tid & 15) * 4;
    lrow = tid >> 4;
    Ci = g.nhwc; K2 = g.K2; Lh = g.Lh; Lw = g.Lw;
#pragma unroll
    for (int p = 0; p < 4; ++p) {
      const RowInfo ri = row_info(g, row0 + lrow + 16 * p, R);
      rbase[p] = ri.base + (ri.h * g.Lw + ri.w) * Ci + kq;
      rh[p] = ri.h;
      rw[p] = ri.w;
      rv[p] = ri.valid;
    }
    const int tap = kbeg / Ci;
    c6 = kbeg - tap * Ci;
    i6 = tap / K2;
    j6 = tap - i6 * K2;
  }
  __device__ __forceinline__ void load(float4 (&r)[4], int p) {
    const int h = rh[p] + i6, w = rw[p] + j6;
    const bool ok = rv[p] && (unsigned)h < (unsigned)Lh && (unsigned)w < (unsigned)Lw;
    r[p] = pipe_load(rs, ok ? (uint32_t)(rbase[p] + (i6 * Lw + j6) * Ci + c6) * 4u : kPipeOOB);
    if (p == 3) {
      c6 += 64;
      if (c6 == Ci) {
        c6 = 0;
        if (++j6 == K2) { j6 = 0; ++i6; }
      }
    }
  }
  __device__ __forceinline__ void store(float* st, const float4 (&r)[4], int s) const {
    *reinterpret_cast<uint2*>(reinterpret_cast<__bf16*>(st) + (lrow + 16 * s) * kHK + kq) =
        make_uint2(hpack2(r[s].x, r[s].y), hpack2(r[s].z, r[s].w));
  }
};

// row-contiguous operand (mode 3, plain case; element (n, k) at b * sr0 + t + k * sk0, n = b *
// R2 + t): thread (lrow / 4, kp) loads 4 consecutive rows of k = kp, kp + 1, kp + 32, kp + 33 as
// one float4 each and writes each row's k pair as one packed 32-bit store (the lanes of a wave
// cover 16 k pairs x 4 row groups: conflict-free)
struct PipeRowsTH {
  static constexpr int NST = 2;
  __amdgpu_buffer_rsrc_t rs;
  uint32_t off;     // byte offset of the thread's 4 rows at the next load's k = kp (kPipeOOB: invalid)
  int kp, lrow, knext, K, sk0;
  __device__ __forceinline__ void init(const Gather& g, int z, int row0, int R, int KK, int tid, int kbeg) {
    rs = pipe_rsrc(g.base + (int64_t)z * g.bstride);
    lrow = (tid >> 4) * 4;
    kp = (tid & 15) * 2;
    K = KK;
    knext = kbeg;
    sk0 = g.sk0;
    const int n = row0 + lrow;
    const int b = n / g.R2, t = n - b * g.R2;
    off = n < R ? (uint32_t)(b * g.sr0 + t + (kbeg + kp) * sk0) * 4u : kPipeOOB;
  }
  __device__ __forceinline__ void load(float4 (&r)[4], int p) {
    const int dk = (p & 1) + 32 * (p >> 1);
    r[p] = pipe_load(rs, knext + kp + dk < K ? off + 4u * dk * sk0 : kPipeOOB);
    if (p == 3) {
      knext += 64;
      off += 4u * 64 * sk0;
    }
  }
  // k pair kp + 32 s of the 4 rows
  __device__ __forceinline__ void store(float* st, const float4 (&r)[4], int s) const {
    uint32_t* w = reinterpret_cast<uint32_t*>(st);
    const int o = (lrow * kHK + kp + 32 * s) >> 1;
    w[o] = hpack2(r[2 * s].x, r[2 * s + 1].x);
    w[o + kHK / 2] = hpack2(r[2 * s].y, r[2 * s + 1].y);
    w[o + kHK] = hpack2(r[2 * s].z, r[2 * s + 1].z);
    w[o + 3 * kHK / 2] = hpack2(r[2 * s].w, r[2 * s + 1].w);
  }
};

// tap-chunked conv1d / ConvTranspose phase (mode 5, NT = 1-3 taps, any shift cw, clips of T <= 64
// rows that tile the 64 rows): per 64-channel chunk the x window is loaded once (k-pair map as
// PipeRowsTH) and stored for every tap j, shifted by j + cw rows within each clip; rows whose
// source leaves the clip receive 0 (gemm_tile's mode-5 map, PipeTap's)
template <int NT>
struct PipeTapH {
  static constexpr int NST = 2;
  __amdgpu_buffer_rsrc_t rs;
  uint32_t off;      // byte offset of x[b][next chunk * 64 + kp][t] (kPipeOOB: rows invalid)
  int kp, lrow, ch, Ci, sk0;
  int o5[NT][4];     // per tap: half offsets of the thread's 4 rows in a [64][72] stage
  int ok5;           // per tap and row: carries data (else 0 is stored)
  __device__ __forceinline__ void init(const Gather& g, int z, int row0, int R, int KK, int tid, int kbeg) {
    rs = pipe_rsrc(g.base + (int64_t)z * g.bstride);
    lrow = (tid >> 4) * 4;
    kp = (tid & 15) * 2;
    const int T = g.R2;
    const int n = row0 + lrow;
    const int b = n / T, tt = n - b * T;
    Ci = KK / NT;
    sk0 = g.sk0;
    ch = (kbeg / (64 * NT)) * 64 + kp;
    off = n < R ? (uint32_t)(b * g.sr0 + tt + ch * sk0) * 4u : kPipeOOB;
    ok5 = 0;
#pragma unroll
    for (int t = 0; t < NT; ++t)
#pragma unroll
      for (int e = 0; e < 4; ++e) {
        const int ts = tt + e;
        int td = ts - (t + g.cw);
        const bool ok = td >= 0 && td < T;
        td += td < 0 ? T : (td >= T ? -T : 0);
        o5[t][e] = (lrow + e + (td - ts)) * kHK + kp;
        ok5 |= (ok ? 1 : 0) << (t * 4 + e);
      }
  }
  __device__ __forceinline__ void load(float4 (&r)[4], int p) {
    const int dk = (p & 1) + 32 * (p >> 1);
    r[p] = pipe_load(rs, ch + dk < Ci ? off + 4u * dk * sk0 : kPipeOOB);
    if (p == 3) {
      ch += 64;
      off += 4u * 64 * sk0;
    }
  }
  // k pair kp + 32 s of the chunk's registers, shifted for tap TAP
  template <int TAP>
  __device__ __forceinline__ void store(float* st, const float4 (&r)[4], int s) const {
    uint32_t* w = reinterpret_cast<uint32_t*>(st);
    const float a[4] = {r[2 * s].x, r[2 * s].y, r[2 * s].z, r[2 * s].w};
    const float b[4] = {r[2 * s + 1].x, r[2 * s + 1].y, r[2 * s + 1].z, r[2 * s + 1].w};
#pragma unroll
    for (int e = 0; e < 4; ++e)
      w[(o5[TAP][e] + 32 * s) >> 1] = ((ok5 >> (TAP * 4 + e)) & 1) ? hpack2(a[e], b[e]) : 0u;
  }
};

// tap-chunked conv1d in the halo layout (mode 5, Gather::halo: 3 taps, pad 1, clips T >= 16 that
// tile the 64 rows; PipeHalo's bf16 twin): the chunk's 64-channel x window is loaded and stored
// ONCE (k-pair map), row n of the tile at halo row (n / T) (T + 2) + 1 + n % T of a chunk-parity
// stage whose rows before and after each clip are zero; tap j reads it shifted by j - 1 rows
struct PipeHaloH {
  static constexpr int HR = 64 + 2 * 4;   // halo stage rows (at most four clips)
  static constexpr int NST = 2;
  __amdgpu_buffer_rsrc_t rs;
  uint32_t off;      // byte offset of x[b][next chunk * 64 + kp][t] (kPipeOOB: rows invalid)
  int kp, lrow, ch, Ci, sk0;
  int h5[4];         // half offsets of the thread's 4 rows in a halo stage
  __device__ __forceinline__ void init(const Gather& g, int z, int row0, int R, int KK, int tid, int kbeg) {
    rs = pipe_rsrc(g.base + (int64_t)z * g.bstride);
    lrow = (tid >> 4) * 4;
    kp = (tid & 15) * 2;
    const int T = g.R2;
    const int n = row0 + lrow;
    const int b = n / T, tt = n - b * T;
    Ci = KK / 3;
    sk0 = g.sk0;
    ch = (kbeg / 192) * 64 + kp;
    off = n < R ? (uint32_t)(b * g.sr0 + tt + ch * sk0) * 4u : kPipeOOB;
#pragma unroll
    for (int e = 0; e < 4; ++e) {
      const int nn = lrow + e;
      h5[e] = ((nn / T) * (T + 2) + 1 + nn % T) * kHK + kp;
    }
  }
  __device__ __forceinline__ void load(float4 (&r)[4], int p) {
    const int dk = (p & 1) + 32 * (p >> 1);
    r[p] = pipe_load(rs, ch + dk < Ci ? off + 4u * dk * sk0 : kPipeOOB);
    if (p == 3) {
      ch += 64;
      off += 4u * 64 * sk0;
    }
  }
  // k pair kp + 32 s of the window's 4 rows
  __device__ __forceinline__ void store(float* st, const float4 (&r)[4], int s) const {
    uint32_t* w = reinterpret_cast<uint32_t*>(st);
    w[(h5[0] + 32 * s) >> 1] = hpack2(r[2 * s].x, r[2 * s + 1].x);
    w[(h5[1] + 32 * s) >> 1] = hpack2(r[2 * s].y, r[2 * s + 1].y);
    w[(h5[2] + 32 * s) >> 1] = hpack2(r[2 * s].z, r[2 * s + 1].z);
    w[(h5[3] + 32 * s) >> 1] = hpack2(r[2 * s].w, r[2 * s + 1].w);
  }
};

// One 64-k step.  ca / cb: this lane's fragment rows of tile i (A, B), na / nb: those of tile
// i + 1 (halves).  fa0 / fb0 hold tile i's K16 chunks 0-1 on entry and tile i + 1's on exit.
// work(HS<s>), s = 0..15: 0-7 behind the first two MFMAs (the stores of tile i + 1: they must
// land before the barrier), 8-15 behind the last (the loads of the tile two steps ahead).
template <class W>
__device__ __forceinline__ void pipe_step_h(floatx16& acc, bf16x8 (&fa0)[2], bf16x8 (&fb0)[2], const __bf16* ca,
                                            const __bf16* cb, const __bf16* na, const __bf16* nb, W&& work) {
  bf16x8 fa1[2], fb1[2];
  fa1[0] = hld(ca + 32); fa1[1] = hld(ca + 48);
  fb1[0] = hld(cb + 32); fb1[1] = hld(cb + 48);
  A2M_SB();
  hmfma(acc, fa0[0], fb0[0]);
  if (A2M_PIPE_ABL != 1) { work(HS<0>()); work(HS<1>()); work(HS<2>()); work(HS<3>()); }
  A2M_SB();
  hmfma(acc, fa0[1], fb0[1]);
  if (A2M_PIPE_ABL != 1) { work(HS<4>()); work(HS<5>()); work(HS<6>()); work(HS<7>()); }
  A2M_SB();
  // every wave's stores of tile i + 1 have landed, and no wave reads tile i's chunks 0-1 any more
  __builtin_amdgcn_s_waitcnt(0xC07F);   // lgkmcnt(0)
  if (A2M_PIPE_ABL != 2) __builtin_amdgcn_s_barrier();
  A2M_SB();
  hmfma(acc, fa1[0], fb1[0]);
  A2M_SB();
  fa0[0] = hld(na); fa0[1] = hld(na + 16);
  fb0[0] = hld(nb); fb0[1] = hld(nb + 16);
  A2M_SB();
  hmfma(acc, fa1[1], fb1[1]);
  if (A2M_PIPE_ABL != 1) {
    work(HS<8>()); work(HS<9>()); work(HS<10>()); work(HS<11>());
    work(HS<12>()); work(HS<13>()); work(HS<14>()); work(HS<15>());
  }
  A2M_SB();
}

template <int MB, int NT = 0, int MA = 0>   // MB 5: NT = taps (1-3); MA: A's mode (0, 3 or 4)
__global__ __launch_bounds__(256) void gemm_pipe_bf16_kernel(GemmArgs args) {
  span_begin(args.ts);
  constexpr int BM = 64;
  constexpr bool HALO = MB == 5 && NT == 0;
  constexpr bool TAPS = MB == 5 && NT > 0;
  constexpr int TBH = PipeHaloH::HR * kHK / 2;   // a halo B stage, in floats
  constexpr int TB = HALO ? TBH : kHStage;
  __shared__ __attribute__((aligned(16))) float lds[2 * kHStage + 2 * TB];   // A stages, then B stages
  __shared__ EpiRow epr[BM];
  const int tid = threadIdx.x;
  const int lane = tid & 63, wave = tid >> 6;
  const int wm = wave >> 1, wn = wave & 1;
  const int li = lane & 31, lh = lane >> 5;
  int bx, by, bz;
  pipe_block(args, bx, by, bz);
  const int zz = bz;
  const int batch = zz / args.splits, split = zz % args.splits;
  const int m0 = by * BM, n0 = bx * 64;
  const int kbeg = split * args.kchunk;
  const int kend = min(args.K, kbeg + args.kchunk);
  const int nk = __builtin_amdgcn_readfirstlane(kbeg < kend ? (kend - kbeg + 63) / 64 : 0);

  // MB 7: stride-2 runs (PipeRunsH<2>; gemm_tile's mode 1 for them)
  static_assert(MA == 0 || (MA == 3 && (MB == 0 || MB == 3)) || (MA == 4 && (MB == 4 || MB == 7)),
                "A in mode 3 with B in mode 0 / 3, in mode 4 with B in runs");
  using LA = typename std::conditional<MA == 4, PipeRunsH<1>, typename std::conditional<MA == 3, PipeRowsTH, PipeRowsH>::type>::type;
  LA la;
  la.init(args.A, batch, m0, args.M, args.K, tid, kbeg);
  using LB = typename std::conditional<
      MB == 5, typename std::conditional<TAPS, PipeTapH<NT ? NT : 1>, PipeHaloH>::type,
      typename std::conditional<MB == 6, PipeNhwcH,
                                typename std::conditional<MB == 3, PipeRowsTH,
                                                          typename std::conditional<MB == 4, PipeRunsH<1>,
                                                                                    typename std::conditional<MB == 7, PipeRunsH<2>, PipeRowsH>::type>::type>::type>::type>::type;
  LB lb;
  lb.init(args.B, batch, n0, args.N, args.K, tid, kbeg);

  float* const As = lds;
  float* const Bs = lds + 2 * kHStage;
  auto H = [](float* p) { return reinterpret_cast<const __bf16*>(p); };
  const int arow = (wm * 32 + li) * kHK + lh * 8;   // this lane's fragment rows (halves)
  const int brow = (wn * 32 + li) * kHK + lh * 8;
  floatx16 acc;
#pragma unroll
  for (int q = 0; q < 16; ++q) acc[q] = 0.f;
  bf16x8 fa0[2], fb0[2];
  float4 ra[2][4], rb[2][4];   // two operand register sets (tile t in set t & 1)
  using P0 = std::integral_constant<int, 0>;
  using P1 = std::integral_constant<int, 1>;
  auto epi_consts = [&]() {
    if (!args.partial && tid < BM && m0 + tid < args.M) epr[tid] = epi_row(args.E, m0 + tid + batch * args.E.pstride);
  };
  auto load4 = [](auto& l, float4 (&r)[4]) { l.load(r, 0); l.load(r, 1); l.load(r, 2); l.load(r, 3); };
  auto first_frags = [&]() {
    fa0[0] = hld(H(As) + arow); fa0[1] = hld(H(As) + arow + 16);
    fb0[0] = hld(H(Bs) + brow); fb0[1] = hld(H(Bs) + brow + 16);
  };

  if constexpr (TAPS) {
    // A in per-k-tile sets; B's registers hold a whole 64-channel chunk (two sets, by chunk
    // parity): step i stores tile i + 1 (A from set (i + 1) & 1, B tap (i + 1) % NT of chunk
    // (i + 1) / NT) and loads A tile i + 3, plus chunk (i + 3) / NT when tile i + 3 starts a chunk
    load4(la, ra[0]);
    load4(lb, rb[0]);                      // chunk 0 -> set 0
    epi_consts();
    load4(la, ra[1]);
    if (NT == 1) load4(lb, rb[1]);         // chunk 1 (tile 1)
#pragma unroll
    for (int s = 0; s < 4; ++s) la.store(As, ra[0], s);
    lb.template store<0>(Bs, rb[0], 0); lb.template store<0>(Bs, rb[0], 1);
    load4(la, ra[0]);                      // tile 2
    if (NT == 2) load4(lb, rb[1]);         // chunk 1 (tile 2)
    if (NT == 1) load4(lb, rb[0]);         // chunk 2 (tile 2)
    __syncthreads();
    first_frags();
    auto chunk = [&](auto par, int cc) {
      constexpr int P = decltype(par)::value;
      auto tap_step = [&](auto jj) {
        constexpr int J = decltype(jj)::value;
        constexpr int QA = ((NT % 2 ? P : 0) + J + 1) & 1;       // A set of tile i + 1 (= of tile i + 3)
        constexpr int TS = (J + 1) % NT;                          // tap of tile i + 1
        constexpr int QB = (P + (J + 1) / NT) & 1;                // B set of tile i + 1's chunk
        constexpr bool LB3 = (J + 3) % NT == 0;                   // tile i + 3 starts a chunk
        constexpr int QL = (P + (J + 3) / NT) & 1;                // its set
        const int i = NT * cc + J;
        const int c = (i & 1) * kHStage, n = kHStage - c;
        float* const nA = As + n;
        float* const nB = Bs + n;
        pipe_step_h(acc, fa0, fb0, H(As + c) + arow, H(Bs + c) + brow, H(nA) + arow, H(nB) + brow, [&](auto sc) {
          constexpr int s = decltype(sc)::value;
          if constexpr (s < 4) la.store(nA, ra[QA], s);
          else if constexpr (s < 6) lb.template store<TS>(nB, rb[QB], s - 4);
          else if constexpr (s >= 8 && s < 12) { if (!(A2M_PIPE_HALF_A && (s & 1))) la.load(ra[QA], s - 8); }
          else if constexpr (s >= 12) { if (LB3) lb.load(rb[QL], s - 12); }
        });
      };
      tap_step(std::integral_constant<int, 0>());
      if constexpr (NT > 1) tap_step(std::integral_constant<int, 1>());
      if constexpr (NT > 2) tap_step(std::integral_constant<int, 2>());
    };
    const int nch = nk / NT;
    int cc = 0;
    for (; cc + 1 < nch; cc += 2) {
      chunk(P0(), cc);
      chunk(P1(), cc + 1);
    }
    if (cc < nch) chunk(P0(), cc);
  } else if constexpr (HALO) {
    // A in k-tile parity stages, B in chunk parity stages (one per 3 k-tiles); the next chunk's
    // x window is loaded at the chunk's tap 0 and stored at its tap 2 (gemm_pipe.h's schedule)
    const int T = args.B.R2;
    for (int idx = tid; idx < 2 * (64 / T) * 2 * (kHK / 2); idx += 256) {   // zero rows around each clip
      const int col = idx % (kHK / 2), q = idx / (kHK / 2);
      const int which = q & 1, clip = (q >> 1) % (64 / T), stage = (q >> 1) / (64 / T);
      Bs[stage * TB + (clip * (T + 2) + (which ? T + 1 : 0)) * (kHK / 2) + col] = 0.f;
    }
    const int bsh = 2 * ((wn * 32 + li) / T) + 1;                   // halo rows above this lane's B row
    const int hrow = (wn * 32 + li + bsh) * kHK + lh * 8;           // tap 1 (shift 0), halves
    float4 rx[4];                                                   // a chunk's x window
    load4(la, ra[0]);
    load4(lb, rx);
    epi_consts();
    load4(la, ra[1]);
#pragma unroll
    for (int s = 0; s < 4; ++s) la.store(As, ra[0], s);
    lb.store(Bs, rx, 0); lb.store(Bs, rx, 1);
    load4(la, ra[0]);
    __syncthreads();
    fa0[0] = hld(H(As) + arow); fa0[1] = hld(H(As) + arow + 16);
    fb0[0] = hld(H(Bs) + hrow - kHK); fb0[1] = hld(H(Bs) + hrow - kHK + 16);   // tile 0 = tap 0
    const int nch = nk / 3;
    // chunk cc (parity P): tap j stores A(3 cc + j + 1) from set (P + j + 1) & 1 and loads
    // A(3 cc + j + 3) into it
    auto chunk = [&](auto par, int cc) {
      constexpr int P = decltype(par)::value;
      constexpr int Q0 = (P + 1) & 1, Q1 = P, Q2 = (P + 1) & 1;
      const int i0 = 3 * cc;
      float* const bc = Bs + (cc & 1) * TB;          // this chunk's B stage
      float* const bn = Bs + ((cc & 1) ^ 1) * TB;    // the next chunk's
      {   // tap 0 (+ the next chunk's x window loads)
        const int c = (i0 & 1) * kHStage, n = kHStage - c;
        float* const nA = As + n;
        pipe_step_h(acc, fa0, fb0, H(As + c) + arow, H(bc) + hrow - kHK, H(nA) + arow, H(bc) + hrow, [&](auto sc) {
          constexpr int s = decltype(sc)::value;
          if constexpr (s < 4) la.store(nA, ra[Q0], s);
          else if constexpr (s >= 8 && s < 12) la.load(ra[Q0], s - 8);
          else if constexpr (s >= 12) lb.load(rx, s - 12);
        });
      }
      {   // tap 1
        const int c = ((i0 + 1) & 1) * kHStage, n = kHStage - c;
        float* const nA = As + n;
        pipe_step_h(acc, fa0, fb0, H(As + c) + arow, H(bc) + hrow, H(nA) + arow, H(bc) + hrow + kHK, [&](auto sc) {
          constexpr int s = decltype(sc)::value;
          if constexpr (s < 4) la.store(nA, ra[Q1], s);
          else if constexpr (s >= 8 && s < 12) la.load(ra[Q1], s - 8);
        });
      }
      {   // tap 2 (+ the next chunk's x window stores)
        const int c = ((i0 + 2) & 1) * kHStage, n = kHStage - c;
        float* const nA = As + n;
        pipe_step_h(acc, fa0, fb0, H(As + c) + arow, H(bc) + hrow + kHK, H(nA) + arow, H(bn) + hrow - kHK, [&](auto sc) {
          constexpr int s = decltype(sc)::value;
          if constexpr (s < 4) la.store(nA, ra[Q2], s);
          else if constexpr (s < 6) lb.store(bn, rx, s - 4);
          else if constexpr (s >= 8 && s < 12) la.load(ra[Q2], s - 8);
        });
      }
    };
    int cc = 0;
    for (; cc + 1 < nch; cc += 2) {
      chunk(P0(), cc);
      chunk(P1(), cc + 1);
    }
    if (cc < nch) chunk(P0(), cc);
  } else {
    // D register sets, tile t in set t % D: step i stores tile i + 1 from set (i + 1) % D, then
    // loads tile i + 1 + D into it; the loop is unrolled by D so the set indices are static
    constexpr int D = A2M_PIPE_H_DEPTH;
    float4 xa[D][4], xb[D][4];
    load4(la, xa[0]);
    load4(lb, xb[0]);
    epi_consts();
#pragma unroll
    for (int d = 1; d < D; ++d) { load4(la, xa[d]); load4(lb, xb[d]); }
#pragma unroll
    for (int s = 0; s < LA::NST; ++s) la.store(As, xa[0], s);
#pragma unroll
    for (int s = 0; s < LB::NST; ++s) lb.store(Bs, xb[0], s);
    load4(la, xa[0]);
    load4(lb, xb[0]);
    __syncthreads();
    first_frags();
    auto step = [&](auto par, int i) {
      constexpr int Q = (decltype(par)::value + 1) % D;
      const int c = (i & 1) * kHStage, n = kHStage - c;
      float* const nA = As + n;
      float* const nB = Bs + n;
      pipe_step_h(acc, fa0, fb0, H(As + c) + arow, H(Bs + c) + brow, H(nA) + arow, H(nB) + brow, [&](auto sc) {
        constexpr int s = decltype(sc)::value;
        if constexpr (s < 4) { if constexpr (s < LA::NST) la.store(nA, xa[Q], s); }
        else if constexpr (s < 4 + LB::NST) lb.store(nB, xb[Q], s - 4);
        else if constexpr (s >= 8 && s < 12) { if (!(A2M_PIPE_HALF_A && (s & 1))) la.load(xa[Q], s - 8); }
        else if constexpr (s >= 12) lb.load(xb[Q], s - 12);
      });
    };
    int i = 0;
    for (; i + D - 1 < nk; i += D) {
      step(HS<0>(), i);
      if constexpr (D > 1) step(HS<1>(), i + 1);
      if constexpr (D > 2) step(HS<2>(), i + 2);
      if constexpr (D > 3) step(HS<3>(), i + 3);
    }
    if (i < nk) step(HS<0>(), i);
    if constexpr (D > 2) { if (i + 1 < nk) step(HS<1>(), i + 1); }
    if constexpr (D > 3) { if (i + 2 < nk) step(HS<2>(), i + 2); }
  }
  __syncthreads();   // the epilogue reuses the stages
  floatx16 accs[1][1];
  accs[0][0] = acc;
  if (args.vec4) pipe_epilogue_vec4(args, acc, lds, epr, args.partial != nullptr, zz, batch, m0, n0, tid, wm, wn, li, lh);
  else tile_epilogue<64, 64, 1, 1>(args, accs, lds, epr, args.partial != nullptr, zz, batch, m0, n0, tid, wm, wn, li, lh);
  span_end(args.ts);
}

void launch_pipe_bf16(const GemmArgs& a, int ma, int mb, int batch, hipStream_t st);

}  // namespace a2m
