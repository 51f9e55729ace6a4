// Software-pipelined 64x64 fp32 tile of the implicit-GEMM engine (one wave per SIMD).
//
// gemm_tile's k loop issues a k-step's operand work (global loads, their LDS stores, address
// arithmetic, exec-masked bound checks) as one block in front of the step's 16 MFMAs.  A wave
// issues in order, so with one wave per SIMD -- every launch of at most 256 64x64 tiles, which
// is most of the decoders' and the encoder's -- that block and the MFMAs add up: without its
// MFMAs the decoder conv's k loop still took 14.2 of its 24.7 us (profiles/r02_gemm_ablation.txt).
// A v_mfma_f32_32x32x2_f32 occupies the matrix pipe for 64 cycles, during which the wave can
// issue other, independent instructions.  This kernel puts the operand work INTO those shadows:
//   * every operand load is a raw buffer load (out-of-range rows, k and padding taps get an
//     offset past the buffer and read 0), so the k-step body has no branches;
//   * a k-step is written as explicit slices -- one MFMA, then one piece of operand work --
//     separated by sched_barrier, so the scheduler cannot hoist the pieces back into a block.
// The LDS schedule is gemm_tile's (double-buffered [row][36] stages, one barrier per k-step
// after the first half's MFMAs, the next tile's first fragments read behind the second half's
// first MFMAs), so the MFMAs see the same operands in the same order: results are bitwise
// those of gemm_tile's one-group (KS = 1) tile.
//
// B operand modes: 0 dense k-contiguous rows, 3 row-contiguous [B][C][T] / [K][R] operands (the
// 1x1 projections), 6 channels-last conv rows (Gather::nhwc), 5 the tap-chunked conv1d in the
// halo layout (Gather::halo: 3 taps, pad 1, clips T >= 16 that tile the 64 rows), 4 k-contiguous
// runs (the 1-D conv weight gradients, with A in mode 4 too).  A is dense rows (mode 0; the packed
// conv weights), a plain [K][M] operand (mode 3, with B in mode 0 / 3: the weight gradients of the
// linears and graph layers) or mode 4.
#pragma once
#include "gemm_kernel.h"

// Diagnostic builds only (never the shipped library): A2M_PIPE_ABL = 1 drops the k loop's global
// loads, 2 its barriers, 3 its MFMAs (results wrong; what remains times the rest)
#ifndef A2M_PIPE_ABL
#define A2M_PIPE_ABL 0
#endif
// Diagnostic builds only: A2M_PIPE_STAMPS = 1 records per block the shader clock at kernel entry,
// after the prologue's barrier, after the k loop and after the epilogue, plus the constant-rate
// clock at entry and exit, into g_pipe_stamps (read by a2m_debug_pipe_stamps, gemm_f32_pipe.hip)
#ifndef A2M_PIPE_STAMPS
#define A2M_PIPE_STAMPS 0
#endif
#if A2M_PIPE_STAMPS
constexpr int kPipeStampBlocks = 4096;
extern __device__ unsigned long long g_pipe_stamps[kPipeStampBlocks * 6];
#define A2M_PSTAMP(i, v) do { if (threadIdx.x == 0) { const unsigned lin = blockIdx.x + gridDim.x * (blockIdx.y + gridDim.y * blockIdx.z); if (lin < kPipeStampBlocks) g_pipe_stamps[lin * 6 + (i)] = (v); } } while (0)
#else
#define A2M_PSTAMP(i, v) do { } while (0)
#endif

namespace a2m {

constexpr uint32_t kPipeOOB = 0x80000000u;   // a buffer offset past every operand: loads read 0

__device__ __forceinline__ __amdgpu_buffer_rsrc_t pipe_rsrc(const float* base) {
  // raw buffer, 2 GB range: the host keeps every valid element offset below 2^29 floats
  return __builtin_amdgcn_make_buffer_rsrc(const_cast<float*>(base), (short)0, 0x7FFFFFFF, 0x00020000);
}
__device__ __forceinline__ float4 pipe_load(__amdgpu_buffer_rsrc_t rs, uint32_t off) {
  return __builtin_bit_cast(float4, __builtin_amdgcn_raw_buffer_load_b128(rs, off, 0, 0));
}
__device__ __forceinline__ void pipe_mfma(floatx16& acc, float a, float b) {
  if (A2M_PIPE_ABL == 3) acc[0] += a * b;
  else acc = __builtin_amdgcn_mfma_f32_32x32x2f32(a, b, acc, 0, 0, 0);
}

constexpr int kPipeLDK = 36;   // [row][k] pitch of a 32-k stage (conflict-free ds_read_b128)

// k-contiguous rows (mode 0): a 64-row x 32-k tile, two float4 per thread (rows tid/8 and
// tid/8 + 32 at k offset 4 (tid % 8)), advanced one k-tile per load
struct PipeRows {
  __amdgpu_buffer_rsrc_t rs;
  uint32_t off[2];   // byte offsets of the thread's rows at the next load's k (kPipeOOB: row invalid)
  int kq, lrow, knext, K;
  __device__ __forceinline__ void init(const Gather& g, int z, int row0, int R, int KK, int tid, int kbeg) {
    rs = pipe_rsrc(g.base + (int64_t)z * g.bstride);
    kq = (tid & 7) * 4;
    lrow = tid >> 3;
    K = KK;
    knext = kbeg;
#pragma unroll
    for (int p = 0; p < 2; ++p) {
      const int row = row0 + lrow + 32 * p;
      off[p] = row < R ? (uint32_t)(row * g.sr0 + kbeg + kq) * 4u : kPipeOOB;
    }
  }
  __device__ __forceinline__ void load(float4 (&r)[2], int p) {
    r[p] = pipe_load(rs, knext + kq < K ? off[p] : kPipeOOB);
    off[p] += 4u * 32;
    if (p == 1) knext += 32;
  }
  __device__ __forceinline__ void store(float* st, const float4 (&r)[2], int p) const {
    *reinterpret_cast<float4*>(st + (lrow + 32 * p) * kPipeLDK + kq) = r[p];
  }
};

// k-contiguous runs (mode 4, the weight-gradient operands of the 1-D convs): element (r, k) at
// r0 * sr0 + h * sh + w + k0 * sk0 with k = k0 * K2 + k2, w = r2 * ar2 + cw + k2 (h = r1 * ar1 + ch,
// K1 = 1), zero where w falls outside [0, Lw) or h outside [0, Lh).  K2 % 4 == 0 (host), so a
// lane's quad of k lies in one run (each lane tracks its own run k0 and offset k2, the tile's 32 k
// may span several short runs); the quad is one float4 unless it crosses the row's edge (the
// padding taps), where it loads element by element.  Thread map and LDS layout of PipeRows, so
// the stages hold what gemm_tile's mode-4 loader stores.  S = 2: the runs of a stride-2 conv's input
// (w = r2 * ar2 + cw + 2 k2, gemm_tile's mode 1 for it): a quad's 4 elements from two float4 (their
// even elements) unless it reaches past the row, element by element there
template <int S = 1>
struct PipeRuns {
  __amdgpu_buffer_rsrc_t rs;
  int rbase[2], w0[2];   // element offset of the thread's rows at (k0, k2) = (0, 0); their w origin
  bool rv[2];
  int kq, lrow, knext, K, k0, k2, K2, sk0, Lw;   // k0 / k2: this lane's quad at the next load
  __device__ __forceinline__ void init(const Gather& g, int z, int row0, int R, int KK, int tid, int kbeg) {
    rs = pipe_rsrc(g.base + (int64_t)z * g.bstride);
    kq = (tid & 7) * 4;
    lrow = tid >> 3;
    K = KK;
    knext = kbeg;
    K2 = g.K2; sk0 = g.sk0; Lw = g.Lw;
    k0 = (kbeg + kq) / K2;
    k2 = kbeg + kq - k0 * K2;
#pragma unroll
    for (int p = 0; p < 2; ++p) {
      const RowInfo ri = row_info(g, row0 + lrow + 32 * p, R);
      rv[p] = ri.valid && ri.h >= 0 && ri.h < g.Lh;
      rbase[p] = ri.base + ri.h * g.sh + ri.w;
      w0[p] = ri.w;
    }
  }
  __device__ __forceinline__ void load(float4 (&r)[2], int p) {
    const int w = w0[p] + S * k2;                   // the quad's first element along the run
    const int e0 = rbase[p] + k0 * sk0 + S * k2;    // its element offset (>= 0 where w >= 0)
    const bool inb = rv[p] && knext + kq < K;
    const bool full = inb && w >= 0 && w + 4 * S - 1 < Lw;
    if constexpr (S == 1) {
      r[p] = pipe_load(rs, full ? (uint32_t)e0 * 4u : kPipeOOB);
    } else {
      const float4 lo = pipe_load(rs, full ? (uint32_t)e0 * 4u : kPipeOOB);
      const float4 hi = pipe_load(rs, full ? (uint32_t)(e0 + 4) * 4u : kPipeOOB);
      r[p] = make_float4(lo.x, lo.z, hi.x, hi.z);
    }
    if (inb && !full) {   // a quad across the row's edge: the elements inside it, the rest 0
      float e[4];
#pragma unroll
      for (int j = 0; j < 4; ++j)
        e[j] = __builtin_bit_cast(float, __builtin_amdgcn_raw_buffer_load_b32(
                   rs, (unsigned)(w + S * j) < (unsigned)Lw ? (uint32_t)(e0 + S * j) * 4u : kPipeOOB, 0, 0));
      r[p] = make_float4(e[0], e[1], e[2], e[3]);
    }
    if (p == 1) {
      knext += 32;
      k2 += 32;
      while (k2 >= K2) { k2 -= K2; ++k0; }
    }
  }
  __device__ __forceinline__ void store(float* st, const float4 (&r)[2], int p) const {
    *reinterpret_cast<float4*>(st + (lrow + 32 * p) * kPipeLDK + kq) = r[p];
  }
};

// channels-last conv rows (mode 6): a k-tile is 32 channels of one tap (i, j); each row reads its
// pixel (h + i, w + j) if it lies in the image
struct PipeNhwc {
  __amdgpu_buffer_rsrc_t rs;
  int rbase[2], rh[2], rw[2];
  bool rv[2];
  int kq, lrow;
  int i6, j6, c6;   // tap and channel offset of the next load's k-tile (uniform)
  int Ci, K2, Lh, Lw;
  __device__ __forceinline__ void init(const Gather& g, int z, int row0, int R, int KK, int tid, int kbeg) {
    (void)KK;
    rs = pipe_rsrc(g.base + (int64_t)z * g.bstride);
    kq = (tid & 7) * 4;
    lrow = tid >> 3;
    Ci = g.nhwc; K2 = g.K2; Lh = g.Lh; Lw = g.Lw;
#pragma unroll
    for (int p = 0; p < 2; ++p) {
      const RowInfo ri = row_info(g, row0 + lrow + 32 * p, R);
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
  __device__ __forceinline__ void load(float4 (&r)[2], int p) {
    const int h = rh[p] + i6, w = rw[p] + j6;
    const bool ok = rv[p] && (unsigned)h < (unsigned)Lh && (unsigned)w < (unsigned)Lw;
    r[p] = pipe_load(rs, ok ? (uint32_t)(rbase[p] + (i6 * Lw + j6) * Ci + c6) * 4u : kPipeOOB);
    if (p == 1) {
      c6 += 32;
      if (c6 == Ci) {
        c6 = 0;
        if (++j6 == K2) { j6 = 0; ++i6; }
      }
    }
  }
  __device__ __forceinline__ void store(float* st, const float4 (&r)[2], int p) const {
    *reinterpret_cast<float4*>(st + (lrow + 32 * p) * kPipeLDK + kq) = r[p];
  }
};

// row-contiguous operand (mode 3, plain case): element (n, k) at b * sr0 + t + k * sk0 with
// n = b * R2 + t -- a [K][R] matrix (R2 = 1, sr0 = 1) or a [B][C][T] activation read as rows
// (b, t) and k = c (the 1x1 convs / projections).  Thread (lrow / 4, kq) loads 4 consecutive rows
// of k = kq and kq + 16 as one float4 each and writes them transposed into the [row][36] stage
// (gemm_tile's mode-3 map)
struct PipeRowsT {
  __amdgpu_buffer_rsrc_t rs;
  uint32_t off;     // byte offset of the thread's 4 rows at the next load's k = kq (kPipeOOB: invalid)
  int kq, lrow, knext, K, sk0;
  __device__ __forceinline__ void init(const Gather& g, int z, int row0, int R, int KK, int tid, int kbeg) {
    rs = pipe_rsrc(g.base + (int64_t)z * g.bstride);
    lrow = (tid >> 4) * 4;
    kq = tid & 15;
    K = KK;
    knext = kbeg;
    sk0 = g.sk0;
    const int n = row0 + lrow;
    const int b = n / g.R2, t = n - b * g.R2;
    off = n < R ? (uint32_t)(b * g.sr0 + t + (kbeg + kq) * sk0) * 4u : kPipeOOB;
  }
  __device__ __forceinline__ void load(float4 (&r)[2], int p) {
    r[p] = pipe_load(rs, knext + kq + 16 * p < K ? off + 4u * 16 * sk0 * p : kPipeOOB);
    if (p == 1) {
      knext += 32;
      off += 4u * 32 * sk0;
    }
  }
  __device__ __forceinline__ void store(float* st, const float4 (&r)[2], int p) const {
    float* q = st + lrow * kPipeLDK + kq + 16 * p;
    q[0] = r[p].x;
    q[kPipeLDK] = r[p].y;
    q[2 * kPipeLDK] = r[p].z;
    q[3 * kPipeLDK] = r[p].w;
  }
};

// tap-chunked conv1d, halo layout (mode 5, Gather::halo): per 32-channel chunk the x window
// x[b][c][t] of the tile's 64 rows (whole clips of T >= 16) is loaded once -- thread (lrow / 4,
// kq) reads 4 consecutive t of channels kq and kq + 16 -- and stored once, row n of the tile at
// halo row (n / T) (T + 2) + 1 + n % T of a chunk-parity stage whose rows before and after each
// clip are zero; tap j then reads the stage shifted by j - 1 rows
struct PipeHalo {
  static constexpr int HR = 64 + 2 * 4;   // halo stage rows (at most four clips)
  __amdgpu_buffer_rsrc_t rs;
  uint32_t off;      // byte offset of x[b][next chunk * 32 + kq][t] (kPipeOOB: rows invalid)
  int kq, lrow, ch, Ci, sk0;
  int h5[4];         // LDS offsets of the thread's 4 rows in a halo stage
  __device__ __forceinline__ void init(const Gather& g, int z, int row0, int R, int KK, int tid, int kbeg) {
    rs = pipe_rsrc(g.base + (int64_t)z * g.bstride);
    lrow = (tid >> 4) * 4;
    kq = tid & 15;
    const int T = g.R2;
    const int n = row0 + lrow;
    const int b = n / T, tt = n - b * T;
    Ci = KK / 3;
    sk0 = g.sk0;
    ch = (kbeg / 96) * 32 + kq;
    off = n < R ? (uint32_t)(b * g.sr0 + tt + ch * sk0) * 4u : kPipeOOB;
#pragma unroll
    for (int e = 0; e < 4; ++e) {
      const int nn = lrow + e;
      h5[e] = ((nn / T) * (T + 2) + 1 + nn % T) * kPipeLDK + kq;
    }
  }
  __device__ __forceinline__ void load(float4 (&r)[2], int p) {
    r[p] = pipe_load(rs, ch + 16 * p < Ci ? off + 4u * 16 * sk0 * p : kPipeOOB);
    if (p == 1) {
      ch += 32;
      off += 4u * 32 * sk0;
    }
  }
  // half p of the chunk's registers: channel kq + 16 p of the 4 rows
  __device__ __forceinline__ void store(float* st, const float4 (&r)[2], int p) const {
    st[h5[0] + 16 * p] = r[p].x;
    st[h5[1] + 16 * p] = r[p].y;
    st[h5[2] + 16 * p] = r[p].z;
    st[h5[3] + 16 * p] = r[p].w;
  }
};

// tap-chunked conv1d / ConvTranspose phase, general layout (mode 5 without Gather::halo; NT =
// 1-3 taps, any shift cw, clips of T <= 64 rows that tile the 64 rows): per 32-channel chunk the
// x window is loaded once (as PipeHalo) and stored for every tap j, shifted by j + cw rows within
// each clip -- gemm_tile's mode-5 store: element e of the thread's 4-row group lands on the row
// whose source t + j + cw is its t, and the rows whose source leaves the clip receive 0 (written
// by the element that wraps onto them)
template <int NT>
struct PipeTap {
  __amdgpu_buffer_rsrc_t rs;
  uint32_t off;      // byte offset of x[b][next chunk * 32 + kq][t] (kPipeOOB: rows invalid)
  int kq, lrow, ch, Ci, sk0;
  int o5[NT][4];     // per tap: LDS offsets of the thread's 4 elements in a [64][36] stage
  int ok5;           // per tap and element: carries data (else 0 is stored)
  __device__ __forceinline__ void init(const Gather& g, int z, int row0, int R, int KK, int tid, int kbeg) {
    rs = pipe_rsrc(g.base + (int64_t)z * g.bstride);
    lrow = (tid >> 4) * 4;
    kq = tid & 15;
    const int T = g.R2;
    const int n = row0 + lrow;
    const int b = n / T, tt = n - b * T;
    Ci = KK / NT;
    sk0 = g.sk0;
    ch = (kbeg / (32 * NT)) * 32 + kq;
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
        o5[t][e] = (lrow + e + (td - ts)) * kPipeLDK + kq;
        ok5 |= (ok ? 1 : 0) << (t * 4 + e);
      }
  }
  __device__ __forceinline__ void load(float4 (&r)[2], int p) {
    r[p] = pipe_load(rs, ch + 16 * p < Ci ? off + 4u * 16 * sk0 * p : kPipeOOB);
    if (p == 1) {
      ch += 32;
      off += 4u * 32 * sk0;
    }
  }
  // half p of the chunk's registers, shifted for tap `tap` (compile-time)
  template <int TAP>
  __device__ __forceinline__ void store(float* st, const float4 (&r)[2], int p) const {
    const float v[4] = {r[p].x, r[p].y, r[p].z, r[p].w};
#pragma unroll
    for (int e = 0; e < 4; ++e) st[o5[TAP][e] + 16 * p] = ((ok5 >> (TAP * 4 + e)) & 1) ? v[e] : 0.f;
  }
};

__device__ __forceinline__ void pipe_frag(const float* p, float (&f)[8]) {
  const float4 v0 = *reinterpret_cast<const float4*>(p);
  const float4 v1 = *reinterpret_cast<const float4*>(p + 4);
  f[0] = v0.x; f[1] = v0.y; f[2] = v0.z; f[3] = v0.w;
  f[4] = v1.x; f[5] = v1.y; f[6] = v1.z; f[7] = v1.w;
}

// Epilogue for outputs whose n index is contiguous in 16-byte groups (args.vec4): the 64 x 64
// accumulator tile goes to LDS as C[m][n] (pitch 68), then each thread finishes 4 float4 runs
// of one row: the row's epilogue constants once, the residual / accumulate operands as float4
// loads, one global_store_dwordx4 per 4 outputs (16 scalar stores per lane before: the
// epilogue's store issue was ~7k cycles, the largest fixed cost of a one-block-per-CU launch).
// Split-K slabs ([M][N] rows) take the same path.
__device__ __forceinline__ void pipe_epilogue_vec4(const GemmArgs& args, const floatx16& acc, float* lds,
                                                   const EpiRow* epr, bool slab, int zz, int batch, int m0,
                                                   int n0, int tid, int wm, int wn, int li, int lh) {
  constexpr int LDC = 68;
#pragma unroll
  for (int q = 0; q < 16; ++q)
    lds[(wm * 32 + (q & 3) + 8 * (q >> 2) + 4 * lh) * LDC + wn * 32 + li] = acc[q];
  __syncthreads();
  const Epilogue& E = args.E;
#pragma unroll
  for (int j = 0; j < 4; ++j) {
    const int idx = tid + 256 * j;
    const int ml = idx >> 4, nl = (idx & 15) * 4;
    const int m = m0 + ml, n = n0 + nl;
    if (m >= args.M || n >= args.N) continue;
    float4 v = *reinterpret_cast<const float4*>(lds + ml * LDC + nl);
    if (slab) {
      *reinterpret_cast<float4*>(args.partial + (int64_t)zz * args.M * args.N + (int64_t)m * args.N + n) = v;
      continue;
    }
    const EpiRow r = epr[ml];
    const int64_t off = (int64_t)batch * E.bstride + epi_addr(E, m, n);
    v.x = epi_value_p(E, v.x, r); v.y = epi_value_p(E, v.y, r);
    v.z = epi_value_p(E, v.z, r); v.w = epi_value_p(E, v.w, r);
    if (E.res1) {
      const float4 a = *reinterpret_cast<const float4*>(E.res1 + off);
      v.x += a.x; v.y += a.y; v.z += a.z; v.w += a.w;
    }
    if (E.res2) {
      const float4 a = *reinterpret_cast<const float4*>(E.res2 + off);
      v.x += a.x; v.y += a.y; v.z += a.z; v.w += a.w;
    }
    if (E.accumulate) {
      const float4 a = *reinterpret_cast<const float4*>(E.out + off);
      v.x += a.x; v.y += a.y; v.z += a.z; v.w += a.w;
    }
    *reinterpret_cast<float4*>(E.out + off) = v;
  }
}

#define A2M_SB() __builtin_amdgcn_sched_barrier(0)

// block -> (n-tile, m-tile, batch * split), XCD-grouped as in gemm_tile (block-uniform: SGPRs)
__device__ __forceinline__ void pipe_block(const GemmArgs& args, int& bx, int& by, int& bz) {
  bx = blockIdx.x; by = blockIdx.y; bz = blockIdx.z;
  if (args.xcd_group > 0) {
    const int gx = gridDim.x, gy = gridDim.y;
    const int total = gx * gy * gridDim.z;
    const int L = blockIdx.x + gx * (blockIdx.y + gy * blockIdx.z);
    const int q = total / 8, r = total % 8, x = L % 8;
    const int t = (x < r ? x * (q + 1) : r * (q + 1) + (x - r) * q) + L / 8;
    bz = t / (gx * gy);
    const int rem = t - bz * gx * gy;
    const int gm = args.xcd_group;
    const int group = rem / (gm * gx);
    const int first_m = group * gm;
    const int gsz = min(gy - first_m, gm);
    const int in = rem - group * gm * gx;
    by = first_m + in % gsz;
    bx = in / gsz;
  }
  bx = __builtin_amdgcn_readfirstlane(bx);
  by = __builtin_amdgcn_readfirstlane(by);
  bz = __builtin_amdgcn_readfirstlane(bz);
}

// One k-step.  ca / cb: this lane's fragment rows of tile i (A, B) at half 0 (the half-1
// fragments are 16 floats further); na / nb: those of tile i + 1.  f0 holds tile i's half-0
// fragments on entry and tile i + 1's on exit.  work(s), s = 0..7, is the operand work placed
// behind half-0 MFMA s (stores of tile i + 1 first, then loads of tile i + 2).
template <class W>
__device__ __forceinline__ void pipe_step(floatx16& acc, float (&fa0)[8], float (&fb0)[8], const float* ca,
                                          const float* cb, const float* na, const float* nb, W&& work) {
  float fa1[8], fb1[8];
  pipe_frag(ca + 16, fa1);
  pipe_frag(cb + 16, fb1);
  A2M_SB();
#pragma unroll
  for (int s = 0; s < 8; ++s) {
    pipe_mfma(acc, fa0[s], fb0[s]);
    if (A2M_PIPE_ABL != 1 || s < 4) work(s);
    A2M_SB();
  }
  // every wave's stores of tile i + 1 have landed (LDS ops retire in order, so after the
  // fragment reads issued before them), and no wave reads tile i's half 0 any more
  __builtin_amdgcn_s_waitcnt(0xC07F);   // lgkmcnt(0)
  if (A2M_PIPE_ABL != 2) __builtin_amdgcn_s_barrier();
  A2M_SB();
  pipe_mfma(acc, fa1[0], fb1[0]);
  pipe_mfma(acc, fa1[1], fb1[1]);
  A2M_SB();
  pipe_frag(na, fa0);
  pipe_frag(nb, fb0);
  A2M_SB();
#pragma unroll
  for (int s = 2; s < 8; ++s) pipe_mfma(acc, fa1[s], fb1[s]);
  A2M_SB();
}

template <int MB, int NT = 0, int MA = 0>   // NT > 0: mode 5 in the general (per-tap store) layout
__global__ __launch_bounds__(256) void gemm_pipe_kernel(GemmArgs args) {
  A2M_PSTAMP(4, __builtin_amdgcn_s_memrealtime());
  A2M_PSTAMP(0, __builtin_amdgcn_s_memtime());
  span_begin(args.ts);
  constexpr int BM = 64, BN = 64, BK = 32, LDK = kPipeLDK;
  constexpr bool HALO = MB == 5 && NT == 0;
  constexpr bool TAPS = MB == 5 && NT > 0;
  constexpr int TA = BM * LDK;
  constexpr int TB = (HALO ? PipeHalo::HR : BN) * LDK;
  __shared__ __attribute__((aligned(16))) float lds[2 * TA + 2 * TB];   // A stages, then B stages
  __shared__ EpiRow epr[BM];
  const int tid = threadIdx.x;
  const int lane = tid & 63, wave = tid >> 6;
  const int wm = wave >> 1, wn = wave & 1;
  const int li = lane & 31, lh = lane >> 5;

  int bx, by, bz;
  pipe_block(args, bx, by, bz);
  const int zz = bz;
  const int batch = zz / args.splits, split = zz % args.splits;
  const int m0 = by * BM, n0 = bx * BN;
  const int kbeg = split * args.kchunk;
  const int kend = min(args.K, kbeg + args.kchunk);
  const int nk = __builtin_amdgcn_readfirstlane(kbeg < kend ? (kend - kbeg + BK - 1) / BK : 0);

  // MB 7: stride-2 runs (PipeRuns<2>; gemm_tile's mode 1 for them)
  static_assert(MA == 0 || (MA == 3 && (MB == 0 || MB == 3)) || (MA == 4 && (MB == 4 || MB == 7)),
                "A in mode 3 with B in mode 0 / 3, in mode 4 with B in runs");
  typename std::conditional<MA == 4, PipeRuns<1>, typename std::conditional<MA == 3, PipeRowsT, PipeRows>::type>::type la;
  la.init(args.A, batch, m0, args.M, args.K, tid, kbeg);
  using LB = typename std::conditional<
      MB == 5, typename std::conditional<TAPS, PipeTap<NT ? NT : 1>, PipeHalo>::type,
      typename std::conditional<MB == 6, PipeNhwc,
                                typename std::conditional<MB == 3, PipeRowsT,
                                                          typename std::conditional<MB == 4, PipeRuns<1>,
                                                                                    typename std::conditional<MB == 7, PipeRuns<2>, PipeRows>::type>::type>::type>::type>::type;
  LB lb;
  lb.init(args.B, batch, n0, args.N, args.K, tid, kbeg);

  float* const As = lds;
  float* const Bs = lds + 2 * TA;
  const int arow = (wm * 32 + li) * LDK + lh * 8;   // this lane's fragment row offsets
  const int brow_i = wn * 32 + li;
  floatx16 acc;
#pragma unroll
  for (int q = 0; q < 16; ++q) acc[q] = 0.f;
  float fa0[8], fb0[8];
  // Operand registers, two sets: tile t is loaded two k-steps before it is stored (set t & 1;
  // the store of tile i + 1 at step i frees the set that the load of tile i + 3 then takes), so
  // every global load has about two k-steps (~2,000 cycles) to land.  The loop is unrolled by
  // two (by two channel chunks in the halo layout) so that the set indices are static.
  float4 ra[2][2], rb[2][2];
  using P0 = std::integral_constant<int, 0>;
  using P1 = std::integral_constant<int, 1>;
  // the block's epilogue constants: their loads are issued after tile 0's, so both round trips
  // overlap (visible after the prologue's barrier)
  auto epi_consts = [&]() {
    if (!args.partial && tid < BM && m0 + tid < args.M) epr[tid] = epi_row(args.E, m0 + tid + batch * args.E.pstride);
  };

  if constexpr (TAPS) {
    // per k-tile stages for A and B (as mode 0); B's registers hold a whole chunk (two sets, by
    // chunk parity): step i stores tile i + 1 (A from set (i + 1) & 1, B tap (i + 1) % NT of chunk
    // (i + 1) / NT) and loads A tile i + 3, plus chunk (i + 3) / NT when tile i + 3 starts a chunk
    // -- two k-steps before its first store, after the last store of the chunk that held its set
    const int brow = brow_i * LDK + lh * 8;
    la.load(ra[0], 0); la.load(ra[0], 1);
    lb.load(rb[0], 0); lb.load(rb[0], 1);            // chunk 0 -> set 0
    epi_consts();
    la.load(ra[1], 0); la.load(ra[1], 1);
    if (NT == 1) { lb.load(rb[1], 0); lb.load(rb[1], 1); }   // chunk 1 (tile 1)
    la.store(As, ra[0], 0); la.store(As, ra[0], 1);
    lb.template store<0>(Bs, rb[0], 0); lb.template store<0>(Bs, rb[0], 1);
    la.load(ra[0], 0); la.load(ra[0], 1);            // tile 2
    if (NT == 2) { lb.load(rb[1], 0); lb.load(rb[1], 1); }   // chunk 1 (tile 2)
    if (NT == 1) { lb.load(rb[0], 0); lb.load(rb[0], 1); }   // chunk 2 (tile 2)
    __syncthreads();
    A2M_PSTAMP(1, __builtin_amdgcn_s_memtime());
    pipe_frag(As + arow, fa0);
    pipe_frag(Bs + brow, fb0);
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
        const int c = (i & 1) * TA, n = TA - c;
        float* const nA = As + n;
        float* const nB = Bs + n;
        pipe_step(acc, fa0, fb0, As + c + arow, Bs + c + brow, nA + arow, nB + brow, [&](int s) {
          switch (s) {
            case 0: la.store(nA, ra[QA], 0); break;
            case 1: la.store(nA, ra[QA], 1); break;
            case 2: lb.template store<TS>(nB, rb[QB], 0); break;
            case 3: lb.template store<TS>(nB, rb[QB], 1); break;
            case 4: la.load(ra[QA], 0); break;
            case 5: la.load(ra[QA], 1); break;
            case 6: if (LB3) lb.load(rb[QL], 0); break;
            default: if (LB3) lb.load(rb[QL], 1); break;
          }
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
  } else if constexpr (!HALO) {
    const int brow = brow_i * LDK + lh * 8;
    la.load(ra[0], 0); la.load(ra[0], 1);
    lb.load(rb[0], 0); lb.load(rb[0], 1);
    epi_consts();
    la.load(ra[1], 0); la.load(ra[1], 1);
    lb.load(rb[1], 0); lb.load(rb[1], 1);
    la.store(As, ra[0], 0); la.store(As, ra[0], 1);
    lb.store(Bs, rb[0], 0); lb.store(Bs, rb[0], 1);
    la.load(ra[0], 0); la.load(ra[0], 1);
    lb.load(rb[0], 0); lb.load(rb[0], 1);
    __syncthreads();
    A2M_PSTAMP(1, __builtin_amdgcn_s_memtime());
    pipe_frag(As + arow, fa0);
    pipe_frag(Bs + brow, fb0);
    // step i (parity P = i & 1): stores of tile i + 1 from set (P + 1) & 1, then the loads of
    // tile i + 3 into that set
    auto step = [&](auto par, int i) {
      constexpr int Q = (decltype(par)::value + 1) & 1;
      const int c = (i & 1) * TA, n = TA - c;   // stage offsets of tiles i, i + 1 (TA == TB)
      float* const nA = As + n;
      float* const nB = Bs + n;
      pipe_step(acc, fa0, fb0, As + c + arow, Bs + c + brow, nA + arow, nB + brow, [&](int s) {
        switch (s) {
          case 0: la.store(nA, ra[Q], 0); break;
          case 1: la.store(nA, ra[Q], 1); break;
          case 2: lb.store(nB, rb[Q], 0); break;
          case 3: lb.store(nB, rb[Q], 1); break;
          case 4: la.load(ra[Q], 0); break;
          case 5: la.load(ra[Q], 1); break;
          case 6: lb.load(rb[Q], 0); break;
          default: lb.load(rb[Q], 1); break;
        }
      });
    };
    int i = 0;
    for (; i + 1 < nk; i += 2) {
      step(P0(), i);
      step(P1(), i + 1);
    }
    if (i < nk) step(P0(), i);
  } else {
    // halo layout: A in k-tile parity stages, B in chunk parity stages (one per 3 k-tiles); the
    // next chunk's x window is loaded at the chunk's tap 0 and stored at its tap 2
    const int T = args.B.R2;
    for (int idx = tid; idx < 2 * (BN / T) * 2 * LDK; idx += 256) {   // zero rows around each clip
      const int col = idx % LDK, q = idx / LDK;
      const int which = q & 1, clip = (q >> 1) % (BN / T), stage = (q >> 1) / (BN / T);
      Bs[stage * TB + (clip * (T + 2) + (which ? T + 1 : 0)) * LDK + col] = 0.f;
    }
    const int bsh = 2 * (brow_i / T) + 1;                     // halo rows above this lane's B row
    const int brow = (brow_i + bsh) * LDK + lh * 8;           // tap 1 (shift 0)
    float4 rx[2];                                             // a chunk's x window
    la.load(ra[0], 0); la.load(ra[0], 1);
    lb.load(rx, 0); lb.load(rx, 1);
    epi_consts();
    la.load(ra[1], 0); la.load(ra[1], 1);
    la.store(As, ra[0], 0); la.store(As, ra[0], 1);
    lb.store(Bs, rx, 0); lb.store(Bs, rx, 1);
    la.load(ra[0], 0); la.load(ra[0], 1);
    __syncthreads();
    A2M_PSTAMP(1, __builtin_amdgcn_s_memtime());
    pipe_frag(As + arow, fa0);
    pipe_frag(Bs + brow - LDK, fb0);   // tile 0 = tap 0: shift -1
    const int nch = nk / 3;
    // chunk cc (parity P = cc & 1, so tile 3 cc + j has parity (P + j) & 1): tap j stores
    // A(3 cc + j + 1) from set (P + j + 1) & 1 and loads A(3 cc + j + 3) into it
    auto chunk = [&](auto par, int cc) {
      constexpr int P = decltype(par)::value;
      constexpr int Q0 = (P + 1) & 1, Q1 = P, Q2 = (P + 1) & 1;
      const int i0 = 3 * cc;
      float* const bc = Bs + (cc & 1) * TB;          // this chunk's B stage
      float* const bn = Bs + ((cc & 1) ^ 1) * TB;    // the next chunk's
      {   // tap 0 (+ the next chunk's x window loads)
        const int c = (i0 & 1) * TA, n = TA - c;
        float* const nA = As + n;
        pipe_step(acc, fa0, fb0, As + c + arow, bc + brow - LDK, nA + arow, bc + brow, [&](int s) {
          switch (s) {
            case 0: la.store(nA, ra[Q0], 0); break;
            case 1: la.store(nA, ra[Q0], 1); break;
            case 4: la.load(ra[Q0], 0); break;
            case 5: la.load(ra[Q0], 1); break;
            case 6: lb.load(rx, 0); break;
            case 7: lb.load(rx, 1); break;
            default: break;
          }
        });
      }
      {   // tap 1
        const int c = ((i0 + 1) & 1) * TA, n = TA - c;
        float* const nA = As + n;
        pipe_step(acc, fa0, fb0, As + c + arow, bc + brow, nA + arow, bc + brow + LDK, [&](int s) {
          switch (s) {
            case 0: la.store(nA, ra[Q1], 0); break;
            case 1: la.store(nA, ra[Q1], 1); break;
            case 4: la.load(ra[Q1], 0); break;
            case 5: la.load(ra[Q1], 1); break;
            default: break;
          }
        });
      }
      {   // tap 2 (+ the next chunk's x window stores)
        const int c = ((i0 + 2) & 1) * TA, n = TA - c;
        float* const nA = As + n;
        pipe_step(acc, fa0, fb0, As + c + arow, bc + brow + LDK, nA + arow, bn + brow - LDK, [&](int s) {
          switch (s) {
            case 0: la.store(nA, ra[Q2], 0); break;
            case 1: la.store(nA, ra[Q2], 1); break;
            case 2: lb.store(bn, rx, 0); break;
            case 3: lb.store(bn, rx, 1); break;
            case 4: la.load(ra[Q2], 0); break;
            case 5: la.load(ra[Q2], 1); break;
            default: break;
          }
        });
      }
    };
    int cc = 0;
    for (; cc + 1 < nch; cc += 2) {
      chunk(P0(), cc);
      chunk(P1(), cc + 1);
    }
    if (cc < nch) chunk(P0(), cc);
  }
  A2M_PSTAMP(2, __builtin_amdgcn_s_memtime());
  __syncthreads();   // the m-contiguous epilogue reuses the stages
  floatx16 accs[1][1];
  accs[0][0] = acc;
  if (args.vec4) pipe_epilogue_vec4(args, acc, lds, epr, args.partial != nullptr, zz, batch, m0, n0, tid, wm, wn, li, lh);
  else tile_epilogue<BM, BN, 1, 1>(args, accs, lds, epr, args.partial != nullptr, zz, batch, m0, n0, tid, wm, wn, li, lh);
  span_end(args.ts);
#if A2M_PIPE_STAMPS
  __syncthreads();
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  A2M_PSTAMP(3, __builtin_amdgcn_s_memtime());
  A2M_PSTAMP(5, __builtin_amdgcn_s_memrealtime());
#endif
}

void launch_pipe(const GemmArgs& a, int ma, int mb, int batch, hipStream_t st);

}  // namespace a2m
