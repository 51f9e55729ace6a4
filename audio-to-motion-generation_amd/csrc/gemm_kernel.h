// Implicit-GEMM engine device code (shared by the per-tile translation units and gemm.hip).
// Implicit-GEMM engine on gfx950 fp32 MFMA (v_mfma_f32_32x32x2_f32, exact f32 FMA chain).
//
// C[m][n] = sum_k A(m,k) * B(n,k) with A, B described by a2m::Gather (dense matrices,
// conv im2col, transposed-conv / dgrad gathers, wgrad operands) and a fused epilogue
// (bias, BatchNorm-eval affine, activation, gamma scale, residual adds, strided store).
//
// Tiling: 256 threads = 4 waves in a 2x2 layout, block tile BM x BN (128x128 or 64x64),
// BK = 16 or 32.  Both operands are staged in LDS as [row][k] with a (BK+4)-float row pitch:
// a wave64 lane (i = lane&31, h = lane>>5) reads its k-values of row i 8 at a time as two
// ds_read_b128 (conflict-free at this pitch) and feeds MFMA sub-step s with k = (BK/2)h + s
// -- the MFMA's k slot assignment is free as long as A and B agree.  Global loads for tile
// k+1 are issued into registers before the MFMAs of tile k; LDS is double-buffered so one
// barrier per K-step suffices.  Split-K writes fp32 partial slabs to a workspace that a
// second kernel reduces in a fixed order (bitwise reproducible) and runs the epilogue on.
#pragma once
#include "a2m_internal.h"

// Diagnostic builds only (tools/gemm_ablate.sh; never the shipped library): A2M_ABLATE = 1 drops
// the k-loop MFMAs, 2 its global loads after the prologue, 3 its barriers (results wrong; the
// timing of what remains tells which part holds the loop).
#ifndef A2M_ABLATE
#define A2M_ABLATE 0
#endif

namespace a2m {

typedef float floatx16 __attribute__((ext_vector_type(16)));
typedef unsigned v4u32_t __attribute__((ext_vector_type(4)));
typedef __bf16 bf16x8 __attribute__((ext_vector_type(8)));

// K-tile depth BK = 32 (the kernels are templated on it).  LDS row pitch BK+4 floats keeps the
// per-lane ds_read_b128 fragment reads conflict-free (row*pitch mod 64 banks distinct over 16 rows).

struct GemmArgs {
  Gather A, B;
  Epilogue E;
  int M, N, K;
  int splits, kchunk;
  float* partial;
  int xcd_group;   // >0: XCD-aware block remap with this many M-tiles per group; 0: identity
  int vec4;        // (pipelined tile) output rows contiguous along n in 16-byte groups: the tile is
                   // staged through LDS and written as float4 rows (host: gemm.hip)
  int mcontig;     // output has unit m stride: the tile is staged through LDS and written
                   // along m (split-K slabs then are [N][M])
  unsigned long long* ts;   // measurement only (a2m_gemm_timing_*; null otherwise): this launch's
                            // span stamps, [tile | reduce][XCD][first start, last end]
};

// Launch-span stamps (bench.py's in-step roofline): per XCD, the earliest block start and the
// latest block end of a launch on the constant-rate wall clock, by vector atomics into the
// launch's slots.  Each block stamps once at its start and once after a final barrier, into
// one of kSpanLanes slot pairs of its XCD chosen by its linear block id, so a short launch of
// thousands of blocks does not serialise on a handful of addresses (one pair per XCD inflated
// a 7 us split-K reduce to 40 us).  Kept per XCD because the XCDs' clocks need not agree: a
// launch's duration is taken as its longest per-XCD span (every XCD receives blocks from the
// dispatch's first moment).  They work identically eagerly and inside a replayed HIP graph
// (where event records between kernels are not timestamps of the kernel: DESIGN.md 6).
constexpr int kSpanLanes = 32;
constexpr int kSpanSlots = 8 * kSpanLanes * 2;   // XCD x lane x (start, end) per kernel
__device__ __forceinline__ unsigned long long* span_slot(unsigned long long* p) {
  const unsigned xcd = __builtin_amdgcn_s_getreg((3 << 11) | 20) & 7;   // hwreg(HW_REG_XCC_ID, 0, 4)
  const unsigned lin = blockIdx.x + gridDim.x * (blockIdx.y + gridDim.y * blockIdx.z);
  return p + 2 * (xcd * kSpanLanes + lin % kSpanLanes);
}
__device__ __forceinline__ void span_begin(unsigned long long* p) {
  if (p && threadIdx.x == 0) atomicMin(span_slot(p), (unsigned long long)wall_clock64());
}
__device__ __forceinline__ void span_end(unsigned long long* p) {
  if (p) {   // uniform: the whole block takes the barrier
    __syncthreads();
    if (threadIdx.x == 0) atomicMax(span_slot(p) + 1, (unsigned long long)wall_clock64());
  }
}

struct RowInfo {
  int base, h, w;
  bool valid;
};

__device__ __forceinline__ RowInfo row_info(const Gather& g, int r, int R) {
  RowInfo ri;
  ri.valid = r < R;
  int rr = ri.valid ? r : 0;
  int r2 = rr % g.R2;
  int t = rr / g.R2;
  int r1 = t % g.R1;
  int r0 = t / g.R1;
  ri.base = r0 * g.sr0;
  ri.h = r1 * g.ar1 + g.ch;
  ri.w = r2 * g.ar2 + g.cw;
  return ri;
}

struct KPos {
  int k, k0, k1, k2;
};

__device__ __forceinline__ KPos kpos(const Gather& g, int k) {
  KPos p;
  p.k = k;
  p.k2 = k % g.K2;
  int t = k / g.K2;
  p.k1 = t % g.K1;
  p.k0 = t / g.K1;
  return p;
}

// p += d in the mixed radix (k0, K1, K2) with d.k1 < K1, d.k2 < K2: branch-free, no division
// (the loaders advance their k positions by BK per k-step this way).
__device__ __forceinline__ void kadd(const Gather& g, KPos& p, const KPos& d) {
  p.k += d.k;
  int k2 = p.k2 + d.k2;
  const int c2 = k2 >= g.K2;
  k2 -= c2 ? g.K2 : 0;
  int k1 = p.k1 + d.k1 + c2;
  const int c1 = k1 >= g.K1;
  k1 -= c1 ? g.K1 : 0;
  p.k0 += d.k0 + c1;
  p.k1 = k1;
  p.k2 = k2;
}

__device__ __forceinline__ void kinc(const Gather& g, KPos& p) {
  ++p.k;
  if (++p.k2 == g.K2) {
    p.k2 = 0;
    if (++p.k1 == g.K1) {
      p.k1 = 0;
      ++p.k0;
    }
  }
}

__device__ __forceinline__ float gather_elem(const Gather& g, const float* base, const RowInfo& ri,
                                             const KPos& p, int K) {
  int h = ri.h + p.k1 * g.bk1;
  int w = ri.w + p.k2 * g.bk2;
  bool v = ri.valid && p.k < K && h >= 0 && w >= 0;
  if (g.divh > 1) {
    v = v && (h % g.divh) == 0;
    h /= g.divh;
  }
  if (g.divw > 1) {
    v = v && (w % g.divw) == 0;
    w /= g.divw;
  }
  v = v && h < g.Lh && w < g.Lw;
  return v ? base[ri.base + p.k0 * g.sk0 + h * g.sh + w * g.sw] : 0.f;
}

typedef float float4u __attribute__((ext_vector_type(4), aligned(4)));

// Operand staging.  The MFMA k-slot order is k = 16*half + 8*h + s (h = lane>>5, s = 0..7,
// half = 0..BK/16-1) for both operands.
//   MODE 0: dense k-contiguous rows, float4 loads, LDS [row][k].
//   MODE 1: k-contiguous gather (scalar loads), LDS [row][k].
//   MODE 2: row-contiguous gather (scalar loads, lanes along rows), LDS [row][k].
//   MODE 3: row-contiguous rows loaded 4 at a time (float4 along the row axis: [K][R] matrices
//           and stride-1/2 conv im2col over [B][C][T]); written transposed into LDS [row][k]
//           (A2M_M3_TRANSPOSE, default) or kept k-major with ds_read_b32 fragments.
//   MODE 4: k-contiguous runs (the inner k digit has unit stride, K2 % 4 == 0: wgrad operands
//           over [B][C][T]) loaded 4 k at a time, LDS [row][k].
//   MODE 5: stride-1 conv1d over [B][C][T] in tap-chunked k order (k-tile j = chunk j / ntap,
//           tap j % ntap; Gather::tapconv): the chunk's x[b][c0..c0+BK)[t] rows are loaded as
//           float4 along t once (tap 0) and stored transposed, shifted by tap - pad within each
//           clip, for every tap -- the im2col operand without its 3x global traffic.  Tiles
//           hold whole clips (BR % T == 0) so the shift wraps inside the tile (wrapped rows = 0).
//   MODE 6: channels-last conv rows (Gather::nhwc): a k-tile is BK channels of one tap, so every
//           row's slice is a contiguous run loaded as float4 along k like a dense row; the tap
//           (i, j) and channel offset are uniform per tile, each row only adds its pixel offset
//           and checks the pixel against the image (padding reads 0).
#ifndef A2M_M3_TRANSPOSE
#define A2M_M3_TRANSPOSE 1
#endif
template <int BR, int BK, int MODE, int P = 0>
struct TileLoader {
  static constexpr bool H = P != 0;   // bf16 LDS image (P = 1 one plane, P = 2 three planes)
  // MODE 3 with A2M_M3_TRANSPOSE: the float4 of 4 rows is written as 4 scalars into the
  // [row][k] layout (lanes spread over k so the writes stay conflict-free), and fragments are
  // the same two ds_read_b128 as the other modes.
  static constexpr bool KMAJ = MODE == 3 && !A2M_M3_TRANSPOSE && !H;
  // [row][k] pitch in elements: fp32 BK + 4 floats; bf16 BK + 8 halves (a 16-B multiple, and
  // 36 dwords for BK = 64 so the ds_read_b128 fragments stay conflict-free)
  static constexpr int LDK = H ? BK + 8 : BK + 4;
  static constexpr int LDR = BR + 4;                // [k][row] pitch: 8*LDR = 32 mod 64 banks
  static constexpr int PLANE = BR * LDK;             // bf16 plane size in halves (P >= 1)
  static constexpr int NPLANE = P == 2 ? 3 : 1;      // bf16 planes (hi / mid / lo for P = 2)
  static constexpr int TILE = KMAJ ? BK * LDR : (H ? NPLANE * BR * LDK / 2 : BR * LDK);  // in floats
  static constexpr int QPR = BK / 4;                // k-major maps: float4 quads per row
  static constexpr int RPP = 256 / QPR;             //   rows per pass
  static constexpr int NPASS = BR / RPP;
  static constexpr int KPT = BK * BR / 256;         // row-major map: k per thread
  static constexpr int NREG = BK * BR / 256;        // floats per thread
  static constexpr int QR = BR / 4;                 // mode 3: float4 row groups per k
  static constexpr int KPP = 256 / QR;              //   k per pass
  static constexpr int NP3 = BK / KPP;
  // bf16 images of the row-vector modes (3, 5) use a k-pair map: each thread loads the float4
  // row groups of two adjacent k and writes each row's pair as one 32-bit LDS store per plane
  // (not 2-byte stores); the lanes of a wave hit 16 k-pairs x 4 row groups, conflict-free
  static constexpr bool PAIR = H && (MODE == 3 || MODE == 5);
  static constexpr int NKE = PAIR ? BK / KPP : NP3;   // k entries (a float4 of 4 rows each)
  static constexpr int NPP = BK / (2 * KPP);          // pair map: passes
  // k offset (relative to kq) of k entry e
  __device__ __forceinline__ static constexpr int eofs(int e) {
    return PAIR ? (e >> 1) * 2 * KPP + (e & 1) : e * KPP;
  }
  const Gather* g;
  const float* base;
  int K;
  RowInfo ri[MODE == 2 || MODE == 3 || MODE == 5 ? 1 : NPASS];
  int lrow[MODE == 2 || MODE == 3 || MODE == 5 ? 1 : NPASS];
  int kq;  // k offset of this thread inside the tile
  int nrow;  // mode 3: rows of this group that exist (0..4)
  int rdim;   // mode 3: 0 rows via r0, 1 rows along h, 2 rows along w
  int rstep;  // mode 3: element step between consecutive rows (1, or 2 for stride-2 convs)
  static constexpr int NKP = MODE == 3 ? NKE : 1;
  // mode 5
  int tt;        // t of this thread's first row within its clip
  int64_t rb;    // element offset of (b, t) of that row
  int st_j;      // k-tile index of the next store (its tap)
  int st_tap, ld_tap, ld_cc;   // tap of the next store; tap / channel chunk of the next load
  // fp32, up to 3 taps: each tap's LDS offsets of this thread's 4 rows and their data bits
  // (row5 evaluated once here instead of per element and k-tile)
  static constexpr int T5 = 3;
  int o5[MODE == 5 && !H ? T5 : 1][4];
  int ok5;
  // halo layout (Gather::halo; fp32, 3 taps, pad 1, clips T >= 16): the chunk's x window is
  // stored ONCE, at rows hrow(n) = (n / T) (T + 2) + 1 + n % T of its own LDS stage, with a zero
  // row before and after every clip; tap j reads it shifted by j - 1 rows
  static constexpr int HR = BR + 2 * (BR / 16);   // rows of a halo stage (T >= 16)
  static constexpr int TILE_H = HR * LDK;
  int h5[MODE == 5 && !H ? 4 : 1];
  // mode 6: the tap (i6, j6) and channel offset c6 of k-tile k6 (the next load's, normally):
  // advanced by whole k-tiles instead of dividing k0 by Ci and the tap by kw every k-step
  int k6, i6, j6, c6;
  KPos kp[NKP];   // k position of each of this thread's k groups at the next load (modes 1-3)
  KPos kstep;     // BK in (k0, k1, k2) digits
  float r[NREG];

  __device__ __forceinline__ void init(const Gather& gg, int z, int row0, int R, int KK, int tid,
                                       int kbeg, int kstride = BK) {
    g = &gg;
    base = gg.base + (int64_t)z * gg.bstride;
    K = KK;
    if (MODE == 5) {
      lrow[0] = (tid / KPP) * 4;
      kq = (tid % KPP) * (PAIR ? 2 : 1);
      // rows past R still get their true t (tiles hold whole clips, so the shifted stores of
      // an invalid group stay inside its own clip-sized span of the tile); only the address
      // of the (unused) load is clamped
      const int n = row0 + lrow[0];
      nrow = min(4, max(0, R - n));
      const int b = n / gg.R2;
      tt = n - b * gg.R2;
      rb = nrow > 0 ? (int64_t)b * gg.sr0 + tt : 0;
      st_j = kbeg / BK;
      st_tap = ld_tap = st_j % gg.tapconv;
      ld_cc = st_j / gg.tapconv;
      if constexpr (!H) {
        if (gg.halo) {
          const int T = gg.R2;
#pragma unroll
          for (int e = 0; e < 4; ++e) {
            const int n = lrow[0] + e;   // tile row (whole clips per tile: n / T is the clip)
            h5[e] = ((n / T) * (T + 2) + 1 + n % T) * LDK + kq;
          }
        }
        ok5 = 0;
#pragma unroll
        for (int t = 0; t < T5; ++t)
#pragma unroll
          for (int e = 0; e < 4; ++e) {
            bool ok;
            o5[t][e] = row5(e, t + gg.cw, ok) * LDK + kq;
            ok5 |= (ok ? 1 : 0) << (t * 4 + e);
          }
      }
      return;
    }
    if (MODE == 3) {
      if (KMAJ) {
        lrow[0] = (tid % QR) * 4;
        kq = tid / QR;
      } else {
        lrow[0] = (tid / KPP) * 4;
        kq = (tid % KPP) * (PAIR ? 2 : 1);
      }
      ri[0] = row_info(gg, row0 + lrow[0], R);
      nrow = min(4, max(0, R - (row0 + lrow[0])));
      rdim = gg.R2 > 1 ? 2 : (gg.R1 > 1 ? 1 : 0);
      rstep = rdim == 2 ? gg.ar2 : (rdim == 1 ? gg.ar1 : 1);
    } else if (MODE == 2) {
      lrow[0] = tid % BR;
      kq = (tid / BR) * KPT;
      ri[0] = row_info(gg, row0 + lrow[0], R);
    } else {
#pragma unroll
      for (int p = 0; p < NPASS; ++p) {
        lrow[p] = tid / QPR + p * RPP;
        ri[p] = row_info(gg, row0 + lrow[p], R);
        // mode 6: row_info gives base = image offset, h / w = the row's input pixel origin
        // (r1*ar1 + ch, r2*ar2 + cw); fold the origin into the base once
        if (MODE == 6) ri[p].base += (ri[p].h * gg.Lw + ri[p].w) * gg.nhwc;
      }
      kq = (tid % QPR) * 4;
      if (MODE == 6) {
        const int tap = kbeg / gg.nhwc;
        k6 = kbeg;
        c6 = kbeg - tap * gg.nhwc;
        i6 = tap / gg.K2;
        j6 = tap - i6 * gg.K2;
      }
    }
    if (MODE != 0 && MODE != 6) {
      kstep = kpos(gg, kstride);
#pragma unroll
      for (int p = 0; p < NKP; ++p) kp[p] = kpos(gg, kbeg + kq + (MODE == 3 ? eofs(p) : 0));
    }
  }

  __device__ __forceinline__ void load(int k0) {
    if (MODE == 5) {
      // loads come in k-tile order (k0 = kbeg, kbeg + BK, ...): tap / chunk kept as counters
      const int cc = ld_cc;
      const bool first = ld_tap == 0;
      if (++ld_tap == g->tapconv) { ld_tap = 0; ++ld_cc; }
      if (!first) return;   // taps 1.. re-store the registers of tap 0
      (void)k0;
#pragma unroll
      for (int p = 0; p < NKE; ++p) {
        const float* src = base + rb + (int64_t)(cc * BK + kq + eofs(p)) * g->sk0;
        if (nrow == 4) {
          const float4u u = *reinterpret_cast<const float4u*>(src);
          r[p * 4 + 0] = u.x; r[p * 4 + 1] = u.y; r[p * 4 + 2] = u.z; r[p * 4 + 3] = u.w;
        } else {
#pragma unroll
          for (int j2 = 0; j2 < 4; ++j2) r[p * 4 + j2] = j2 < nrow ? src[j2] : 0.f;
        }
      }
      return;
    }
    if (MODE == 0) {
#pragma unroll
      for (int p = 0; p < NPASS; ++p) {
        int k = k0 + kq;
        float4 v = make_float4(0.f, 0.f, 0.f, 0.f);
        if (ri[p].valid && k < K) v = *reinterpret_cast<const float4*>(base + ri[p].base + k);
        r[p * 4 + 0] = v.x; r[p * 4 + 1] = v.y; r[p * 4 + 2] = v.z; r[p * 4 + 3] = v.w;
      }
    } else if (MODE == 6) {
      const int Ci = g->nhwc;
      // k0 comes in whole k-tiles after k6 (one for the one-group tile); Ci % BK == 0 (host)
      while (k6 < k0) {
        k6 += BK;
        c6 += BK;
        if (c6 == Ci) {
          c6 = 0;
          if (++j6 == g->K2) { j6 = 0; ++i6; }
        }
      }
      const int i = i6, j = j6;
      const int toff = (i * g->Lw + j) * Ci + c6 + kq;
#pragma unroll
      for (int p = 0; p < NPASS; ++p) {
        const int h = ri[p].h + i, w = ri[p].w + j;
        float4 v = make_float4(0.f, 0.f, 0.f, 0.f);
        if (ri[p].valid && k0 < K && (unsigned)h < (unsigned)g->Lh && (unsigned)w < (unsigned)g->Lw)
          v = *reinterpret_cast<const float4*>(base + ri[p].base + toff);
        r[p * 4 + 0] = v.x; r[p * 4 + 1] = v.y; r[p * 4 + 2] = v.z; r[p * 4 + 3] = v.w;
      }
    } else if (MODE == 4) {
      // k-contiguous runs: the 4 k of a quad share k0, k1 (host: K2 % 4 == 0) and sit at
      // consecutive addresses (bk2 * sw == 1), so one float4 unless the quad crosses an edge
#pragma unroll
      for (int p = 0; p < NPASS; ++p) {
        const KPos q = kp[0];
        int h = ri[p].h + q.k1 * g->bk1;
        const int w = ri[p].w + q.k2;
        bool hv = ri[p].valid && h >= 0;
        if (g->divh > 1) {
          hv = hv && (h % g->divh) == 0;
          h = h / g->divh;
        }
        hv = hv && h < g->Lh;
        float4 v;
        if (hv && q.k + 3 < K && w >= 0 && w + 3 < g->Lw) {
          const float4u u = *reinterpret_cast<const float4u*>(
              base + ri[p].base + (int64_t)q.k0 * g->sk0 + (int64_t)h * g->sh + w);
          v = make_float4(u.x, u.y, u.z, u.w);
        } else {
          KPos qq = q;
          float e[4];
#pragma unroll
          for (int j = 0; j < 4; ++j) {
            e[j] = gather_elem(*g, base, ri[p], qq, K);
            kinc(*g, qq);
          }
          v = make_float4(e[0], e[1], e[2], e[3]);
        }
        r[p * 4 + 0] = v.x; r[p * 4 + 1] = v.y; r[p * 4 + 2] = v.z; r[p * 4 + 3] = v.w;
      }
      kadd(*g, kp[0], kstep);
    } else if (MODE == 1) {
#pragma unroll
      for (int p = 0; p < NPASS; ++p) {
        KPos q = kp[0];
#pragma unroll
        for (int j = 0; j < 4; ++j) {
          r[p * 4 + j] = gather_elem(*g, base, ri[p], q, K);
          kinc(*g, q);
        }
      }
      kadd(*g, kp[0], kstep);
    } else if (MODE == 2) {
      KPos q = kp[0];
#pragma unroll
      for (int j = 0; j < KPT; ++j) {
        r[j] = gather_elem(*g, base, ri[0], q, K);
        kinc(*g, q);
      }
      kadd(*g, kp[0], kstep);
    } else {
      // 4 consecutive rows differ only in the row axis (host guarantees it): rdim 0 = rows via
      // r0 with unit stride, 1 = rows along h (sh == 1), 2 = rows along w (sw == 1), so their
      // elements are consecutive floats (rstep 1) or every other float (stride-2 convs).
      const int dh = rdim == 1 ? rstep : 0, dw = rdim == 2 ? rstep : 0;
#pragma unroll
      for (int p = 0; p < NKE; ++p) {
        const KPos q = kp[p];
        kadd(*g, kp[p], kstep);
        int h = ri[0].h + q.k1 * g->bk1;
        const int w = ri[0].w + q.k2 * g->bk2;
        bool kv = q.k < K && nrow > 0;
        if (g->divh > 1) {  // only with rdim != 1
          kv = kv && h >= 0 && (h % g->divh) == 0;
          h = h / g->divh;
        }
        const int64_t a = (int64_t)ri[0].base + (int64_t)q.k0 * g->sk0 + (int64_t)h * g->sh +
                          (int64_t)w * g->sw;
        float4 v;
        if (kv && nrow == 4 && h >= 0 && h + 3 * dh < g->Lh && w >= 0 && w + 3 * dw < g->Lw) {
          const float4u u = *reinterpret_cast<const float4u*>(base + a);
          if (rstep == 1) {
            v = make_float4(u.x, u.y, u.z, u.w);
          } else {  // stride-2 rows: elements a, a+2 | a+4, a+6 (second load ends at a+6)
            const float4u u1 = *reinterpret_cast<const float4u*>(base + a + 3);
            v = make_float4(u.x, u.z, u1.y, u1.w);
          }
        } else {
          float e[4];
#pragma unroll
          for (int j = 0; j < 4; ++j) {
            const int hj = h + j * dh, wj = w + j * dw;
            e[j] = (kv && j < nrow && hj >= 0 && hj < g->Lh && wj >= 0 && wj < g->Lw)
                       ? base[a + j * rstep] : 0.f;
          }
          v = make_float4(e[0], e[1], e[2], e[3]);
        }
        r[p * 4 + 0] = v.x; r[p * 4 + 1] = v.y; r[p * 4 + 2] = v.z; r[p * 4 + 3] = v.w;
      }
    }
  }

  // halo layout: the tap-0 registers of the chunk to their unshifted rows (rows past R hold 0)
  __device__ __forceinline__ void store_h(float* lds) {
    if constexpr (MODE == 5 && !H) {
#pragma unroll
      for (int p = 0; p < NP3; ++p)
#pragma unroll
        for (int e = 0; e < 4; ++e) lds[h5[e] + p * KPP] = r[p * 4 + e];
    }
  }

  // mode 5: the row (within the tile) that element e of this thread's 4-row group lands on for
  // the shift s = tap - pad, and whether it carries data (rows whose source t + s leaves the
  // clip take 0, written by the element that wraps onto them)
  __device__ __forceinline__ int row5(int e, int s, bool& ok) const {
    const int ts = tt + e;
    int td = ts - s;
    const int T = g->R2;
    ok = td >= 0 && td < T;
    td += td < 0 ? T : (td >= T ? -T : 0);
    return lrow[0] + e + (td - ts);
  }

  __device__ __forceinline__ void store(float* lds) {
    if constexpr (MODE == 5) {
      const int tap = st_tap;
      if (++st_tap == g->tapconv) st_tap = 0;
      ++st_j;
      if constexpr (!H) {
        if (g->tapconv <= T5) {   // precomputed offsets (tap is uniform: one branch per tile)
          auto put = [&](const int (&o)[4], int sh) {
#pragma unroll
            for (int p = 0; p < NP3; ++p)
#pragma unroll
              for (int e = 0; e < 4; ++e)
                lds[o[e] + p * KPP] = ((ok5 >> (sh + e)) & 1) ? r[p * 4 + e] : 0.f;
          };
          if (tap == 0) put(o5[0], 0);
          else if (tap == 1) put(o5[T5 > 1 ? 1 : 0], 4);
          else put(o5[T5 > 2 ? 2 : 0], 8);
          return;
        }
      }
      const int s = tap + g->cw;   // cw = -pad
      if constexpr (H) {
#pragma unroll
        for (int pp = 0; pp < NPP; ++pp)
#pragma unroll
          for (int e = 0; e < 4; ++e) {
            bool ok;
            const int o = row5(e, s, ok) * LDK + kq + pp * 2 * KPP;
            store_pair(lds, o, ok ? r[(2 * pp) * 4 + e] : 0.f, ok ? r[(2 * pp + 1) * 4 + e] : 0.f);
          }
      } else {
#pragma unroll
        for (int p = 0; p < NP3; ++p)
#pragma unroll
          for (int e = 0; e < 4; ++e) {
            bool ok;
            const int o = row5(e, s, ok) * LDK + kq + p * KPP;
            lds[o] = ok ? r[p * 4 + e] : 0.f;
          }
      }
      return;
    }
    if constexpr (P == 2) {  // three-way bf16 split (hi + mid + lo == v) on the way into LDS
      __bf16* hl = reinterpret_cast<__bf16*>(lds);
      if (MODE == 3) {
        store_pairs3(lds);
      } else if (MODE == 2) {
#pragma unroll
        for (int j = 0; j < KPT; j += 4) {
          uint2 q[3];
          split4(&r[j], q);
          const int o = lrow[0] * LDK + kq + j;
#pragma unroll
          for (int c = 0; c < 3; ++c) *reinterpret_cast<uint2*>(hl + c * PLANE + o) = q[c];
        }
      } else {
#pragma unroll
        for (int p = 0; p < NPASS; ++p) {
          uint2 q[3];
          split4(&r[p * 4], q);
          const int o = lrow[p] * LDK + kq;
#pragma unroll
          for (int c = 0; c < 3; ++c) *reinterpret_cast<uint2*>(hl + c * PLANE + o) = q[c];
        }
      }
      return;
    } else if constexpr (H) {  // round to bf16 (RNE) on the way into LDS
      __bf16* hl = reinterpret_cast<__bf16*>(lds);
      if (MODE == 3) {
        store_pairs3(lds);
      } else if (MODE == 2) {
        __bf16* dst = hl + lrow[0] * LDK + kq;
#pragma unroll
        for (int j = 0; j < KPT; j += 4) *reinterpret_cast<uint2*>(dst + j) = pack4(&r[j]);
      } else {
#pragma unroll
        for (int p = 0; p < NPASS; ++p)
          *reinterpret_cast<uint2*>(hl + lrow[p] * LDK + kq) = pack4(&r[p * 4]);
      }
      return;
    }
    if (MODE == 3 && KMAJ) {
#pragma unroll
      for (int p = 0; p < NP3; ++p)
        *reinterpret_cast<float4*>(lds + (kq + p * KPP) * LDR + lrow[0]) =
            make_float4(r[p * 4], r[p * 4 + 1], r[p * 4 + 2], r[p * 4 + 3]);
    } else if (MODE == 3) {
#pragma unroll
      for (int p = 0; p < NP3; ++p)
#pragma unroll
        for (int j = 0; j < 4; ++j) lds[(lrow[0] + j) * LDK + kq + p * KPP] = r[p * 4 + j];
    } else if (MODE == 2) {
      float* dst = lds + lrow[0] * LDK + kq;
#pragma unroll
      for (int j = 0; j < KPT; j += 4)
        *reinterpret_cast<float4*>(dst + j) = make_float4(r[j], r[j + 1], r[j + 2], r[j + 3]);
    } else {
#pragma unroll
      for (int p = 0; p < NPASS; ++p)
        *reinterpret_cast<float4*>(lds + lrow[p] * LDK + kq) =
            make_float4(r[p * 4], r[p * 4 + 1], r[p * 4 + 2], r[p * 4 + 3]);
    }
  }

  __device__ __forceinline__ static uint2 pack4(const float* v) {
    const __bf16 a = (__bf16)v[0], b = (__bf16)v[1], c = (__bf16)v[2], d = (__bf16)v[3];
    return make_uint2((uint32_t)__builtin_bit_cast(uint16_t, a) |
                          ((uint32_t)__builtin_bit_cast(uint16_t, b) << 16),
                      (uint32_t)__builtin_bit_cast(uint16_t, c) |
                          ((uint32_t)__builtin_bit_cast(uint16_t, d) << 16));
  }

  // Three-way split of an fp32 value: hi = rne_bf16(v), mid = rne_bf16(v - hi),
  // lo = rne_bf16(v - hi - mid).  Both differences are exact in fp32 (each removes the leading
  // 8 significant bits), so hi + mid + lo == v for every finite v whose pieces stay normal, and
  // |mid| <= 2^-8 |v|, |lo| <= 2^-16 |v|.
  __device__ __forceinline__ static void split3(float v, __bf16* o) {
    const __bf16 h = (__bf16)v;
    const float r1 = v - (float)h;
    const __bf16 m = (__bf16)r1;
    o[0] = h;
    o[1] = m;
    o[2] = (__bf16)(r1 - (float)m);
  }
  // split3 of two values at once, each piece as a packed bf16 pair (v_cvt_pk_bf16_f32 and
  // v_pk_add_f32 do both lanes: ~9 instructions per pair)
  __device__ __forceinline__ static void split_pair(float a, float b, uint32_t* q) {
    typedef float f2 __attribute__((ext_vector_type(2)));
    typedef __bf16 h2 __attribute__((ext_vector_type(2)));
    const f2 v = {a, b};
    const uint32_t hu = __builtin_bit_cast(uint32_t, __builtin_convertvector(v, h2));
    const f2 hf = {__builtin_bit_cast(float, hu << 16), __builtin_bit_cast(float, hu & 0xffff0000u)};
    const f2 r1 = v - hf;
    const uint32_t mu = __builtin_bit_cast(uint32_t, __builtin_convertvector(r1, h2));
    const f2 mf = {__builtin_bit_cast(float, mu << 16), __builtin_bit_cast(float, mu & 0xffff0000u)};
    const f2 r2 = r1 - mf;
    q[0] = hu;
    q[1] = mu;
    q[2] = __builtin_bit_cast(uint32_t, __builtin_convertvector(r2, h2));
  }
  __device__ __forceinline__ static void split4(const float* v, uint2* q) {
    uint32_t a[3], b[3];
    split_pair(v[0], v[1], a);
    split_pair(v[2], v[3], b);
#pragma unroll
    for (int c = 0; c < 3; ++c) q[c] = make_uint2(a[c], b[c]);
  }
  // one k-pair of one row into the bf16 image(s) at half offset o (o even)
  __device__ __forceinline__ static void store_pair(float* lds, int o, float v0, float v1) {
    uint32_t* w = reinterpret_cast<uint32_t*>(lds);
    if constexpr (P == 2) {
      uint32_t q[3];
      split_pair(v0, v1, q);
#pragma unroll
      for (int c = 0; c < 3; ++c) w[(c * PLANE + o) >> 1] = q[c];
    } else {
      typedef float f2 __attribute__((ext_vector_type(2)));
      typedef __bf16 h2 __attribute__((ext_vector_type(2)));
      const f2 v = {v0, v1};
      w[o >> 1] = __builtin_bit_cast(uint32_t, __builtin_convertvector(v, h2));
    }
  }
  // mode 3, bf16 images: the k-pair map's row groups
  __device__ __forceinline__ void store_pairs3(float* lds) const {
#pragma unroll
    for (int pp = 0; pp < NPP; ++pp)
#pragma unroll
      for (int j = 0; j < 4; ++j)
        store_pair(lds, (lrow[0] + j) * LDK + kq + pp * 2 * KPP, r[(2 * pp) * 4 + j],
                   r[(2 * pp + 1) * 4 + j]);
  }

  // bf16: the 8 k-values k = 16*sub + 8*lh + s of tile row `row` (one ds_read_b128) of plane c
  __device__ __forceinline__ static bf16x8 hfrag(const float* lds, int row, int sub, int lh, int c = 0) {
    const __bf16* q = reinterpret_cast<const __bf16*>(lds) + c * PLANE + row * LDK + sub * 16 + lh * 8;
    return *reinterpret_cast<const bf16x8*>(q);
  }

  // The 8 k-values (k = 16*half + 8*lh + s, s = 0..7) of tile row `row` for one lane.
  __device__ __forceinline__ static void frag(const float* lds, int row, int half, int lh, float* f) {
    if (KMAJ) {
      const float* q = lds + (half * 16 + lh * 8) * LDR + row;
#pragma unroll
      for (int s = 0; s < 8; ++s) f[s] = q[s * LDR];
    } else {
      const float* q = lds + row * LDK + half * 16 + lh * 8;
      const float4 v0 = *reinterpret_cast<const float4*>(q);
      const float4 v1 = *reinterpret_cast<const float4*>(q + 4);
      f[0] = v0.x; f[1] = v0.y; f[2] = v0.z; f[3] = v0.w;
      f[4] = v1.x; f[5] = v1.y; f[6] = v1.z; f[7] = v1.w;
    }
  }
};

__device__ __forceinline__ int64_t epi_addr(const Epilogue& E, int m, int n) {
  int n2 = n % E.N2;
  int t = n / E.N2;
  int n1 = t % E.N1;
  int n0 = t / E.N1;
  return (int64_t)n0 * E.so0 + (int64_t)n1 * E.so1 + (int64_t)n2 * E.so2 + (int64_t)m * E.som;
}

__device__ __forceinline__ float epi_value(const Epilogue& E, float v, int m) {
  if (E.bias) v += E.bias[m];
  if (E.bn_w) v = (v - E.bn_rm[m]) * (E.bn_w[m] / sqrtf(E.bn_rv[m] + E.bn_eps)) + E.bn_b[m];
  if (E.act == ACT_RELU) v = v > 0.f ? v : 0.f;
  else if (E.act == ACT_LRELU) v = v > 0.f ? v : v * E.slope;
  else if (E.act == ACT_SIGMOID) v = 1.f / (1.f + expf(-v));
  if (E.gamma) v *= E.gamma[0];
  return v;
}

__device__ __forceinline__ void epi_store(const Epilogue& E, int z, float v, int m, int64_t a) {
  int64_t off = (int64_t)z * E.bstride + a;
  v = epi_value(E, v, m + z * E.pstride);
  if (E.res1) v += E.res1[off];
  if (E.res2) v += E.res2[off];
  if (E.accumulate) v += E.out[off];
  E.out[off] = v;
}

// The per-channel epilogue constants of one output row m (bias, BN running mean, BN scale
// w / sqrt(var + eps), BN shift), loaded and computed once per row instead of per element;
// epi_value_p applies them with exactly epi_value's operations (same results).
struct __attribute__((aligned(16))) EpiRow {
  float bias, rm, sc, bb;
};
__device__ __forceinline__ EpiRow epi_row(const Epilogue& E, int m) {
  EpiRow r{0.f, 0.f, 1.f, 0.f};
  if (E.bias) r.bias = E.bias[m];
  if (E.bn_w) {
    r.rm = E.bn_rm[m];
    r.sc = E.bn_w[m] / sqrtf(E.bn_rv[m] + E.bn_eps);
    r.bb = E.bn_b[m];
  }
  return r;
}
__device__ __forceinline__ float epi_value_p(const Epilogue& E, float v, const EpiRow& r) {
  if (E.bias) v += r.bias;
  if (E.bn_w) v = (v - r.rm) * r.sc + r.bb;
  if (E.act == ACT_RELU) v = v > 0.f ? v : 0.f;
  else if (E.act == ACT_LRELU) v = v > 0.f ? v : v * E.slope;
  else if (E.act == ACT_SIGMOID) v = 1.f / (1.f + expf(-v));
  if (E.gamma) v *= E.gamma[0];
  return v;
}
__device__ __forceinline__ void epi_store_p(const Epilogue& E, int z, float v, const EpiRow& r, int64_t a) {
  const int64_t off = (int64_t)z * E.bstride + a;
  v = epi_value_p(E, v, r);
  if (E.res1) v += E.res1[off];
  if (E.res2) v += E.res2[off];
  if (E.accumulate) v += E.out[off];
  E.out[off] = v;
}
// n -> (n0, n1, n2) of the output's 3-level column index, advanced incrementally
struct EpiCol {
  int n0, n1, n2;
  __device__ __forceinline__ void set(const Epilogue& E, int n) {
    n2 = n % E.N2;
    const int t = n / E.N2;
    n1 = t % E.N1;
    n0 = t / E.N1;
  }
  __device__ __forceinline__ void advance(const Epilogue& E, int d) {
    n2 += d;
    while (n2 >= E.N2) {
      n2 -= E.N2;
      if (++n1 == E.N1) { n1 = 0; ++n0; }
    }
  }
  __device__ __forceinline__ int64_t addr(const Epilogue& E) const {
    return (int64_t)n0 * E.so0 + (int64_t)n1 * E.so1 + (int64_t)n2 * E.so2;
  }
};

// Main loop, BK = 32 (two 16-k halves per k-tile), one barrier per k-step placed mid-step:
//   step i:  store tile i+1 (registers) -> LDS[(i+1)&1]; issue global loads of tile i+2;
//            read half-1 fragments of tile i; MFMAs of half 0 (fragments read last step);
//            barrier (tile i+1 visible, every read of tile i complete);
//            read half-0 fragments of tile i+1; MFMAs of half 1.
// The next tile's first fragments are read while this tile's second half is on the matrix
// pipe, so no LDS latency sits between k-steps.  LDS[(i+1)&1] is free at the start of step i:
// its last reads (tile i-1, half 1) preceded step i-1's barrier.
template <int TM, int TN, int P, int NS = 1>
struct Frags;
template <int TM, int TN, int NS>
struct Frags<TM, TN, 0, NS> {  // fp32: 16 NS k per half (BK = 32 NS), 8 NS per lane
  float a[TM][8 * NS], b[TN][8 * NS];
};
template <int TM, int TN>
struct Frags<TM, TN, 1, 1> {   // bf16: 32 k per half = two K16 chunks, 8 per lane each
  bf16x8 a[TM][2], b[TN][2];
};
template <int TM, int TN>
struct Frags<TM, TN, 2, 1> {   // bf16x6: 16 k per half (one K16 chunk), the three planes
  bf16x8 a[TM][3], b[TN][3];
};

template <int BM, int BN, int TM, int TN, int P, int NS, class LA, class LB>
__device__ __forceinline__ void read_frags(const float* As, const float* Bs, int half, int wm, int wn,
                                           int li, int lh, Frags<TM, TN, P, NS>& f) {
  if constexpr (P == 2) {
#pragma unroll
    for (int c = 0; c < 3; ++c) {
#pragma unroll
      for (int t = 0; t < TM; ++t) f.a[t][c] = LA::hfrag(As, wm * (BM / 2) + t * 32 + li, half, lh, c);
#pragma unroll
      for (int u = 0; u < TN; ++u) f.b[u][c] = LB::hfrag(Bs, wn * (BN / 2) + u * 32 + li, half, lh, c);
    }
  } else if constexpr (P == 1) {
#pragma unroll
    for (int c = 0; c < 2; ++c) {
#pragma unroll
      for (int t = 0; t < TM; ++t) f.a[t][c] = LA::hfrag(As, wm * (BM / 2) + t * 32 + li, 2 * half + c, lh);
#pragma unroll
      for (int u = 0; u < TN; ++u) f.b[u][c] = LB::hfrag(Bs, wn * (BN / 2) + u * 32 + li, 2 * half + c, lh);
    }
  } else {
#pragma unroll
    for (int sub = 0; sub < NS; ++sub) {
#pragma unroll
      for (int t = 0; t < TM; ++t) LA::frag(As, wm * (BM / 2) + t * 32 + li, half * NS + sub, lh, &f.a[t][8 * sub]);
#pragma unroll
      for (int u = 0; u < TN; ++u) LB::frag(Bs, wn * (BN / 2) + u * 32 + li, half * NS + sub, lh, &f.b[u][8 * sub]);
    }
  }
}

// MFMA sub-steps [S0, S1) of a half (fp32: s = 0..7, bf16: c = 0..1)
// bf16x6: the six products of the split operands whose order is >= 2^-16 (a_i b_j, i + j <= 2),
// smallest first; the dropped a1 b2, a2 b1, a2 b2 are below 2^-24 |a b|.  Term j of the list:
__device__ __forceinline__ constexpr int x6_ia(int j) { return j == 0 ? 2 : j == 1 ? 1 : j == 2 ? 0 : j == 3 ? 1 : j == 4 ? 0 : 0; }
__device__ __forceinline__ constexpr int x6_ib(int j) { return j == 0 ? 0 : j == 1 ? 1 : j == 2 ? 2 : j == 3 ? 0 : j == 4 ? 1 : 0; }
template <int S0, int S1, int TM, int TN>
__device__ __forceinline__ void mfma_part(const Frags<TM, TN, 2, 1>& f, floatx16 (&acc)[TM][TN]) {
#pragma unroll
  for (int j = S0; j < S1; ++j)
#pragma unroll
    for (int t = 0; t < TM; ++t)
#pragma unroll
      for (int u = 0; u < TN; ++u)
        acc[t][u] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(f.a[t][x6_ia(j)], f.b[u][x6_ib(j)], acc[t][u], 0, 0, 0);
}
template <int TM, int TN>
__device__ __forceinline__ void mfma_half(const Frags<TM, TN, 2, 1>& f, floatx16 (&acc)[TM][TN]) {
  mfma_part<0, 6>(f, acc);
}

template <int S0, int S1, int TM, int TN, int NS>
__device__ __forceinline__ void mfma_part(const Frags<TM, TN, 0, NS>& f, floatx16 (&acc)[TM][TN]) {
#pragma unroll
  for (int s = S0; s < S1; ++s)
#pragma unroll
    for (int t = 0; t < TM; ++t)
#pragma unroll
      for (int u = 0; u < TN; ++u)
        acc[t][u] = __builtin_amdgcn_mfma_f32_32x32x2f32(f.a[t][s], f.b[u][s], acc[t][u], 0, 0, 0);
}
template <int S0, int S1, int TM, int TN>
__device__ __forceinline__ void mfma_part(const Frags<TM, TN, 1, 1>& f, floatx16 (&acc)[TM][TN]) {
#pragma unroll
  for (int c = S0; c < S1; ++c)
#pragma unroll
    for (int t = 0; t < TM; ++t)
#pragma unroll
      for (int u = 0; u < TN; ++u)
        acc[t][u] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(f.a[t][c], f.b[u][c], acc[t][u], 0, 0, 0);
}

template <int TM, int TN, int NS>
__device__ __forceinline__ void mfma_half(const Frags<TM, TN, 0, NS>& f, floatx16 (&acc)[TM][TN]) {
#pragma unroll
  for (int s = 0; s < 8 * NS; ++s)
#pragma unroll
    for (int t = 0; t < TM; ++t)
#pragma unroll
      for (int u = 0; u < TN; ++u)
        acc[t][u] = __builtin_amdgcn_mfma_f32_32x32x2f32(f.a[t][s], f.b[u][s], acc[t][u], 0, 0, 0);
}

template <int TM, int TN>
__device__ __forceinline__ void mfma_half(const Frags<TM, TN, 1, 1>& f, floatx16 (&acc)[TM][TN]) {
#pragma unroll
  for (int c = 0; c < 2; ++c)
#pragma unroll
    for (int t = 0; t < TM; ++t)
#pragma unroll
      for (int u = 0; u < TN; ++u)
        acc[t][u] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(f.a[t][c], f.b[u][c], acc[t][u], 0, 0, 0);
}

// A2M_ABLATE = 1: keep the fragments live with one VALU op instead of the MFMAs
template <class FR, int TM, int TN>
__device__ __forceinline__ void ablate_touch(const FR& f, floatx16 (&acc)[TM][TN]) {
  if constexpr (sizeof(f.a[0][0]) == 4)
    acc[0][0][0] += __builtin_bit_cast(float, __builtin_bit_cast(uint32_t, f.a[0][0]) ^
                                                  __builtin_bit_cast(uint32_t, f.b[0][0])) * 1e-30f;
}

// Tile epilogue (shared by gemm_tile and gemm_pipe_kernel): the accumulators of the block's
// BM x BN tile (wave (wm, wn) holds rows wm*BM/2 + t*32 + (q&3) + 8(q>>2) + 4lh, columns
// wn*BN/2 + u*32 + li) as split-K slabs (slab_out) or through the fused epilogue; m-contiguous
// outputs are staged through lds (>= BN * (BM + 1) floats, free when called).
template <int BM, int BN, int TM, int TN>
__device__ __forceinline__ void tile_epilogue(const GemmArgs& args, const floatx16 (&acc)[TM][TN], float* lds,
                                              const EpiRow* epr, bool slab_out, int zz, int batch, int m0,
                                              int n0, int tid, int wm, int wn, int li, int lh) {
  if (args.mcontig) {
    // m-contiguous output (node-feature layouts [.., J*64]): a direct store would put the 32
    // lanes of each instruction (consecutive n) M floats apart.  Stage the tile as Cs[n][m]
    // (pitch BM + 1) in the now idle LDS and write it out along m instead.
    constexpr int LDC = BM + 1;
#pragma unroll
    for (int u = 0; u < TN; ++u)
#pragma unroll
      for (int t = 0; t < TM; ++t)
#pragma unroll
        for (int q = 0; q < 16; ++q)
          lds[(wn * (BN / 2) + u * 32 + li) * LDC + wm * (BM / 2) + t * 32 + (q & 3) + 8 * (q >> 2) +
              4 * lh] = acc[t][u][q];
    __syncthreads();
    const int ml = tid % BM;
    const int m = m0 + ml;
    if (m < args.M) {
      if (slab_out) {
        for (int nl = tid / BM; nl < BN; nl += 256 / BM) {
          const int n = n0 + nl;
          if (n >= args.N) break;
          args.partial[(int64_t)zz * args.M * args.N + (int64_t)n * args.M + m] = lds[nl * LDC + ml];
        }
      } else {
        const EpiRow r = epr[ml];
        const int64_t am = (int64_t)m * args.E.som;
        EpiCol c;
        c.set(args.E, n0 + tid / BM);
        for (int nl = tid / BM; nl < BN; nl += 256 / BM) {
          if (n0 + nl >= args.N) break;
          epi_store_p(args.E, batch, lds[nl * LDC + ml], r, c.addr(args.E) + am);
          c.advance(args.E, 256 / BM);
        }
      }
    }
    return;
  }
#pragma unroll
  for (int u = 0; u < TN; ++u) {
    const int n = n0 + wn * (BN / 2) + u * 32 + li;
    if (n >= args.N) continue;
    if (slab_out) {
      float* dst = args.partial + (int64_t)zz * args.M * args.N + n;
#pragma unroll
      for (int t = 0; t < TM; ++t)
#pragma unroll
        for (int q = 0; q < 16; ++q) {
          const int m = m0 + wm * (BM / 2) + t * 32 + (q & 3) + 8 * (q >> 2) + 4 * lh;
          if (m < args.M) dst[(int64_t)m * args.N] = acc[t][u][q];
        }
    } else {
      const int64_t an = epi_addr(args.E, 0, n);
#pragma unroll
      for (int t = 0; t < TM; ++t)
#pragma unroll
        for (int q = 0; q < 16; ++q) {
          const int ml = wm * (BM / 2) + t * 32 + (q & 3) + 8 * (q >> 2) + 4 * lh;
          const int m = m0 + ml;
          if (m < args.M) epi_store_p(args.E, batch, acc[t][u][q], epr[ml], an + (int64_t)m * args.E.som);
        }
    }
  }
}

// H = false: fp32 operands, v_mfma_f32_32x32x2_f32, BK = 32 (two 16-k halves).
// H = true:  operands rounded to bf16 (RNE) when staged in LDS, v_mfma_f32_32x32x16_bf16 with
//            fp32 accumulation, BK = 64 (two 32-k halves of two K16 chunks).
// KS = 2 (64x64 fp32 tile): 512 threads, two wave groups on the same output subtiles, group g
// running the MFMAs of k-half g of every k-tile (so each SIMD holds two waves that fill each
// other's issue gaps at one block per CU); the groups stage alternate k-tiles, the partial
// accumulators are summed through LDS before the epilogue.  (The k-halves of one k-tile are added in a
// different order than KS = 1: results agree to fp32 rounding, not bitwise.)
template <int BM, int BN, int BK, int MA, int MB, int P, int KS = 1>
__device__ __forceinline__ void gemm_tile(const GemmArgs& args) {
  static_assert(P == 0 ? (BK == 32 || BK == 64) : BK == (P == 1 ? 64 : 32),
                "the k-step pipeline assumes two halves per k-tile");
  constexpr int NS = P == 0 ? BK / 32 : 1;   // fp32: 16-k fragment chunks per half
  static_assert(KS == 1 || (KS == 2 && P == 0), "two wave groups: fp32 tiles only");
  constexpr int TM = BM / 64, TN = BN / 64;
  using LA = TileLoader<BM, BK, MA, P>;
  using LB = TileLoader<BN, BK, MB, P>;
  constexpr int STAGE = LA::TILE + LB::TILE;
  // mode-5 halo layout: two A stages + two chunk-wide B stages (tile_halo below)
  constexpr bool HALO = MB == 5 && P == 0 && KS == 1 && BN == 64;
  constexpr int LDS_F = 2 * STAGE;
  constexpr int LDS_H = HALO ? 2 * LA::TILE + 2 * LB::TILE_H : 0;
  constexpr int LDS_T = LDS_F > LDS_H ? LDS_F : LDS_H;
  __shared__ __attribute__((aligned(16))) float lds[LDS_T];
  __shared__ EpiRow epr[BM];   // the block's per-row epilogue constants (final-output launches)
  static_assert(KS == 1 || (TM * TN * 16 * 256 <= 2 * STAGE), "KS = 2 partials must fit the stages");
  const int grp = KS == 1 ? 0 : (int)(threadIdx.x >> 8);
  const int tid = threadIdx.x & 255;
  const int lane = tid & 63, wave = tid >> 6;
  const int wm = wave >> 1, wn = wave & 1;
  const int li = lane & 31, lh = lane >> 5;

  // Block -> (n-tile, m-tile, batch*split).  With xcd_group > 0 the linear block id, which the
  // dispatcher deals round-robin over the 8 XCDs, is first made contiguous per XCD (bijective
  // for any grid size) and then walked in groups of xcd_group M-tiles, so the blocks that share
  // an XCD's L2 share A panels (weights) and B panels (activations).
  int bx = blockIdx.x, by = blockIdx.y, bz = blockIdx.z;
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
  // block-uniform values kept in SGPRs (readfirstlane): the k-loop's tile-count branches then
  // compile to scalar branches instead of exec-masked regions
  bx = __builtin_amdgcn_readfirstlane(bx);
  by = __builtin_amdgcn_readfirstlane(by);
  bz = __builtin_amdgcn_readfirstlane(bz);
  const int zz = bz;
  const int batch = zz / args.splits, split = zz % args.splits;
  const int m0 = by * BM, n0 = bx * BN;
  const int kbeg = split * args.kchunk;
  const int kend = min(args.K, kbeg + args.kchunk);

  // epilogue constants of the block's rows, visible after the k loop's first barrier
  if (!args.partial && grp == 0 && tid < BM && m0 + tid < args.M)
    epr[tid] = epi_row(args.E, m0 + tid + batch * args.E.pstride);

  LA la;
  LB lb;
  la.init(args.A, batch, m0, args.M, args.K, tid, kbeg);
  lb.init(args.B, batch, n0, args.N, args.K, tid, kbeg);

  floatx16 acc[TM][TN];
#pragma unroll
  for (int t = 0; t < TM; ++t)
#pragma unroll
    for (int u = 0; u < TN; ++u)
#pragma unroll
      for (int q = 0; q < 16; ++q) acc[t][u][q] = 0.f;

  const int nk = __builtin_amdgcn_readfirstlane(kbeg < kend ? (kend - kbeg + BK - 1) / BK : 0);
  bool halo_done = false;
  if constexpr (HALO) {
    if (args.B.halo) {
      // Tap-chunked conv1d with the halo B layout (LB::store_h): per channel chunk the x window
      // is loaded AND stored once; the chunk's three k-tiles (taps) read it at row shifts -1, 0,
      // +1 (a lane's B rows move by its clip's halo offset too), so taps 1 and 2 store only A.
      // A keeps its k-tile-parity stages; B has chunk-parity stages after them.
      const int T = args.B.R2;
      float* const bst0 = lds + 2 * LA::TILE;
      // zero rows of both B stages: rows c (T + 2) and c (T + 2) + T + 1 of every clip c
      {
        const int nclip = BN / T;
        for (int idx = tid; idx < 2 * nclip * 2 * LB::LDK; idx += 256) {
          const int col = idx % LB::LDK, q = idx / LB::LDK;
          const int which = q & 1, clip = (q >> 1) % nclip, stage = (q >> 1) / nclip;
          bst0[stage * LB::TILE_H + (clip * (T + 2) + (which ? T + 1 : 0)) * LB::LDK + col] = 0.f;
        }
      }
      const int brow = wn * (BN / 2) + li;          // this lane's B fragment row (TN = 1)
      const int bsh = 2 * (brow / T) + 1;           // its halo row offset at tap shift 0
      const int ntap = args.B.tapconv;              // 3 (host)
      int tap_i = (kbeg / BK) % ntap;               // tap / chunk parity of k-tile i
      int cpar = 0;
      auto bfrag = [&](int tap, int par) { return bst0 + par * LB::TILE_H + (bsh + tap - 1) * LB::LDK; };
      Frags<TM, TN, P, NS> f0, f1;
      if (nk > 0) {
        la.load(kbeg);
        lb.load(kbeg);
        la.store(lds);
        lb.store_h(bst0);
        if (nk > 1) {
          la.load(kbeg + BK);
          lb.load(kbeg + BK);
        }
      }
      __syncthreads();
      if (nk > 0) read_frags<BM, BN, TM, TN, P, NS, LA, LB>(lds, bfrag(tap_i, 0), 0, wm, wn, li, lh, f0);
      for (int i = 0; i < nk; ++i) {
        const float* cur = lds + (i & 1) * LA::TILE;
        float* nxt = lds + ((i + 1) & 1) * LA::TILE;
        const int tap_n = tap_i + 1 == ntap ? 0 : tap_i + 1;   // tile i + 1
        const int cpar_n = tap_n == 0 ? cpar ^ 1 : cpar;
        if (i + 1 < nk) {
          la.store(nxt);
          if (tap_n == 0) lb.store_h(bst0 + cpar_n * LB::TILE_H);
        }
        __builtin_amdgcn_sched_barrier(0);
        if (i + 2 < nk) {
          la.load(kbeg + (i + 2) * BK);
          lb.load(kbeg + (i + 2) * BK);
        }
        read_frags<BM, BN, TM, TN, P, NS, LA, LB>(cur, bfrag(tap_i, cpar), 1, wm, wn, li, lh, f1);
        mfma_half(f0, acc);
        __builtin_amdgcn_sched_barrier(0);
        constexpr int RD = 2 * NS * (TM + TN);
        __builtin_amdgcn_s_waitcnt(0xC07F | ((RD < 15 ? RD : 15) << 8));
        __builtin_amdgcn_s_barrier();
        __builtin_amdgcn_sched_barrier(0);
        mfma_part<0, 2>(f1, acc);
        __builtin_amdgcn_sched_barrier(0);
        read_frags<BM, BN, TM, TN, P, NS, LA, LB>(nxt, bfrag(tap_n, cpar_n), 0, wm, wn, li, lh, f0);
        __builtin_amdgcn_sched_barrier(0);
        mfma_part<2, 8 * NS>(f1, acc);
        tap_i = tap_n;
        cpar = cpar_n;
      }
      __syncthreads();  // the m-contiguous epilogue reuses the stages
      halo_done = true;
    }
  }
  if constexpr (KS == 1) {
   if (!halo_done) {
    Frags<TM, TN, P, NS> f0, f1;
    if (nk > 0) {
      la.load(kbeg);
      lb.load(kbeg);
      la.store(lds);
      lb.store(lds + LA::TILE);
      if (nk > 1) {
        la.load(kbeg + BK);
        lb.load(kbeg + BK);
      }
    }
    __syncthreads();
    if (nk > 0) read_frags<BM, BN, TM, TN, P, NS, LA, LB>(lds, lds + LA::TILE, 0, wm, wn, li, lh, f0);
    for (int i = 0; i < nk; ++i) {
      const float* cur = lds + (i & 1) * STAGE;
      float* nxt = lds + ((i + 1) & 1) * STAGE;
      if (i + 1 < nk) {
        la.store(nxt);
        lb.store(nxt + LA::TILE);
      }
      __builtin_amdgcn_sched_barrier(0);  // the tile stores stay ahead of the fragment reads
      if (A2M_ABLATE != 2 && i + 2 < nk) {
        la.load(kbeg + (i + 2) * BK);
        lb.load(kbeg + (i + 2) * BK);
      }
      read_frags<BM, BN, TM, TN, P, NS, LA, LB>(cur, cur + LA::TILE, 1, wm, wn, li, lh, f1);
      if (A2M_ABLATE != 1) mfma_half(f0, acc);
      else ablate_touch(f0, acc);
      // The step's barrier, pinned after the first half's MFMAs (left to itself the compiler
      // hoists it above them, and __syncthreads' fence would also wait for the second half's
      // fragment reads).  Only this wave's tile stores must have landed: LDS ops retire in
      // order, so the 2 (TM + TN) fragment reads issued after them may stay in flight (the
      // second half's MFMAs wait for them where they are used).  s_waitcnt simm16 on gfx950:
      // vmcnt / expcnt at their maxima (no wait), lgkmcnt in bits 11:8.
      __builtin_amdgcn_sched_barrier(0);
      constexpr int RD = P == 0 ? 2 * NS * (TM + TN) : 2 * (TM + TN);   // fragment reads after the stores
      __builtin_amdgcn_s_waitcnt(0xC07F | ((RD < 15 ? RD : 15) << 8));
      if (A2M_ABLATE != 3) __builtin_amdgcn_s_barrier();
      __builtin_amdgcn_sched_barrier(0);
      // the next tile's first fragments are read behind the first MFMAs of this second half
      // (issued right after the barrier they would be waited for before any MFMA: the compiler
      // cannot tell them apart from the second half's own reads in the LDS counter)
      constexpr int SPLIT = P == 1 ? 1 : 2;
      constexpr int NSUB = P == 0 ? 8 * NS : (P == 1 ? 2 : 6);
      if (A2M_ABLATE != 1) mfma_part<0, SPLIT>(f1, acc);
      __builtin_amdgcn_sched_barrier(0);
      // unconditional (after the last k-step the stale stage is read and never used): behind a
      // branch the compiler split these reads (b96 / b32 / read2 + moves, a wait inside the
      // MFMA cluster) and, not knowing how many were in flight after the join, waited for all
      // of them (lgkmcnt(0)) before this half's remaining MFMAs
      read_frags<BM, BN, TM, TN, P, NS, LA, LB>(nxt, nxt + LA::TILE, 0, wm, wn, li, lh, f0);
      __builtin_amdgcn_sched_barrier(0);
      if (A2M_ABLATE != 1) mfma_part<SPLIT, NSUB>(f1, acc);
      else ablate_touch(f1, acc);
    }
    __syncthreads();  // the m-contiguous epilogue reuses the stages
   }
  } else if constexpr (KS == 2) {
    // The groups take turns staging: group j % 2 loads k-tile j three steps ahead and stores it
    // one step ahead, so a tile's global loads have two k-steps to land (one with a single
    // staging group) at no extra registers.
    Frags<TM, TN, P, NS> f;
    if (nk > 0) {
      if (grp == 0) {
        la.load(kbeg);
        lb.load(kbeg);
        la.store(lds);
        lb.store(lds + LA::TILE);
        if (nk > 2) {
          la.load(kbeg + 2 * BK);
          lb.load(kbeg + 2 * BK);
        }
      } else if (nk > 1) {
        la.load(kbeg + BK);
        lb.load(kbeg + BK);
      }
    }
    __syncthreads();
    if (nk > 0) read_frags<BM, BN, TM, TN, P, NS, LA, LB>(lds, lds + LA::TILE, grp, wm, wn, li, lh, f);
    for (int i = 0; i < nk; ++i) {
      float* nxt = lds + ((i + 1) & 1) * STAGE;
      if (grp == ((i + 1) & 1)) {
        if (i + 1 < nk) {
          la.store(nxt);
          lb.store(nxt + LA::TILE);
        }
        if (A2M_ABLATE != 2 && i + 3 < nk) {
          la.load(kbeg + (i + 3) * BK);
          lb.load(kbeg + (i + 3) * BK);
        }
      }
      if (A2M_ABLATE != 1) mfma_half(f, acc);
      else ablate_touch(f, acc);
      if (A2M_ABLATE != 3) __syncthreads();
      read_frags<BM, BN, TM, TN, P, NS, LA, LB>(nxt, nxt + LA::TILE, grp, wm, wn, li, lh, f);
    }
    // sum the two groups' partial accumulators (group 1 -> LDS -> group 0)
    __syncthreads();
    constexpr int NQ = TM * TN * 16;
    if (grp == 1) {
#pragma unroll
      for (int t = 0; t < TM; ++t)
#pragma unroll
        for (int u = 0; u < TN; ++u)
#pragma unroll
          for (int q = 0; q < 16; ++q) lds[((t * TN + u) * 16 + q) * 256 + tid] = acc[t][u][q];
    }
    __syncthreads();
    if (grp == 0) {
#pragma unroll
      for (int t = 0; t < TM; ++t)
#pragma unroll
        for (int u = 0; u < TN; ++u)
#pragma unroll
          for (int q = 0; q < 16; ++q) acc[t][u][q] += lds[((t * TN + u) * 16 + q) * 256 + tid];
    }
    (void)NQ;
    __syncthreads();  // the partials region is free again
    if (grp == 1) {
      if (args.mcontig) __syncthreads();  // the epilogue's one barrier
      return;
    }
  }

  const bool slab_out = args.partial != nullptr;
  static_assert(BN * (BM + 1) <= 2 * STAGE, "C tile must fit the LDS stages");
  tile_epilogue<BM, BN, TM, TN>(args, acc, lds, epr, slab_out, zz, batch, m0, n0, tid, wm, wn, li, lh);
}

template <int BM, int BN, int BK, int MA, int MB, int P, int KS = 1>
__global__ __launch_bounds__(256 * KS) void gemm_kernel(GemmArgs args) {
  span_begin(args.ts);
  gemm_tile<BM, BN, BK, MA, MB, P, KS>(args);
  span_end(args.ts);
}


// Launch one tile configuration for the operand modes (ma, mb).  Instantiated per (tile, type)
// in its own translation unit (gemm_f32_64.hip, ...), so the 25 mode pairs compile in parallel.
template <int BM, int BN, int BK, int P, int KS = 1>
void launch_tile(const GemmArgs& a, int ma, int mb, int batch, hipStream_t st) {
  dim3 grid((unsigned)cdiv(a.N, BN), (unsigned)cdiv(a.M, BM), (unsigned)(batch * a.splits));
#define A2M_L(MA_, MB_) \
  if (ma == MA_ && mb == MB_) { hipLaunchKernelGGL((gemm_kernel<BM, BN, BK, MA_, MB_, P, KS>), grid, dim3(256 * KS), 0, st, a); return; }
  // (else-chained, so a wave-group variant instantiates only the mode pairs it serves)
  if constexpr (KS == 2) {  // dense (or channels-last conv, mode 6) operands only (gemm.hip)
    A2M_L(0, 0) A2M_L(0, 6)
  } else {
    A2M_L(0, 0) A2M_L(0, 1) A2M_L(0, 2) A2M_L(0, 3) A2M_L(0, 4)
    A2M_L(1, 0) A2M_L(1, 1) A2M_L(1, 2) A2M_L(1, 3) A2M_L(1, 4)
    A2M_L(2, 0) A2M_L(2, 1) A2M_L(2, 2) A2M_L(2, 3) A2M_L(2, 4)
    A2M_L(3, 0) A2M_L(3, 1) A2M_L(3, 2) A2M_L(3, 3) A2M_L(3, 4)
    A2M_L(4, 0) A2M_L(4, 1) A2M_L(4, 2) A2M_L(4, 3) A2M_L(4, 4)
    A2M_L(0, 5) A2M_L(0, 6)
  }
#undef A2M_L
}

extern template void launch_tile<64, 64, 32, 0>(const GemmArgs&, int, int, int, hipStream_t);
extern template void launch_tile<64, 64, 32, 0, 2>(const GemmArgs&, int, int, int, hipStream_t);
extern template void launch_tile<128, 128, 32, 0>(const GemmArgs&, int, int, int, hipStream_t);
extern template void launch_tile<64, 64, 64, 1>(const GemmArgs&, int, int, int, hipStream_t);
extern template void launch_tile<128, 128, 64, 1>(const GemmArgs&, int, int, int, hipStream_t);
extern template void launch_tile<64, 64, 32, 2>(const GemmArgs&, int, int, int, hipStream_t);
extern template void launch_tile<128, 128, 32, 2>(const GemmArgs&, int, int, int, hipStream_t);

}  // namespace a2m
