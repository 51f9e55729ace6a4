// Implicit-GEMM engine: host side (operand modes, planner, split-K reduce, launch, timing).
// The kernels and their description are in gemm_kernel.h.
#include <algorithm>
#include <cstdlib>
#include <mutex>
#include <vector>

#include "gemm_kernel.h"
#include "gemm_pipe_bf16.h"

namespace a2m {

// Fixed-order (s = 0, 1, ...) sum of the split-K slabs + epilogue.  Slabs are [M][N], or
// [N][M] for m-contiguous outputs (args.mcontig), so the inner slab index is also the output's
// contiguous one.  Four consecutive inner elements per thread (float4) when the inner extent
// is a multiple of 4, and the slab loads of four splits are issued before their adds, so the
// pass is bandwidth- rather than latency-bound.
__device__ __forceinline__ void reduce_store(const GemmArgs& args, int z, float v, int o, int in) {
  const int m = args.mcontig ? in : o, n = args.mcontig ? o : in;
  epi_store(args.E, z, v, m, epi_addr(args.E, m, n));
}

// Four consecutive inner elements (in .. in+3) of output row / column o: the epilogue
// constants and the column decomposition are computed once per float4 (mcontig: one column n,
// rows in..in+3; otherwise one row m, columns in..in+3).
__device__ __forceinline__ void reduce_store4(const GemmArgs& args, int z, const float4& v, int o, int in) {
  const Epilogue& E = args.E;
  const float vv[4] = {v.x, v.y, v.z, v.w};
  if (args.mcontig) {
    EpiCol c;
    c.set(E, o);
    const int64_t an = c.addr(E);
    const int64_t off = (int64_t)z * E.bstride + an + in;
    const int mp = in + z * E.pstride;
    auto al16 = [](const void* q) { return (reinterpret_cast<uintptr_t>(q) & 15) == 0; };
    if (E.som == 1 && !E.res1 && !E.res2 && !E.gamma && al16(E.out + off) && (!E.bias || al16(E.bias + mp)) &&
        (!E.bn_w || (al16(E.bn_w + mp) && al16(E.bn_b + mp) && al16(E.bn_rm + mp) && al16(E.bn_rv + mp)))) {
      // four consecutive channels of one output position: vector parameter loads and store
      float4 bi = make_float4(0.f, 0.f, 0.f, 0.f), w = bi, b = bi, rm = bi, rv = bi;
      if (E.bias) bi = *reinterpret_cast<const float4*>(E.bias + mp);
      if (E.bn_w) {
        w = *reinterpret_cast<const float4*>(E.bn_w + mp);
        b = *reinterpret_cast<const float4*>(E.bn_b + mp);
        rm = *reinterpret_cast<const float4*>(E.bn_rm + mp);
        rv = *reinterpret_cast<const float4*>(E.bn_rv + mp);
      }
      const float bia[4] = {bi.x, bi.y, bi.z, bi.w}, wa[4] = {w.x, w.y, w.z, w.w};
      const float ba[4] = {b.x, b.y, b.z, b.w}, rma[4] = {rm.x, rm.y, rm.z, rm.w};
      const float rva[4] = {rv.x, rv.y, rv.z, rv.w};
      float o4[4];
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        const EpiRow r{bia[j], rma[j], E.bn_w ? wa[j] / sqrtf(rva[j] + E.bn_eps) : 1.f, ba[j]};
        o4[j] = epi_value_p(E, vv[j], r);
      }
      float4 out4 = make_float4(o4[0], o4[1], o4[2], o4[3]);
      if (E.accumulate) {
        const float4 q = *reinterpret_cast<const float4*>(E.out + off);
        out4.x += q.x; out4.y += q.y; out4.z += q.z; out4.w += q.w;
      }
      *reinterpret_cast<float4*>(E.out + off) = out4;
      return;
    }
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      const int m = in + j;
      epi_store_p(E, z, vv[j], epi_row(E, m + z * E.pstride), an + (int64_t)m * E.som);
    }
  } else {
    const EpiRow r = epi_row(E, o + z * E.pstride);
    const int64_t am = (int64_t)o * E.som;
    EpiCol c;
    c.set(E, in);
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      if (j) c.advance(E, 1);
      epi_store_p(E, z, vv[j], r, c.addr(E) + am);
    }
  }
}

template <typename I>
__device__ __forceinline__ void splitk_reduce4(const GemmArgs& args, int batch) {
  const I MN = (I)args.M * args.N;
  const int S = args.splits;
  const I inner = args.mcontig ? args.M : args.N;
  const I total4 = MN * batch / 4;
  for (I i = blockIdx.x * (I)blockDim.x + threadIdx.x; i < total4; i += (I)gridDim.x * blockDim.x) {
    const I e = i * 4;
    const int z = (int)(e / MN);
    const I mn = e - (I)z * MN;
    const int o = (int)(mn / inner), in = (int)(mn - (I)o * inner);
    const float* p = args.partial + (int64_t)z * S * MN + mn;
    float4 v = make_float4(0.f, 0.f, 0.f, 0.f);
    int s = 0;
    for (; s + 4 <= S; s += 4) {
      const float4 a0 = *reinterpret_cast<const float4*>(p + (int64_t)(s + 0) * MN);
      const float4 a1 = *reinterpret_cast<const float4*>(p + (int64_t)(s + 1) * MN);
      const float4 a2 = *reinterpret_cast<const float4*>(p + (int64_t)(s + 2) * MN);
      const float4 a3 = *reinterpret_cast<const float4*>(p + (int64_t)(s + 3) * MN);
      v.x += a0.x; v.y += a0.y; v.z += a0.z; v.w += a0.w;
      v.x += a1.x; v.y += a1.y; v.z += a1.z; v.w += a1.w;
      v.x += a2.x; v.y += a2.y; v.z += a2.z; v.w += a2.w;
      v.x += a3.x; v.y += a3.y; v.z += a3.z; v.w += a3.w;
    }
    for (; s < S; ++s) {
      const float4 a = *reinterpret_cast<const float4*>(p + (int64_t)s * MN);
      v.x += a.x; v.y += a.y; v.z += a.z; v.w += a.w;
    }
    reduce_store4(args, z, v, o, in);
  }
}

__device__ __forceinline__ void splitk_reduce(const GemmArgs& args, int batch) {
  const int64_t MN = (int64_t)args.M * args.N;
  const int S = args.splits;
  const int inner = args.mcontig ? args.M : args.N;
  if ((inner & 3) == 0) {
    // 32-bit index arithmetic whenever the slab set fits (the 64-bit divisions cost more than
    // the float4 loads they address)
    if (MN * batch < (int64_t)1 << 31) splitk_reduce4<int>(args, batch);
    else splitk_reduce4<int64_t>(args, batch);
    return;
  }
  const int64_t total = MN * batch;
  for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < total;
       i += (int64_t)gridDim.x * blockDim.x) {
    const int z = (int)(i / MN);
    const int64_t mn = i - (int64_t)z * MN;
    const int o = (int)(mn / inner), in = (int)(mn - (int64_t)o * inner);
    const float* p = args.partial + (int64_t)z * S * MN + mn;
    float v = 0.f;
    for (int s = 0; s < S; ++s) v += p[s * MN];
    reduce_store(args, z, v, o, in);
  }
}

// the reduce's span stamps follow the tile kernel's in the launch's record
__device__ __forceinline__ unsigned long long* reduce_span(const GemmArgs& args) {
  return args.ts ? args.ts + kSpanSlots : nullptr;
}

__global__ void splitk_reduce_kernel(GemmArgs args, int batch) {
  span_begin(reduce_span(args));
  splitk_reduce(args, batch);
  span_end(reduce_span(args));
}

// Many splits over few outputs (graph-layer weight gradients: 64 x 64 outputs, K up to 172,032
// nodes, 128-256 splits): the per-thread serial sum above would be latency-bound on a handful of
// blocks, so here 16 lanes of a block share one float4 of outputs, each summing the splits
// s = lane, lane + 16, ... in order, and the 16 lane sums are added in lane order (a fixed order:
// still bitwise reproducible).  Inner extent a multiple of 4.
constexpr int RW_LANES = 16, RW_COLS = 16;
__device__ __forceinline__ void splitk_reduce_wide(const GemmArgs& args, int batch) {
  __shared__ float4 red[RW_LANES][RW_COLS];
  const int64_t MN = (int64_t)args.M * args.N;
  const int S = args.splits;
  const int inner = args.mcontig ? args.M : args.N;
  const int col = threadIdx.x % RW_COLS, lane = threadIdx.x / RW_COLS;
  const int64_t i = (int64_t)blockIdx.x * RW_COLS + col;
  const int64_t total4 = MN * batch / 4;
  const int64_t e = i * 4;
  const int z = (int)(e / MN);
  const int64_t mn = e - (int64_t)z * MN;
  float4 v = make_float4(0.f, 0.f, 0.f, 0.f);
  if (i < total4) {
    const float* p = args.partial + (int64_t)z * S * MN + mn;
    int s = lane;
    for (; s + 3 * RW_LANES < S; s += 4 * RW_LANES) {
      const float4 a0 = *reinterpret_cast<const float4*>(p + (int64_t)s * MN);
      const float4 a1 = *reinterpret_cast<const float4*>(p + (int64_t)(s + RW_LANES) * MN);
      const float4 a2 = *reinterpret_cast<const float4*>(p + (int64_t)(s + 2 * RW_LANES) * MN);
      const float4 a3 = *reinterpret_cast<const float4*>(p + (int64_t)(s + 3 * RW_LANES) * MN);
      v.x += a0.x; v.y += a0.y; v.z += a0.z; v.w += a0.w;
      v.x += a1.x; v.y += a1.y; v.z += a1.z; v.w += a1.w;
      v.x += a2.x; v.y += a2.y; v.z += a2.z; v.w += a2.w;
      v.x += a3.x; v.y += a3.y; v.z += a3.z; v.w += a3.w;
    }
    for (; s < S; s += RW_LANES) {
      const float4 a = *reinterpret_cast<const float4*>(p + (int64_t)s * MN);
      v.x += a.x; v.y += a.y; v.z += a.z; v.w += a.w;
    }
  }
  red[lane][col] = v;
  __syncthreads();
  if (lane != 0 || i >= total4) return;
  for (int l = 1; l < RW_LANES; ++l) {
    const float4 a = red[l][col];
    v.x += a.x; v.y += a.y; v.z += a.z; v.w += a.w;
  }
  const int o = (int)(mn / inner), in = (int)(mn - (int64_t)o * inner);
  reduce_store4(args, z, v, o, in);
}

__global__ __launch_bounds__(RW_LANES * RW_COLS) void splitk_reduce_wide_kernel(GemmArgs args,
                                                                               int batch) {
  span_begin(reduce_span(args));
  splitk_reduce_wide(args, batch);
  span_end(reduce_span(args));
}

// The AudioEncoder's last conv (one live output column, model_layers.py:272) with the
// bilinear time resample (model_layers.py:277-279) fused into its split-K reduce: phase 1 sums
// the slabs of RB whole (m, b) rows of H values in fixed order s = 0, 1, ... (the order of
// splitk_reduce_kernel, or splitk_reduce_wide_kernel's where the unfused path would use that
// kernel) and applies the epilogue into LDS; phase 2 writes those rows' T
// outputs y[b][m][t] from the LDS rows with exactly interp_time_at's operations (ops.hip), so
// the result is the unfused conv + interp_time_kernel's bit for bit, without the [B][Co][H][W]
// round trip and the second launch.  Slabs are [M][N], n = b * H + h (rows (m, b) contiguous).
__global__ __launch_bounds__(256) void splitk_reduce_interp_kernel(GemmArgs args, int nb, int RB, int wide) {
  span_begin(reduce_span(args));
  extern __shared__ float sv[];   // [RB][H]
  const Epilogue& E = args.E;
  const int H = E.interp_H, T = E.interp_T, M = args.M, S = args.splits;
  const int64_t MN = (int64_t)M * args.N;
  const int rows = M * nb;
  const int r0 = blockIdx.x * RB;
  const int nr = min(RB, rows - r0);
  for (int e = threadIdx.x; e < nr * H; e += blockDim.x) {
    const float* p = args.partial + (int64_t)r0 * H + e;   // row r0 + e / H, h = e % H
    float v = 0.f;
    if (wide) {
      // the order of splitk_reduce_wide_kernel (which the unfused path uses at these sizes):
      // RW_LANES strided partial sums, then added in lane order
      for (int l = 0; l < RW_LANES; ++l) {
        float vl = 0.f;
        for (int s = l; s < S; s += RW_LANES) vl += p[s * MN];
        if (l == 0) v = vl;
        else v += vl;
      }
    } else {
      int s = 0;
      for (; s + 4 <= S; s += 4) {
        const float a0 = p[(s + 0) * MN], a1 = p[(s + 1) * MN], a2 = p[(s + 2) * MN], a3 = p[(s + 3) * MN];
        v += a0; v += a1; v += a2; v += a3;
      }
      for (; s < S; ++s) v += p[s * MN];
    }
    const int m = (r0 + e / H) / nb;
    sv[e] = epi_value_p(E, v, epi_row(E, m));
  }
  __syncthreads();
  const float sh = (float)H / (float)T, lw0 = E.interp_lw0;
  for (int o = threadIdx.x; o < nr * T; o += blockDim.x) {
    const int rl = o / T, t = o - rl * T;
    const int r = r0 + rl, m = r / nb, b = r - m * nb;
    float src = sh * ((float)t + 0.5f) - 0.5f;
    src = src < 0.f ? 0.f : src;
    const int h0 = (int)src;
    const int h1 = h0 + (h0 < H - 1 ? 1 : 0);
    const float lh1 = src - (float)h0, lh0 = 1.f - lh1;
    float v = lh0 * (lw0 * sv[rl * H + h0]);
    if (lh1 != 0.f) v += lh1 * (lw0 * sv[rl * H + h1]);
    E.out[((int64_t)b * M + m) * T + t] = v;
  }
  span_end(reduce_span(args));
}

static int env_int(const char* name, int dflt) {
  const char* v = std::getenv(name);
  return v ? std::atoi(v) : dflt;
}

static int operand_mode(const Gather& g, int K) {
  if (g.tapconv > 0) return 5;
  if (g.nhwc > 0) return 6;
  if (!g.kcontig) {
    // rows 4-at-a-time contiguous: plain [K][R] (rows via r0, unit stride), or stride-1 im2col
    // rows along w (R2 % 4 == 0) or along h (R2 == 1, R1 % 4 == 0), unit element stride
    const bool plain = g.R1 == 1 && g.R2 == 1 && g.sr0 == 1;
    const bool along_w = g.R2 > 1 && g.R2 % 4 == 0 && (g.ar2 == 1 || g.ar2 == 2) && g.sw == 1 &&
                         g.divw == 1;
    const bool along_h = g.R2 == 1 && g.R1 > 1 && g.R1 % 4 == 0 && (g.ar1 == 1 || g.ar1 == 2) &&
                         g.sh == 1 && g.divh == 1;
    return plain || along_w || along_h ? 3 : 2;
  }
  const bool dense = g.K1 == 1 && g.K2 == 1 && g.sk0 == 1 && g.Lh == 1 && g.Lw == 1 &&
                     g.sh == 0 && g.sw == 0 && g.ch == 0 && g.cw == 0 && g.divh == 1 && g.divw == 1;
  const bool aligned = (reinterpret_cast<uintptr_t>(g.base) % 16 == 0) && (g.sr0 % 4 == 0) &&
                       (g.bstride % 4 == 0) && (K % 4 == 0);
  if (dense && aligned) return 0;
  const bool runs = g.K2 % 4 == 0 && g.bk2 == 1 && g.sw == 1 && g.divw == 1;
  return runs ? 4 : 1;
}

struct Plan {
  int bm, bk, splits, kchunk;
};

// fixed cost of a split-K reduce launch in the planner's model (us)
#ifndef A2M_RED_FIXED_US
#define A2M_RED_FIXED_US 3.0
#endif
#ifndef A2M_RED_FIXED_US_BF16
#define A2M_RED_FIXED_US_BF16 6.0
#endif

// Tile / split-K choice by a cost model fitted to measured sweeps of the engine on MI355X
// (tools/gemm_tune.py; DESIGN.md "GEMM planner").  For each candidate (tile, splits):
//   blocks = tiles * splits, per_cu = ceil(blocks / 256) (the busiest CU), c = min(per_cu,
//   resident blocks per CU: 4 at 64x64, 2 at 128x128 -- LDS-bound),
//   t = per_cu * block_flops / thr(tile, c) + ceil(per_cu / occ) * t_fixed(tile) + t_launch
//       + (splits > 1 ? (splits + 1) * M * N * 4 B / 3.5 TB/s + 3 us : 0)   (the slab reduce)
// thr is the per-CU fp32 MFMA throughput measured at c co-resident blocks; a row-gathered
// operand (modes 2/3: transposed LDS staging) costs the 64x64 tile ~16 % of throughput and
// the 128x128 tile ~6 us more per round of blocks.  The model is
// deterministic in (M, N, K, batch, gathered), so a shape always gets the same plan and the
// same (bitwise-reproducible) split order.  a2m_gemm_plan_override and A2M_GEMM_PLAN_RULES
// (per-shape "M,N,K:tile:splits;...") override it (experiments).
// Operand precision of the engine: 0 = fp32 (v_mfma_f32_32x32x2_f32, BK 32; the default and
// the parity configuration), 1 = bf16 (operands rounded to bf16 in LDS, fp32 accumulation,
// BK 64; a2m_set_gemm_precision, configs[4]), 2 = bf16x6 (fp32 operands split exactly into
// three bf16 planes in LDS, the six products of order >= 2^-16 on v_mfma_f32_32x32x16_bf16 with
// fp32 accumulation: fp32-class accuracy at 16/6 of the f32 MFMA rate; BK 32).
// (BK = 16 measured slower end to end.)
static int g_gemm_prec = 0;
// (fp32 at BK = 64 -- fewer barriers per MFMA -- measured 10-20 % slower on every G shape:
// the k-loop's non-MFMA cost scales with the staged bytes, not with the barrier count;
// profiles/r02_gemm_ablation.txt)
static int gemm_bk(int prec) { return prec == 1 ? 64 : 32; }
int gemm_k_tile() { return gemm_bk(g_gemm_prec); }

// XCD-aware block order: groups of 8 M-tiles share an XCD's L2 (40 MB a launch instead of ~64 MB
// at a 0.5 % step cost; identity order and groups of 2 / 4 measured within noise)
static int gemm_xcd_group() { return 8; }

static int g_override_tile = 0, g_override_split = 0;   // a2m_gemm_plan_override (tuning)
static int g_pipe_override = -1;   // a2m_gemm_pipe_override: -1 default (pipelined), 0 gemm_tile, 1 pipelined

struct PlanRule {
  int M, N, K, tile, splits;
};
static const PlanRule* plan_rule(int M, int N, int K) {
  static const std::vector<PlanRule> rules = [] {
    std::vector<PlanRule> v;
    const char* e = std::getenv("A2M_GEMM_PLAN_RULES");
    while (e && *e) {
      PlanRule r{};
      int used = 0;
      if (std::sscanf(e, "%d,%d,%d:%d:%d%n", &r.M, &r.N, &r.K, &r.tile, &r.splits, &used) != 5) break;
      if ((r.tile == 0 || r.tile == 64 || r.tile == 128) && r.splits >= 0 && r.splits <= 256) v.push_back(r);
      else std::fprintf(stderr, "a2m: A2M_GEMM_PLAN_RULES entry %d,%d,%d:%d:%d ignored (tile 0/64/128, splits 0..256)\n",
                        r.M, r.N, r.K, r.tile, r.splits);
      e += used;
      while (*e == ';' || *e == ' ') ++e;
    }
    return v;
  }();
  for (const PlanRule& r : rules)
    if (r.M == M && r.N == N && r.K == K) return &r;
  return nullptr;
}

// (Rounds 4-5 kept a table of seven fp32 plans tuned in the replayed bench step -- 64x64 tiles
// with 2 splits on the UNet's large tap convs, 1 split on the hand stack's proj_out.  With the
// round-6 kernels the planner's own choices measured faster: 2.245 vs 2.228 ms and 2.473 vs
// 2.448 ms, three interleaved rounds on each of two boxes, training neutral
// (profiles/r06_r_tuned_plans_ab.txt); the table is gone.)

// bf16 (prec 1) throughput per CU by resident blocks, flop / us: staging- and latency-bound
// rather than MFMA-bound (16x the f32 MFMA rate), so it grows with the blocks a CU holds far more
// than the f32 tile's (kflop / us per CU by resident blocks: 64x64 at 1..4, 128x128 at 1 / 2)
static double bf16_thr(int tile, int c) {
  // fitted in the replayed bf16 bench step (r05 sweeps, two interleaved rounds each: 1.658 ms
  // against 1.831 ms with round 4's 4 x the f32 table, {1360, 1712, 1740, 1760, 1856, 2000}e3,
  // at {530, 750, 900, 1060, 1500, 2000}e3; refitted with the bf16 pipelined tile, whose 64x64
  // launches run faster: 1.416-1.422 ms against 1.447-1.449)
  static constexpr double t[6] = {600e3, 850e3, 1000e3, 1150e3, 1500e3, 2000e3};
  return tile == 128 ? t[4 + (c > 1)] : t[std::min(std::max(c, 1), 4) - 1];
}

static double plan_cost_us(int M, int N, int K, int batch, bool gathered, int tile, int kchunk,
                           int splits, int prec, bool conv_rows = false) {
  static const double thr64[4] = {340e3, 428e3, 435e3, 440e3};   // flop / us per CU
  static const double thr128[2] = {464e3, 500e3};
  // bf16x6 (fitted to a plan sweep of the G forward's shapes, tools/sweep_summary.py): three
  // bf16 planes per operand halve the resident blocks (LDS: 61 KB at 64x64, 120 KB at
  // 128x128) and the 128x128 tile gains most from the faster MFMA
  static const double x6_thr64[2] = {272e3, 342e3};
  static const double x6_thr128[1] = {557e3};
  const int occ = prec == 2 ? (tile == 128 ? 1 : 2) : (tile == 128 ? 2 : 4);
  const int64_t tiles = cdiv(M, tile) * cdiv(N, tile) * (int64_t)batch;
  const int64_t per_cu = cdiv(tiles * splits, 256);
  const int c = (int)std::min<int64_t>(per_cu, occ);
  double thr = prec == 2 ? (tile == 128 ? x6_thr128[c - 1] : x6_thr64[c - 1])
                         : (tile == 128 ? thr128[c - 1] : thr64[c - 1]);
#ifndef A2M_THR64_SCALE
#define A2M_THR64_SCALE 1.0   // diagnostic: the 64x64 tile's fitted throughput scaled
#endif
#ifndef A2M_GATHER_F
#define A2M_GATHER_F 0.84
#endif
  if (prec == 0 && tile == 64) thr *= A2M_THR64_SCALE;
  if (gathered && tile == 64) thr *= A2M_GATHER_F;
  // (channels-last conv rows, mode 6, run at the dense fit on the one-group 64x64 tile: a 0.87
  // factor measured slower, encoder 303.2 vs 300.0 us, tools/enc_plan_ab.py, round 3)
#ifndef A2M_BF16_THR128_SCALE
#define A2M_BF16_THR128_SCALE 1.0   // diagnostic: the bf16 128x128 tile's fitted throughput scaled
#endif
  if (prec == 1) thr = bf16_thr(tile, c) * (gathered && tile == 64 ? 0.84 : 1.0) * (tile == 128 ? A2M_BF16_THR128_SCALE : 1.0);
  const double block_flops = 2.0 * tile * tile * (double)kchunk;
  const double fixed = prec == 2 ? (tile == 128 ? 15.0 : 2.0)
                                 : (tile == 128 ? (gathered ? 16.0 : 10.0) : 3.0);
  double t = per_cu * block_flops / thr + cdiv(per_cu, occ) * fixed + 4.0;
  // (the reduce term scaled by 0.6 / 1.5 / 2 measured slower in-step, round 2: it is right as fitted)
  constexpr double red_scale = 1.0;
  // channels-last conv rows (the encoder): the reduce priced at A2M_GEMM_SPLIT_COST_ROWS
  // (default 200 %), so its launches take fewer splits (conv2: 3 instead of 4).  With every
  // launch's reduce at 200 % the encoder measured 0.2906-0.2937 vs 0.2951-0.2971 ms but the step
  // neutral to slightly slower (three rounds); on the encoder's launches only: in-step
  // path_frac 0.480-0.484 vs 0.473-0.476, step 2.718-2.727 vs 2.721-2.737 ms (four rounds, r04s)
#ifndef A2M_RED_SCALE_ROWS
#define A2M_RED_SCALE_ROWS 2.0
#endif
  constexpr double red_scale_rows = A2M_RED_SCALE_ROWS;
  if (splits > 1)
    t += (conv_rows ? red_scale_rows : red_scale) *
         ((splits + 1.0) * M * N * (double)batch * 4.0 / 3.5e6 + (prec == 1 ? A2M_RED_FIXED_US_BF16 : A2M_RED_FIXED_US));
  return t;
}

static Plan plan_for(int M, int N, int K, int batch, bool gathered, int prec, int kquant = 1,
                     bool conv_rows = false, bool pipe64 = false) {
  const int force_tile = g_override_tile;     // a2m_gemm_plan_override (tuning sweeps)
  const int force_split = g_override_split;
  const int BK = gemm_bk(prec);
  const int KQ = BK * kquant;   // split boundaries on whole k-tile groups (mode 5: all taps of a chunk)
  static const int cand_splits[] = {1, 2, 3, 4, 6, 8, 12, 16, 24, 32, 48, 64, 96, 128, 192, 256};
  Plan p{64, BK, 1, (int)(cdiv(std::max(K, 1), KQ) * KQ)};
  double best = 1e300;
  for (int tile : {64, 128}) {
    if (force_tile && tile != force_tile) continue;
    // operands the fp32 pipelined 64x64 tile takes: the cost table is gemm_tile's, which the
    // pipelined tile outruns -- kept to 64 (training iteration 66.0 -> 64.5 ms, r05_n)
    if (!force_tile && pipe64 && tile != 64) continue;
    for (int s : cand_splits) {
      if (force_split && s != force_split) continue;
      const int kchunk = (int)(cdiv(cdiv(std::max(K, 1), s), KQ) * KQ);
      const int se = (int)cdiv(std::max(K, 1), kchunk);
      if (!force_split && se > 1 && kchunk < 128) continue;
      if (se != s && s > 1 && !force_split) continue;   // the same plan at a smaller s
      const double t = plan_cost_us(M, N, K, batch, gathered, tile, kchunk, se, prec, conv_rows);
      if (t < best) {
        best = t;
        p.bm = tile;
        p.kchunk = kchunk;
        p.splits = se;
      }
    }
  }
  if (force_split && best == 1e300) {   // a forced split outside the candidate list
    p.bm = force_tile ? force_tile : 64;
    p.kchunk = (int)(cdiv(cdiv(std::max(K, 1), force_split), KQ) * KQ);
    p.splits = (int)cdiv(std::max(K, 1), p.kchunk);
  }
  return p;
}

// slab workspace of a split plan: [splits][batch][M][N] for the reduce kernel
static size_t split_ws_bytes(const Plan& p, int M, int N, int batch) {
  return (size_t)p.splits * batch * M * (size_t)N * sizeof(float);
}

// the plan gemm() launches: the planner's, unless an A2M_GEMM_PLAN_RULES rule fixes the tile /
// split count for the shape
static Plan launch_plan(int M, int N, int K, int batch, bool gathered, int prec, int kquant, bool rows6,
                        int force_split, bool pipe64 = false) {
  Plan p = plan_for(M, N, K, batch, gathered, prec, kquant, rows6, pipe64);
  if (force_split > 0) {
    p.kchunk = (int)(cdiv(cdiv(K, force_split), p.bk * kquant) * p.bk * kquant);
    p.splits = (int)cdiv(K, p.kchunk);
  }
  if (const PlanRule* r = plan_rule(M, N, K)) {
    if (r->tile) p.bm = r->tile;
    if (r->splits > 0) {
      p.kchunk = (int)(cdiv(cdiv(K, r->splits), p.bk * kquant) * p.bk * kquant);
      p.splits = (int)cdiv(K, p.kchunk);
    }
  }
  if (K == 0) { p.splits = 1; p.kchunk = p.bk; }
  return p;
}

size_t gemm_ws_bytes(int M, int N, int K, int batch) {
  // every plan gemm() may launch for the shape: either operand orientation (the plan depends on
  // whether an operand is row-gathered), either precision, conv rows or not, the tap-chunk
  // quantum of a tap-chunked conv (1-3 taps), and the tuned / rule overrides
  size_t need = 0;
  for (bool gathered : {false, true})
    for (int prec : {0, 1, 2})
      for (bool rows6 : {false, true})
        for (int kq : {1, 2, 3})
          for (bool p64 : {false, true}) {
            const Plan p = launch_plan(M, N, K, batch, gathered, prec, kq, rows6, 0, p64);
            if (p.splits > 1) need = std::max(need, split_ws_bytes(p, M, N, batch));
          }
  return need;
}

// Optional per-launch timing of the engine (bench.py's live roofline).  While enabled, every
// launch gets a record of four span stamps in a device buffer (GemmArgs::ts): the tile kernel's
// earliest block start / latest wave end and the split-K reduce's, on the GPU's constant-rate
// wall clock (span_begin / span_end, gemm_kernel.h).  The stamps are written by the kernels
// themselves, so they time the same launches eagerly and in every replay of a graph captured
// while timing was on (bench.py's in-step roofline: the step captured once more, replayed, read
// after each replay).  HIP event records were tried first: inside a graph they become
// separate nodes whose timestamps include each kernel's dispatch (+3.5 us a launch against the
// rocprof kernel trace, r04_v1), and hipExtLaunchKernel's kernel-timestamp events are not
// updated under capture (tools/micro/ext_events.hip).  Off by default, no cost when off.
struct GemmTiming {
  double flops;
  bool reduce;
  char desc[96];   // shape/plan, printed per launch by a2m_gemm_timing_read under A2M_GEMM_LOG=2
};
constexpr int kTimingRecs = 1024;   // launches per timing window
static std::mutex g_timing_mu;
static bool g_timing = false;
static bool g_timing_overflow = false;
static std::vector<GemmTiming> g_timing_recs;
// tile spans + reduce spans + the launch's ready mark (and a pad slot; A2M_GEMM_TIMING_READY=1):
// the wall clock at which a one-thread mark kernel, enqueued right before the tile kernel on its
// stream, ran -- i.e.
// when the stream reached the launch (its previous kernel done), so last end - ready counts the
// launch's dispatch and any wait for free CUs behind the other decoder branch, as a kernel
// trace's duration does
constexpr int kRecSlots = 2 * kSpanSlots + 2;
constexpr int kReadySlot = 2 * kSpanSlots;
static unsigned long long* g_ts = nullptr;   // [kTimingRecs][kRecSlots] + [A2M_TIMING_MARKS] mark slots
static double g_wall_mhz = 0.0;

// (re)arm the stamps: start slots at the maximum, end slots at 0
static int timing_reset_stamps() {
  std::vector<unsigned long long> init((size_t)kTimingRecs * kRecSlots, 0ull);
  for (size_t i = 0; i < init.size(); i += 2) init[i] = ~0ull;
  return hipMemcpy(g_ts, init.data(), init.size() * sizeof(unsigned long long), hipMemcpyHostToDevice) ==
         hipSuccess ? A2M_OK : A2M_EHIP;
}

__global__ void timing_mark_kernel(unsigned long long* p) {
  if (threadIdx.x == 0) *p = (unsigned long long)wall_clock64();
}

static int timing_alloc() {
  if (g_ts) return A2M_OK;
  int dev = 0, khz = 0;
  if (hipGetDevice(&dev) != hipSuccess ||
      hipDeviceGetAttribute(&khz, hipDeviceAttributeWallClockRate, dev) != hipSuccess || khz <= 0 ||
      hipMalloc(&g_ts, ((size_t)kTimingRecs * kRecSlots + A2M_TIMING_MARKS) * sizeof(unsigned long long)) != hipSuccess) {
    set_error("gemm timing: device stamp buffer / wall clock rate unavailable");
    g_ts = nullptr;
    return A2M_EHIP;
  }
  g_wall_mhz = khz / 1e3;
  return hipMemset(g_ts, 0, ((size_t)kTimingRecs * kRecSlots + A2M_TIMING_MARKS) * sizeof(unsigned long long)) ==
         hipSuccess ? A2M_OK : A2M_EHIP;
}

static unsigned long long* timing_open(double flops, const char* desc) {
  std::lock_guard<std::mutex> lk(g_timing_mu);
  if (!g_timing || !g_ts) return nullptr;
  if ((int)g_timing_recs.size() >= kTimingRecs) {
    g_timing_overflow = true;
    return nullptr;
  }
  GemmTiming t{};
  t.flops = flops;
  std::snprintf(t.desc, sizeof(t.desc), "%s", desc);
  g_timing_recs.push_back(t);
  return g_ts + kRecSlots * (g_timing_recs.size() - 1);
}

int gemm(const Gather& A, const Gather& B, const Epilogue& E, int M, int N, int K, int batch,
         void* ws, size_t ws_bytes, hipStream_t stream, int force_split) {
  A2M_CHECK_ARG(M > 0 && N > 0 && K >= 0 && batch > 0, "gemm: bad sizes M=%d N=%d K=%d batch=%d",
                M, N, K, batch);
  GemmArgs a;
  a.A = A; a.B = B; a.E = E; a.M = M; a.N = N; a.K = K;
  const int ma = operand_mode(A, K), mb = operand_mode(B, K);
  const int prec = g_gemm_prec;
  const int kquant = mb == 5 ? B.tapconv : 1;
  // gathered: row-vector staging (modes 2 / 3) or gathers; k-contiguous conv rows (mode 6) load
  // like dense rows
  // software-pipelined one-wave-per-SIMD tile (gemm_pipe.h; a2m_gemm_pipe_override(0) restores
  // gemm_tile): fp32 64x64, dense weights x dense rows / channels-last rows / halo tap conv, every
  // element offset below 2^29 floats (raw buffer loads)
  const int pipe_on = g_pipe_override >= 0 ? g_pipe_override : 1;
  auto below = [](int64_t v) { return v >= 0 && v < ((int64_t)1 << 29); };
  bool pipe_ext = below((int64_t)(M - 1) * A.sr0 + K);
  if (mb == 0) pipe_ext = pipe_ext && below((int64_t)(N - 1) * B.sr0 + K);
  else if (mb == 6) pipe_ext = pipe_ext && below((int64_t)((N - 1) / (B.R1 * B.R2)) * B.sr0 + (int64_t)B.Lh * B.Lw * B.nhwc);
  else if (mb == 5) pipe_ext = pipe_ext && below((int64_t)((N - 1) / B.R2) * B.sr0 + B.R2 + (int64_t)(K / B.tapconv) * B.sk0);
  else if (mb == 3) pipe_ext = pipe_ext && below((int64_t)((N - 1) / B.R2) * B.sr0 + B.R2 + (int64_t)K * B.sk0);
  // mode 3 in its plain form only: k = channel, rows (b, t) at unit stride in groups of 4
  const bool rows3 = mb == 3 && B.K1 == 1 && B.K2 == 1 && B.R1 == 1 && B.ch == 0 && B.cw == 0 &&
                     B.divh == 1 && B.divw == 1 && N % 4 == 0 &&
                     ((B.R2 == 1 && B.sr0 == 1) || (B.R2 % 4 == 0 && B.ar2 == 1 && B.sw == 1 && B.Lw >= B.R2));
  // mode 4 on both sides (the 1-D conv weight gradients): one k digit (K1 = 1) in runs of a
  // multiple of 4, every split a whole number of k-tiles, offsets below 2^29
  auto runs4 = [&](const Gather& g, int R) {
    const int64_t rmax = (int64_t)((R - 1) / (g.R1 * g.R2)) * g.sr0 +
                         (int64_t)std::max(0, g.Lh - 1) * std::abs(g.sh) + g.Lw + (int64_t)(K / g.K2) * g.sk0;
    return g.K1 == 1 && g.K2 % 4 == 0 && g.bk2 == 1 && g.sw == 1 && g.divh == 1 && g.divw == 1 &&
           g.sr0 >= 0 && g.sk0 >= 0 && below(rmax);
  };
  // ... and B as stride-2 runs (a stride-2 conv's input: gemm_tile gathers it, mode 1)
  const bool runs_s2 = mb == 1 && B.K1 == 1 && B.K2 % 4 == 0 && B.bk2 == 2 && B.sw == 1 && B.divh == 1 &&
                       B.divw == 1 && B.sr0 >= 0 && B.sk0 >= 0 &&
                       below((int64_t)((N - 1) / (B.R1 * B.R2)) * B.sr0 + (int64_t)std::max(0, B.Lh - 1) * std::abs(B.sh) +
                             B.Lw + (int64_t)(K / B.K2) * B.sk0);
  const bool m4_ok = ma == 4 && runs4(A, M) && ((mb == 4 && runs4(B, N)) || runs_s2);
  // A as a plain [K][M] operand (mode 3: rows at unit stride, loaded 4 at a time) with B dense or
  // plain mode 3 (the weight gradients of the linears / graph layers)
  const bool plainA3 = ma == 3 && A.K1 == 1 && A.K2 == 1 && A.R1 == 1 && A.R2 == 1 && A.sr0 == 1 && A.ch == 0 &&
                       A.cw == 0 && A.divh == 1 && A.divw == 1 && M % 4 == 0 && A.sk0 >= 0 &&
                       below((int64_t)(M - 1) + (int64_t)K * A.sk0);
  const bool pipe_a3 = plainA3 &&
                       ((mb == 0 && below((int64_t)(N - 1) * B.sr0 + K)) ||
                        (rows3 && below((int64_t)((N - 1) / B.R2) * B.sr0 + B.R2 + (int64_t)K * B.sk0)));
  // the operand modes the fp32 pipelined tile takes (at a 64-row tile)
  const bool tap5 = mb == 5 && B.tapconv >= 1 && B.tapconv <= 3 && B.R2 % 4 == 0 && 64 % B.R2 == 0;
  const bool pipe_modes = (ma == 0 && (mb == 0 || mb == 6 || rows3 || tap5) && pipe_ext) || m4_ok || pipe_a3;
  // launches the pipelined tile takes are planned on 64x64 tiles: fp32 every such launch, bf16 its
  // training modes (mode-4 / plain mode-3 A: bf16 B=32 training kernel time 43.0 -> 41.7 ms a step,
  // r05_p; the bf16 planner table was refitted on the inference launches with its pipelined tile)
  const Plan p = launch_plan(M, N, K, batch, ma == 2 || ma == 3 || mb == 2 || (mb >= 3 && mb != 6), prec,
                             kquant, mb == 6, force_split,
                             pipe_on && ((prec == 0 && pipe_modes) || (prec == 1 && (m4_ok || pipe_a3))));
  // A2M_GEMM_HALO=0: mode 5 re-stores the window shifted for every tap (the round-3 loader)
  static const int halo_on = env_int("A2M_GEMM_HALO", 1);
  a.B.halo = halo_on && mb == 5 && prec == 0 && p.bm == 64 && B.tapconv == 3 &&
             B.cw == -1 && B.R2 >= 16 && 64 % B.R2 == 0;
  a.splits = p.splits;
  a.kchunk = p.kchunk;
  a.partial = nullptr;
  a.xcd_group = gemm_xcd_group();
  // fused resample (E.interp_T): the tile always writes raw slabs (also at one split) and the
  // reduce kernel runs epilogue + resample
  const bool interp = E.interp_T > 0;
  A2M_CHECK_ARG(!interp || (batch == 1 && E.interp_H > 0 && N % E.interp_H == 0 &&
                            (size_t)E.interp_H * sizeof(float) <= 32768),
                "gemm: fused resample needs batch 1, N a multiple of H = %d <= 8192", E.interp_H);
  a.mcontig = E.som == 1 && M > 1 && !interp;
  // float4 output rows (pipelined tile): n contiguous within 4-aligned groups of one n2 run, every
  // other stride and base 16-byte aligned; split-K slabs ([M][N]) whenever N % 4 == 0
  auto al16 = [](const void* q) { return (reinterpret_cast<uintptr_t>(q) & 15) == 0; };
  const bool slab_out = p.splits > 1 || interp;
  // the innermost index that varies with n: n2 (N2 > 1), else n1 (N1 > 1), else n0
  const int in_lvl = E.N2 > 1 ? 2 : (E.N1 > 1 ? 1 : 0);
  const int in_stride = in_lvl == 2 ? E.so2 : (in_lvl == 1 ? E.so1 : E.so0);
  const int in_len = in_lvl == 2 ? E.N2 : (in_lvl == 1 ? E.N1 : 4);
  const bool outer4 = (in_lvl == 0 || E.so0 % 4 == 0) && (in_lvl != 2 || E.N1 == 1 || E.so1 % 4 == 0) &&
                      E.som % 4 == 0 && E.bstride % 4 == 0;
  a.vec4 = !a.mcontig && N % 4 == 0 &&
           (slab_out || (in_stride == 1 && in_len % 4 == 0 && outer4 && al16(E.out) &&
                         (!E.res1 || al16(E.res1)) && (!E.res2 || al16(E.res2))));
  const bool pipe_m4 = m4_ok && p.kchunk % 32 == 0;
  const bool pipe_launch = pipe_on && prec == 0 && p.bm == 64 &&
                           ((ma == 0 && (mb == 0 || mb == 6 || rows3 || (mb == 5 && (a.B.halo || tap5))) && pipe_ext) ||
                            pipe_m4 || pipe_a3);
  // the bf16-operand pipelined tile (gemm_pipe_bf16.h): the same operand modes, 64-channel
  // k-tiles (mode 6: Ci % 64 == 0), no halo layout (mode 5 takes the per-tap stores)
  // (and, as the fp32 tile, mode-4 runs on both sides -- runs of a multiple of its 64-k tile --
  // and plain [K][M] A operands)
  const bool pipe_bf16 = pipe_on && prec == 1 && p.bm == 64 &&
                         ((ma == 0 && (mb == 0 || (mb == 6 && B.nhwc % 64 == 0) || rows3 ||
                                       (mb == 5 && B.tapconv >= 1 && B.tapconv <= 3 && B.R2 % 4 == 0 && 64 % B.R2 == 0)) &&
                           pipe_ext) ||
                          (m4_ok && p.kchunk % 64 == 0) || pipe_a3);
  // ... and its halo layout for the 3-tap pad-1 convs over clips of T >= 16 (the window stored
  // once per chunk instead of once per tap); gemm_tile's bf16 tile takes the per-tap stores
  if (pipe_bf16 && halo_on && mb == 5 && B.tapconv == 3 && B.cw == -1 && B.R2 >= 16 && 64 % B.R2 == 0)
    a.B.halo = 1;
  if (p.splits > 1 || interp) {
    const size_t need = split_ws_bytes(p, M, N, batch);
    if (ws == nullptr || ws_bytes < need) {
      set_error("gemm: workspace too small (%zu < %zu bytes)", ws_bytes, need);
      return A2M_EWS;
    }
    a.partial = static_cast<float*>(ws);
  }
  static const int log_launches = env_int("A2M_GEMM_LOG", 0);
  if (log_launches)
    std::fprintf(stderr, "a2m gemm M=%d N=%d K=%d batch=%d tile=%d bk=%d splits=%d%s modes=%d,%d som=%d so=%d,%d,%d N12=%d,%d\n",
                 M, N, K, batch, p.bm, p.bk, p.splits, pipe_launch || pipe_bf16 ? " (pipe)" : "", ma, mb, E.som, E.so0, E.so1,
                 E.so2, E.N1, E.N2);
  a.ts = nullptr;
  if (g_timing) {
    char desc[96];
    std::snprintf(desc, sizeof(desc), "M=%d N=%d K=%d b=%d tile=%d split=%d modes=%d,%d", M, N, K,
                  batch, p.bm, p.splits, ma, mb);
    a.ts = timing_open(2.0 * M * N * (double)K * batch, desc);
    if (a.ts) {
      g_timing_recs.back().reduce = p.splits > 1 || interp;
      // A2M_GEMM_TIMING_READY=1 (diagnostic): the ready mark.  Off by default: the extra kernel
      // per launch shifts how the two decoder branches share the CUs (tools/stamp_vs_trace.py)
      static const int ready = env_int("A2M_GEMM_TIMING_READY", 0);
      if (ready) hipLaunchKernelGGL(timing_mark_kernel, dim3(1), dim3(64), 0, stream, a.ts + kReadySlot);
    }
  }
  if (prec == 1) {
    if (pipe_bf16) launch_pipe_bf16(a, ma, mb, batch, stream);
    else if (p.bm == 128) launch_tile<128, 128, 64, 1>(a, ma, mb, batch, stream);
    else launch_tile<64, 64, 64, 1>(a, ma, mb, batch, stream);
#ifdef A2M_WITH_X6
  } else if (prec == 2) {
    if (p.bm == 128) launch_tile<128, 128, 32, 2>(a, ma, mb, batch, stream);
    else launch_tile<64, 64, 32, 2>(a, ma, mb, batch, stream);
#endif
  } else {
    if (pipe_launch) launch_pipe(a, ma, mb, batch, stream);
    else if (p.bm == 128) launch_tile<128, 128, 32, 0>(a, ma, mb, batch, stream);
    // two wave groups per 64x64 tile pay off for dense operands (measured -9 % on the decoder
    // convs after im2col); with gathered operands (modes 1-4) they measured slower end to end
    // (also for channels-last conv rows, mode 6, the encoder measured 305.8 us against 303.2
    // without, tools/enc_plan_ab.py, four interleaved rounds)
    else if (ma == 0 && mb == 0) launch_tile<64, 64, 32, 0, 2>(a, ma, mb, batch, stream);
    else launch_tile<64, 64, 32, 0>(a, ma, mb, batch, stream);
  }
  A2M_LAUNCH_CHECK();
  if (interp) {
    const int H = E.interp_H, nb = N / H;
    // whole (m, b) rows per block: ~2,048 outputs, the rows' H values staged in LDS
    const int RB = std::max(1, std::min(2048 / std::max(E.interp_T, 1), 8192 / H));
    const int wide = (N & 3) == 0 && p.splits >= 2 * RW_LANES && (int64_t)M * N / 4 <= 65536;
    hipLaunchKernelGGL(splitk_reduce_interp_kernel, dim3((unsigned)cdiv((int64_t)M * nb, RB)), dim3(256),
                       (size_t)RB * H * sizeof(float), stream, a, nb, RB, wide);
    A2M_LAUNCH_CHECK();
  } else if (p.splits > 1) {
    const int inner = a.mcontig ? M : N;
    const int64_t total = (int64_t)M * N * batch / ((inner & 3) == 0 ? 4 : 1);
    if ((inner & 3) == 0 && p.splits >= 2 * RW_LANES && total <= 65536) {
      hipLaunchKernelGGL(splitk_reduce_wide_kernel, dim3((unsigned)cdiv(total, RW_COLS)),
                         dim3(RW_LANES * RW_COLS), 0, stream, a, batch);
    } else {
      const int blocks = (int)std::min<int64_t>(cdiv(total, 256), 8192);
      hipLaunchKernelGGL(splitk_reduce_kernel, dim3(blocks), dim3(256), 0, stream, a, batch);
    }
    A2M_LAUNCH_CHECK();
  }
  return A2M_OK;
}

}  // namespace a2m

extern "C" {

int a2m_gemm_plan_override(int32_t tile, int32_t splits) {
  A2M_CHECK_ARG((tile == 0 || tile == 64 || tile == 128) && splits >= 0 && splits <= 256,
                "gemm_plan_override: tile %d splits %d", tile, splits);
  a2m::g_override_tile = tile;
  a2m::g_override_split = splits;
  return A2M_OK;
}

int a2m_gemm_pipe_override(int32_t mode) {
  A2M_CHECK_ARG(mode >= -1 && mode <= 1, "gemm_pipe_override: %d (-1 env, 0 off, 1 on)", mode);
  a2m::g_pipe_override = mode;
  return A2M_OK;
}

int a2m_set_gemm_precision(int32_t prec) {
#ifdef A2M_WITH_X6
  A2M_CHECK_ARG(prec >= 0 && prec <= 2, "set_gemm_precision: %d (0 = fp32, 1 = bf16, 2 = bf16x6)", prec);
#else
  // bf16x6 (2) is a build-time option (make EXTRA=-DA2M_WITH_X6): an experiment that measured
  // slower than fp32 end to end, so the shipped library carries fp32 and bf16 only
  A2M_CHECK_ARG(prec >= 0 && prec <= 1, "set_gemm_precision: %d (0 = fp32, 1 = bf16)", prec);
#endif
  a2m::g_gemm_prec = prec;
  return A2M_OK;
}

int32_t a2m_get_gemm_precision(void) { return a2m::g_gemm_prec; }

int a2m_gemm_timing_begin(void) {
  std::lock_guard<std::mutex> lk(a2m::g_timing_mu);
  int rc = a2m::timing_alloc();
  if (rc == A2M_OK) rc = a2m::timing_reset_stamps();
  if (rc != A2M_OK) return rc;
  a2m::g_timing_recs.clear();
  a2m::g_timing_overflow = false;
  a2m::g_timing = true;
  return A2M_OK;
}

int a2m_gemm_timing_stop(void) {
  std::lock_guard<std::mutex> lk(a2m::g_timing_mu);
  a2m::g_timing = false;
  return A2M_OK;
}

int a2m_gemm_timing_read(int64_t* launches, double* flops, double* ms_tile, double* ms_reduce,
                         int64_t* reduces) {
  return a2m_gemm_timing_read_ex(launches, flops, ms_tile, ms_reduce, reduces, nullptr);
}

int a2m_gemm_timing_read_ex(int64_t* launches, double* flops, double* ms_tile, double* ms_reduce,
                            int64_t* reduces, double* ms_queued) {
  std::lock_guard<std::mutex> lk(a2m::g_timing_mu);
  A2M_CHECK_ARG(a2m::g_ts != nullptr, "gemm_timing_read: timing was never begun");
  A2M_CHECK_ARG(!a2m::g_timing_overflow, "gemm_timing_read: more than %d launches in the window",
                a2m::kTimingRecs);
  const size_t nrec = a2m::g_timing_recs.size();
  const int R = a2m::kRecSlots, S = a2m::kSpanSlots;
  std::vector<unsigned long long> st(nrec * R + 1);
  if (hipDeviceSynchronize() != hipSuccess ||
      (nrec && hipMemcpy(st.data(), a2m::g_ts, nrec * R * sizeof(unsigned long long), hipMemcpyDeviceToHost) !=
                   hipSuccess)) {
    a2m::set_error("gemm timing: stamp read failed");
    return A2M_EHIP;
  }
  // a kernel's duration: last block end - first block start over all XCDs (s_memrealtime is the
  // chip's one constant-rate clock, so stamps from different XCDs are comparable: the same
  // assumption as ms_queued and a2m_timing_mark_to_launch_end); -1: nothing stamped since the
  // last reset.  *global is that interval, the return value too (kept for the log line).
  auto span = [](const unsigned long long* s, double* global) {
    double best = -1.0;
    unsigned long long glo = ~0ull, ghi = 0;
    for (int x = 0; x < 8; ++x) {
      unsigned long long lo = ~0ull, hi = 0;
      for (int l = 0; l < a2m::kSpanLanes; ++l) {
        const unsigned long long* q = s + 2 * (x * a2m::kSpanLanes + l);
        if (q[0] == ~0ull || q[1] < q[0]) continue;
        lo = std::min(lo, q[0]);
        hi = std::max(hi, q[1]);
      }
      if (lo == ~0ull) continue;
      best = std::max(best, (double)(hi - lo));
      glo = std::min(glo, lo);
      ghi = std::max(ghi, hi);
    }
    *global = ghi >= glo ? (double)(ghi - glo) : -1.0;
    return best < 0 ? -1.0 : *global;
  };
  int64_t n = 0, nr = 0;
  double f = 0, mt = 0, mr = 0, mq = 0;
  int rc = A2M_OK;
  const double tick_ms = 1.0 / (a2m::g_wall_mhz * 1e3);
  for (size_t i = 0; i < nrec; ++i) {
    const a2m::GemmTiming& t = a2m::g_timing_recs[i];
    double ga = 0, gb = 0;
    const double sa = span(&st[i * R], &ga), sb = t.reduce ? span(&st[i * R + S], &gb) : 0.0;
    if (sa < 0 || sb < 0) {
      a2m::set_error("gemm timing: launch %zu (%s) has no stamps", i, t.desc);
      rc = A2M_EHIP;
      continue;
    }
    const double a = sa * tick_ms, b = sb * tick_ms;
    // ready mark .. last block end over all XCDs (the constant-rate clock is common to them)
    const unsigned long long rdy = st[i * R + a2m::kReadySlot];
    if (ms_queued && rdy != ~0ull && ga >= 0) {
      unsigned long long hi = 0;
      for (int q = 1; q < S; q += 2)
        if (st[i * R + q - 1] != ~0ull && st[i * R + q] >= st[i * R + q - 1]) hi = std::max(hi, st[i * R + q]);
      mq += hi > rdy ? (double)(hi - rdy) * tick_ms : a;
    }
    ++n;
    f += t.flops;
    static const int log_launches = a2m::env_int("A2M_GEMM_LOG", 0);
    if (log_launches >= 2)
      std::fprintf(stderr, "a2m gemm-time %s tile %.1f us (all-XCD span %.1f) reduce %.1f us %.1f TF\n", t.desc,
                   1e3 * a, 1e3 * ga * tick_ms, 1e3 * b, a > 0 ? t.flops / (1e9 * a) : 0.0);
    mt += a;
    if (t.reduce) { mr += b; ++nr; }
  }
  if (launches) *launches = n;
  if (flops) *flops = f;
  if (ms_tile) *ms_tile = mt;
  if (ms_reduce) *ms_reduce = mr;
  if (reduces) *reduces = nr;
  if (ms_queued) *ms_queued = mq;
  // re-arm for the next replay of a graph that carries these launches
  if (a2m::timing_reset_stamps() != A2M_OK) {
    a2m::set_error("gemm timing: stamp reset failed");
    return A2M_EHIP;
  }
  return rc;
}

int a2m_gemm_timing_read_spans(int64_t cap, double* start_us, double* end_us, int64_t* n) {
  return a2m_gemm_timing_read_spans_ex(cap, nullptr, start_us, end_us, n);
}

int a2m_gemm_timing_read_spans_ex(int64_t cap, double* ready_us, double* start_us, double* end_us,
                                  int64_t* n) {
  std::lock_guard<std::mutex> lk(a2m::g_timing_mu);
  A2M_CHECK_ARG(a2m::g_ts != nullptr && start_us && end_us && n && cap >= 0,
                "gemm_timing_read_spans: bad arguments (or timing never begun)");
  const size_t nrec = std::min<size_t>(a2m::g_timing_recs.size(), (size_t)cap);
  const int R = a2m::kRecSlots;
  std::vector<unsigned long long> st(nrec * R + 1);
  if (hipDeviceSynchronize() != hipSuccess ||
      (nrec && hipMemcpy(st.data(), a2m::g_ts, nrec * R * sizeof(unsigned long long), hipMemcpyDeviceToHost) !=
                   hipSuccess)) {
    a2m::set_error("gemm timing: stamp read failed");
    return A2M_EHIP;
  }
  for (size_t i = 0; i < nrec; ++i) {
    unsigned long long lo = ~0ull, hi = 0;
    for (int s = 0; s < a2m::kSpanSlots; s += 2) {
      const unsigned long long* q = &st[i * R + s];
      if (q[0] == ~0ull || q[1] < q[0]) continue;
      lo = std::min(lo, q[0]);
      hi = std::max(hi, q[1]);
    }
    start_us[i] = lo == ~0ull ? -1.0 : (double)lo / a2m::g_wall_mhz;
    end_us[i] = lo == ~0ull ? -1.0 : (double)hi / a2m::g_wall_mhz;
    if (ready_us) {
      const unsigned long long r = st[i * R + a2m::kReadySlot];
      ready_us[i] = r == ~0ull ? -1.0 : (double)r / a2m::g_wall_mhz;
    }
  }
  *n = (int64_t)nrec;
  return a2m::timing_reset_stamps() == A2M_OK ? A2M_OK : A2M_EHIP;
}

int a2m_gemm_timing_end(int64_t* launches, double* flops, double* ms_tile, double* ms_reduce,
                        int64_t* reduces) {
  a2m_gemm_timing_stop();
  const int rc = a2m_gemm_timing_read(launches, flops, ms_tile, ms_reduce, reduces);
  std::lock_guard<std::mutex> lk(a2m::g_timing_mu);
  a2m::g_timing_recs.clear();
  return rc;
}

int a2m_gemm_timing_clear(void) {
  std::lock_guard<std::mutex> lk(a2m::g_timing_mu);
  a2m::g_timing = false;
  a2m::g_timing_recs.clear();
  return A2M_OK;
}

// Named wall-clock marks (bench.py's in-step phase split: step start, log-mel done, encoder
// done): a one-thread kernel stores the clock into the mark's slot, so a mark captured into a
// graph re-stamps on every replay.  Its own dispatch is ~1-2 us of the interval it opens.
int a2m_timing_mark(int32_t slot, void* stream) {
  A2M_CHECK_ARG(slot >= 0 && slot < A2M_TIMING_MARKS, "timing_mark: slot %d", slot);
  if (!a2m::g_ts) {   // allocate the stamp buffer here unless the stream is being captured
    hipStreamCaptureStatus cs = hipStreamCaptureStatusNone;
    A2M_CHECK_ARG(hipStreamIsCapturing(static_cast<hipStream_t>(stream), &cs) == hipSuccess &&
                      cs == hipStreamCaptureStatusNone,
                  "timing_mark: first mark inside a stream capture (call a2m_gemm_timing_begin first)");
    std::lock_guard<std::mutex> lk(a2m::g_timing_mu);
    const int rc = a2m::timing_alloc();
    if (rc != A2M_OK) return rc;
  }
  hipLaunchKernelGGL(a2m::timing_mark_kernel, dim3(1), dim3(64), 0, static_cast<hipStream_t>(stream),
                     a2m::g_ts + (size_t)a2m::kTimingRecs * a2m::kRecSlots + slot);
  A2M_LAUNCH_CHECK();
  return A2M_OK;
}

int a2m_timing_mark_elapsed(int32_t a, int32_t b, float* ms) {
  A2M_CHECK_ARG(a >= 0 && a < A2M_TIMING_MARKS && b >= 0 && b < A2M_TIMING_MARKS && a2m::g_ts && ms,
                "timing_mark_elapsed: slots %d, %d", a, b);
  unsigned long long m[A2M_TIMING_MARKS];
  if (hipDeviceSynchronize() != hipSuccess ||
      hipMemcpy(m, a2m::g_ts + (size_t)a2m::kTimingRecs * a2m::kRecSlots, sizeof(m), hipMemcpyDeviceToHost) != hipSuccess) {
    a2m::set_error("timing_mark_elapsed: stamp read failed");
    return A2M_EHIP;
  }
  *ms = (float)((double)((long long)(m[b] - m[a])) / (a2m::g_wall_mhz * 1e3));
  return A2M_OK;
}

int a2m_timing_mark_to_launch_end(int32_t slot, int64_t rec, float* ms) {
  std::lock_guard<std::mutex> lk(a2m::g_timing_mu);
  A2M_CHECK_ARG(slot >= 0 && slot < A2M_TIMING_MARKS && a2m::g_ts && ms && rec >= 0 &&
                    rec < (int64_t)a2m::g_timing_recs.size(),
                "timing_mark_to_launch_end: slot %d, record %lld", slot, (long long)rec);
  const int R = a2m::kRecSlots;
  std::vector<unsigned long long> st(R);
  unsigned long long m[A2M_TIMING_MARKS];
  if (hipDeviceSynchronize() != hipSuccess ||
      hipMemcpy(st.data(), a2m::g_ts + (size_t)rec * R, R * sizeof(unsigned long long), hipMemcpyDeviceToHost) != hipSuccess ||
      hipMemcpy(m, a2m::g_ts + (size_t)a2m::kTimingRecs * R, sizeof(m), hipMemcpyDeviceToHost) != hipSuccess) {
    a2m::set_error("timing_mark_to_launch_end: stamp read failed");
    return A2M_EHIP;
  }
  unsigned long long hi = 0;
  for (int q = 0; q < 2 * a2m::kSpanSlots; q += 2)   // tile and reduce slots
    if (st[q] != ~0ull && st[q + 1] >= st[q]) hi = std::max(hi, st[q + 1]);
  A2M_CHECK_ARG(hi > 0, "timing_mark_to_launch_end: record %lld has no stamps", (long long)rec);
  *ms = (float)((double)((long long)(hi - m[slot])) / (a2m::g_wall_mhz * 1e3));
  return A2M_OK;
}

}  // extern "C"
