// Internal helpers shared by the a2m HIP translation units (not part of the C-ABI).
#pragma once
#include <hip/hip_runtime.h>

#include <cstdarg>
#include <cstdint>
#include <cstdio>
#include <string>

#include "../../include/a2m.h"

namespace a2m {

void set_error(const char* fmt, ...);

#define A2M_CHECK_ARG(cond, ...)                      \
  do {                                                \
    if (!(cond)) {                                    \
      ::a2m::set_error(__VA_ARGS__);                  \
      return A2M_EINVAL;                              \
    }                                                 \
  } while (0)

#define A2M_CHECK_HIP(expr)                                                     \
  do {                                                                          \
    hipError_t _e = (expr);                                                     \
    if (_e != hipSuccess) {                                                     \
      ::a2m::set_error("%s failed: %s", #expr, hipGetErrorString(_e));          \
      return A2M_EHIP;                                                          \
    }                                                                           \
  } while (0)

#define A2M_LAUNCH_CHECK()                                                      \
  do {                                                                          \
    hipError_t _e = hipGetLastError();                                          \
    if (_e != hipSuccess) {                                                     \
      ::a2m::set_error("kernel launch failed: %s", hipGetErrorString(_e));      \
      return A2M_EHIP;                                                          \
    }                                                                           \
  } while (0)

inline hipStream_t as_stream(void* s) { return reinterpret_cast<hipStream_t>(s); }

inline int64_t cdiv(int64_t a, int64_t b) { return (a + b - 1) / b; }

// ---------------------------------------------------------------------------------------
// Implicit-GEMM operand description.  Element (r, k) of an operand viewed as [R][K]:
//   r = (r0*R1 + r1)*R2 + r2          k = (k0*K1 + k1)*K2 + k2
//   h = r1*ar1 + k1*bk1 + ch          w = r2*ar2 + k2*bk2 + cw
//   valid iff h, w >= 0, h % divh == 0, w % divw == 0, h/divh < Lh, w/divw < Lw
//   value = base[z*bstride + r0*sr0 + k0*sk0 + (h/divh)*sh + (w/divw)*sw]   (0 if invalid)
// This one form covers dense row/col-major matrices, conv1d/conv2d im2col (forward),
// transposed-conv / dgrad gathers (div = stride) and wgrad operands.
// ---------------------------------------------------------------------------------------
struct Gather {
  const float* base;
  int64_t bstride;
  int sr0, sk0, sh, sw;
  int R1, R2, K1, K2;
  int ar1, ar2, bk1, bk2, ch, cw;
  int divh, divw, Lh, Lw;
  int kcontig;  // 1: consecutive k are (usually) adjacent in memory -> k-major thread map
  int nhwc;     // > 0: channels-last conv rows (loader mode 6), the channel count Ci (a multiple
                // of the k-tile): rows n = (r0 = image, r1 = output row, r2 = live output
                // column), k = (i, j, c) with K2 = kw taps per kernel row; pixel (r1*ar1 + ch + i,
                // r2*ar2 + cw + j) of an Lh x Lw image, sr0 = the image stride; every k-tile is
                // one tap's channel slice, a contiguous run
  int tapconv;  // > 0: stride-1 conv1d operand in tap-chunked k order (loader mode 5): k =
                // (chunk, tap, ci) with BK-channel chunks, rows n = b*R2 + t; the chunk's
                // x[b][c][t] window is loaded once and re-stored shifted for each of the
                // `tapconv` taps (sr0 = batch stride, sk0 = channel stride, cw = -pad)
  int halo;     // set by the engine (not the caller): mode 5 with 3 taps, pad 1, R2 >= 16 on the
                // fp32 64x64 one-group tile stores the window once with zero rows around each
                // clip and reads each tap at a row shift (gemm_kernel.h, TileLoader::store_h)
};

inline Gather dense_rk(const float* p, int ld, int64_t bstride = 0) {  // [R][K] row-major, ld >= K
  Gather g{};
  g.base = p; g.bstride = bstride; g.sr0 = ld; g.sk0 = 1;
  g.R1 = g.R2 = g.K1 = g.K2 = 1; g.divh = g.divw = 1; g.Lh = g.Lw = 1; g.kcontig = 1;
  return g;
}
inline Gather dense_kr(const float* p, int ld, int64_t bstride = 0) {  // [K][R] (r contiguous)
  Gather g = dense_rk(p, 1, bstride);
  g.sr0 = 1; g.sk0 = ld; g.kcontig = 0;
  return g;
}

// Output / epilogue: C[m][n] -> out[z*bstride + n0*so0 + n1*so1 + n2*so2 + m*som],
// n = (n0*N1 + n1)*N2 + n2.  v = acc (+bias[m]); BN-eval affine; activation;
// (grouped launches: problem z reads bias / BN entry m + z*pstride)
// v = v*gamma[0] (if gamma); v += res1[addr] + res2[addr] (same addressing as out).
enum Act { ACT_NONE = 0, ACT_RELU = 1, ACT_LRELU = 2, ACT_SIGMOID = 3 };

struct Epilogue {
  float* out;
  int64_t bstride;
  int so0, so1, so2, som;
  int N1, N2;
  const float* bias;
  const float* bn_w; const float* bn_b; const float* bn_rm; const float* bn_rv;
  float bn_eps;
  int act;
  float slope;
  const float* gamma;
  const float* res1; const float* res2;
  int accumulate;  // 1: out += v
  int pstride;     // grouped launches: bias / BN arrays of problem z start at z * pstride
  // > 0: the AudioEncoder's last conv with its bilinear time resample fused into the split-K
  // reduce (gemm.hip splitk_reduce_interp_kernel): C[m][n], n = b * interp_H + h, is one live
  // output column of weight interp_lw0, and out is y[b][m][t] with t < interp_T
  int interp_T, interp_H;
  float interp_lw0;
};

inline Epilogue epi_dense(float* out, int ldn, int64_t bstride = 0) {  // out[m][n], ld = ldn
  Epilogue e{};
  e.out = out; e.bstride = bstride; e.so0 = 1; e.so1 = 0; e.so2 = 0; e.som = ldn;
  e.N1 = e.N2 = 1; e.bn_eps = 1e-5f; e.slope = 0.2f;
  return e;
}

// Runs C = A . B^T-style implicit GEMM: C[m][n] = sum_k A(m,k) * B(n,k), over `batch`
// independent problems (grid z), with optional split-K through workspace `ws`.
// k-tile depth of the engine at the current precision (the chunk of tap-chunked conv weights)
int gemm_k_tile();
int gemm(const Gather& A, const Gather& B, const Epilogue& E, int M, int N, int K, int batch,
         void* ws, size_t ws_bytes, hipStream_t stream, int force_split = 0);
size_t gemm_ws_bytes(int M, int N, int K, int batch);

// shared host-side launch helpers (defined next to their kernels)
int softmax_rows(float* x, int rows, int n, hipStream_t st);                       // ops.hip
int stack_qkv(const float* wq, const float* bq, const float* wk, const float* bk,  // ops.hip
              const float* wv, const float* bv, int C, float* wcat, float* bcat, hipStream_t st);
// Output segments of reduce_cols: column j goes to out[i][j - start[i]] for the last i with
// start[i] <= j (start[0] = 0, n <= 4).
struct ColOuts {
  float* out[4];
  int start[4];
  int n;
};
int reduce_cols(const float* part, int rows, int stride, int cols, float* out,     // train_norm.hip
                int accumulate, hipStream_t st);
int reduce_cols(const float* part, int rows, int stride, int cols, const ColOuts& outs,
                int accumulate, hipStream_t st);                                  // train_norm.hip

inline Gather gather_bct(const float* x, int64_t bs, int cs, int T) {  // rows n=(b,t), k=c of [B][C][T]
  Gather g{};
  g.base = x; g.sr0 = (int)bs; g.R1 = 1; g.R2 = T; g.ar2 = 1; g.sw = 1; g.Lw = T;
  g.sk0 = cs; g.K1 = 1; g.K2 = 1; g.Lh = 1; g.divh = g.divw = 1; g.kcontig = 0;
  return g;
}

// ---------------------------------------------------------------------------------------
// Wave reductions.  __shfl_xor lowers to ds_bpermute (an LDS round trip per step, each
// waited for); within a 16-lane row the DPP forms below are register-to-register.  After
// xor1 + xor2 every lane of a quad holds the quad's value, so the mirror patterns (which pair
// lane i with 7-i / 15-i) combine whole groups exactly like xor 4 / xor 8 would.
// ---------------------------------------------------------------------------------------
template <int CTRL>
__device__ __forceinline__ float dpp_f(float v) {
  return __int_as_float(__builtin_amdgcn_mov_dpp(__float_as_int(v), CTRL, 0xF, 0xF, true));
}
constexpr int DPP_XOR1 = 0xB1, DPP_XOR2 = 0x4E, DPP_HALF_MIRROR = 0x141, DPP_MIRROR = 0x140;

__device__ __forceinline__ float quad_sum(float v) {
  v += dpp_f<DPP_XOR1>(v);
  return v + dpp_f<DPP_XOR2>(v);
}
__device__ __forceinline__ float quad_max(float v) {
  v = fmaxf(v, dpp_f<DPP_XOR1>(v));
  return fmaxf(v, dpp_f<DPP_XOR2>(v));
}
__device__ __forceinline__ float row16_sum(float v) {
  v = quad_sum(v);
  v += dpp_f<DPP_HALF_MIRROR>(v);
  return v + dpp_f<DPP_MIRROR>(v);
}
__device__ __forceinline__ float row16_max(float v) {
  v = quad_max(v);
  v = fmaxf(v, dpp_f<DPP_HALF_MIRROR>(v));
  return fmaxf(v, dpp_f<DPP_MIRROR>(v));
}
// sum over the 32 lanes of each wave half: lanes l and l^16 combined by v_permlane16_swap (gfx950:
// exchanges 16-lane rows 0<->1 and 2<->3 in VALU, no LDS round trip), so r[0] + r[1] is v_l + v_{l^16}
// on every lane (the same two addends in either order: bit-identical to a shuffle)
__device__ __forceinline__ float half32_sum(float v) {
  v = row16_sum(v);
  const auto r = __builtin_amdgcn_permlane16_swap(__float_as_uint(v), __float_as_uint(v), false, false);
  return __uint_as_float(r[0]) + __uint_as_float(r[1]);
}
__device__ __forceinline__ float wave64_sum(float v) {
  v = half32_sum(v);
  const auto r = __builtin_amdgcn_permlane32_swap(__float_as_uint(v), __float_as_uint(v), false, false);
  return __uint_as_float(r[0]) + __uint_as_float(r[1]);
}
__device__ __forceinline__ float wave64_max(float v) {
  v = row16_max(v);
  v = fmaxf(v, __shfl_xor(v, 16));
  return fmaxf(v, __shfl_xor(v, 32));
}

// Fused attention core for T <= 64, C/8 <= 64 (attn_core.hip).
bool attn_core_fits(int C, int T);
bool attn_core_wide_fits(int C, int T);
int attn_core_wide(const float* qkv, int64_t qs_b, int B, int C, int T, const float* gamma,
                   const float* x, int64_t x_bs, const float* res, float* y, float* attn_out,
                   hipStream_t st);
int attn_core(const float* qkv, int64_t qs_b, int B, int C, int T, const float* gamma,
              const float* x, int64_t x_bs, const float* res, float* y, float* attn_out,
              hipStream_t st);
// Eval-only QKV + attention in one launch (C in {128, 256}, T <= 64, T % 4 == 0).
bool attn_fused_eval_fits(int C, int T);
// G > 1: G problems with their own weights (wqkv / bqkv / gamma stacked per problem) over
// x + g*x_gs, res + g*res_gs, y + g*y_gs (grouped decoder branches)
// wqkv_h (bf16 mode only, may be null): wqkv rounded to bf16 (a2m_to_bf16_f32), staged as is
int attn_fused_eval(const float* x, int64_t x_bs, int B, int C, int T, const float* wqkv,
                    const float* bqkv, const float* gamma, const float* res, float* y,
                    hipStream_t st, int G = 1, int64_t x_gs = 0, int64_t res_gs = 0, int64_t y_gs = 0,
                    const void* wqkv_h = nullptr);

}  // namespace a2m
