// Log-mel front end (replaces pose_video/mel_features.py:192-223).
//
// One workgroup (256 threads) per analysis frame:
//   1. coalesced load of the frame's `window` samples (frame :21-45, no padding, hop stride),
//      multiplied by the periodic Hann window (:48-68), packed as a complex sequence
//      z[n] = xw[2n] + i xw[2n+1] of length M = fft_len/2 (zero-padded past the window);
//   2. Stockham autosort FFT of size M in LDS (radix-4 stages, one radix-2 stage when
//      log2 M is odd), twiddles from the plan's table exp(-2 pi i t / fft_len);
//   3. real-FFT split: X[k] = Ze[k] + W^k Zo[k], k = 0..M, magnitude |X[k]| (:71-92);
//   4. banded mel filterbank (CSR, <= a few dozen taps per band, built on the host in
//      float64 exactly as spectrogram_to_mel_matrix :114-189 does) and log(mel + offset).
// HBM traffic per frame: the window (mostly L2 hits for overlapping frames) + n_mels*4 B.
#include <algorithm>
#include <cmath>
#include <cstdlib>
#include <cstring>
#include <vector>

#include "a2m_internal.h"

namespace a2m {

struct PlanHeader {
  int32_t window, hop, fft_len, n_mels, n_bins, nnz;
  int32_t off_window, off_twiddle, off_start, off_len, off_woff, off_weights;  // byte offsets
  int32_t off_tw1, off_tw2;  // fft_len == 2048 only: per-lane stage twiddles (0 otherwise)
  int32_t n_w4, off_band, off_w4;  // fft_len == 2048 only: band rows padded to float4 (see build_plan)
  int32_t la, lb;                   // fft_len == 2048 only: float4 rows per lane for bands A / B
};

static size_t align16(size_t x) { return (x + 15) & ~size_t(15); }

static void plan_layout(int win, int nfft, int n_mels, int nnz, int n_w4, PlanHeader* h,
                        size_t* total) {
  size_t off = align16(sizeof(PlanHeader));
  h->off_window = (int32_t)off; off = align16(off + sizeof(float) * win);
  h->off_twiddle = (int32_t)off; off = align16(off + sizeof(float) * 2 * nfft);
  h->off_start = (int32_t)off; off = align16(off + sizeof(int32_t) * n_mels);
  h->off_len = (int32_t)off; off = align16(off + sizeof(int32_t) * n_mels);
  h->off_woff = (int32_t)off; off = align16(off + sizeof(int32_t) * n_mels);
  h->off_weights = (int32_t)off; off = align16(off + sizeof(float) * nnz);
  h->off_tw1 = h->off_tw2 = h->n_w4 = h->off_band = h->off_w4 = 0;
  if (nfft == 2048) {
    h->off_tw1 = (int32_t)off; off = align16(off + sizeof(float) * 2 * 16 * 64);
    h->off_tw2 = (int32_t)off; off = align16(off + sizeof(float) * 2 * 16 * 4);
    h->n_w4 = n_w4;
    h->off_band = (int32_t)off; off = align16(off + sizeof(int32_t) * 4 * 64);
    h->off_w4 = (int32_t)off; off = align16(off + sizeof(float) * 4 * (size_t)n_w4);
  }
  *total = off;
}

static bool geometry(int sr, double win_s, double hop_s, int* win, int* hop, int* nfft) {
  // int(round(sr * secs)) (mel_features.py:212-213): Python rounds the double product half to
  // even, which nearbyint does under the default FE_TONEAREST mode (lround would not: 44.1 kHz x
  // 25 ms = 1102.5 -> 1102, 22.05 kHz x 10 ms = 220.5 -> 220)
  *win = (int)std::nearbyint((double)sr * win_s);
  *hop = (int)std::nearbyint((double)sr * hop_s);
  if (*win < 2 || *hop < 1) return false;
  *nfft = 1 << (int)std::ceil(std::log((double)*win) / std::log(2.0));
  return *nfft >= 4 && *nfft <= 16384;
}

// Mel weights in float64 following spectrogram_to_mel_matrix (mel_features.py:114-189).
static int mel_weights(int n_mels, int n_bins, int sr, double lo, double hi,
                       std::vector<double>* w) {
  const double nyq = sr / 2.0;
  if (lo < 0.0) { set_error("lower_edge_hertz %.1f must be >= 0", lo); return A2M_EINVAL; }
  if (lo >= hi) { set_error("lower_edge_hertz %.1f >= upper_edge_hertz %.1f", lo, hi); return A2M_EINVAL; }
  if (hi > nyq) { set_error("upper_edge_hertz %.1f is greater than Nyquist %.1f", hi, nyq); return A2M_EINVAL; }
  auto mel = [](double f) { return 1127.0 * std::log(1.0 + f / 700.0); };
  std::vector<double> bins(n_bins), edges(n_mels + 2);
  // np.linspace(start, stop, num): start + i*step, last element exactly stop
  const double bstep = n_bins > 1 ? nyq / (n_bins - 1) : 0.0;
  for (int i = 0; i < n_bins; ++i) bins[i] = mel(i == n_bins - 1 ? nyq : i * bstep);
  const double m0 = mel(lo), m1 = mel(hi);
  const double estep = (m1 - m0) / (n_mels + 1);
  for (int i = 0; i < n_mels + 2; ++i) edges[i] = (i == n_mels + 1) ? m1 : m0 + i * estep;
  w->assign((size_t)n_bins * n_mels, 0.0);
  for (int m = 0; m < n_mels; ++m) {
    const double l = edges[m], c = edges[m + 1], u = edges[m + 2];
    for (int k = 1; k < n_bins; ++k) {  // row 0 (DC) is zeroed (:188)
      const double rise = (bins[k] - l) / (c - l);
      const double fall = (u - bins[k]) / (u - c);
      (*w)[(size_t)k * n_mels + m] = std::max(0.0, std::min(rise, fall));
    }
  }
  return A2M_OK;
}

// ------------------------------------------------------------------------------ device
__device__ __forceinline__ float2 cmul(float2 a, float2 b) {
  return make_float2(a.x * b.x - a.y * b.y, a.x * b.y + a.y * b.x);
}

__global__ __launch_bounds__(256) void logmel_kernel(const float* __restrict__ wave,
                                                     int64_t clip_stride, int n_frames,
                                                     const unsigned char* __restrict__ plan,
                                                     float log_offset, float* __restrict__ out) {
  extern __shared__ __attribute__((aligned(16))) float smem[];
  const PlanHeader* ph = reinterpret_cast<const PlanHeader*>(plan);
  const int win = ph->window, hop = ph->hop, nfft = ph->fft_len, n_mels = ph->n_mels;
  const int M = nfft / 2;
  const float* window = reinterpret_cast<const float*>(plan + ph->off_window);
  const float2* tw = reinterpret_cast<const float2*>(plan + ph->off_twiddle);
  const int32_t* mstart = reinterpret_cast<const int32_t*>(plan + ph->off_start);
  const int32_t* mlen = reinterpret_cast<const int32_t*>(plan + ph->off_len);
  const int32_t* mwoff = reinterpret_cast<const int32_t*>(plan + ph->off_woff);
  const float* mw = reinterpret_cast<const float*>(plan + ph->off_weights);

  float2* buf0 = reinterpret_cast<float2*>(smem);
  float2* buf1 = buf0 + M;
  float* mag = reinterpret_cast<float*>(buf1 + M);

  const int frame = blockIdx.x % n_frames;
  const int clip = blockIdx.x / n_frames;
  const float* src = wave + clip * clip_stride + (int64_t)frame * hop;
  float* xs = reinterpret_cast<float*>(buf0);
  // all of this thread's sample (and window) loads are issued before the first LDS write
  // (a blockDim-strided loop would wait for each load in turn)
  constexpr int PF = 16;  // fft_len <= 4096 (host check)
  float sv[PF], wv[PF];
#pragma unroll
  for (int j = 0; j < PF; ++j) {
    const int n = threadIdx.x + j * 256;
    const bool in = n < win && n < nfft;
    sv[j] = in ? src[n] : 0.f;
    wv[j] = in ? window[n] : 0.f;
  }
#pragma unroll
  for (int j = 0; j < PF; ++j) {
    const int n = threadIdx.x + j * 256;
    if (n < nfft) xs[n] = sv[j] * wv[j];
  }
  __syncthreads();

  // Stockham autosort FFT of size M (complex), out-of-place ping-pong buffer0 <-> buffer1.
  float2* in = buf0;
  float2* outb = buf1;
  int Ns = 1;
  const int lg = __builtin_ctz(M);
  if (lg & 1) {  // one radix-2 stage first
    for (int j = threadIdx.x; j < M / 2; j += blockDim.x) {
      float2 v0 = in[j], v1 = in[j + M / 2];  // Ns = 1: no twiddle
      outb[2 * j] = make_float2(v0.x + v1.x, v0.y + v1.y);
      outb[2 * j + 1] = make_float2(v0.x - v1.x, v0.y - v1.y);
    }
    __syncthreads();
    float2* t = in; in = outb; outb = t;
    Ns = 2;
  }
  for (; Ns < M; Ns *= 4) {
    const int tstep = nfft / (Ns * 4);  // table index step for angle 2 pi k r / (4 Ns)
    for (int j = threadIdx.x; j < M / 4; j += blockDim.x) {
      const int k = j % Ns;
      float2 v0 = in[j];
      float2 v1 = cmul(in[j + M / 4], tw[k * tstep]);
      float2 v2 = cmul(in[j + M / 2], tw[2 * k * tstep]);
      float2 v3 = cmul(in[j + 3 * M / 4], tw[3 * k * tstep]);
      float2 a = make_float2(v0.x + v2.x, v0.y + v2.y), b = make_float2(v0.x - v2.x, v0.y - v2.y);
      float2 c = make_float2(v1.x + v3.x, v1.y + v3.y), d = make_float2(v1.x - v3.x, v1.y - v3.y);
      const int o = (j / Ns) * Ns * 4 + k;
      outb[o] = make_float2(a.x + c.x, a.y + c.y);
      outb[o + Ns] = make_float2(b.x + d.y, b.y - d.x);       // b - i d
      outb[o + 2 * Ns] = make_float2(a.x - c.x, a.y - c.y);
      outb[o + 3 * Ns] = make_float2(b.x - d.y, b.y + d.x);   // b + i d
    }
    __syncthreads();
    float2* t = in; in = outb; outb = t;
  }

  // real-input split and magnitude, k = 0..M
  for (int k = threadIdx.x; k <= M; k += blockDim.x) {
    const float2 zk = in[k == M ? 0 : k];
    const float2 zc = in[k == 0 ? 0 : M - k];                  // Z[M-k], conj below
    const float2 e = make_float2(0.5f * (zk.x + zc.x), 0.5f * (zk.y - zc.y));
    const float2 dd = make_float2(zk.x - zc.x, zk.y + zc.y);   // Z[k] - conj(Z[M-k])
    const float2 o = make_float2(0.5f * dd.y, -0.5f * dd.x);   // / (2i)
    const float2 wo = cmul(tw[k], o);
    const float re = e.x + wo.x, im = e.y + wo.y;
    mag[k] = sqrtf(re * re + im * im);
  }
  __syncthreads();

  float* dst = out + ((int64_t)clip * n_frames + frame) * n_mels;
  for (int m = threadIdx.x; m < n_mels; m += blockDim.x) {
    const int s = mstart[m], len = mlen[m];
    const float* wp = mw + mwoff[m];
    float acc = 0.f;
#pragma unroll 8
    for (int q = 0; q < len; ++q) acc += wp[q] * mag[s + q];
    dst[m] = logf(acc + log_offset);
  }
}



// LDS ordering between the lanes of ONE wave (each wave owns its exchange region): a
// wavefront-scope fence pair around a wave barrier (the rocPRIM wave_barrier form).
__device__ __forceinline__ void wave_lds_sync() {
  __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
  __builtin_amdgcn_wave_barrier();
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
}

// ---- packed complex arithmetic: (re, im) in one 64-bit register pair, so every add / mul /
// fma is one v_pk_*_f32 (two fp32 results per lane and instruction).  Swaps are op_sel
// modifiers; where a partial negation rides on a swapped or single half (conj, +-i, the
// complex product) the backend does not fold it into neg_lo / neg_hi and would emit
// v_xor + v_mov first, so those forms are written out as single instructions.
typedef float f2 __attribute__((ext_vector_type(2)));

__device__ __forceinline__ f2 pmul(f2 a, f2 b) {  // a * b: (a.x b.x - a.y b.y, a.x b.y + a.y b.x)
  const f2 t = a.xx * b;
  f2 r;
  asm("v_pk_fma_f32 %0, %1, %2, %3 op_sel:[1,1,0] op_sel_hi:[1,0,1] neg_lo:[1,0,0]"
      : "=v"(r) : "v"(a), "v"(b), "v"(t));
  return r;
}
__device__ __forceinline__ f2 add_mi(f2 a, f2 b) {  // a - i b = (a.x + b.y, a.y - b.x)
  f2 r;
  asm("v_pk_add_f32 %0, %1, %2 op_sel:[0,1] op_sel_hi:[1,0] neg_hi:[0,1]" : "=v"(r) : "v"(a), "v"(b));
  return r;
}
__device__ __forceinline__ f2 sub_mi(f2 a, f2 b) {  // a + i b = (a.x - b.y, a.y + b.x)
  f2 r;
  asm("v_pk_add_f32 %0, %1, %2 op_sel:[0,1] op_sel_hi:[1,0] neg_lo:[0,1]" : "=v"(r) : "v"(a), "v"(b));
  return r;
}
__device__ __forceinline__ f2 add_conj(f2 a, f2 b) {  // a + conj b
  f2 r;
  asm("v_pk_add_f32 %0, %1, %2 neg_hi:[0,1]" : "=v"(r) : "v"(a), "v"(b));
  return r;
}
__device__ __forceinline__ f2 sub_conj(f2 a, f2 b) {  // a - conj b
  f2 r;
  asm("v_pk_add_f32 %0, %1, %2 neg_lo:[0,1]" : "=v"(r) : "v"(a), "v"(b));
  return r;
}

constexpr float kR2 = 0.70710678118654752f;

__device__ __forceinline__ void dft4p(f2& a0, f2& a1, f2& a2, f2& a3) {  // W4 = -i
  const f2 s02 = a0 + a2, d02 = a0 - a2, s13 = a1 + a3, d13 = a1 - a3;
  a0 = s02 + s13;
  a2 = s02 - s13;
  a1 = add_mi(d02, d13);
  a3 = sub_mi(d02, d13);
}

template <int m>  // v * W16^m, m in {1, 2, 3, 4, 6, 9}
__device__ __forceinline__ f2 tw16p(f2 v) {
  if constexpr (m == 4) {
    return (f2){1.f, -1.f} * v.yx;                                                 // -i
  } else if constexpr (m == 2) {
    return __builtin_elementwise_fma(v.yx, (f2){kR2, -kR2}, kR2 * v);             // (1 - i)/sqrt 2
  } else if constexpr (m == 6) {
    return __builtin_elementwise_fma(v.yx, (f2){kR2, -kR2}, -kR2 * v);            // (-1 - i)/sqrt 2
  } else {
    constexpr float C1 = 0.92387953251128674f, S1 = 0.38268343236508978f;
    constexpr float c = m == 1 ? C1 : m == 3 ? S1 : -C1;
    constexpr float s = m == 1 ? S1 : m == 3 ? C1 : -S1;
    static_assert(m == 1 || m == 3 || m == 9, "tw16p");
    return __builtin_elementwise_fma(v.yx, (f2){s, -s}, c * v);                    // (c - i s) v
  }
}

__device__ __forceinline__ void dft16p(f2 (&v)[16]) {  // v[k] = sum_j v[j] W16^(j k)
#pragma unroll
  for (int j0 = 0; j0 < 4; ++j0) dft4p(v[j0], v[j0 + 4], v[j0 + 8], v[j0 + 12]);
  v[5] = tw16p<1>(v[5]); v[9] = tw16p<2>(v[9]); v[13] = tw16p<3>(v[13]);
  v[6] = tw16p<2>(v[6]); v[10] = tw16p<4>(v[10]); v[14] = tw16p<6>(v[14]);
  v[7] = tw16p<3>(v[7]); v[11] = tw16p<6>(v[11]); v[15] = tw16p<9>(v[15]);
#pragma unroll
  for (int ka = 0; ka < 4; ++ka) dft4p(v[4 * ka], v[4 * ka + 1], v[4 * ka + 2], v[4 * ka + 3]);
  f2 t[16];
#pragma unroll
  for (int i = 0; i < 16; ++i) t[i] = v[i];
#pragma unroll
  for (int ka = 0; ka < 4; ++ka)
#pragma unroll
    for (int kb = 0; kb < 4; ++kb) v[ka + 4 * kb] = t[kb + 4 * ka];
}

// Compile-time twiddles W16^j and W16^j W2048: the periodic Hann window of samples
// 2(lane + 64 j) and 2(lane + 64 j) + 1 from the lane's W1024^lane.
__constant__ const float HANN_C0_RE[16] = {1.f, 0.92387953251128674f, 0.70710678118654757f, 0.38268343236508984f, 6.123233995736766e-17f, -0.38268343236508973f, -0.70710678118654746f, -0.92387953251128674f, -1.f, -0.92387953251128685f, -0.70710678118654768f, -0.38268343236509034f, -1.8369701987210297e-16f, 0.38268343236509f, 0.70710678118654735f, 0.92387953251128652f};
__constant__ const float HANN_C0_IM[16] = {0.f, -0.38268343236508978f, -0.70710678118654746f, -0.92387953251128674f, -1.f, -0.92387953251128674f, -0.70710678118654757f, -0.38268343236508989f, -1.2246467991473532e-16f, 0.38268343236508967f, 0.70710678118654746f, 0.92387953251128652f, 1.f, 0.92387953251128663f, 0.70710678118654768f, 0.38268343236509039f};
__constant__ const float HANN_C1_RE[16] = {0.99999529380957619f, 0.92270112833387863f, 0.70493408037590499f, 0.37984720892405111f, -0.0030679567629660156f, -0.3855160538439189f, -0.70927282643886547f, -0.92504924078267747f, -0.99999529380957619f, -0.92270112833387863f, -0.7049340803759051f, -0.37984720892405144f, 0.0030679567629661149f, 0.38551605384391857f, 0.70927282643886569f, 0.92504924078267747f};
__constant__ const float HANN_C1_IM[16] = {-0.0030679567629659761f, -0.38551605384391885f, -0.70927282643886558f, -0.92504924078267758f, -0.99999529380957619f, -0.92270112833387852f, -0.7049340803759051f, -0.37984720892405138f, 0.0030679567629657324f, 0.38551605384391863f, 0.70927282643886547f, 0.92504924078267747f, 0.99999529380957619f, 0.92270112833387874f, 0.70493408037590488f, 0.37984720892405149f};

// v[k] *= b^k, k = 1..15 (powers by a product tree: each at most 4 roundings from b).
// Computed, not loaded: a wave-wide table load costs ~20 TA cycles whatever its footprint,
// more than the 2 x 14 packed products it replaces (measured: TA-bound with table twiddles).
__device__ __forceinline__ void twiddle15p(f2 (&v)[16], f2 b) {
  f2 p[16];
  p[1] = b;
  p[2] = pmul(b, b);
  p[3] = pmul(p[2], b);
  p[4] = pmul(p[2], p[2]);
  p[5] = pmul(p[4], b);
  p[6] = pmul(p[4], p[2]);
  p[7] = pmul(p[4], p[3]);
  p[8] = pmul(p[4], p[4]);
#pragma unroll
  for (int k = 9; k < 16; ++k) p[k] = pmul(p[8], p[k - 8]);
#pragma unroll
  for (int k = 1; k < 16; ++k) v[k] = pmul(v[k], p[k]);
}

constexpr int LM_WAVES = 8;            // frames (one per wave) per workgroup
constexpr int LM_P2 = 68;              // complex pitch of the stage-1 -> stage-2 exchange rows
constexpr int LM_EP = 260;             // complex pitch of the stage-2 output planes E[m0][.]
constexpr int LM_REGION = 16 * LM_P2;  // complex words per wave (exchange, E, then magnitudes)
constexpr int LM_ROWS = 12;            // float4 mel-weight rows per lane kept in LDS (build config 3 + 9)
constexpr int LM_MAX_W4 = 64 * LM_ROWS;

// ---------------------------------------------------------------------------------------
// fft_len == 2048 (the build configuration, W = 2048, M = 1024): one wave64 per frame, the
// 1024-point complex FFT of z[n] = xw[2n] + i xw[2n+1] register-resident, all complex
// arithmetic packed (v_pk_*_f32).  M = 16 x 16 x 4:
//   stage 1  lane n0 holds z[n0 + 64 n1]: B = DFT16_n1, C[n0][k1] = B W1024^(n0 k1)
//   LDS exchange (rows k1, pitch 68 complex: ds_*_b64 conflict-free both ways)
//   stage 2  lane (k1, m0): DFT16 over m1 of C[m0 + 4 m1][k1], times W64^(m0 k2)
//            -> E[m0][b], b = k1 + 16 k2, stored to LDS planes m0 (pitch 260)
//   split    Z[b + 256 k3] = DFT4_m0 E[m0][b] (W4 = -i).  A lane takes the two bases b and
//            256 - b (their DFT4s hold exactly the partners Z[M - k] of each other's Z[k]):
//            units b = lane + 1 and b = lane + 65 (b = 128 pairs with itself), lane 63's
//            second unit is {0, 128}.  Each (k, M - k) pair gives both magnitudes:
//            s = Z[k] + conj Z[M-k], d = Z[k] - conj Z[M-k], wd = -i W2048^k d,
//            2|X[k]| = |s + wd|, 2|X[M-k]| = |s - wd| (the 1/2 is folded into the mel rows)
//   mel      lane owns bands lane and 127 - lane (narrow + wide: balanced), rows aligned to
//            4 bins so weights and magnitudes are both read as float4
// then log(mel + offset).  LDS per wave: 8.7 KB; the mel rows once per workgroup.
// ---------------------------------------------------------------------------------------
template <bool FULL>  // FULL: window == fft_len == 2048 (Hann from twiddles, no predicated loads)
__global__ __launch_bounds__(64 * LM_WAVES) void logmel2048_kernel(
    const float* __restrict__ wave, int64_t clip_stride, int n_frames, int total_frames,
    const unsigned char* __restrict__ plan, float log_offset, float* __restrict__ out) {
  constexpr int M = 1024;
  __shared__ f2 s_region[LM_WAVES][LM_REGION];
  __shared__ float4 s_w4[LM_MAX_W4];
  const PlanHeader* ph = reinterpret_cast<const PlanHeader*>(plan);
  const int win = ph->window, hop = ph->hop, n_mels = ph->n_mels, n_w4 = ph->n_w4;
  const int la = ph->la, lb = ph->lb;
  const bool lds_rows = la + lb <= LM_ROWS;      // else the mel rows are read from L2
  const float* window = reinterpret_cast<const float*>(plan + ph->off_window);
  const f2* tw = reinterpret_cast<const f2*>(plan + ph->off_twiddle);   // W2048^t
  const int4* band = reinterpret_cast<const int4*>(plan + ph->off_band);
  const float4* w4 = reinterpret_cast<const float4*>(plan + ph->off_w4);

  const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
  const int gframe = blockIdx.x * LM_WAVES + wv;
  const bool active = gframe < total_frames;
  const int frame = active ? gframe % n_frames : 0;
  const int clip = active ? gframe / n_frames : 0;
  const float* src = wave + clip * clip_stride + (int64_t)frame * hop;
  f2* sx = s_region[wv];

  // mel weight rows: one copy per workgroup in LDS (loads issued before the frame's samples)
  float4 wst[2];
#pragma unroll
  for (int i = 0; i < 2; ++i) {
    const int q = threadIdx.x + i * 64 * LM_WAVES;
    wst[i] = lds_rows && q < n_w4 ? w4[q] : make_float4(0.f, 0.f, 0.f, 0.f);
  }
  // per-lane values used later, fetched now (L2-resident plan)
  const f2 b1 = tw[2 * lane];                    // W1024^lane
  const int k1 = lane >> 2, m0 = lane & 3;
  const f2 b2 = tw[32 * m0];                     // W64^m0
  const bool sp = lane == 63;                    // unit 1 of lane 63 is {0, 128}
  const int ub0 = lane + 1, ub1 = sp ? 0 : lane + 65;
  const f2 t0 = tw[ub0], t1 = tw[ub1], t128 = tw[128];
  const int4 bd = band[lane];

  // ---- stage 1
  f2 v[16];
  {
    f2 x[16], w[16];
#pragma unroll
    for (int j = 0; j < 16; ++j) {
      const int n = 2 * (lane + 64 * j);
      if (FULL) {  // 0.5 - 0.5 cos(2 pi n / 2048) = 0.5 - 0.5 Re(W1024^lane W16^j [W2048])
        x[j] = (f2){src[n], src[n + 1]};
        const f2 cre = (f2){HANN_C0_RE[j], HANN_C1_RE[j]}, cim = (f2){HANN_C0_IM[j], HANN_C1_IM[j]};
        const f2 r = __builtin_elementwise_fma(-b1.yy, cim, b1.xx * cre);
        w[j] = __builtin_elementwise_fma((f2)(-0.5f), r, (f2)(0.5f));
      } else {
        x[j] = (f2){n < win ? src[n] : 0.f, n + 1 < win ? src[n + 1] : 0.f};
        w[j] = (f2){n < win ? window[n] : 0.f, n + 1 < win ? window[n + 1] : 0.f};
      }
    }
#pragma unroll
    for (int i = 0; i < 2; ++i) {
      const int q = threadIdx.x + i * 64 * LM_WAVES;
      if (q < LM_MAX_W4) s_w4[q] = wst[i];
    }
#pragma unroll
    for (int j = 0; j < 16; ++j) v[j] = x[j] * w[j];
  }
  dft16p(v);
  twiddle15p(v, b1);                             // W1024^(n0 k1)
#pragma unroll
  for (int k = 0; k < 16; ++k) sx[k * LM_P2 + lane] = v[k];
  wave_lds_sync();  // the exchange region is this wave's own

  // ---- stage 2: lane (k1, m0)
#pragma unroll
  for (int m1 = 0; m1 < 16; ++m1) v[m1] = sx[k1 * LM_P2 + m0 + 4 * m1];
  dft16p(v);
  twiddle15p(v, b2);                             // W64^(m0 k2)
  wave_lds_sync();  // every stage-2 read of this wave before E overwrites the region
#pragma unroll
  for (int k2 = 0; k2 < 16; ++k2) sx[m0 * LM_EP + k1 + 16 * k2] = v[k2];
  wave_lds_sync();

  // ---- split: DFT4 over m0, real-input split, magnitudes (x2)
  float mg[17];
  int ki[17];
#pragma unroll
  for (int u = 0; u < 2; ++u) {
    const int b = u == 0 ? ub0 : ub1;
    const int bp = u == 0 ? 256 - ub0 : (sp ? 128 : 256 - ub1);
    const f2 t = u == 0 ? t0 : t1;
    f2 za[4], zb[4];
#pragma unroll
    for (int q = 0; q < 4; ++q) {
      za[q] = sx[q * LM_EP + b];
      zb[q] = sx[q * LM_EP + bp];
    }
    dft4p(za[0], za[1], za[2], za[3]);
    dft4p(zb[0], zb[1], zb[2], zb[3]);
#pragma unroll
    for (int k3 = 0; k3 < 4; ++k3) {
      f2 first = za[k3], second = zb[3 - k3];
      f2 w = k3 == 0 ? t : k3 == 1 ? tw16p<2>(t) : k3 == 2 ? tw16p<4>(t) : tw16p<6>(t);  // W8^k3
      int ka = b + 256 * k3;
      if (u == 1) {  // lane 63: pairs (0,1024), (256,768) from Z[0..3*256]; (128,896), (384,640)
        if (k3 < 2) {
          second = sp ? za[(4 - k3) & 3] : second;
        } else {
          first = sp ? zb[k3 - 2] : first;
          second = sp ? zb[5 - k3] : second;
          const f2 ws = k3 == 2 ? t128 : tw16p<2>(t128);
          w = sp ? ws : w;
          ka = sp ? 128 + 256 * (k3 - 2) : ka;
        }
      }
      const f2 s = add_conj(first, second), d = sub_conj(first, second);
      const f2 wd = pmul(w, d);                  // X2 = s -+ i wd
      const f2 xa = add_mi(s, wd), xb = sub_mi(s, wd);
      const f2 qa = xa * xa, qb = xb * xb;
      mg[8 * u + 2 * k3] = __builtin_amdgcn_sqrtf(qa.x + qa.y);
      mg[8 * u + 2 * k3 + 1] = __builtin_amdgcn_sqrtf(qb.x + qb.y);
      ki[8 * u + 2 * k3] = ka;
      ki[8 * u + 2 * k3 + 1] = M - ka;
    }
    if (u == 1) {  // lane 63 also owns X[512] = |Z[512]| (stored x2 like the others)
      const f2 q = za[2] * za[2];
      mg[16] = 2.f * __builtin_amdgcn_sqrtf(q.x + q.y);
      ki[16] = 512;
    }
  }
  wave_lds_sync();  // every E read of this wave before the magnitudes overwrite the region
  float* s_mag = reinterpret_cast<float*>(sx);
#pragma unroll
  for (int i = 0; i < 16; ++i) s_mag[ki[i]] = mg[i];
  if (sp) s_mag[ki[16]] = mg[16];
  s_mag[M + 1 + lane] = 0.f;  // zero tail: aligned band rows may read past bin 1024
  wave_lds_sync();

  // ---- banded mel + log: bands A = lane and B = 127 - lane, rows contiguous in s_w4.  The
  // workgroup's only barrier publishes s_w4 here, so until now every wave ran its FFT as soon
  // as its own samples arrived, overlapping the other frames' loads.
  __syncthreads();
  if (!active) return;
  const int stA = bd.x, stB = bd.y, r0 = lane * (la + lb);
  f2 accA = (f2)(0.f), accB = (f2)(0.f);
  if (lds_rows) {
    for (int c = 0; c < la; ++c) {
      const float4 wq = s_w4[r0 + c], mq = *reinterpret_cast<const float4*>(s_mag + stA + 4 * c);
      accA = __builtin_elementwise_fma((f2){wq.x, wq.y}, (f2){mq.x, mq.y}, accA);
      accA = __builtin_elementwise_fma((f2){wq.z, wq.w}, (f2){mq.z, mq.w}, accA);
    }
    for (int c = 0; c < lb; ++c) {
      const float4 wq = s_w4[r0 + la + c], mq = *reinterpret_cast<const float4*>(s_mag + stB + 4 * c);
      accB = __builtin_elementwise_fma((f2){wq.x, wq.y}, (f2){mq.x, mq.y}, accB);
      accB = __builtin_elementwise_fma((f2){wq.z, wq.w}, (f2){mq.z, mq.w}, accB);
    }
  } else {
    for (int c = 0; c < la; ++c) {
      const float4 wq = w4[r0 + c], mq = *reinterpret_cast<const float4*>(s_mag + stA + 4 * c);
      accA = __builtin_elementwise_fma((f2){wq.x, wq.y}, (f2){mq.x, mq.y}, accA);
      accA = __builtin_elementwise_fma((f2){wq.z, wq.w}, (f2){mq.z, mq.w}, accA);
    }
    for (int c = 0; c < lb; ++c) {
      const float4 wq = w4[r0 + la + c], mq = *reinterpret_cast<const float4*>(s_mag + stB + 4 * c);
      accB = __builtin_elementwise_fma((f2){wq.x, wq.y}, (f2){mq.x, mq.y}, accB);
      accB = __builtin_elementwise_fma((f2){wq.z, wq.w}, (f2){mq.z, mq.w}, accB);
    }
  }
  float* dst = out + (int64_t)gframe * n_mels;
  const int mA = lane, mB = 127 - lane;
  if (mA < n_mels) dst[mA] = __logf(accA.x + accA.y + log_offset);
  if (mB >= 64 && mB < n_mels) dst[mB] = __logf(accB.x + accB.y + log_offset);
}

}  // namespace a2m

using namespace a2m;

extern "C" {

int64_t a2m_logmel_num_frames(int64_t n_samples, int32_t window, int32_t hop) {
  if (hop <= 0) return 0;
  const int64_t n = 1 + (int64_t)std::floor((double)(n_samples - window) / hop);
  return n > 0 ? n : 0;
}

int a2m_logmel_geometry(int32_t sample_rate, double window_secs, double hop_secs,
                        int32_t* window, int32_t* hop, int32_t* fft_len) {
  int w, h, n;
  A2M_CHECK_ARG(geometry(sample_rate, window_secs, hop_secs, &w, &h, &n),
                "logmel: unsupported geometry sr=%d win=%g hop=%g", sample_rate, window_secs,
                hop_secs);
  *window = w; *hop = h; *fft_len = n;
  return A2M_OK;
}

static int build_plan(int32_t sr, double win_s, double hop_s, int32_t n_mels, double lo, double hi,
                      void* host, size_t bytes, size_t* need) {
  int win, hop, nfft;
  A2M_CHECK_ARG(geometry(sr, win_s, hop_s, &win, &hop, &nfft), "logmel: unsupported geometry");
  A2M_CHECK_ARG(n_mels > 0 && n_mels <= 4096, "logmel: bad n_mels %d", n_mels);
  const int n_bins = nfft / 2 + 1;
  std::vector<double> w;
  int rc = mel_weights(n_mels, n_bins, sr, lo, hi, &w);
  if (rc) return rc;
  std::vector<int32_t> start(n_mels), len(n_mels), woff(n_mels);
  std::vector<float> vals;
  for (int m = 0; m < n_mels; ++m) {
    int first = -1, last = -1;
    for (int k = 0; k < n_bins; ++k)
      if (w[(size_t)k * n_mels + m] != 0.0) { if (first < 0) first = k; last = k; }
    if (first < 0) { first = 0; last = -1; }
    start[m] = first; len[m] = last - first + 1; woff[m] = (int32_t)vals.size();
    for (int k = first; k <= last; ++k) vals.push_back((float)w[(size_t)k * n_mels + m]);
  }
  PlanHeader h{};
  h.window = win; h.hop = hop; h.fft_len = nfft; h.n_mels = n_mels; h.n_bins = n_bins;
  h.nnz = (int32_t)vals.size();
  // register-FFT path (fft_len 2048, <= 128 mels): lane l owns bands A = l and B = 127 - l;
  // each band's row starts at a multiple of 4 bins and every lane's A (B) row is zero-padded
  // to the widest A (B) row, la (lb) float4s, so the kernel's loops have uniform trip counts
  auto row4 = [&](int m) { return m < n_mels && len[m] > 0 ? (start[m] % 4 + len[m] + 3) / 4 : 0; };
  int la = 0, lb = 0;
  for (int l = 0; l < 64; ++l) {
    la = std::max(la, row4(l));
    lb = std::max(lb, row4(127 - l));
  }
  const int n_w4 = 64 * (la + lb);
  size_t total;
  plan_layout(win, nfft, n_mels, h.nnz, n_w4, &h, &total);
  h.la = la;
  h.lb = lb;
  *need = total;
  if (host == nullptr) return A2M_OK;
  if (bytes < total) { set_error("logmel plan buffer too small (%zu < %zu)", bytes, total); return A2M_EWS; }
  unsigned char* p = static_cast<unsigned char*>(host);
  std::memset(p, 0, total);
  std::memcpy(p, &h, sizeof(h));
  float* wp = reinterpret_cast<float*>(p + h.off_window);
  const double pi = 3.14159265358979323846;
  for (int n = 0; n < win; ++n) wp[n] = (float)(0.5 - 0.5 * std::cos(2.0 * pi / win * n));
  float* tp = reinterpret_cast<float*>(p + h.off_twiddle);
  for (int t = 0; t < nfft; ++t) {
    const double a = -2.0 * pi * t / nfft;
    tp[2 * t] = (float)std::cos(a);
    tp[2 * t + 1] = (float)std::sin(a);
  }
  if (nfft == 2048) {  // see logmel2048_kernel: W_1024^(n0 k1) as [k1][n0], W_64^(m0 k2) as [k2][m0]
    float* t1 = reinterpret_cast<float*>(p + h.off_tw1);
    for (int k1 = 0; k1 < 16; ++k1)
      for (int n0 = 0; n0 < 64; ++n0) {
        const double a = -2.0 * pi * (n0 * k1) / 1024.0;
        t1[2 * (k1 * 64 + n0)] = (float)std::cos(a);
        t1[2 * (k1 * 64 + n0) + 1] = (float)std::sin(a);
      }
    float* t2 = reinterpret_cast<float*>(p + h.off_tw2);
    for (int k2 = 0; k2 < 16; ++k2)
      for (int m0 = 0; m0 < 4; ++m0) {
        const double a = -2.0 * pi * (m0 * k2) / 64.0;
        t2[2 * (k2 * 4 + m0)] = (float)std::cos(a);
        t2[2 * (k2 * 4 + m0) + 1] = (float)std::sin(a);
      }
  }
  if (nfft == 2048 && n_mels <= 128) {
    // band[lane] = {A start, B start, 0, 0} (starts rounded down to a multiple of 4); rows of
    // lane l at float4 l (la + lb): A then B; weights x 0.5 (the kernel's magnitudes are 2 |X|)
    int32_t* band = reinterpret_cast<int32_t*>(p + h.off_band);
    float* w4 = reinterpret_cast<float*>(p + h.off_w4);
    for (int lane = 0; lane < 64; ++lane) {
      for (int half = 0; half < 2; ++half) {
        const int m = half == 0 ? lane : 127 - lane;
        const int l4 = row4(m);
        const int st4 = l4 ? start[m] & ~3 : 0;
        band[4 * lane + half] = st4;
        float* row = w4 + 4 * (lane * (la + lb) + (half == 0 ? 0 : la));
        for (int q = 0; q < (l4 ? len[m] : 0); ++q) row[(start[m] - st4) + q] = 0.5f * vals[woff[m] + q];
      }
    }
  }
  std::memcpy(p + h.off_start, start.data(), sizeof(int32_t) * n_mels);
  std::memcpy(p + h.off_len, len.data(), sizeof(int32_t) * n_mels);
  std::memcpy(p + h.off_woff, woff.data(), sizeof(int32_t) * n_mels);
  if (!vals.empty()) std::memcpy(p + h.off_weights, vals.data(), sizeof(float) * vals.size());
  return A2M_OK;
}

size_t a2m_logmel_plan_bytes(int32_t sample_rate, double window_secs, double hop_secs,
                             int32_t n_mels, double lower_hz, double upper_hz) {
  size_t need = 0;
  if (build_plan(sample_rate, window_secs, hop_secs, n_mels, lower_hz, upper_hz, nullptr, 0, &need))
    return 0;
  return need;
}

int a2m_logmel_plan_build(int32_t sample_rate, double window_secs, double hop_secs,
                          int32_t n_mels, double lower_hz, double upper_hz, void* host_plan,
                          size_t plan_bytes) {
  size_t need = 0;
  return build_plan(sample_rate, window_secs, hop_secs, n_mels, lower_hz, upper_hz, host_plan,
                    plan_bytes, &need);
}

int a2m_logmel_f32(const float* wave, int64_t n_clips, int64_t clip_stride, int64_t n_samples,
                   int32_t window, int32_t hop, int32_t fft_len, int32_t n_mels,
                   const void* dev_plan, float log_offset, float* out, void* stream) {
  A2M_CHECK_ARG(fft_len >= 4 && (fft_len & (fft_len - 1)) == 0 && window <= fft_len && hop > 0,
                "logmel: bad geometry window=%d hop=%d fft_len=%d", window, hop, fft_len);
  const int64_t nf = a2m_logmel_num_frames(n_samples, window, hop);
  if (nf == 0 || n_clips == 0) return A2M_OK;  // empty output, like the reference's (0, n_mels)
  A2M_CHECK_ARG(wave && out && dev_plan, "logmel: null pointer");
  A2M_CHECK_ARG(n_clips * nf < (1LL << 31), "logmel: too many frames");
  A2M_CHECK_ARG(fft_len <= 4096, "logmel: fft_len %d > 4096", fft_len);
  const size_t lds = sizeof(float) * (2 * (size_t)fft_len + fft_len / 2 + 1 + 3);
  A2M_CHECK_ARG(lds <= 160 * 1024, "logmel: fft_len %d too large for LDS", fft_len);
  // register-FFT path (its mel rows sit in LDS when each lane's fit in LM_ROWS float4s, as
  // for the build configuration, and are read from L2 otherwise)
  if (fft_len == 2048 && n_mels <= 128) {
    auto kern = window == 2048 ? logmel2048_kernel<true> : logmel2048_kernel<false>;
    const int64_t total = n_clips * nf;
    hipLaunchKernelGGL(kern, dim3((unsigned)cdiv(total, LM_WAVES)), dim3(64 * LM_WAVES), 0,
                       as_stream(stream), wave, clip_stride, (int)nf, (int)total,
                       static_cast<const unsigned char*>(dev_plan), log_offset, out);
    A2M_LAUNCH_CHECK();
    return A2M_OK;
  }
  hipLaunchKernelGGL(logmel_kernel, dim3((unsigned)(n_clips * nf)), dim3(256), lds,
                     as_stream(stream), wave, clip_stride, (int)nf,
                     static_cast<const unsigned char*>(dev_plan), log_offset, out);
  A2M_LAUNCH_CHECK();
  return A2M_OK;
}

}  // extern "C"
