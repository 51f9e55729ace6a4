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
    h->off_band = (int32_t)off; off = align16(off + sizeof(int32_t) * 2 * n_mels);
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


// ---------------------------------------------------------------------------------------
// fft_len == 2048 (the build configuration, W = 2048, M = 1024): one wave64 per frame, the
// FFT register-resident.  M = 1024 is split 16 x 16 x 4:
//   z[n0 + 64 n1]                                    lane n0 holds n1 = 0..15
//   stage 1  B[n0][k1] = DFT16_n1, C = B * W1024^(n0 k1)          (registers)
//   LDS transpose (re/im planes, pitch 68: conflict-free both ways)
//   stage 2  lane (k1, m0): D[k2] = DFT16_m1 C[m0 + 4 m1][k1], E = D * W64^(m0 k2)
//   stage 3  DFT4 over m0 across the lane quad (two DPP butterflies, xor 2 then xor 1):
//            lane m0 = a + 2b ends with Z[k1 + 16 k2 + 256 (b + 2a)]
// then the real-input split / magnitude (:71-92) and the banded mel + log as above.
// LDS per frame: 2 x 1088 floats (exchange, then Z, then magnitudes) = 8.7 KB.
// ---------------------------------------------------------------------------------------
__device__ __forceinline__ float2 c_add(float2 a, float2 b) { return make_float2(a.x + b.x, a.y + b.y); }
__device__ __forceinline__ float2 c_sub(float2 a, float2 b) { return make_float2(a.x - b.x, a.y - b.y); }

// forward DFT4 in place (W4 = -i)
__device__ __forceinline__ void dft4(float2& a0, float2& a1, float2& a2, float2& a3) {
  const float2 s02 = c_add(a0, a2), d02 = c_sub(a0, a2);
  const float2 s13 = c_add(a1, a3), d13 = c_sub(a1, a3);
  a0 = c_add(s02, s13);
  a2 = c_sub(s02, s13);
  a1 = make_float2(d02.x + d13.y, d02.y - d13.x);  // d02 - i d13
  a3 = make_float2(d02.x - d13.y, d02.y + d13.x);  // d02 + i d13
}

// v * W16^m for a compile-time m in 1..9
template <int m>
__device__ __forceinline__ float2 tw16(float2 v) {
  constexpr float C1 = 0.92387953251128674f, S1 = 0.38268343236508978f, R2 = 0.70710678118654752f;
  if constexpr (m == 4) return make_float2(v.y, -v.x);  // -i
  else if constexpr (m == 2) return make_float2(R2 * (v.x + v.y), R2 * (v.y - v.x));
  else if constexpr (m == 6) return make_float2(R2 * (v.y - v.x), -R2 * (v.x + v.y));
  else {
    constexpr float c = m == 1 ? C1 : m == 3 ? S1 : m == 9 ? -C1 : 0.f;
    constexpr float s = m == 1 ? S1 : m == 3 ? C1 : m == 9 ? -S1 : 0.f;
    static_assert(m == 1 || m == 3 || m == 9, "tw16");
    // W16^m = c - i s
    return make_float2(c * v.x + s * v.y, c * v.y - s * v.x);
  }
}

// in place: on return v[k] = sum_j v_in[j] W16^(j k)
__device__ __forceinline__ void dft16(float2 (&v)[16]) {
#pragma unroll
  for (int j0 = 0; j0 < 4; ++j0) dft4(v[j0], v[j0 + 4], v[j0 + 8], v[j0 + 12]);  // v[j0+4ka] = T[j0][ka]
  v[5] = tw16<1>(v[5]); v[9] = tw16<2>(v[9]); v[13] = tw16<3>(v[13]);
  v[6] = tw16<2>(v[6]); v[10] = tw16<4>(v[10]); v[14] = tw16<6>(v[14]);
  v[7] = tw16<3>(v[7]); v[11] = tw16<6>(v[11]); v[15] = tw16<9>(v[15]);
#pragma unroll
  for (int ka = 0; ka < 4; ++ka) dft4(v[4 * ka], v[4 * ka + 1], v[4 * ka + 2], v[4 * ka + 3]);
  // position kb + 4 ka holds B[ka + 4 kb]: transpose the 4x4 index
  float2 t[16];
#pragma unroll
  for (int i = 0; i < 16; ++i) t[i] = v[i];
#pragma unroll
  for (int ka = 0; ka < 4; ++ka)
#pragma unroll
    for (int kb = 0; kb < 4; ++kb) v[ka + 4 * kb] = t[kb + 4 * ka];
}

template <int CTRL>
__device__ __forceinline__ float2 dpp_c(float2 v) {
  return make_float2(dpp_f<CTRL>(v.x), dpp_f<CTRL>(v.y));
}

// Compile-time twiddles: W16^j, W16^j * W2048 (Hann window from the lane's W1024^lane for
// samples 2(lane + 64 j) and 2(lane + 64 j) + 1), W32^i (split twiddles W2048^(lane + 64 i)).
__constant__ const float HANN_C0_RE[16] = {1.f, 0.92387953251128674f, 0.70710678118654757f, 0.38268343236508984f, 6.123233995736766e-17f, -0.38268343236508973f, -0.70710678118654746f, -0.92387953251128674f, -1.f, -0.92387953251128685f, -0.70710678118654768f, -0.38268343236509034f, -1.8369701987210297e-16f, 0.38268343236509f, 0.70710678118654735f, 0.92387953251128652f};
__constant__ const float HANN_C0_IM[16] = {0.f, -0.38268343236508978f, -0.70710678118654746f, -0.92387953251128674f, -1.f, -0.92387953251128674f, -0.70710678118654757f, -0.38268343236508989f, -1.2246467991473532e-16f, 0.38268343236508967f, 0.70710678118654746f, 0.92387953251128652f, 1.f, 0.92387953251128663f, 0.70710678118654768f, 0.38268343236509039f};
__constant__ const float HANN_C1_RE[16] = {0.99999529380957619f, 0.92270112833387863f, 0.70493408037590499f, 0.37984720892405111f, -0.0030679567629660156f, -0.3855160538439189f, -0.70927282643886547f, -0.92504924078267747f, -0.99999529380957619f, -0.92270112833387863f, -0.7049340803759051f, -0.37984720892405144f, 0.0030679567629661149f, 0.38551605384391857f, 0.70927282643886569f, 0.92504924078267747f};
__constant__ const float HANN_C1_IM[16] = {-0.0030679567629659761f, -0.38551605384391885f, -0.70927282643886558f, -0.92504924078267758f, -0.99999529380957619f, -0.92270112833387852f, -0.7049340803759051f, -0.37984720892405138f, 0.0030679567629657324f, 0.38551605384391863f, 0.70927282643886547f, 0.92504924078267747f, 0.99999529380957619f, 0.92270112833387874f, 0.70493408037590488f, 0.37984720892405149f};
__constant__ const float W32_RE[9] = {1.f, 0.98078528040323043f, 0.92387953251128674f, 0.83146961230254524f, 0.70710678118654757f, 0.55557023301960229f, 0.38268343236508984f, 0.19509032201612833f, 6.123233995736766e-17f};
__constant__ const float W32_IM[9] = {0.f, -0.19509032201612825f, -0.38268343236508978f, -0.55557023301960218f, -0.70710678118654746f, -0.83146961230254524f, -0.92387953251128674f, -0.98078528040323043f, -1.f};

// p[k] = b^k, k = 1..15, by a product tree (each power at most 4 roundings from the table value)
__device__ __forceinline__ void powers15(float2 b, float2 (&p)[16]) {
  p[0] = make_float2(1.f, 0.f);
  p[1] = b;
  p[2] = cmul(b, b);
  p[3] = cmul(p[2], b);
  p[4] = cmul(p[2], p[2]);
  p[5] = cmul(p[4], b);
  p[6] = cmul(p[4], p[2]);
  p[7] = cmul(p[4], p[3]);
  p[8] = cmul(p[4], p[4]);
#pragma unroll
  for (int k = 9; k < 16; ++k) p[k] = cmul(p[8], p[k - 8]);
}

// LDS ordering between the lanes of ONE wave (each wave owns its exchange planes): a
// wavefront-scope fence pair around a wave barrier (the rocPRIM wave_barrier form).
__device__ __forceinline__ void wave_lds_sync() {
  __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
  __builtin_amdgcn_wave_barrier();
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
}

constexpr int LM_WAVES = 8;          // frames (one per wave) per workgroup
constexpr int LM_PLANE = 16 * 68;    // floats per exchange plane (pitch 68; Z / magnitudes reuse it)
constexpr int LM_MAX_W4 = 640;       // float4 mel-weight rows staged in LDS (build config: ~520)

template <bool FULL>  // FULL: window == fft_len == 2048 (Hann from twiddles, no predicated loads)
__global__ __launch_bounds__(64 * LM_WAVES) void logmel2048_kernel(
    const float* __restrict__ wave, int64_t clip_stride, int n_frames, int total_frames,
    const unsigned char* __restrict__ plan, float log_offset, float* __restrict__ out) {
  constexpr int M = 1024, P = 68;
  __shared__ float s_plane[LM_WAVES][2][LM_PLANE];
  __shared__ float4 s_w4[LM_MAX_W4];
  const PlanHeader* ph = reinterpret_cast<const PlanHeader*>(plan);
  const int win = ph->window, hop = ph->hop, n_mels = ph->n_mels, n_w4 = ph->n_w4;
  const float* window = reinterpret_cast<const float*>(plan + ph->off_window);
  const float2* tw = reinterpret_cast<const float2*>(plan + ph->off_twiddle);
  const int2* band = reinterpret_cast<const int2*>(plan + ph->off_band);
  const float4* w4 = reinterpret_cast<const float4*>(plan + ph->off_w4);

  const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
  const int gframe = blockIdx.x * LM_WAVES + wv;
  const bool active = gframe < total_frames;
  const int frame = active ? gframe % n_frames : 0;
  const int clip = active ? gframe / n_frames : 0;
  const float* src = wave + clip * clip_stride + (int64_t)frame * hop;
  float* s_re = s_plane[wv][0];
  float* s_im = s_plane[wv][1];

  // mel weight rows: one copy per workgroup in LDS (loads issued before the frame's samples)
  float4 wst[2];
#pragma unroll
  for (int i = 0; i < 2; ++i) {
    const int q = threadIdx.x + i * 64 * LM_WAVES;
    wst[i] = q < n_w4 ? w4[q] : make_float4(0.f, 0.f, 0.f, 0.f);
  }

  // ---- stage 1: lane n0 = lane holds z[n0 + 64 j] = xw[2n] + i xw[2n+1], n = n0 + 64 j
  const float2 b1 = tw[2 * lane];  // W1024^lane
  float2 v[16];
  {
    float a[16], b[16];
#pragma unroll
    for (int j = 0; j < 16; ++j) {
      const int n = 2 * (lane + 64 * j);
      if (FULL) {
        a[j] = src[n];
        b[j] = src[n + 1];
      } else {
        a[j] = n < win ? src[n] : 0.f;
        b[j] = n + 1 < win ? src[n + 1] : 0.f;
      }
    }
#pragma unroll
    for (int i = 0; i < 2; ++i) {
      const int q = threadIdx.x + i * 64 * LM_WAVES;
      if (q < LM_MAX_W4) s_w4[q] = wst[i];
    }
#pragma unroll
    for (int j = 0; j < 16; ++j) {
      float wa, wb;
      if (FULL) {  // 0.5 - 0.5 cos(2 pi n / 2048) = 0.5 - 0.5 Re(W1024^lane W16^j [W2048])
        wa = fmaf(-0.5f, b1.x * HANN_C0_RE[j] - b1.y * HANN_C0_IM[j], 0.5f);
        wb = fmaf(-0.5f, b1.x * HANN_C1_RE[j] - b1.y * HANN_C1_IM[j], 0.5f);
      } else {
        const int n = 2 * (lane + 64 * j);
        wa = n < win ? window[n] : 0.f;
        wb = n + 1 < win ? window[n + 1] : 0.f;
      }
      v[j] = make_float2(a[j] * wa, b[j] * wb);
    }
  }
  dft16(v);
  {
    float2 t[16];
    powers15(b1, t);  // W1024^(n0 k1)
#pragma unroll
    for (int k = 1; k < 16; ++k) v[k] = cmul(v[k], t[k]);
  }
#pragma unroll
  for (int k = 0; k < 16; ++k) { s_re[k * P + lane] = v[k].x; s_im[k * P + lane] = v[k].y; }
  __syncthreads();  // also publishes s_w4 (the only workgroup-wide barrier)

  // ---- stage 2: lane (k1, m0)
  const int k1 = lane >> 2, m0 = lane & 3;
#pragma unroll
  for (int m1 = 0; m1 < 16; ++m1) {
    const int a = k1 * P + m0 + 4 * m1;
    v[m1] = make_float2(s_re[a], s_im[a]);
  }
  dft16(v);
  {
    float2 t[16];
    powers15(tw[32 * m0], t);  // W64^(m0 k2)
#pragma unroll
    for (int k = 1; k < 16; ++k) v[k] = cmul(v[k], t[k]);
  }

  // ---- stage 3: DFT4 over m0 = a + 2b across the quad
  const int qa = m0 & 1, qb = m0 >> 1;
  const float sb = qb ? -1.f : 1.f, sa = qa ? -1.f : 1.f;
  const bool rot = qa & qb;
#pragma unroll
  for (int k = 0; k < 16; ++k) {
    const float2 p = dpp_c<DPP_XOR2>(v[k]);
    float2 u = make_float2(fmaf(sb, v[k].x, p.x), fmaf(sb, v[k].y, p.y));
    if (rot) u = make_float2(u.y, -u.x);  // (-i)^(a b)
    const float2 q = dpp_c<DPP_XOR1>(u);
    v[k] = make_float2(fmaf(sa, u.x, q.x), fmaf(sa, u.y, q.y));
  }
  wave_lds_sync();  // stage-2 reads done before the planes are reused for Z
  const int k3 = qb + 2 * qa;
#pragma unroll
  for (int k = 0; k < 16; ++k) {
    const int idx = k1 + 16 * k + 264 * k3;  // Z index + 8 * (index >> 8)
    s_re[idx] = v[k].x;
    s_im[idx] = v[k].y;
  }
  wave_lds_sync();

  // ---- real-input split and magnitude.  Lane pairs k with M-k: with e = (Z[k] + conj Z[M-k])/2,
  // o = (Z[k] - conj Z[M-k])/(2i): X[k] = e + W^k o and X[M-k] = conj(e - W^k o), so one pair
  // of Z reads gives both magnitudes (k = 0 gives X[0] and X[M]).  All Z reads finish before the
  // magnitudes overwrite the re plane (mag[k] at plain index k).
  const float2 bs = tw[lane];  // W2048^lane; W2048^(lane + 64 i) = bs * W32^i
  float mk[9], mc[9];
#pragma unroll
  for (int i = 0; i < 9; ++i) {
    const int k = lane + 64 * i;
    const int kk = k <= M / 2 ? k : 0;
    const int ic = kk == 0 ? 0 : M - kk;
    const int ak = kk + 8 * (kk >> 8), ac = ic + 8 * (ic >> 8);
    const float2 zk = make_float2(s_re[ak], s_im[ak]);
    const float2 zc = make_float2(s_re[ac], s_im[ac]);
    const float2 e = make_float2(0.5f * (zk.x + zc.x), 0.5f * (zk.y - zc.y));
    const float2 dd = make_float2(zk.x - zc.x, zk.y + zc.y);
    const float2 o = make_float2(0.5f * dd.y, -0.5f * dd.x);
    const float2 wk = i == 0 ? bs : cmul(bs, make_float2(W32_RE[i], W32_IM[i]));
    const float2 wo = cmul(wk, o);
    const float pr = e.x + wo.x, pi = e.y + wo.y, qr = e.x - wo.x, qi = e.y - wo.y;
    mk[i] = __builtin_amdgcn_sqrtf(pr * pr + pi * pi);
    mc[i] = __builtin_amdgcn_sqrtf(qr * qr + qi * qi);
  }
  wave_lds_sync();
  float* s_mag = s_re;
#pragma unroll
  for (int i = 0; i < 9; ++i) {
    const int k = lane + 64 * i;
    if (k <= M / 2) {
      s_mag[k] = mk[i];
      if (k < M / 2) s_mag[M - k] = mc[i];
    }
  }
  wave_lds_sync();

  // ---- banded mel + log: lane owns bands lane and lane + 64 (host: n_mels <= 128), weights
  // from the workgroup's LDS rows (zero past a band's support; magnitude index clamped)
  if (!active) return;
  float* dst = out + (int64_t)gframe * n_mels;
#pragma unroll
  for (int h = 0; h < 2; ++h) {
    const int m = lane + 64 * h;
    if (m < n_mels) {
      const int2 bd = band[m];
      const int st = bd.x & 0xFFFF, l4 = bd.x >> 16;
      const float4* wr = s_w4 + bd.y;
      float acc = 0.f;
      for (int c = 0; c < l4; ++c) {
        const float4 wq = wr[c];
        const int bi = st + 4 * c;
        acc += wq.x * s_mag[min(bi, M)];
        acc += wq.y * s_mag[min(bi + 1, M)];
        acc += wq.z * s_mag[min(bi + 2, M)];
        acc += wq.w * s_mag[min(bi + 3, M)];
      }
      dst[m] = __logf(acc + log_offset);
    }
  }
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
  int n_w4 = 0;
  for (int m = 0; m < n_mels; ++m) n_w4 += (len[m] + 3) / 4;
  A2M_CHECK_ARG(nfft != 2048 || n_mels > 128 || n_w4 <= LM_MAX_W4,
                "logmel: %d weight rows exceed the kernel's LDS copy", n_w4);
  size_t total;
  plan_layout(win, nfft, n_mels, h.nnz, n_w4, &h, &total);
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
  if (nfft == 2048) {  // same CSR weights, each band's row zero-padded to whole float4s:
    // band[m] = {start | len4 << 16, row offset in float4s}
    int32_t* band = reinterpret_cast<int32_t*>(p + h.off_band);
    float* w4 = reinterpret_cast<float*>(p + h.off_w4);
    int o4 = 0;
    for (int m = 0; m < n_mels; ++m) {
      const int l4 = (len[m] + 3) / 4;
      band[2 * m] = start[m] | (l4 << 16);
      band[2 * m + 1] = o4;
      for (int q = 0; q < len[m]; ++q) w4[4 * o4 + q] = vals[woff[m] + q];
      o4 += l4;
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
  static const bool generic_only = std::getenv("A2M_LOGMEL_GENERIC") != nullptr;
  // register-FFT path.  Its LDS copy of the band rows always fits: with strictly increasing
  // mel edges a bin lies inside at most two triangles, so nnz <= 2 * 1025 and
  // n_w4 <= (nnz + 3 n_mels) / 4 <= 609 < LM_MAX_W4 (build_plan asserts it).
  if (fft_len == 2048 && n_mels <= 128 && !generic_only) {
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
