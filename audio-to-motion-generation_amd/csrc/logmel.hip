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
#include <cstring>
#include <vector>

#include "a2m_internal.h"

namespace a2m {

struct PlanHeader {
  int32_t window, hop, fft_len, n_mels, n_bins, nnz;
  int32_t off_window, off_twiddle, off_start, off_len, off_woff, off_weights;  // byte offsets
};

static size_t align16(size_t x) { return (x + 15) & ~size_t(15); }

static void plan_layout(int win, int nfft, int n_mels, int nnz, PlanHeader* h, size_t* total) {
  size_t off = align16(sizeof(PlanHeader));
  h->off_window = (int32_t)off; off = align16(off + sizeof(float) * win);
  h->off_twiddle = (int32_t)off; off = align16(off + sizeof(float) * 2 * nfft);
  h->off_start = (int32_t)off; off = align16(off + sizeof(int32_t) * n_mels);
  h->off_len = (int32_t)off; off = align16(off + sizeof(int32_t) * n_mels);
  h->off_woff = (int32_t)off; off = align16(off + sizeof(int32_t) * n_mels);
  h->off_weights = (int32_t)off; off = align16(off + sizeof(float) * nnz);
  *total = off;
}

static bool geometry(int sr, double win_s, double hop_s, int* win, int* hop, int* nfft) {
  *win = (int)std::lround(sr * win_s);
  *hop = (int)std::lround(sr * hop_s);
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
  size_t total;
  plan_layout(win, nfft, n_mels, h.nnz, &h, &total);
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
  hipLaunchKernelGGL(logmel_kernel, dim3((unsigned)(n_clips * nf)), dim3(256), lds,
                     as_stream(stream), wave, clip_stride, (int)nf,
                     static_cast<const unsigned char*>(dev_plan), log_offset, out);
  A2M_LAUNCH_CHECK();
  return A2M_OK;
}

}  // extern "C"
