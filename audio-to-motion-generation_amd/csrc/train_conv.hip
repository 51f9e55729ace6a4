// Convolution backward on the implicit-GEMM engine.
//
// dgrad: dX = conv_transpose(dY, W).  Decomposed by output phase (rh, rw) so a stride-s
// conv's dgrad never multiplies the (s^2 - 1)/s^2 structural zeros a naive transposed
// convolution would: phase (rh, rw) of dX only meets the taps with (r + pad - k) % s == 0,
// each a dense GEMM over K = Co * taps_h * taps_w with per-phase packed weights.
// wgrad: dW[co][ci,kh,kw] = sum_{b,ho,wo} dY[b][co][ho][wo] X[b][ci][ho*s+kh-ph][wo*s+kw-pw],
// a GEMM over K = B*Ho*Wo with split-K (partials reduced in a fixed order).
// 1-D convs are the H = 1 case; ConvTranspose1d's dgrad / wgrad are a plain conv forward /
// this wgrad with the operands' roles exchanged (see a2m.autograd).
#include <algorithm>
#include <cstdlib>

#include "a2m_internal.h"

namespace a2m {

struct PhaseTaps {
  int k0, n;  // first tap, tap count (taps are k0, k0 + s, ...)
};

static PhaseTaps phase_taps_h(int r, int k, int s, int pad) {
  PhaseTaps t{-1, 0};
  for (int kk = 0; kk < k; ++kk)
    if ((((r + pad - kk) % s) + s) % s == 0) { if (t.k0 < 0) t.k0 = kk; ++t.n; }
  return t;
}

// P_(rh,rw)[ci][(co*nth + th)*ntw + tw] = W[co][ci][kh0 + s*th][kw0 + s*tw]
// One block row per ci (blockIdx.y) and 32-bit index math: the flat 64-bit form spent four
// 64-bit divisions per element, which made the large UNet weights' packs VALU-bound.
__global__ void dgrad_pack_kernel(const float* w, int Co, int Ci, int kh, int kw, int nth, int ntw,
                                  int kh0, int kw0, int sh, int sw, float* out) {
  const int ci = blockIdx.y;
  const int per = Co * nth * ntw;   // packed row length (< 2^31: host)
  const int ntap = nth * ntw;
  float* orow = out + (int64_t)ci * per;
  for (int j = blockIdx.x * blockDim.x + threadIdx.x; j < per; j += gridDim.x * blockDim.x) {
    const int co = j / ntap;
    const int t = j - co * ntap;
    const int th = ntw == 1 ? t : t / ntw;
    const int tw = t - th * ntw;
    orow[j] = w[(((int64_t)co * Ci + ci) * kh + kh0 + sh * th) * kw + kw0 + sw * tw];
  }
}

// The dgrad of a stride-1 "same" conv1d is that conv1d of dY with W'[ci][co][j] = W[co][ci][ks-1-j]:
// W' packed tap-chunked ([Ci][Co/CH][ks][CH], the k order of loader mode 5) so the engine runs it
// as the forward's tap conv (the pipelined tile's halo / per-tap layouts) instead of a mode-3
// gather over (co, tap)
__global__ void dgrad_tap_pack_kernel(const float* w, int Co, int Ci, int ks, int ch, float* out) {
  // one block row per ci (blockIdx.y), 32-bit index math, the packed row written contiguously
  // (dgrad_pack_kernel's layout of the work)
  const int ci = blockIdx.y;
  const int per = Co * ks;   // packed row length (< 2^31: host)
  const int cch = ks * ch;
  float* orow = out + (int64_t)ci * per;
  for (int o = blockIdx.x * blockDim.x + threadIdx.x; o < per; o += gridDim.x * blockDim.x) {
    const int cc = o / cch, rem = o - cc * cch;
    const int j = rem / ch, cl = rem - j * ch;
    orow[o] = w[((int64_t)(cc * ch + cl) * Ci + ci) * ks + (ks - 1 - j)];
  }
}

}  // namespace a2m

using namespace a2m;

extern "C" {

int a2m_conv2d_dgrad_f32(const float* dy, int32_t B, int32_t Co, int32_t Ho, int32_t Wo,
                         const float* w, int32_t Ci, int32_t H, int32_t W, int32_t kh, int32_t kw,
                         int32_t stride_h, int32_t stride_w, int32_t pad_h, int32_t pad_w,
                         float* dx, int64_t dxs_b, int64_t dxs_c, int64_t dxs_h, int64_t dxs_w,
                         int32_t accumulate, void* ws, size_t ws_bytes, void* stream) {
  A2M_CHECK_ARG(dy && w && dx && B > 0 && Co > 0 && Ci > 0 && H > 0 && W > 0 && kh > 0 && kw > 0 &&
                    stride_h > 0 && stride_w > 0 && pad_h >= 0 && pad_w >= 0,
                "conv_dgrad: bad args");
  A2M_CHECK_ARG(Ho == (H + 2 * pad_h - kh) / stride_h + 1 && Wo == (W + 2 * pad_w - kw) / stride_w + 1,
                "conv_dgrad: output geometry mismatch");
  A2M_CHECK_ARG((int64_t)B * Co * Ho * Wo < (1LL << 31) && (int64_t)B * dxs_b < (1LL << 31),
                "conv_dgrad: too large");
  A2M_CHECK_ARG(Ci <= 65535 && (int64_t)Co * kh * kw < (1LL << 31), "conv_dgrad: Ci %d > 65535 (pack grid)", Ci);
  const size_t pack_bytes = ((size_t)Ci * Co * kh * kw * sizeof(float) + 255) & ~size_t(255);
  if (!ws || ws_bytes < pack_bytes) {
    set_error("conv_dgrad: workspace too small (%zu < %zu bytes)", ws_bytes, pack_bytes);
    return A2M_EWS;
  }
  hipStream_t st = as_stream(stream);
  float* packed = static_cast<float*>(ws);
  // 1-D, stride 1, 3 taps, pad 1, clips that tile the 64-row block: the tap conv (A2M_DGRAD_TAP=0:
  // the phase GEMM below for every conv)
  const int chunk = gemm_k_tile();
  if (H == 1 && kh == 1 && pad_h == 0 && stride_h == 1 && stride_w == 1 && kw == 3 && pad_w == 1 &&
      Wo == W && W % 4 == 0 && 64 % W == 0 && Co % chunk == 0 &&
      (reinterpret_cast<uintptr_t>(dy) % 16) == 0 && ((int64_t)Co * W) % 4 == 0) {
    hipLaunchKernelGGL(dgrad_tap_pack_kernel, dim3((unsigned)std::min<int64_t>(cdiv((int64_t)Co * kw, 256), 64), (unsigned)Ci),
                       dim3(256), 0, st, w, Co, Ci, kw, chunk, packed);
    A2M_LAUNCH_CHECK();
    Gather A = dense_rk(packed, Co * kw);
    Gather Bg{};
    Bg.base = dy; Bg.bstride = 0;
    Bg.sr0 = Co * W; Bg.R1 = 1; Bg.R2 = W; Bg.sk0 = W;
    Bg.K1 = Bg.K2 = 1; Bg.divh = Bg.divw = 1; Bg.Lh = Bg.Lw = 1;
    Bg.cw = -pad_w; Bg.tapconv = kw;
    Epilogue E = epi_dense(dx, 0);
    E.N1 = 1; E.N2 = W; E.so0 = (int)dxs_b; E.so1 = 0; E.so2 = (int)dxs_w; E.som = (int)dxs_c;
    E.accumulate = accumulate;
    int rc = gemm(A, Bg, E, Ci, B * W, Co * kw, 1, static_cast<char*>(ws) + pack_bytes, ws_bytes - pack_bytes, st);
    if (rc == A2M_EWS)
      set_error("conv_dgrad: workspace too small (%zu < %zu bytes)", ws_bytes,
                pack_bytes + gemm_ws_bytes(Ci, B * W, Co * kw, 1));
    return rc;
  }
  // 1-D, stride s > 1 with s * Wo == W: dX is the ConvTranspose1d of dY with W read as its
  // [in = Co][out = Ci][k] weight -- per output phase a tap conv of dY (the eval ConvTranspose's
  // tap-chunked pack and phases), clips of Wo rows that tile the 64-row block
  if (H == 1 && kh == 1 && pad_h == 0 && stride_h == 1 && stride_w > 1 && stride_w * Wo == W &&
      Wo % 4 == 0 && 64 % Wo == 0 && Co % chunk == 0 && (reinterpret_cast<uintptr_t>(dy) % 16) == 0) {
    bool shifts_ok = true;
    for (int r = 0; r < stride_w; ++r) {
      const PhaseTaps tw = phase_taps_h(r, kw, stride_w, pad_w);
      if (tw.n == 0) continue;
      const int cw = (r + pad_w - tw.k0) / stride_w - tw.n + 1;
      shifts_ok = shifts_ok && tw.n <= 3 && cw > -Wo && cw + tw.n - 1 < Wo;
    }
    if (shifts_ok) {
      int rc = a2m_convt1d_tap_pack_f32(w, Co, Ci, kw, stride_w, pad_w, chunk, packed, stream);
      if (rc) return rc;
      size_t off = 0;
      for (int r = 0; r < stride_w; ++r) {
        const PhaseTaps tw = phase_taps_h(r, kw, stride_w, pad_w);
        Epilogue E = epi_dense(dx + r * dxs_w, 0);
        E.N1 = 1; E.N2 = Wo; E.so0 = (int)dxs_b; E.so1 = 0; E.so2 = (int)(stride_w * dxs_w); E.som = (int)dxs_c;
        E.accumulate = accumulate;
        if (tw.n == 0) {   // no tap reaches this phase: zeros (or nothing added)
          rc = gemm(dense_rk(packed, 1), dense_rk(dy, 1), E, Ci, B * Wo, 0, 1, nullptr, 0, st);
          if (rc) return rc;
          continue;
        }
        Gather Bg{};
        Bg.base = dy; Bg.bstride = 0;
        Bg.sr0 = Co * Wo; Bg.R1 = 1; Bg.R2 = Wo; Bg.sk0 = Wo;
        Bg.K1 = Bg.K2 = 1; Bg.divh = Bg.divw = 1; Bg.Lh = Bg.Lw = 1;
        Bg.cw = (r + pad_w - tw.k0) / stride_w - tw.n + 1; Bg.tapconv = tw.n;
        rc = gemm(dense_rk(packed + off, tw.n * Co), Bg, E, Ci, B * Wo, tw.n * Co, 1,
                  static_cast<char*>(ws) + pack_bytes, ws_bytes - pack_bytes, st);
        if (rc == A2M_EWS)
          set_error("conv_dgrad: workspace too small (%zu < %zu bytes)", ws_bytes,
                    pack_bytes + gemm_ws_bytes(Ci, B * Wo, tw.n * Co, 1));
        if (rc) return rc;
        off += (size_t)Ci * tw.n * Co;
      }
      return A2M_OK;
    }
  }
  for (int rh = 0; rh < stride_h; ++rh) {
    const int nuh = (H - rh + stride_h - 1) / stride_h;
    if (nuh <= 0) continue;
    const PhaseTaps th = phase_taps_h(rh, kh, stride_h, pad_h);
    for (int rw = 0; rw < stride_w; ++rw) {
      const int nuw = (W - rw + stride_w - 1) / stride_w;
      if (nuw <= 0) continue;
      const PhaseTaps tw = phase_taps_h(rw, kw, stride_w, pad_w);
      const int K = Co * th.n * tw.n;
      Epilogue E = epi_dense(dx + rh * dxs_h + rw * dxs_w, 0);
      E.N1 = nuh; E.N2 = nuw; E.so0 = (int)dxs_b; E.so1 = (int)(stride_h * dxs_h);
      E.so2 = (int)(stride_w * dxs_w); E.som = (int)dxs_c; E.accumulate = accumulate;
      Gather A = dense_rk(packed, std::max(K, 1));
      Gather Bg{};
      Bg.base = dy; Bg.sr0 = Co * Ho * Wo; Bg.R1 = nuh; Bg.R2 = nuw; Bg.ar1 = 1; Bg.ar2 = 1;
      Bg.sk0 = Ho * Wo; Bg.K1 = std::max(th.n, 1); Bg.K2 = std::max(tw.n, 1); Bg.bk1 = -1; Bg.bk2 = -1;
      Bg.ch = K ? (rh + pad_h - th.k0) / stride_h : 0;
      Bg.cw = K ? (rw + pad_w - tw.k0) / stride_w : 0;
      Bg.divh = Bg.divw = 1; Bg.Lh = Ho; Bg.Lw = Wo; Bg.sh = Wo; Bg.sw = 1; Bg.kcontig = 0;
      if (K > 0) {
        hipLaunchKernelGGL(dgrad_pack_kernel, dim3((unsigned)std::min<int64_t>(cdiv(K, 256), 64), (unsigned)Ci),
                           dim3(256), 0, st, w, Co, Ci, kh, kw, th.n, tw.n, th.k0, tw.k0, stride_h,
                           stride_w, packed);
        A2M_LAUNCH_CHECK();
      }
      int rc = gemm(A, Bg, E, Ci, B * nuh * nuw, K, 1, static_cast<char*>(ws) + pack_bytes,
                    ws_bytes - pack_bytes, st);
      if (rc == A2M_EWS) {
        set_error("conv_dgrad: workspace too small (%zu < %zu bytes)", ws_bytes,
                  pack_bytes + gemm_ws_bytes(Ci, B * nuh * nuw, K, 1));
        return rc;
      }
      if (rc) return rc;
    }
  }
  return A2M_OK;
}

int a2m_conv2d_wgrad_f32(const float* dy, int32_t B, int32_t Co, int32_t Ho, int32_t Wo,
                         const float* x, int64_t xs_b, int64_t xs_c, int64_t xs_h, int64_t xs_w,
                         int32_t Ci, int32_t H, int32_t W, int32_t kh, int32_t kw,
                         int32_t stride_h, int32_t stride_w, int32_t pad_h, int32_t pad_w,
                         float* dw, int32_t accumulate, void* ws, size_t ws_bytes, void* stream) {
  A2M_CHECK_ARG(dy && x && dw && B > 0 && Co > 0 && Ci > 0 && Ho > 0 && Wo > 0, "conv_wgrad: bad args");
  A2M_CHECK_ARG((int64_t)B * Co * Ho * Wo < (1LL << 31) && (int64_t)B * xs_b < (1LL << 31),
                "conv_wgrad: too large");
  // k = (b, ho, wo).  (Padding wo up to a multiple of 4 so that Wo = 15 rows load as mode-4
  // float4 runs measured slower: the encoder's (3, 8) conv wgrad 0.91 -> 1.12 ms a call, the
  // shifted x runs being unaligned; so odd widths keep the element gathers.)
  const int Wk = Wo;
  // A(m=co, k=(b,ho,wo)) = dY[b][co][ho][wo]   (dY contiguous): (ho, wo) is one unit-stride
  // digit of Ho * Wo, so the rows load as float4 runs (loader mode 4) whenever Ho * Wo % 4 == 0,
  // also for odd Wo (the encoder's (3, 8) conv, Wo = 15) -- the same k order as X's (b, ho, wo)
  // digits, so the same products in the same order as the element gather it replaces
  Gather A{};
  A.base = dy; A.sr0 = Ho * Wo; A.R1 = A.R2 = 1;
  A.sk0 = Co * Ho * Wo; A.K1 = 1; A.K2 = Ho * Wk; A.bk1 = 1; A.bk2 = 1; A.Lh = 1; A.Lw = Ho * Wo;
  A.sh = 0; A.sw = 1; A.divh = A.divw = 1; A.kcontig = 1;
  // B(n=(ci,ih,iw), k=(b,ho,wo)) = X[b][ci][ho*s + ih - ph][wo*s + iw - pw]
  Gather Bg{};
  Bg.base = x; Bg.sr0 = (int)xs_c; Bg.R1 = kh; Bg.R2 = kw; Bg.ar1 = 1; Bg.ar2 = 1;
  Bg.sk0 = (int)xs_b; Bg.K1 = Ho; Bg.K2 = Wk; Bg.bk1 = stride_h; Bg.bk2 = stride_w;
  Bg.ch = -pad_h; Bg.cw = -pad_w; Bg.divh = Bg.divw = 1; Bg.Lh = H; Bg.Lw = W;
  Bg.sh = (int)xs_h; Bg.sw = (int)xs_w; Bg.kcontig = 1;
  Epilogue E = epi_dense(dw, Ci * kh * kw);
  E.accumulate = accumulate;
  return gemm(A, Bg, E, Co, Ci * kh * kw, B * Ho * Wk, 1, ws, ws_bytes, as_stream(stream));
}

int a2m_gemm_f32(int32_t M, int32_t N, int32_t N1, int32_t K, int32_t K1, int32_t batch,
                 const float* A, int64_t a_bs, int64_t a_m, int64_t a_k0, int64_t a_k1,
                 const float* B, int64_t b_bs, int64_t b_n0, int64_t b_n1, int64_t b_k0,
                 int64_t b_k1, float* C, int64_t c_bs, int64_t c_m, int64_t c_n0, int64_t c_n1,
                 const float* bias, float alpha, int32_t accumulate, void* ws, size_t ws_bytes,
                 void* stream) {
  A2M_CHECK_ARG(A && B && C && M > 0 && N > 0 && K >= 0 && batch > 0 && N1 > 0 && K1 > 0 &&
                    N % N1 == 0 && K % K1 == 0, "gemm: bad args");
  A2M_CHECK_ARG(alpha == 1.f, "gemm: only alpha = 1 is supported");
  auto fits = [](int64_t v) { return v > -(1LL << 31) && v < (1LL << 31); };
  A2M_CHECK_ARG(fits(a_m) && fits(a_k0) && fits(a_k1) && fits(b_n0) && fits(b_n1) && fits(b_k0) &&
                    fits(b_k1) && fits(c_m) && fits(c_n0) && fits(c_n1), "gemm: stride too large");
  Gather Ag{};
  Ag.base = A; Ag.bstride = a_bs; Ag.sr0 = (int)a_m; Ag.R1 = Ag.R2 = 1;
  Ag.sk0 = (int)a_k0; Ag.K1 = K1; Ag.K2 = 1; Ag.bk1 = 1; Ag.sh = (int)a_k1; Ag.Lh = K1; Ag.Lw = 1;
  Ag.divh = Ag.divw = 1;
  Ag.kcontig = (K1 > 1 ? a_k1 == 1 : a_k0 == 1) ? 1 : 0;
  if (K1 == 1 && Ag.kcontig) { Ag.sh = 0; Ag.bk1 = 0; }  // plain [M][K] -> vectorisable
  Gather Bg{};
  Bg.base = B; Bg.bstride = b_bs; Bg.sr0 = (int)b_n0; Bg.R1 = 1; Bg.R2 = N1; Bg.ar2 = 1;
  Bg.sw = (int)b_n1; Bg.Lw = N1; Bg.sk0 = (int)b_k0; Bg.K1 = K1; Bg.K2 = 1; Bg.bk1 = 1;
  Bg.sh = (int)b_k1; Bg.Lh = K1; Bg.divh = Bg.divw = 1;
  Bg.kcontig = (K1 > 1 ? b_k1 == 1 : b_k0 == 1) ? 1 : 0;
  if (N1 == 1 && K1 == 1 && Bg.kcontig) { Bg.R2 = 1; Bg.ar2 = 0; Bg.sw = 0; Bg.sh = 0; Bg.bk1 = 0; }
  Epilogue E = epi_dense(C, 0, c_bs);
  E.N1 = 1; E.N2 = N1; E.so0 = (int)c_n0; E.so2 = (int)c_n1; E.som = (int)c_m;
  E.bias = bias; E.accumulate = accumulate;
  return gemm(Ag, Bg, E, M, N, K, batch, ws, ws_bytes, as_stream(stream));
}

}  // extern "C"
