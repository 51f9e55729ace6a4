/*
 * a2m.h -- C-ABI of liba2m_hip.so, the MI355X (gfx950) audio -> 2-D pose hot path.
 *
 * Every entry point takes caller-owned DEVICE pointers, explicit sizes / element strides
 * and a hipStream_t passed as void*.  Nothing allocates device memory: scratch comes from
 * the caller through (ws, ws_bytes).  Calls are stream-ordered and reentrant (no hidden
 * global state besides the thread-local error string), so they are safe to capture into
 * a hipGraph.  Return value: 0 = ok, A2M_EINVAL (bad shape / argument), A2M_EHIP (HIP
 * error), A2M_EWS (workspace too small); a2m_last_error() holds the message.
 *
 * The reference (Xukai-UoA/Audio-to-Motion-Generation) is pure Python/PyTorch; each entry
 * cites the reference code it replaces (file:line, paths relative to the reference root).
 * Tensor layouts follow the reference's PyTorch layouts: [B][C][T] for 1-D feature maps,
 * [B][C][H][W] for 2-D, [B][T][F] for pose / mel.
 */
#ifndef A2M_H_
#define A2M_H_

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define A2M_OK 0
#define A2M_EINVAL -1
#define A2M_EHIP -2
#define A2M_EWS -3

/* activation codes used by the *_fwd entry points */
#define A2M_ACT_NONE 0
#define A2M_ACT_RELU 1
#define A2M_ACT_LRELU 2

const char* a2m_last_error(void);
int a2m_version(void);

/* ---------------------------------------------------------------- log-mel front end
 * Replaces pose_video/mel_features.py:192-223 (log_mel_spectrogram) with its helpers
 * frame :21, periodic_hann :48, stft_magnitude :71, spectrogram_to_mel_matrix :114.
 * Plan = periodic Hann window + FFT twiddles + banded (CSR) mel filterbank, built on the
 * HOST in float64 exactly as the reference builds its matrix, then copied by the caller
 * to device memory once.  a2m_logmel_plan_build returns A2M_EINVAL with the reference's
 * ValueError text for bad band edges (mel_features.py:156-163).
 */
int64_t a2m_logmel_num_frames(int64_t n_samples, int32_t window, int32_t hop);
int a2m_logmel_geometry(int32_t sample_rate, double window_secs, double hop_secs,
                        int32_t* window, int32_t* hop, int32_t* fft_len);
size_t a2m_logmel_plan_bytes(int32_t sample_rate, double window_secs, double hop_secs,
                             int32_t n_mels, double lower_hz, double upper_hz);
int a2m_logmel_plan_build(int32_t sample_rate, double window_secs, double hop_secs,
                          int32_t n_mels, double lower_hz, double upper_hz,
                          void* host_plan, size_t plan_bytes);
/* wave[c][s] at wave + c*clip_stride + s (float32, n_samples per clip);
 * out[c][f][m] at out + (c*n_frames + f)*n_mels + m, n_frames = a2m_logmel_num_frames() */
int a2m_logmel_f32(const float* wave, int64_t n_clips, int64_t clip_stride, int64_t n_samples,
                   int32_t window, int32_t hop, int32_t fft_len, int32_t n_mels,
                   const void* dev_plan, float log_offset, float* out, void* stream);

/* ---------------------------------------------------------------- convolutions
 * ConvNormRelu (model_layers.py:51-118) forward in eval mode: conv + bias, optional
 * BatchNorm (running stats; bn_w == NULL disables it), activation (A2M_ACT_*, LeakyReLU
 * slope), all fused into the MFMA implicit-GEMM epilogue.  Also used for nn.Linear
 * (kernel 1, T = rows) and 1x1 convs.  Element (b, c, t) of x lives at
 * x + b*xs_b + c*xs_c + t*xs_t, same for y; Tout = (Tin + 2*pad - ks)/stride + 1.
 */
int a2m_conv1d_fwd_f32(const float* x, int64_t xs_b, int64_t xs_c, int64_t xs_t,
                       int32_t B, int32_t Ci, int32_t Tin,
                       const float* w, const float* bias, int32_t Co, int32_t ks,
                       int32_t stride, int32_t pad,
                       const float* bn_w, const float* bn_b, const float* bn_rm,
                       const float* bn_rv, float bn_eps, int32_t act, float slope,
                       float* y, int64_t ys_b, int64_t ys_c, int64_t ys_t,
                       void* ws, size_t ws_bytes, void* stream);

/* ConvTranspose1D (model_layers.py:193-215): ConvTranspose1d(k, stride, pad, out_pad)
 * + BN + ReLU.  w is [Ci][Co][ks]; Tout = (Tin-1)*stride - 2*pad + ks + out_pad. */
int a2m_convt1d_fwd_f32(const float* x, int64_t xs_b, int64_t xs_c, int32_t B, int32_t Ci,
                        int32_t Tin, const float* w, const float* bias, int32_t Co, int32_t ks,
                        int32_t stride, int32_t pad, int32_t out_pad,
                        const float* bn_w, const float* bn_b, const float* bn_rm,
                        const float* bn_rv, float bn_eps, int32_t act, float slope,
                        float* y, int64_t ys_b, int64_t ys_c,
                        void* ws, size_t ws_bytes, void* stream);
/* Tap-chunked conv1d (stride 1, "same" padding 2*pad == ks-1): the forward of
 * model_layers.py ConvNormRelu(type='1d') / ResBlock convs (nn.Conv1d(k=3, s=1, p=1),
 * model_layers.py:75-120) without an im2col matrix.  Weights are packed once per weight version
 * by a2m_conv1d_tap_pack_f32 as [Co][Ci/chunk][ks][chunk] with chunk = a2m_conv1d_tap_chunk()
 * (the engine's k-tile at the current precision: 32 fp32 / bf16x6, 64 bf16); the GEMM's B
 * loader reads each chunk's x[b][c][t] window once and re-stores it shifted for every tap.
 * x: [B][Ci][T] with unit t stride and 16-byte aligned rows; T % 4 == 0 and 64 % T == 0 (the
 * tiles hold whole clips).  Epilogue (bias, BN-eval, activation) and output strides as
 * a2m_conv1d_fwd_f32. */
int32_t a2m_conv1d_tap_chunk(void);
int a2m_conv1d_tap_pack_f32(const float* w, int32_t Co, int32_t Ci, int32_t ks, int32_t chunk,
                            float* packed, void* stream);
int a2m_conv1d_tap_fwd_f32(const float* x, int64_t xs_b, int64_t xs_c, int32_t B, int32_t Ci,
                           int32_t T, const float* packed, int32_t chunk, const float* bias,
                           int32_t Co, int32_t ks, int32_t pad, const float* bn_w,
                           const float* bn_b, const float* bn_rm, const float* bn_rv, float bn_eps,
                           int32_t act, float slope, float* y, int64_t ys_b, int64_t ys_c,
                           int64_t ys_t, void* ws, size_t ws_bytes, void* stream);
/* G independent tap-chunked conv1d problems in one launch (the body and hand decoders' layers
 * of equal shape): problem g reads x + g*xs_g, weights packed + g*w_gs (each packed by
 * a2m_conv1d_tap_pack_f32), bias / BN arrays at + g*Co, and writes y + g*ys_g (group strides
 * are element offsets of either sign; xs_g may be 0 for a shared input).  Any of
 * bias / BN may be NULL for all problems.  Otherwise as a2m_conv1d_tap_fwd_f32. */
int a2m_conv1d_tap_group_fwd_f32(const float* x, int64_t xs_g, int64_t xs_b, int64_t xs_c, int32_t G,
                                 int32_t B, int32_t Ci, int32_t T, const float* packed, int64_t w_gs,
                                 int32_t chunk, const float* bias, int32_t Co, int32_t ks, int32_t pad,
                                 const float* bn_w, const float* bn_b, const float* bn_rm,
                                 const float* bn_rv, float bn_eps, int32_t act, float slope, float* y,
                                 int64_t ys_g, int64_t ys_b, int64_t ys_c, int64_t ys_t, void* ws,
                                 size_t ws_bytes, void* stream);
/* The same split in two: the per-phase weight packing (packed: Ci*Co*k floats) and the
 * forward on packed weights (callers cache the packing while the weights are unchanged). */
int a2m_convt1d_pack_f32(const float* w, int32_t Ci, int32_t Co, int32_t ks, int32_t stride,
                         int32_t pad, float* packed, void* stream);
int a2m_convt1d_packed_fwd_f32(const float* x, int64_t xs_b, int64_t xs_c, int32_t B, int32_t Ci,
                               int32_t Tin, const float* packed, const float* bias, int32_t Co,
                               int32_t ks, int32_t stride, int32_t pad, int32_t out_pad,
                               const float* bn_w, const float* bn_b, const float* bn_rm,
                               const float* bn_rv, float bn_eps, int32_t act, float slope, float* y,
                               int64_t ys_b, int64_t ys_c, void* ws, size_t ws_bytes, void* stream);
/* The same forward with each phase as a stride-1 tap-chunked conv1d (the GEMM engine's loader
 * mode 5: a channel chunk's x window is loaded once for all of the phase's taps).  Weights
 * packed per phase in `chunk`-channel chunks with reversed taps (chunk = a2m_conv1d_tap_chunk(),
 * Ci % chunk == 0); every phase must hold Tin outputs (Tout = stride * Tin), Tin % 4 == 0 and
 * 64 % Tin == 0, x rows 16-byte aligned.  Replaces nn.ConvTranspose1d.forward at the
 * ConvTranspose1D shapes (model_layers.py:193-215, the UNet up path at :325). */
int a2m_convt1d_tap_pack_f32(const float* w, int32_t Ci, int32_t Co, int32_t ks, int32_t stride,
                             int32_t pad, int32_t chunk, float* packed, void* stream);
int a2m_convt1d_tap_fwd_f32(const float* x, int64_t xs_b, int64_t xs_c, int32_t B, int32_t Ci,
                            int32_t Tin, const float* packed, int32_t chunk, const float* bias,
                            int32_t Co, int32_t ks, int32_t stride, int32_t pad, int32_t out_pad,
                            const float* bn_w, const float* bn_b, const float* bn_rm,
                            const float* bn_rv, float bn_eps, int32_t act, float slope, float* y,
                            int64_t ys_b, int64_t ys_c, void* ws, size_t ws_bytes, void* stream);

/* Channels-last conv2d for the AudioEncoder eval chain (model_layers.py:219-280,
 * ConvNormRelu(type='2d') layers): x NHWC [B][H][W][Ci] (the mel [B][T][F] is already NHWC with
 * Ci = 1), weights packed once by a2m_conv2d_pack_nhwc_f32 as [Co][kh][kw][Ci], output NHWC
 * [B][Hout][Wout][Co] (y_nhwc = 1) or NCHW (0), only columns [w_lo, w_hi) computed.  The GEMM's
 * activation operand is a unit-stride run of kw*Ci floats per (row, kernel row) -- float4 loads,
 * no im2col matrix and no transposed staging.  Requires (kw * Ci) % 4 == 0. */
int a2m_conv2d_pack_nhwc_f32(const float* w, int32_t Co, int32_t Ci, int32_t kh, int32_t kw,
                             float* packed, void* stream);
int a2m_conv2d_nhwc_fwd_f32(const float* x, int32_t B, int32_t Ci, int32_t H, int32_t W,
                            const float* packed, const float* bias, int32_t Co, int32_t kh,
                            int32_t kw, int32_t stride, int32_t pad_h, int32_t pad_w,
                            const float* bn_w, const float* bn_b, const float* bn_rm,
                            const float* bn_rv, float bn_eps, int32_t act, float slope, float* y,
                            int32_t y_nhwc, int32_t Hout, int32_t Wout, int32_t w_lo, int32_t w_hi,
                            void* ws, size_t ws_bytes, void* stream);
/* The AudioEncoder's last ConvNormRelu plus its time resample (model_layers.py:272-279): the
 * channels-last conv of a2m_conv2d_nhwc_fwd_f32 restricted to the one output column w_col that
 * F.interpolate(size=(T,1), mode='bilinear', align_corners=False) reads (it must be that
 * resample's only live column: Wout/2 - 1/2 == w_col, else A2M_EINVAL), with the resample fused
 * into the GEMM's reduce: y [B][Co][T] equals a2m_conv2d_nhwc_fwd_f32 (y_nhwc = 0) followed by
 * a2m_interp_time_f32, bit for bit, without the intermediate tensor or the second launch.
 * Replaces the last conv + interpolate of AudioEncoder.forward (model_layers.py:271-280). */
int a2m_conv2d_nhwc_interp_fwd_f32(const float* x, int32_t B, int32_t Ci, int32_t H, int32_t W,
                                   const float* packed, const float* bias, int32_t Co, int32_t kh,
                                   int32_t kw, int32_t stride, int32_t pad_h, int32_t pad_w,
                                   const float* bn_w, const float* bn_b, const float* bn_rm,
                                   const float* bn_rv, float bn_eps, int32_t act, float slope,
                                   float* y, int32_t T, int32_t Hout, int32_t Wout, int32_t w_col,
                                   void* ws, size_t ws_bytes, void* stream);
/* AudioEncoder's Conv2d ConvNormRelu layers (model_layers.py:219-276) on contiguous
 * [B][Ci][H][W] -> [B][Co][Hout][Wout].  Only output columns [w_lo, w_hi) are computed
 * (the encoder's dead-column pruning); the rest of y is untouched. */
int a2m_conv2d_fwd_f32(const float* x, int32_t B, int32_t Ci, int32_t H, int32_t W,
                       const float* w, const float* bias, int32_t Co, int32_t kh, int32_t kw,
                       int32_t stride, int32_t pad_h, int32_t pad_w,
                       const float* bn_w, const float* bn_b, const float* bn_rm,
                       const float* bn_rv, float bn_eps, int32_t act, float slope,
                       float* y, int32_t Hout, int32_t Wout, int32_t w_lo, int32_t w_hi,
                       void* ws, size_t ws_bytes, void* stream);

/* F.interpolate(x, size=(T,1), mode='bilinear', align_corners=False).squeeze(-1)
 * (model_layers.py:277-279) on x [B][C][H][W] -> y [B][C][T]. */
/* y[b][t][c] = x[b][c][t] (x channel stride T, batch stride xs_b; T <= 64): the [B*T][C]
 * row layout of an activation for GEMMs that want it as dense k-contiguous rows (the UNet's
 * wide attentions do this internally; the decoders' graph-stack input projection,
 * real_motion_model.py:173-176).  No reference counterpart: a layout change. */
int a2m_bct_to_btc_f32(const float* x, int64_t xs_b, int32_t B, int32_t C, int32_t T, float* y,
                       void* stream);
int a2m_interp_time_f32(const float* x, int32_t B, int32_t C, int32_t H, int32_t W,
                        float* y, int32_t T, void* stream);

/* Discriminator plumbing (real_motion_model.py:599,609,620): y[b][c] = scale * mean_t x[b][c][t]
 * and y[b][c][t] = scale * x[b][c] (repeat over time into a strided, e.g. concatenated,
 * buffer).  Each is the other's adjoint up to the scale (used by the backward pass). */
int a2m_mean_time_f32(const float* x, int64_t xs_b, int64_t xs_c, int32_t B, int32_t C,
                      int32_t T, float scale, float* y, void* stream);
int a2m_repeat_time_f32(const float* x, int32_t B, int32_t C, int32_t T, float scale, float* y,
                        int64_t ys_b, int64_t ys_c, void* stream);

/* ---------------------------------------------------------------- attention blocks
 * SelfAttention (model_layers.py:121-146): q,k = 1x1 conv C->C/8, v = 1x1 conv C->C,
 * A = softmax(q^T k) (no 1/sqrt(d) scaling), y = gamma*(v A^T) + x (+ res if not NULL).
 * x, res, y are [B][C][T] with batch stride x_bs / y_bs (res uses y's layout).
 * qkv_out [B][C/4 + C][T] and attn_out [B][T][T] receive the intermediates (kept for the
 * backward pass); ws is split-K scratch. */
int a2m_self_attention_fwd_f32(const float* x, int64_t x_bs, int32_t B, int32_t C, int32_t T,
                               const float* wq, const float* bq, const float* wk,
                               const float* bk, const float* wv, const float* bv,
                               const float* gamma, const float* res,
                               float* y, int64_t y_bs, float* qkv_out, float* attn_out,
                               void* ws, size_t ws_bytes, void* stream);
size_t a2m_self_attention_ws_bytes(int32_t B, int32_t C, int32_t T);
/* The same with the q/k/v 1x1-conv weights pre-stacked by a2m_stack_qkv_f32 into
 * wqkv [C/4 + C][C] and bqkv [C/4 + C] (callers cache these while the weights are unchanged). */
int a2m_stack_qkv_f32(const float* wq, const float* bq, const float* wk, const float* bk,
                      const float* wv, const float* bv, int32_t C, float* wqkv, float* bqkv,
                      void* stream);
int a2m_self_attention_packed_fwd_f32(const float* x, int64_t x_bs, int32_t B, int32_t C,
                                      int32_t T, const float* wqkv, const float* bqkv,
                                      const float* gamma, const float* res, float* y, int64_t y_bs,
                                      float* qkv_out, float* attn_out, void* ws, size_t ws_bytes,
                                      void* stream);

/* Inference-only SelfAttention with the q/k/v projections fused into the attention core (one
 * launch; no qkv / attention intermediates).  Supported when a2m_self_attention_eval_fits(C, T):
 * C in {128, 256}, T <= 64, T % 4 == 0 (the decoders' SelfAttention(256) at T = 64).
 * Same arguments and results as a2m_self_attention_packed_fwd_f32 otherwise. */
int32_t a2m_self_attention_eval_fits(int32_t C, int32_t T);
int a2m_self_attention_eval_f32(const float* x, int64_t x_bs, int32_t B, int32_t C, int32_t T,
                                const float* wqkv, const float* bqkv, const float* gamma,
                                const float* res, float* y, int64_t y_bs, void* stream);
/* The same with wqkv_h, wqkv rounded to bf16 (a2m_to_bf16_f32, 16-byte aligned; made once per
 * weight version), for the bf16 operand mode: the projection stages the ready bf16 weights
 * instead of rounding the fp32 ones in every workgroup -- bitwise the same result.  wqkv_h may
 * be NULL; ignored at precision 0. */
int a2m_self_attention_eval_ex_f32(const float* x, int64_t x_bs, int32_t B, int32_t C, int32_t T,
                                   const float* wqkv, const float* bqkv, const float* gamma,
                                   const float* res, float* y, int64_t y_bs, const void* wqkv_h,
                                   void* stream);

/* G such problems in one launch (grid G*B): problem g has its own wqkv + g*(C/4 + C)*C,
 * bqkv + g*(C/4 + C), gamma + g, and reads x + g*x_gs (batch stride x_bs, also y's), res +
 * g*res_gs, writes y + g*y_gs. */
int a2m_self_attention_eval_group_f32(const float* x, int64_t x_gs, int64_t x_bs, int32_t G, int32_t B,
                                      int32_t C, int32_t T, const float* wqkv, const float* bqkv,
                                      const float* gamma, const float* res, int64_t res_gs, float* y,
                                      int64_t y_gs, void* stream);

/* ChannelAttention (model_layers.py:149-174): y = x * (mlp(avg_T x) + mlp(max_T x)),
 * mlp = Linear(C, C/r) -> ReLU -> Linear(C/r, C) -> Sigmoid.  x, y contiguous [B][C][T];
 * att_out [B][C] (required) receives the channel weights; y may alias x. */
int a2m_channel_attention_fwd_f32(const float* x, int32_t B, int32_t C, int32_t T,
                                  const float* w1, const float* b1, int32_t Cr,
                                  const float* w2, const float* b2,
                                  float* y, float* att_out, void* stream);

/* LayerNorm over the last dim of rows [R][D] (real_motion_model.py:176,207).
 * Output element (r, d) goes to y + (r / T)*ys_b + d*ys_d + (r % T)*ys_t so the decoder's
 * permute(0,2,1) back to [B][C][T] is fused. */
int a2m_layernorm_fwd_f32(const float* x, int32_t R, int32_t D, const float* w, const float* b,
                          float eps, float* y, int32_t T, int64_t ys_b, int64_t ys_d,
                          int64_t ys_t, float* mean_out, float* rstd_out, void* stream);

/* GAT attention projections U[q][k] = sum_c W_h[c][k] att_q[c] (q < 4: att_src of head q,
 * q >= 4: att_dst of head q-4) of one GATConv(64, 64, heads=4): the logits a[n][q] = x_n . U[q]
 * without projecting x.  U: [8][64] device buffer; cache it per weight version. */
int a2m_graph_att_proj_f32(const float* w0, const float* att_src, const float* att_dst, float* U,
                           void* stream);
/* Fused eval graph stack (real_motion_model.py:173-201 body / :225-253 hand, eval mode):
 * nlayers x { y = LeakyReLU(LayerNorm64(L(x))) + x } with L = GATConv(64,64,heads=4,concat=False)
 * (kinds[l] = 0: w0 = lin.weight [256][64], U from a2m_graph_att_proj_f32, bias) or GraphConv
 * (kinds[l] = 1: w0 = lin_rel.weight, w1 = lin_root.weight, bias = lin_rel.bias).  The
 * per-layer arrays are host arrays of device pointers.  One launch; each workgroup keeps its
 * frames' node tile in LDS across the layers.  x, y: [F*J][64], distinct.
 * Topology limits (nbr_ptr / nbr_idx are device arrays, so they are NOT checked here; the
 * Python host side validates them where the CSR is built, a2m/skeleton.py in_neighbour_csr):
 * J <= 128, in-degree <= 7 per node, and (J + 1) + nbr_ptr[J] <= 256.  A topology beyond
 * them gives wrong results. */
int a2m_graph_stack_fwd_f32(const float* x, int32_t F, int32_t J, const int32_t* nbr_ptr,
                            const int32_t* nbr_idx, int32_t nlayers, const int32_t* kinds,
                            const float* const* w0, const float* const* w1, const float* const* U,
                            const float* const* bias, const float* const* ln_w,
                            const float* const* ln_b, float slope, float* y, void* stream);
/* The same with bf16 copies of the layer weights for the bf16 operand mode (precision 1):
 * w0h[l] / w1h[l] are device buffers holding w0[l] / w1[l] rounded to bf16 (a2m_to_bf16_f32, same
 * [row][64] layout, 16-byte aligned), made once per weight version, so the layers' k loops load
 * ready bf16 fragments instead of rounding the fp32 weights each time (the same values: the
 * result is bitwise that of a2m_graph_stack_fwd_f32).  w0h / w1h (the arrays or a layer's
 * entries) may be NULL; ignored at precision 0. */
int a2m_graph_stack_fwd_ex_f32(const float* x, int32_t F, int32_t J, const int32_t* nbr_ptr,
                               const int32_t* nbr_idx, int32_t nlayers, const int32_t* kinds,
                               const float* const* w0, const float* const* w1, const float* const* U,
                               const float* const* bias, const float* const* ln_w,
                               const float* const* ln_b, const void* const* w0h,
                               const void* const* w1h, float slope, float* y, void* stream);
/* y[i] = bf16(x[i]), round to nearest even (the rounding the bf16 operand mode applies), n
 * elements; y 4-byte aligned, 2 bytes an element. */
int a2m_to_bf16_f32(const float* x, void* y, int64_t n, void* stream);
/* ---------------------------------------------------------------- skeleton graph layers
 * One fused GNN step of the body / hand decoders (real_motion_model.py:173-201, 225-253):
 *   y = LeakyReLU(LayerNorm64(L(x))) + x
 * for every frame's J-node skeleton graph (nodes [F][J][64] contiguous), where L is
 *   kind 0: GATConv(64,64,heads=4,concat=False) + self loops; wlin [256][64], att_src,
 *           att_dst [4][64], bias [64]
 *   kind 1: GraphConv(64,64): W_rel (sum_nbr x) + b_rel + W_root x
 * The topology is given as an in-neighbour CSR over one graph (nbr_ptr[J+1], nbr_idx,
 * source nodes of the edges into each target, in edge order) and is shared by all F
 * frames (limits as for a2m_graph_stack_fwd_f32: J <= 128, in-degree <= 7,
 * (J + 1) + nbr_ptr[J] <= 256; not checked on the device arrays).  norm_res = 0 gives the bare layer y = L(x) (the discriminator's per-sample
 * GATConv, real_motion_model.py:602-616).  lin_out (GAT: x' [F*J][256]; GraphConv: aggregated x [F*J][64]) and
 * pre_ln [F*J][64] are saved for the backward pass when not NULL. */
int a2m_graph_layer_fwd_f32(const float* x, int32_t F, int32_t J, int32_t kind,
                            int32_t norm_res, const int32_t* nbr_ptr, const int32_t* nbr_idx,
                            const float* w0, const float* w1, const float* att_src,
                            const float* att_dst, const float* bias,
                            const float* ln_w, const float* ln_b, float slope,
                            float* y, float* lin_out, float* pre_ln,
                            void* ws, size_t ws_bytes, void* stream);

/* ---------------------------------------------------------------- pose losses
 * compute_bone_length_loss (real_motion_model.py:307-347) and
 * compute_comprehensive_angle_loss (:449-461, hand :350-392, body :394-447) on interleaved
 * (x, y) poses [B][T][104] with element (b,t,f) at p + b*ps_b + t*ps_t + f.
 * out[0] = bone loss (0 if real == NULL), out[1] = 0.7*hand + 0.3*body angle loss. */
int a2m_pose_losses_f32(const float* gen, int64_t gs_b, int64_t gs_t, const float* real,
                        int64_t rs_b, int64_t rs_t, int32_t B, int32_t T, float* out,
                        void* ws, size_t ws_bytes, void* stream);
/* The same with the angle weights explicit: out[1] = hand_w * hand + body_w * body.
 * (1, 0) is compute_hand_joint_angle_loss (real_motion_model.py:350-392), (0, 1)
 * compute_body_joint_angle_loss (:394-447), (0.7, 0.3) the comprehensive loss (:449-461). */
int a2m_pose_losses_w_f32(const float* gen, int64_t gs_b, int64_t gs_t, const float* real,
                          int64_t rs_b, int64_t rs_t, int32_t B, int32_t T, float hand_w,
                          float body_w, float* out, void* ws, size_t ws_bytes, void* stream);

/* ================================================================ training step
 * Forward-in-train-mode and backward entry points for the per-clip GAN step
 * (version5_model_train.py:342-405).  Gradients are written (accumulate = 0) or added
 * (accumulate = 1) into caller buffers; reductions are done in a fixed order. */

/* BatchNorm in training mode (nn.BatchNorm1d/2d forward with batch statistics, running
 * stats updated in place with `momentum`, unbiased running variance) fused with dropout
 * and the activation.  x is the raw conv output, element (b, c, l) at b*xs_b + c*xs_c + l.
 * drop_mode: 0 none, 1 element dropout before BN (ConvNormRelu 1-d, model_layers.py:118),
 * 2 channel dropout before BN (Dropout2d, 2-d ConvNormRelu), 3 element dropout after the
 * activation (discriminator blocks, real_motion_model.py:504-551).  Masks are a hash of
 * (seed, element index) and are regenerated by the backward pass.  Limit: B * L < 2^31
 * elements per channel (32-bit slice indexing; A2M_EINVAL beyond -- such a channel alone
 * would be 8 GB, more than any tensor of this model at any batch that fits one GPU). */
int a2m_bn_train_fwd_f32(const float* x, int64_t xs_b, int64_t xs_c, int32_t B, int32_t C,
                         int32_t L, const float* gamma, const float* beta, float* running_mean,
                         float* running_var, float momentum, float eps, float drop_p,
                         int32_t drop_mode, uint64_t seed, int32_t act, float slope, float* y,
                         int64_t ys_b, int64_t ys_c, float* save_mean, float* save_rstd,
                         void* ws, size_t ws_bytes, void* stream);
/* dx (contiguous [B][C][L]) = d(loss)/d(raw conv output); dbias = sum over (b, l) of dx. */
int a2m_bn_train_bwd_f32(const float* dy, int64_t dys_b, int64_t dys_c, const float* x,
                         int64_t xs_b, int64_t xs_c, int32_t B, int32_t C, int32_t L,
                         const float* gamma, const float* beta, const float* save_mean,
                         const float* save_rstd, float drop_p, int32_t drop_mode, uint64_t seed,
                         int32_t act, float slope, float* dx, float* dgamma, float* dbeta,
                         float* dbias, void* ws, size_t ws_bytes, void* stream);
/* Eval-mode BatchNorm with gradients (nn.BatchNorm*d after .eval(), model_layers.py:51-118, e.g.
 * fine-tuning or input attribution through a frozen G): normalises with the running statistics,
 * which it does not update, fused with the activation; save_mean / save_rstd receive the running
 * mean and 1 / sqrt(running_var + eps) for the backward.  drop_p / drop_mode / seed as in
 * a2m_bn_train_fwd_f32: the surrounding Dropout module may still be in training mode when only the
 * norm is frozen (bn.eval(), dropout left on); pass drop_p = 0 for a whole module in eval. */
int a2m_bn_eval_fwd_f32(const float* x, int64_t xs_b, int64_t xs_c, int32_t B, int32_t C, int32_t L,
                        const float* gamma, const float* beta, const float* running_mean,
                        const float* running_var, float eps, float drop_p, int32_t drop_mode,
                        uint64_t seed, int32_t act, float slope, float* y, int64_t ys_b, int64_t ys_c,
                        float* save_mean, float* save_rstd, void* stream);
/* Its backward: dx = gamma * rstd * act'(.) * dy (* the dropout scale; fixed statistics: no
 * batch-mean terms), dgamma = sum g * xhat, dbeta = sum g, dbias = sum dx, g = act'(.) * dy. */
int a2m_bn_eval_bwd_f32(const float* dy, int64_t dys_b, int64_t dys_c, const float* x, int64_t xs_b,
                        int64_t xs_c, int32_t B, int32_t C, int32_t L, const float* gamma,
                        const float* beta, const float* save_mean, const float* save_rstd, float drop_p,
                        int32_t drop_mode, uint64_t seed, int32_t act, float slope, float* dx,
                        float* dgamma, float* dbeta, float* dbias, void* ws, size_t ws_bytes,
                        void* stream);
/* Dropout seed offset for training steps captured in a HIP graph (version5_model_train.py:
 * 342-405 replayed per G / D step): every dropout launch issued while `counter` (a device
 * uint64) is registered hashes with seed + counter[0] * K, read when the kernel runs, so a
 * replayed step that advances the counter draws fresh masks although its seeds are baked.
 * NULL (the default) restores the plain seeds.  Library-global; set it around the launches. */
int a2m_set_dropout_seed_offset(const uint64_t* counter);
/* SyncBatchNorm phases for data-parallel training (per-layer all-reduce of the
 * BatchNorm statistics so DP over ranks normalises like the single-device batch,
 * version5_model_train.py:342-414 at B = 64).  The fused bn_train_fwd/bwd above split at their
 * per-channel reductions; the caller all-reduces (SUM) the float64 pairs between the phases:
 *   fwd:  sync_stats -> sums[C][2] = (sum z, sum z^2) -> all-reduce -> sync_apply(n_total)
 *   bwd:  sync_bwd_stats -> sums[C][2] = (sum g, sum g*xhat), local dbeta / dgamma
 *         -> all-reduce -> sync_bwd_apply(n_total).   n_total = sum over ranks of B*L. */
int a2m_bn_sync_stats_f32(const float* x, int64_t xs_b, int64_t xs_c, int32_t B, int32_t C,
                          int32_t L, float drop_p, int32_t drop_mode, uint64_t seed, double* sums,
                          void* ws, size_t ws_bytes, void* stream);
int a2m_bn_sync_apply_f32(const float* x, int64_t xs_b, int64_t xs_c, int32_t B, int32_t C,
                          int32_t L, const double* sums, int64_t n_total, const float* gamma,
                          const float* beta, float* running_mean, float* running_var,
                          float momentum, float eps, float drop_p, int32_t drop_mode,
                          uint64_t seed, int32_t act, float slope, float* y, int64_t ys_b,
                          int64_t ys_c, float* save_mean, float* save_rstd, void* stream);
int a2m_bn_sync_bwd_stats_f32(const float* dy, int64_t dys_b, int64_t dys_c, const float* x,
                              int64_t xs_b, int64_t xs_c, int32_t B, int32_t C, int32_t L,
                              const float* gamma, const float* beta, const float* save_mean,
                              const float* save_rstd, float drop_p, int32_t drop_mode,
                              uint64_t seed, int32_t act, float slope, double* sums,
                              float* dgamma, float* dbeta, void* ws, size_t ws_bytes, void* stream);
int a2m_bn_sync_bwd_apply_f32(const float* dy, int64_t dys_b, int64_t dys_c, const float* x,
                              int64_t xs_b, int64_t xs_c, int32_t B, int32_t C, int32_t L,
                              const float* gamma, const float* beta, const float* save_mean,
                              const float* save_rstd, float drop_p, int32_t drop_mode,
                              uint64_t seed, int32_t act, float slope, const double* sums,
                              int64_t n_total, float* dx, float* dbias, void* ws, size_t ws_bytes,
                              void* stream);
/* nn.Dropout(p) with the hash mask (real_motion_model.py:203,255); backward = same call. */
int a2m_dropout_f32(const float* x, int64_t n, float p, uint64_t seed, float* y, void* stream);
/* y[c] (+)= sum_{b,t} x[b][c][t] (conv / linear bias gradients). */
int a2m_sum_bt_f32(const float* x, int64_t xs_b, int64_t xs_c, int64_t xs_t, int32_t B,
                   int32_t C, int32_t T, float* y, int32_t accumulate, void* stream);
/* LayerNorm backward; dy in the same (permuted) layout the forward wrote. */
int a2m_layernorm_bwd_f32(const float* dy, int64_t dys_b, int64_t dys_d, int64_t dys_t,
                          int32_t T, const float* x, int32_t R, int32_t D, const float* w,
                          const float* mean, const float* rstd, float* dx, float* dw, float* db,
                          void* ws, size_t ws_bytes, void* stream);

/* Conv2d / Conv1d (H = kh = 1) backward.  dgrad: dy contiguous [B][Co][Ho][Wo] ->
 * dx (strided) by output-phase decomposed implicit GEMMs (also ConvTranspose1d's forward
 * algebra); wgrad: dw [Co][Ci][kh][kw] = sum dy (x) im2col(x). */
int a2m_conv2d_dgrad_f32(const float* dy, int32_t B, int32_t Co, int32_t Ho, int32_t Wo,
                         const float* w, int32_t Ci, int32_t H, int32_t W, int32_t kh, int32_t kw,
                         int32_t stride_h, int32_t stride_w, int32_t pad_h, int32_t pad_w,
                         float* dx, int64_t dxs_b, int64_t dxs_c, int64_t dxs_h, int64_t dxs_w,
                         int32_t accumulate, void* ws, size_t ws_bytes, void* stream);
int a2m_conv2d_wgrad_f32(const float* dy, int32_t B, int32_t Co, int32_t Ho, int32_t Wo,
                         const float* x, int64_t xs_b, int64_t xs_c, int64_t xs_h, int64_t xs_w,
                         int32_t Ci, int32_t H, int32_t W, int32_t kh, int32_t kw,
                         int32_t stride_h, int32_t stride_w, int32_t pad_h, int32_t pad_w,
                         float* dw, int32_t accumulate, void* ws, size_t ws_bytes, void* stream);

/* SelfAttention / ChannelAttention backward (inputs: the forward's saved qkv / attention). */
size_t a2m_self_attention_bwd_ws_bytes(int32_t B, int32_t C, int32_t T);
int a2m_self_attention_bwd_f32(const float* dy, const float* x, int64_t bs, int32_t B, int32_t C,
                               int32_t T, const float* wq, const float* bq, const float* wk,
                               const float* bk, const float* wv, const float* bv,
                               const float* gamma, const float* qkv, const float* attn, float* dx,
                               float* dwq, float* dbq, float* dwk, float* dbk, float* dwv,
                               float* dbv, float* dgamma, void* ws, size_t ws_bytes, void* stream);
int a2m_channel_attention_bwd_f32(const float* dy, const float* x, int32_t B, int32_t C, int32_t T,
                                  const float* w1, const float* b1, int32_t Cr, const float* w2,
                                  const float* b2, float* dx, float* dw1, float* db1, float* dw2,
                                  float* db2, void* ws, size_t ws_bytes, void* stream);

/* Skeleton graph layer backward (recomputes the forward from x). */
int a2m_graph_layer_bwd_f32(const float* x, const float* dy, int32_t F, int32_t J, int32_t kind,
                            int32_t norm_res, const int32_t* nbr_ptr, const int32_t* nbr_idx,
                            const float* w0, const float* w1, const float* att_src,
                            const float* att_dst, const float* bias, const float* ln_w,
                            const float* ln_b, float slope, float* dx, float* dw0, float* dw1,
                            float* datt_src, float* datt_dst, float* dbias, float* dln_w,
                            float* dln_b, void* ws, size_t ws_bytes, void* stream);
/* The same with the forward's saved pre-LayerNorm output (a2m_graph_layer_fwd_f32's pre_ln,
   norm_res layers; NULL = recompute): no forward recompute in the backward kernel, and the
   weight gradients contract the aggregation adjoint of dout with x (same sums, another order). */
int a2m_graph_layer_bwd_saved_f32(const float* x, const float* dy, const float* pre_ln, int32_t F,
                                  int32_t J, int32_t kind, int32_t norm_res, const int32_t* nbr_ptr,
                                  const int32_t* nbr_idx, const float* w0, const float* w1,
                                  const float* att_src, const float* att_dst, const float* bias,
                                  const float* ln_w, const float* ln_b, float slope, float* dx,
                                  float* dw0, float* dw1, float* datt_src, float* datt_dst, float* dbias,
                                  float* dln_w, float* dln_b, void* ws, size_t ws_bytes, void* stream);

/* F.interpolate (time) backward: dx [B][C][H][W] (zeros where the forward read nothing). */
int a2m_interp_time_bwd_f32(const float* dy, int32_t B, int32_t C, int32_t H, int32_t W,
                            float* dx, int32_t T, void* stream);

/* Losses of the G / D steps (version5_model_train.py:208-248, 367-403). */
int a2m_pose_losses_bwd_f32(const float* gen, int64_t gs_b, int64_t gs_t, const float* real,
                            int64_t rs_b, int64_t rs_t, int32_t B, int32_t T,
                            const float* grad_out, float* dgen, void* ws, size_t ws_bytes,
                            void* stream);
int a2m_pose_losses_w_bwd_f32(const float* gen, int64_t gs_b, int64_t gs_t, const float* real,
                              int64_t rs_b, int64_t rs_t, int32_t B, int32_t T, float hand_w,
                              float body_w, const float* grad_out, float* dgen, void* ws,
                              size_t ws_bytes, void* stream);
/* terms = [L1(diff(real), diff(fake)), mean||accel||, mean||jerk||] on [B][T][Fd] (contiguous).
 * If grad_terms (device [3], the incoming dL/dterms) and dfake are given, also
 * dfake = sum_i grad_terms[i] * dterms[i]/dfake (overwritten). */
int a2m_motion_losses_f32(const float* fake, const float* real, int32_t B, int32_t T, int32_t Fd,
                          float* terms, const float* grad_terms, float* dfake, void* ws,
                          size_t ws_bytes, void* stream);
/* loss = mean (pred - target)^2; dpred (optional) = grad_loss[0] * 2 (pred - target) / n
 * (grad_loss: device scalar, NULL = 1). */
int a2m_mse_loss_f32(const float* pred, const float* target, int64_t n, float* loss,
                     const float* grad_loss, float* dpred, void* ws, size_t ws_bytes, void* stream);
/* pos_to_motion (version5_model_train.py:208): y[b][t] = x[b][t+1] - x[b][t], and its adjoint. */
int a2m_diff_time_f32(const float* x, int32_t B, int32_t T, int32_t Fd, float* y, void* stream);
int a2m_diff_time_bwd_f32(const float* dy, int32_t B, int32_t T, int32_t Fd, float* dx,
                          int32_t accumulate, void* stream);

/* General strided GEMM on the same MFMA engine (linear layers' backward, 1x1 projections):
 *   C[m][n] (+)= alpha * sum_k A(m,k) B(n,k) (+ bias[m]), per batch z < batch
 *   n = n0*N1 + n1, k = k0*K1 + k1 (two-level index spaces cover [B][C][T] row sets)
 *   A(m,k) = A[z*a_bs + m*a_m + k0*a_k0 + k1*a_k1]
 *   B(n,k) = B[z*b_bs + n0*b_n0 + n1*b_n1 + k0*b_k0 + k1*b_k1]
 *   C(m,n) = C[z*c_bs + m*c_m + n0*c_n0 + n1*c_n1]                                        */
int a2m_gemm_f32(int32_t M, int32_t N, int32_t N1, int32_t K, int32_t K1, int32_t batch,
                 const float* A, int64_t a_bs, int64_t a_m, int64_t a_k0, int64_t a_k1,
                 const float* B, int64_t b_bs, int64_t b_n0, int64_t b_n1, int64_t b_k0,
                 int64_t b_k1, float* C, int64_t c_bs, int64_t c_m, int64_t c_n0, int64_t c_n1,
                 const float* bias, float alpha, int32_t accumulate, void* ws, size_t ws_bytes,
                 void* stream);

/* torch.optim.Adam step (no weight decay by default, no amsgrad) over a flat buffer. */
int a2m_adam_f32(float* param, const float* grad, float* exp_avg, float* exp_avg_sq, int64_t n,
                 float lr, float beta1, float beta2, float eps, float weight_decay, int32_t step,
                 void* stream);

/* The same update for a step captured in a HIP graph: step (device int32) is advanced by one in
 * the launch and the bias corrections derived from it on the device; lr is a device float the
 * host rewrites when DynamicGANTraining changes it (version5_model_train.py:80-107).  Bitwise
 * the update of a2m_adam_f32 at the same step and lr. */
int a2m_adam_dev_f32(float* param, const float* grad, float* exp_avg, float* exp_avg_sq, int64_t n,
                     const float* lr, float beta1, float beta2, float eps, float weight_decay,
                     int32_t* step, void* stream);

/* dst[dst_off[i] .. dst_off[i] + n[i]) = src[i][0 .. n[i]) for i < count (host arrays of device
 * pointers / element counts; segments must not overlap).  The optimiser's gradient collection:
 * per-parameter gradient tensors into the flat gradient buffer, 48 segments per launch.
 * Replaces torch's per-parameter AccumulateGrad add (version5_model_train.py:285-286 Adam over
 * model.parameters()). */
int a2m_gather_segments_f32(const float* const* src, const int64_t* dst_off, const int64_t* n,
                            int32_t count, float* dst, void* stream);

/* ---- Pose normalisation and evaluation ----
 * Poses are [n_frames][104] planar (x of 52 joints, then y), neck = joint 0.
 * a2m_pose_moments_f32: acc[0:104] += mean over the frames of (x - neck) (necksub = 1) or x,
 * acc[104:208] += mean of squares, fp64 -- one batch of normalization_tools.get_mean_std[_necksub]
 * (normalization_tools.py:7-45); the caller averages over batches.
 * a2m_pose_normalize_f32: ((x - neck) - mean) / std  (version5_model_train.py:298-304).
 * a2m_pose_denormalize_f32: x * std + mean  (generate_motion_video.py:259-260).
 * a2m_pck_f32: pred, gt [N][2][K] -> out[N] = fraction of keypoints with
 * |gt - pred| <= alpha * max(x extent, y extent) of gt (motion_evaluation.py:4-22). */
int a2m_pose_moments_f32(const float* pose, int64_t n_frames, int32_t necksub, double* acc,
                         void* stream);
int a2m_pose_normalize_f32(const float* pose, int64_t n_frames, const float* mean, const float* std_,
                           float* out, void* stream);
int a2m_pose_denormalize_f32(const float* pose, int64_t n_frames, const float* mean,
                             const float* std_, float* out, void* stream);
int a2m_pck_f32(const float* pred, const float* gt, int32_t N, int32_t K, double alpha,
                double* out, void* stream);

/* PATS windowing (dataUtils.py:585-665): out[w][j][c] =
 * data[starts[w] + j*interval][c], j < ceil(window/interval), data [length][C] in HBM; with
 * mean/std (both or neither) each value is standardised as (x - mean[c]) / (std[c] < 1e-7 ? 1 : std[c]). */
int a2m_window_gather_f32(const float* data, int64_t length, int32_t C, const int64_t* starts,
                          int32_t n_windows, int32_t window, int32_t interval, const float* mean,
                          const float* std_, float* out, void* stream);

/* Measurement hook (bench.py): while enabled, every launch of the implicit-GEMM engine (up to
 * 1024 per window; more make _read fail) carries a record of span stamps that its tile kernel and
 * split-K reduce write themselves (earliest block start, latest wave end on the GPU's constant-rate
 * wall clock, which all XCDs share; a span is last end - first start over all XCDs), eagerly or inside a graph
 * captured while enabled.  _read synchronises the device and returns the launch count, the
 * launches' algorithmic FLOPs (2*M*N*K*batch), the summed tile-kernel spans and the summed
 * split-K reduce spans (ms) of the latest execution, then re-arms the stamps (so it can follow
 * each replay of such a graph); _stop ends recording of new launches, _end = _stop + _read +
 * forget the records.  No effect when disabled. */
int a2m_gemm_timing_begin(void);
/* Tuning hook: force the engine's tile (64 | 128) and split-K count for subsequent launches
 * (0 = the planner's choice); workspace sizing follows.  Process-global, not for production. */
int a2m_gemm_plan_override(int32_t tile, int32_t splits);
/* Test / tuning hook: which 64x64 tile kernel eligible launches take -- 1 the software-pipelined
 * tile (gemm_pipe.h / gemm_pipe_bf16.h), 0 gemm_tile, -1 the default
 * (1).  Both give bitwise-equal results; process-global, not for production. */
int a2m_gemm_pipe_override(int32_t mode);
/* Test hook: V channels per workgroup of the fused eval SelfAttention at C % 128 == 0 -- 64
 * (default: eight waves, Q / K computed by each of the C / 64 chunks) or 128 (twelve waves, Q / K
 * once per two 64-channel chunks: less kernel time, but measured 0.5-0.7 % slower a step).  Both
 * give bitwise-equal results; A2M_EINVAL for any other value.  Process-global, not for
 * production. */
int a2m_set_attn_eval_chunk(int32_t nv);
/* Operand precision of every GEMM-engine launch (convs, linears, attention products and their
 * backward) issued after the call: 0 = fp32 (default; the parity configuration), 1 = bf16
 * operands with fp32 accumulation (BASELINE configs[4], torch.autocast(bfloat16)-equivalent:
 * weights and activations stay fp32 in HBM, rounded to bf16 where they enter the MFMA),
 * (2 = bf16x6, fp32 operands split into three bf16 pieces, six products: only in a library built
 * with -DA2M_WITH_X6, an experiment measured slower than fp32; A2M_EINVAL otherwise).
 * Process-wide; not thread-safe against concurrent launches. */
int a2m_set_gemm_precision(int32_t prec);
int32_t a2m_get_gemm_precision(void);
int a2m_gemm_timing_end(int64_t* launches, double* flops, double* ms_tile, double* ms_reduce,
                        int64_t* reduces);
int a2m_gemm_timing_stop(void);
/* Per-launch tile-kernel spans of the latest execution instead of their sums: the first block
 * start and last block end (us on the GPU wall clock, -1 for a launch that did not run) of the
 * first min(cap, launches) records; re-arms the stamps like _read. */
int a2m_gemm_timing_read_spans(int64_t cap, double* start_us, double* end_us, int64_t* n);
/* _read_spans plus each launch's ready mark (us; -1 unless A2M_GEMM_TIMING_READY=1 was set when
 * the launch was recorded: the wall clock at which a one-thread mark kernel enqueued right before
 * the tile kernel ran, i.e. when its stream reached the launch) */
int a2m_gemm_timing_read_spans_ex(int64_t cap, double* ready_us, double* start_us, double* end_us,
                                  int64_t* n);
/* _stop + forget the records without reading them (after the last _read of a kept window) */
int a2m_gemm_timing_clear(void);
int a2m_gemm_timing_read(int64_t* launches, double* flops, double* ms_tile, double* ms_reduce,
                         int64_t* reduces);
/* _read plus ms_queued: the sum over launches of (last block end - ready mark), the launch's time
 * from the moment its stream reached it, i.e. including its dispatch and any wait for free CUs
 * (0 without A2M_GEMM_TIMING_READY=1) */
int a2m_gemm_timing_read_ex(int64_t* launches, double* flops, double* ms_tile, double* ms_reduce,
                            int64_t* reduces, double* ms_queued);
/* Named wall-clock marks (measurement only; after a2m_gemm_timing_begin has allocated the stamp
 * buffer): a one-thread kernel on the stream stores the GPU wall clock into mark `slot`
 * (0 .. A2M_TIMING_MARKS-1), also as a node of a graph being captured; _elapsed synchronises the
 * device and returns mark b - mark a in ms. */
#define A2M_TIMING_MARKS 16
int a2m_timing_mark(int32_t slot, void* stream);
int a2m_timing_mark_elapsed(int32_t a, int32_t b, float* ms);
/* ms from mark `slot` to the last block end (tile kernel or its split-K reduce) of engine
 * launch record `rec` of the current timing window, in the latest execution (does not re-arm) */
int a2m_timing_mark_to_launch_end(int32_t slot, int64_t rec, float* ms);

#ifdef __cplusplus
}
#endif
#endif /* A2M_H_ */
