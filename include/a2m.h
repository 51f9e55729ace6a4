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
int a2m_interp_time_f32(const float* x, int32_t B, int32_t C, int32_t H, int32_t W,
                        float* y, int32_t T, void* stream);

/* Discriminator plumbing (real_motion_model.py:599,609,620): y[b][c] = mean_t x[b][c][t]
 * and y[b][c][t] = x[b][c] (repeat over time into a strided, e.g. concatenated, buffer). */
int a2m_mean_time_f32(const float* x, int64_t xs_b, int64_t xs_c, int32_t B, int32_t C,
                      int32_t T, float* y, void* stream);
int a2m_repeat_time_f32(const float* x, int32_t B, int32_t C, int32_t T, float* y,
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

/* ChannelAttention (model_layers.py:149-174): y = x * (mlp(avg_T x) + mlp(max_T x)),
 * mlp = Linear(C, C/r) -> ReLU -> Linear(C/r, C) -> Sigmoid.  x, y contiguous [B][C][T];
 * att_out [B][C] receives the channel weights. */
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

/* ---------------------------------------------------------------- skeleton graph layers
 * One fused GNN step of the body / hand decoders (real_motion_model.py:173-201, 225-253):
 *   y = LeakyReLU(LayerNorm64(L(x))) + x
 * for every frame's J-node skeleton graph (nodes [F][J][64] contiguous), where L is
 *   kind 0: GATConv(64,64,heads=4,concat=False) + self loops; wlin [256][64], att_src,
 *           att_dst [4][64], bias [64]
 *   kind 1: GraphConv(64,64): W_rel (sum_nbr x) + b_rel + W_root x
 * The topology is given as an in-neighbour CSR over one graph (nbr_ptr[J+1], nbr_idx,
 * source nodes of the edges into each target, in edge order) and is shared by all F
 * frames.  norm_res = 0 gives the bare layer y = L(x) (the discriminator's per-sample
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
 * out[0] = bone loss (only if real != NULL), out[1] = 0.7*hand + 0.3*body angle loss. */
int a2m_pose_losses_f32(const float* gen, int64_t gs_b, int64_t gs_t, const float* real,
                        int64_t rs_b, int64_t rs_t, int32_t B, int32_t T, float* out,
                        void* ws, size_t ws_bytes, void* stream);

#ifdef __cplusplus
}
#endif
#endif /* A2M_H_ */
