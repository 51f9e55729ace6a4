"""ctypes binding of liba2m_hip.so (C-ABI declared in include/a2m.h).

The library is REQUIRED: there is no CPU or eager-PyTorch fallback.  Importing a2m on a
machine without the built library raises immediately (build it with
`make -C audio-to-motion-generation_amd` or `python -c "import __graft_entry__ as g; g.build()"`).
"""
import ctypes
import os

_HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.environ.get('A2M_LIB', os.path.join(_HERE, 'liba2m_hip.so'))

P = ctypes.c_void_p
I32 = ctypes.c_int32
I64 = ctypes.c_int64
F32 = ctypes.c_float
F64 = ctypes.c_double
SZ = ctypes.c_size_t
U64 = ctypes.c_uint64

# name -> (restype, argtypes); mirrors include/a2m.h
SIGNATURES = {
    'a2m_last_error': (ctypes.c_char_p, []),
    'a2m_version': (ctypes.c_int, []),
    'a2m_logmel_num_frames': (I64, [I64, I32, I32]),
    'a2m_logmel_geometry': (ctypes.c_int, [I32, F64, F64, ctypes.POINTER(I32), ctypes.POINTER(I32),
                                           ctypes.POINTER(I32)]),
    'a2m_logmel_plan_bytes': (SZ, [I32, F64, F64, I32, F64, F64]),
    'a2m_logmel_plan_build': (ctypes.c_int, [I32, F64, F64, I32, F64, F64, P, SZ]),
    'a2m_logmel_f32': (ctypes.c_int, [P, I64, I64, I64, I32, I32, I32, I32, P, F32, P, P]),
    'a2m_conv1d_fwd_f32': (ctypes.c_int, [P, I64, I64, I64, I32, I32, I32, P, P, I32, I32, I32, I32,
                                          P, P, P, P, F32, I32, F32, P, I64, I64, I64, P, SZ, P]),
    'a2m_convt1d_fwd_f32': (ctypes.c_int, [P, I64, I64, I32, I32, I32, P, P, I32, I32, I32, I32, I32,
                                           P, P, P, P, F32, I32, F32, P, I64, I64, P, SZ, P]),
    'a2m_convt1d_packed_fwd_f32': (ctypes.c_int, [P, I64, I64, I32, I32, I32, P, P, I32, I32, I32, I32, I32,
                                           P, P, P, P, F32, I32, F32, P, I64, I64, P, SZ, P]),
    'a2m_convt1d_pack_f32': (ctypes.c_int, [P, I32, I32, I32, I32, I32, P, P]),
    'a2m_conv1d_tap_chunk': (I32, []),
    'a2m_convt1d_tap_pack_f32': (ctypes.c_int, [P, I32, I32, I32, I32, I32, I32, P, P]),
    'a2m_convt1d_tap_fwd_f32': (ctypes.c_int, [P, I64, I64, I32, I32, I32, P, I32, P, I32, I32, I32, I32,
                                               I32, P, P, P, P, F32, I32, F32, P, I64, I64, P, SZ, P]),
    'a2m_conv2d_pack_nhwc_f32': (ctypes.c_int, [P, I32, I32, I32, I32, P, P]),
    'a2m_conv2d_nhwc_fwd_f32': (ctypes.c_int, [P, I32, I32, I32, I32, P, P, I32, I32, I32, I32, I32,
                                               I32, P, P, P, P, F32, I32, F32, P, I32, I32, I32,
                                               I32, I32, P, SZ, P]),
    'a2m_conv2d_nhwc_interp_fwd_f32': (ctypes.c_int, [P, I32, I32, I32, I32, P, P, I32, I32, I32, I32, I32,
                                                      I32, P, P, P, P, F32, I32, F32, P, I32, I32, I32,
                                                      I32, P, SZ, P]),
    'a2m_graph_att_proj_f32': (ctypes.c_int, [P, P, P, P, P]),
    'a2m_graph_stack_fwd_f32': (ctypes.c_int, [P, I32, I32, P, P, I32, P, P, P, P, P, P, P, F32,
                                               P, P]),
    'a2m_graph_stack_fwd_ex_f32': (ctypes.c_int, [P, I32, I32, P, P, I32, P, P, P, P, P, P, P, P, P,
                                                  F32, P, P]),
    'a2m_to_bf16_f32': (ctypes.c_int, [P, P, I64, P]),
    'a2m_conv1d_tap_pack_f32': (ctypes.c_int, [P, I32, I32, I32, I32, P, P]),
    'a2m_conv1d_tap_fwd_f32': (ctypes.c_int, [P, I64, I64, I32, I32, I32, P, I32, P, I32, I32, I32,
                                              P, P, P, P, F32, I32, F32, P, I64, I64, I64, P, SZ, P]),
    'a2m_conv2d_fwd_f32': (ctypes.c_int, [P, I32, I32, I32, I32, P, P, I32, I32, I32, I32, I32, I32,
                                          P, P, P, P, F32, I32, F32, P, I32, I32, I32, I32, P, SZ, P]),
    'a2m_mean_time_f32': (ctypes.c_int, [P, I64, I64, I32, I32, I32, F32, P, P]),
    'a2m_repeat_time_f32': (ctypes.c_int, [P, I32, I32, I32, F32, P, I64, I64, P]),
    'a2m_interp_time_f32': (ctypes.c_int, [P, I32, I32, I32, I32, P, I32, P]),
    'a2m_self_attention_fwd_f32': (ctypes.c_int, [P, I64, I32, I32, I32, P, P, P, P, P, P, P, P, P,
                                                  I64, P, P, P, SZ, P]),
    'a2m_self_attention_ws_bytes': (SZ, [I32, I32, I32]),
    'a2m_stack_qkv_f32': (ctypes.c_int, [P, P, P, P, P, P, I32, P, P, P]),
    'a2m_self_attention_packed_fwd_f32': (ctypes.c_int, [P, I64, I32, I32, I32, P, P, P, P, P, I64, P, P, P,
                                                         SZ, P]),
    'a2m_channel_attention_fwd_f32': (ctypes.c_int, [P, I32, I32, I32, P, P, I32, P, P, P, P, P]),
    'a2m_layernorm_fwd_f32': (ctypes.c_int, [P, I32, I32, P, P, F32, P, I32, I64, I64, I64, P, P, P]),
    'a2m_graph_layer_fwd_f32': (ctypes.c_int, [P, I32, I32, I32, I32, P, P, P, P, P, P, P, P, P, F32, P, P,
                                               P, P, SZ, P]),
    'a2m_pose_losses_f32': (ctypes.c_int, [P, I64, I64, P, I64, I64, I32, I32, P, P, SZ, P]),
    'a2m_pose_losses_w_f32': (ctypes.c_int, [P, I64, I64, P, I64, I64, I32, I32, F32, F32, P, P, SZ, P]),
    # ---- training step
    'a2m_bn_train_fwd_f32': (ctypes.c_int, [P, I64, I64, I32, I32, I32, P, P, P, P, F32, F32, F32, I32,
                                            U64, I32, F32, P, I64, I64, P, P, P, SZ, P]),
    'a2m_bn_train_bwd_f32': (ctypes.c_int, [P, I64, I64, P, I64, I64, I32, I32, I32, P, P, P, P, F32, I32,
                                            U64, I32, F32, P, P, P, P, P, SZ, P]),
    'a2m_bn_eval_fwd_f32': (ctypes.c_int, [P, I64, I64, I32, I32, I32, P, P, P, P, F32, F32, I32, U64, I32, F32,
                                           P, I64, I64, P, P, P]),
    'a2m_bn_eval_bwd_f32': (ctypes.c_int, [P, I64, I64, P, I64, I64, I32, I32, I32, P, P, P, P, F32, I32, U64,
                                           I32, F32, P, P, P, P, P, SZ, P]),
    'a2m_set_dropout_seed_offset': (ctypes.c_int, [P]),
    'a2m_bn_sync_stats_f32': (ctypes.c_int, [P, I64, I64, I32, I32, I32, F32, I32, U64, P, P, SZ, P]),
    'a2m_bn_sync_apply_f32': (ctypes.c_int, [P, I64, I64, I32, I32, I32, P, I64, P, P, P, P, F32, F32, F32,
                                             I32, U64, I32, F32, P, I64, I64, P, P, P]),
    'a2m_bn_sync_bwd_stats_f32': (ctypes.c_int, [P, I64, I64, P, I64, I64, I32, I32, I32, P, P, P, P, F32,
                                                 I32, U64, I32, F32, P, P, P, P, SZ, P]),
    'a2m_bn_sync_bwd_apply_f32': (ctypes.c_int, [P, I64, I64, P, I64, I64, I32, I32, I32, P, P, P, P, F32,
                                                 I32, U64, I32, F32, P, I64, P, P, P, SZ, P]),
    'a2m_self_attention_eval_fits': (I32, [I32, I32]),
    'a2m_self_attention_eval_f32': (ctypes.c_int, [P, I64, I32, I32, I32, P, P, P, P, P, I64, P]),
    'a2m_self_attention_eval_ex_f32': (ctypes.c_int, [P, I64, I32, I32, I32, P, P, P, P, P, I64, P, P]),
    'a2m_self_attention_eval_group_f32': (ctypes.c_int, [P, I64, I64, I32, I32, I32, I32, P, P, P, P, I64,
                                                         P, I64, P]),
    'a2m_conv1d_tap_group_fwd_f32': (ctypes.c_int, [P, I64, I64, I64, I32, I32, I32, I32, P, I64, I32, P,
                                                    I32, I32, I32, P, P, P, P, F32, I32, F32, P, I64, I64,
                                                    I64, I64, P, SZ, P]),
    'a2m_dropout_f32': (ctypes.c_int, [P, I64, F32, U64, P, P]),
    'a2m_sum_bt_f32': (ctypes.c_int, [P, I64, I64, I64, I32, I32, I32, P, I32, P]),
    'a2m_layernorm_bwd_f32': (ctypes.c_int, [P, I64, I64, I64, I32, P, I32, I32, P, P, P, P, P, P, P, SZ, P]),
    'a2m_conv2d_dgrad_f32': (ctypes.c_int, [P, I32, I32, I32, I32, P, I32, I32, I32, I32, I32, I32, I32, I32,
                                            I32, P, I64, I64, I64, I64, I32, P, SZ, P]),
    'a2m_conv2d_wgrad_f32': (ctypes.c_int, [P, I32, I32, I32, I32, P, I64, I64, I64, I64, I32, I32, I32, I32,
                                            I32, I32, I32, I32, I32, P, I32, P, SZ, P]),
    'a2m_self_attention_bwd_ws_bytes': (SZ, [I32, I32, I32]),
    'a2m_self_attention_bwd_f32': (ctypes.c_int, [P, P, I64, I32, I32, I32, P, P, P, P, P, P, P, P, P, P, P, P,
                                                  P, P, P, P, P, P, SZ, P]),
    'a2m_channel_attention_bwd_f32': (ctypes.c_int, [P, P, I32, I32, I32, P, P, I32, P, P, P, P, P, P, P, P,
                                                     SZ, P]),
    'a2m_graph_layer_bwd_f32': (ctypes.c_int, [P, P, I32, I32, I32, I32, P, P, P, P, P, P, P, P, P, F32, P, P,
                                               P, P, P, P, P, P, P, SZ, P]),
    'a2m_graph_layer_bwd_saved_f32': (ctypes.c_int, [P, P, P, I32, I32, I32, I32, P, P, P, P, P, P, P, P, P, F32,
                                                     P, P, P, P, P, P, P, P, P, SZ, P]),
    'a2m_interp_time_bwd_f32': (ctypes.c_int, [P, I32, I32, I32, I32, P, I32, P]),
    'a2m_pose_losses_bwd_f32': (ctypes.c_int, [P, I64, I64, P, I64, I64, I32, I32, P, P, P, SZ, P]),
    'a2m_pose_losses_w_bwd_f32': (ctypes.c_int, [P, I64, I64, P, I64, I64, I32, I32, F32, F32, P, P, P, SZ, P]),
    'a2m_motion_losses_f32': (ctypes.c_int, [P, P, I32, I32, I32, P, P, P, P, SZ, P]),
    'a2m_mse_loss_f32': (ctypes.c_int, [P, P, I64, P, P, P, P, SZ, P]),
    'a2m_diff_time_f32': (ctypes.c_int, [P, I32, I32, I32, P, P]),
    'a2m_diff_time_bwd_f32': (ctypes.c_int, [P, I32, I32, I32, P, I32, P]),
    'a2m_adam_f32': (ctypes.c_int, [P, P, P, P, I64, F32, F32, F32, F32, F32, I32, P]),
    'a2m_adam_dev_f32': (ctypes.c_int, [P, P, P, P, I64, P, F32, F32, F32, F32, P, P]),
    'a2m_gather_segments_f32': (ctypes.c_int, [P, P, P, I32, P, P]),
    'a2m_gemm_f32': (ctypes.c_int, [I32, I32, I32, I32, I32, I32, P, I64, I64, I64, I64, P, I64, I64, I64,
                                    I64, I64, P, I64, I64, I64, I64, P, F32, I32, P, SZ, P]),
    'a2m_pose_moments_f32': (ctypes.c_int, [P, I64, I32, P, P]),
    'a2m_pose_normalize_f32': (ctypes.c_int, [P, I64, P, P, P, P]),
    'a2m_pose_denormalize_f32': (ctypes.c_int, [P, I64, P, P, P, P]),
    'a2m_pck_f32': (ctypes.c_int, [P, P, I32, I32, F64, P, P]),
    'a2m_window_gather_f32': (ctypes.c_int, [P, I64, I32, P, I32, I32, I32, P, P, P, P]),
    'a2m_gemm_timing_begin': (ctypes.c_int, []),
    'a2m_gemm_plan_override': (ctypes.c_int, [I32, I32]),
    'a2m_gemm_pipe_override': (ctypes.c_int, [I32]),
    'a2m_set_gemm_precision': (ctypes.c_int, [I32]),
    'a2m_set_attn_eval_chunk': (ctypes.c_int, [I32]),
    'a2m_get_gemm_precision': (I32, []),
    'a2m_gemm_timing_end': (ctypes.c_int, [ctypes.POINTER(I64), ctypes.POINTER(F64), ctypes.POINTER(F64),
                                           ctypes.POINTER(F64), ctypes.POINTER(I64)]),
    'a2m_bct_to_btc_f32': (ctypes.c_int, [P, I64, I32, I32, I32, P, P]),
    'a2m_gemm_timing_stop': (ctypes.c_int, []),
    'a2m_gemm_timing_clear': (ctypes.c_int, []),
    'a2m_gemm_timing_read_spans': (ctypes.c_int, [I64, ctypes.POINTER(F64), ctypes.POINTER(F64),
                                                  ctypes.POINTER(I64)]),
    'a2m_gemm_timing_read': (ctypes.c_int, [ctypes.POINTER(I64), ctypes.POINTER(F64), ctypes.POINTER(F64),
                                            ctypes.POINTER(F64), ctypes.POINTER(I64)]),
    'a2m_gemm_timing_read_spans_ex': (ctypes.c_int, [I64, ctypes.POINTER(F64), ctypes.POINTER(F64),
                                                     ctypes.POINTER(F64), ctypes.POINTER(I64)]),
    'a2m_gemm_timing_read_ex': (ctypes.c_int, [ctypes.POINTER(I64), ctypes.POINTER(F64), ctypes.POINTER(F64),
                                               ctypes.POINTER(F64), ctypes.POINTER(I64), ctypes.POINTER(F64)]),
    'a2m_timing_mark_to_launch_end': (ctypes.c_int, [I32, I64, ctypes.POINTER(ctypes.c_float)]),
    'a2m_timing_mark': (ctypes.c_int, [I32, ctypes.c_void_p]),
    'a2m_timing_mark_elapsed': (ctypes.c_int, [I32, I32, ctypes.POINTER(ctypes.c_float)]),
}

A2M_EINVAL, A2M_EHIP, A2M_EWS = -1, -2, -3


class A2MError(RuntimeError):
    pass


class WorkspaceTooSmall(A2MError):
    pass


def _load():
    if not os.path.exists(LIB_PATH):
        raise ImportError(f'a2m: native library not found at {LIB_PATH}; build it first '
                          f'(make -C audio-to-motion-generation_amd)')
    lib = ctypes.CDLL(LIB_PATH)
    for name, (res, args) in SIGNATURES.items():
        fn = getattr(lib, name, None)
        if fn is None and 'A2M_LIB' in os.environ:
            continue   # an older library selected for an A/B run (tools/ab_lib*.sh) may lack newer entry points
        if fn is None:
            raise ImportError(f'a2m: {LIB_PATH} does not export {name}')
        fn.restype = res
        fn.argtypes = args
    return lib


lib = _load()


def last_error():
    return lib.a2m_last_error().decode()


def check(rc, value_error=False):
    """Raise on a non-zero status (ValueError where the reference raises ValueError)."""
    if rc == 0:
        return
    msg = last_error()
    if rc == A2M_EWS:
        raise WorkspaceTooSmall(msg)
    if rc == A2M_EINVAL and value_error:
        raise ValueError(msg)
    raise A2MError(f'a2m error {rc}: {msg}')


def exported_symbols():
    return list(SIGNATURES)
