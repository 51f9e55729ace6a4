"""a2m -- MI355X-native (gfx950) audio -> 2-D pose hot path.

Drop-in modules for the reference's real_motion_model / model_layers / mel_features call
surface; all compute runs in liba2m_hip.so (include/a2m.h) through a2m.functional.
Importing this package loads the native library and fails loudly if it is missing.
"""
import torch  # noqa: F401  (loads the ROCm runtime the library links against first)

from . import _native  # noqa: F401  (raises ImportError if liba2m_hip.so is absent)

__version__ = '0.1.0'


def set_gemm_precision(dtype):
    """Operand precision of every GEMM-engine launch issued afterwards: 'fp32' (default, the
    parity configuration: v_mfma_f32_32x32x2_f32), 'bf16' (bf16 operands, fp32 accumulation,
    fp32 storage -- the torch.autocast(dtype=torch.bfloat16)-equivalent of BASELINE configs[4]).
    ('bf16x6', three-way bf16 operand splits, exists only in a library built with
    -DA2M_WITH_X6: it measured slower than fp32)  Returns the previous setting.
    HIP graphs keep the precision they were captured with."""
    prev = _PREC_NAMES[_native.lib.a2m_get_gemm_precision()]
    if dtype in ('bf16', torch.bfloat16):
        flag = 1
    elif dtype in ('fp32', torch.float32):
        flag = 0
    elif dtype == 'bf16x6':
        flag = 2
    else:
        raise ValueError(f'unsupported GEMM precision {dtype!r} (fp32 or bf16)')
    _native.check(_native.lib.a2m_set_gemm_precision(flag))
    return prev


_PREC_NAMES = ('fp32', 'bf16', 'bf16x6')


class gemm_precision:
    """Context manager: `with a2m.gemm_precision('bf16'): ...`."""

    def __init__(self, dtype):
        self.dtype = dtype
        self.prev = None

    def __enter__(self):
        self.prev = set_gemm_precision(self.dtype)
        return self

    def __exit__(self, *exc):
        set_gemm_precision(self.prev)
        return False
