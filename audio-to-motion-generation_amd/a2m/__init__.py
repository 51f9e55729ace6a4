"""a2m -- MI355X-native (gfx950) audio -> 2-D pose hot path.

Drop-in modules for the reference's real_motion_model / model_layers / mel_features call
surface; all compute runs in liba2m_hip.so (include/a2m.h) through a2m.functional.
Importing this package loads the native library and fails loudly if it is missing.
"""
import torch  # noqa: F401  (loads the ROCm runtime the library links against first)

from . import _native  # noqa: F401  (raises ImportError if liba2m_hip.so is absent)

__version__ = '0.1.0'
