"""Drop-in log-mel front end (pose_video/mel_features.py:192-223) on the HIP path.

log_mel_spectrogram(data, audio_sample_rate=8000, log_offset=0.0, window_length_secs=0.025,
                    hop_length_secs=0.010, **kwargs)
keeps the reference signature (kwargs: num_mel_bins, lower_edge_hertz, upper_edge_hertz) and
its ValueError cases.  `data` may be a 1-D numpy array (returns numpy [frames, mels], as the
reference does) or a device tensor [S] / [C, S] (returns a device tensor [F, M] / [C, F, M]).
Computation is fp32 on the GPU (reference: float64 numpy); see DESIGN.md for the tolerance.
"""
import numpy as np
import torch

from . import functional as F


def _plan(audio_sample_rate, window_length_secs, hop_length_secs, kwargs, device):
    return F.LogMelPlan.get(audio_sample_rate, window_length_secs, hop_length_secs,
                            kwargs.get('num_mel_bins', 20), kwargs.get('lower_edge_hertz', 125.0),
                            kwargs.get('upper_edge_hertz', 3800.0), device)


def log_mel_spectrogram(data, audio_sample_rate=8000, log_offset=0.0, window_length_secs=0.025,
                        hop_length_secs=0.010, **kwargs):
    unknown = set(kwargs) - {'num_mel_bins', 'lower_edge_hertz', 'upper_edge_hertz'}
    if unknown:
        raise TypeError(f'unexpected keyword arguments {sorted(unknown)}')
    as_numpy = not torch.is_tensor(data)
    if as_numpy:
        wave = torch.as_tensor(np.asarray(data, dtype=np.float32)).to('cuda')
    else:
        wave = data.float()
    device = wave.device
    plan = _plan(audio_sample_rate, window_length_secs, hop_length_secs, kwargs, device)
    squeeze = wave.dim() == 1
    w2 = wave.reshape(1, -1) if squeeze else wave
    out = F.log_mel(w2.contiguous(), plan, log_offset)
    if squeeze:
        out = out[0]
    return out.cpu().numpy() if as_numpy else out


def log_mel_batch(wave, audio_sample_rate=16000, log_offset=0.01, window_length_secs=0.128,
                  hop_length_secs=1.0 / 15, num_mel_bins=128, lower_edge_hertz=125.0,
                  upper_edge_hertz=7500.0, out=None):
    """Batched device front end with the build's defaults (128 mels at 15 fps):
    wave [C, S] -> [C, F, 128], the generator's audio input."""
    plan = F.LogMelPlan.get(audio_sample_rate, window_length_secs, hop_length_secs, num_mel_bins,
                            lower_edge_hertz, upper_edge_hertz, wave.device)
    return F.log_mel(wave, plan, log_offset, out=out)
