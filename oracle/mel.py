"""numpy float64 restatement of the log-mel front end.  TEST ORACLE ONLY.

Follows pose_video/mel_features.py of the reference:
  frame                      :21-45   num_frames = 1 + floor((N - W) / H), no padding
  periodic_hann              :48-68   0.5 - 0.5 cos(2 pi n / W)
  stft_magnitude             :71-92   |rfft(frame * window, fft_len)|
  hertz_to_mel               :100-111 HTK 1127 ln(1 + f / 700)
  spectrogram_to_mel_matrix  :114-189 triangular filters linear in mel, DC row zeroed,
                                      ValueError on bad edges (:156-163)
  log_mel_spectrogram        :192-223 int(round(sr*secs)) window/hop, fft_len = 2^ceil(log2 W)
"""
import numpy as np

MEL_BREAK_HZ = 700.0
MEL_HIGH_Q = 1127.0


def frame_count(n_samples, window, hop):
    return 1 + int(np.floor((n_samples - window) / hop))


def frames(wave, window, hop):
    n = max(frame_count(wave.shape[0], window, hop), 0)
    idx = np.arange(window)[None, :] + hop * np.arange(n)[:, None]
    return wave[idx] if n else np.zeros((0, window), dtype=wave.dtype)


def hann_periodic(window):
    return 0.5 - 0.5 * np.cos(2.0 * np.pi * np.arange(window) / window)


def hz_to_mel(f):
    return MEL_HIGH_Q * np.log(1.0 + np.asarray(f, dtype=np.float64) / MEL_BREAK_HZ)


def mel_matrix(num_mel_bins, num_spectrogram_bins, sample_rate, lower_hz, upper_hz):
    nyq = sample_rate / 2.0
    if lower_hz < 0.0:
        raise ValueError("lower_edge_hertz %.1f must be >= 0" % lower_hz)
    if lower_hz >= upper_hz:
        raise ValueError("lower_edge_hertz %.1f >= upper_edge_hertz %.1f" % (lower_hz, upper_hz))
    if upper_hz > nyq:
        raise ValueError("upper_edge_hertz %.1f is greater than Nyquist %.1f" % (upper_hz, nyq))
    bin_mel = hz_to_mel(np.linspace(0.0, nyq, num_spectrogram_bins))[:, None]       # [S,1]
    edges = np.linspace(hz_to_mel(lower_hz), hz_to_mel(upper_hz), num_mel_bins + 2)
    lo, mid, hi = edges[:-2][None, :], edges[1:-1][None, :], edges[2:][None, :]      # [1,M]
    rising = (bin_mel - lo) / (mid - lo)
    falling = (hi - bin_mel) / (hi - mid)
    w = np.maximum(0.0, np.minimum(rising, falling))
    w[0, :] = 0.0
    return w


def log_mel(wave, sample_rate=8000, log_offset=0.0, window_secs=0.025, hop_secs=0.010,
            num_mel_bins=20, lower_hz=125.0, upper_hz=3800.0):
    wave = np.asarray(wave, dtype=np.float64)
    win = int(round(sample_rate * window_secs))
    hop = int(round(sample_rate * hop_secs))
    nfft = 2 ** int(np.ceil(np.log(win) / np.log(2.0)))
    spec = np.abs(np.fft.rfft(frames(wave, win, hop) * hann_periodic(win), nfft))
    mel = spec @ mel_matrix(num_mel_bins, spec.shape[1], sample_rate, lower_hz, upper_hz)
    return np.log(mel + log_offset)


# The build's front-end configuration: 128 mel bins at 15 fps.
BUILD_CFG = dict(sample_rate=16000, log_offset=0.01, window_secs=0.128, hop_secs=1.0 / 15,
                 num_mel_bins=128, lower_hz=125.0, upper_hz=7500.0)
