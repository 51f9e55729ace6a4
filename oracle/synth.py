"""Deterministic synthetic inputs.  TEST ORACLE / BENCH INPUT ONLY.

Audio: 16 kHz float32, 0.1*N(0,1) white noise + 3 harmonics of f0 ~ U(90, 250) Hz,
amplitude-modulated at 4 Hz, clipped to [-1, 1].  numpy PCG64 streams are bit-stable
across machines, so the GPU box regenerates exactly the committed inputs.
"""
import numpy as np

SR = 16000
WIN = 2048          # int(round(16000 * 0.128))
HOP = 1067          # int(round(16000 / 15))


def samples_for_frames(n_frames, win=WIN, hop=HOP):
    """Shortest waveform that yields exactly n_frames mel frames (mel_features.py:42)."""
    return (n_frames - 1) * hop + win


def speech_like(n_clips, n_samples, seed=0, f0_range=(90.0, 250.0), sr=SR):
    rng = np.random.default_rng(seed)
    t = np.arange(n_samples, dtype=np.float64) / sr
    out = np.empty((n_clips, n_samples), dtype=np.float32)
    for c in range(n_clips):
        f0 = rng.uniform(*f0_range)
        phase = rng.uniform(0, 2 * np.pi, size=3)
        amp = np.array([0.3, 0.15, 0.08])
        voiced = sum(a * np.sin(2 * np.pi * f0 * (h + 1) * t + p)
                     for h, (a, p) in enumerate(zip(amp, phase)))
        env = 0.5 * (1.0 + np.sin(2 * np.pi * 4.0 * t + rng.uniform(0, 2 * np.pi)))
        noise = 0.1 * rng.standard_normal(n_samples)
        out[c] = np.clip(voiced * env + noise, -1.0, 1.0).astype(np.float32)
    return out


def pose_targets(n_clips, n_frames, seed=1, feats=104):
    """Already neck-subtracted + normalised pose targets ~ N(0,1)."""
    return np.random.default_rng(seed).standard_normal((n_clips, n_frames, feats)).astype(np.float32)
