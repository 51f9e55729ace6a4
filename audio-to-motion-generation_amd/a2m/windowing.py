"""PATS sample windowing on the device: the index arithmetic of
dataUtils.MiniData.update_idx_list (dataUtils.py:585-624) and the strided window slices of
__getitem__ (:646-665), gathering whole batches of windows from sequences resident in HBM.

  window_index(length, modality, fs_new, time=4.3, window_hop=0) -> (starts, window, interval)
      window = int(time * fs); interval = round(fs / fs_new);
      starts = range(0, length - window, window if window_hop == 0 else window_hop * interval)
      (the reference's bound excludes the last full window; kept)
  gather_windows(data, starts, window, interval, mean=None, std=None) -> [n, ceil(window/interval), C]
  PatsClip(sequences, fs_new, time, window_hop): per-file windows for several modalities,
      len = min over modalities (:624-626), batch(idx) -> {modality: [n, T, C]}

Modality sampling rates: pose 15 (skeleton.py:150-151), audio/log_mel_512 int(45.6e3/512) = 89,
audio/log_mel_400 int(16.52e3/160) = 103 (audio.py:174-180).  HDF5 reading itself is out of
scope (h5py is absent here and the reference's loader chain does not import).
"""
import numpy as np
import torch

from . import functional as F
from ._native import check, lib

FS = {'pose/data': 15, 'audio/log_mel_512': int(45.6 * 1000 / 512),
      'audio/log_mel_400': int(16.52 * 1000 / 160), 'audio/silence': 15}


def window_index(length, modality, fs_new, time=4.3, window_hop=0):
    fs = FS[modality] if isinstance(modality, str) else modality
    window = int(time * fs)
    assert window_hop < window, 'hop size {} must be less than window size {}'.format(window_hop, window)
    interval = round(fs / fs_new)
    step = int(window) if not window_hop else int(window_hop * interval)
    starts = np.arange(0, length - window, step, dtype=np.int64)
    return starts, window, interval


def gather_windows(data, starts, window, interval, mean=None, std=None, out=None):
    """data [L, C] on the device; starts: int64 array/tensor -> [n, ceil(window/interval), C]."""
    F._check_dev(data, mean, std, out)
    data = data.contiguous()
    L, C = data.shape
    st = torch.as_tensor(np.asarray(starts, np.int64)).to(data.device) if not torch.is_tensor(starts) \
        else starts.to(data.device, torch.int64)
    if st.numel() and (int(st.min()) < 0 or int(st.max()) + window > L):
        raise ValueError('window out of range')
    nj = (window + interval - 1) // interval
    if out is None:
        out = torch.empty(st.numel(), nj, C, device=data.device)
    check(lib.a2m_window_gather_f32(F._p(data), L, C, F._p(st), st.numel(), window, interval,
                                    F._p(mean), F._p(std), F._p(out), F._stream()))
    return out


class PatsClip:
    """Windows of one recording's modalities (e.g. {'pose/data': [Lp,104], 'audio/log_mel_512': [La,128]})."""

    def __init__(self, sequences, fs_new=(15, 15), time=4.3, window_hop=0, norm_stats=None):
        self.seq = sequences
        self.index = {}
        for (mod, data), fn in zip(sequences.items(), fs_new):
            self.index[mod] = window_index(data.shape[0], mod, fn, time, window_hop)
        self.norm_stats = norm_stats or {}
        self.fs_new = tuple(fs_new)

    def __len__(self):
        return min(len(ix[0]) for ix in self.index.values())

    @staticmethod
    def window_times(first_index, last_index, fs_new, idx):
        """__getitem__'s meta start / end seconds (dataUtils.py:660,718-725): the start counts
        the LAST modality's strided samples before its window (len(data[0:start:interval]),
        the loop variable left over from the modality loop), the duration is the FIRST
        modality's window length; both over fs_new[-1]."""
        s_last, _, i_last = last_index
        s_first, w_first, i_first = first_index
        out = []
        for k in np.asarray(idx, np.int64).reshape(-1):
            start = len(range(0, int(s_last[k]), i_last)) / fs_new[-1]
            dur = len(range(int(s_first[k]), int(s_first[k]) + w_first, i_first)) / fs_new[-1]
            out.append((start, start + dur))
        return np.array(out, dtype=np.float64).reshape(-1, 2)

    def meta(self, idx):
        mods = list(self.seq)
        return self.window_times(self.index[mods[0]], self.index[mods[-1]], self.fs_new, idx)

    def batch(self, idx):
        idx = np.asarray(idx, np.int64)
        out = {}
        for mod, data in self.seq.items():
            starts, window, interval = self.index[mod]
            ns = self.norm_stats.get(mod)
            out[mod] = gather_windows(data, starts[idx], window, interval,
                                      *(ns if ns is not None else (None, None)))
        return out
