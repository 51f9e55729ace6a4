"""CPU-side checks of the boundary: the C-ABI library loads and exports every symbol that
include/a2m.h declares, host-side plan building matches the reference filterbank, and the
drop-in modules expose the reference's state_dict keys.  No GPU compute here."""
import ctypes
import os
import re

import numpy as np
import pytest
import torch

from conftest import REPO, golden, golden_keys

HEADER = os.path.join(REPO, 'include', 'a2m.h')


def header_symbols():
    src = open(HEADER).read()
    return sorted(set(re.findall(r'^\s*(?:const\s+)?[a-z_0-9]+\*?\s+\*?(a2m_[a-z0-9_]+)\(', src, re.M)))


def test_library_exports_every_header_symbol():
    from a2m import _native
    syms = header_symbols()
    assert len(syms) >= 15
    for s in syms:
        assert hasattr(_native.lib, s), s
    assert sorted(_native.SIGNATURES) == syms
    assert _native.lib.a2m_version() == 1


def test_logmel_geometry_and_frames():
    from a2m import _native as N
    w, h, n = ctypes.c_int32(), ctypes.c_int32(), ctypes.c_int32()
    assert N.lib.a2m_logmel_geometry(16000, 0.128, 1 / 15, ctypes.byref(w), ctypes.byref(h), ctypes.byref(n)) == 0
    assert (w.value, h.value, n.value) == (2048, 1067, 2048)
    assert N.lib.a2m_logmel_num_frames(69269, 2048, 1067) == 64
    assert N.lib.a2m_logmel_num_frames(2048, 2048, 1067) == 1
    assert N.lib.a2m_logmel_num_frames(2047, 2048, 1067) == 0
    assert N.lib.a2m_logmel_num_frames(513141, 2048, 1067) == 480


def test_logmel_geometry_rounds_like_python():
    """window/hop = int(round(sr * secs)) with Python's half-to-even rounding of the double
    product, fft_len = 2 ** ceil(log2(window)) (mel_features.py:212-214), over a sweep of rates
    and durations that includes the .5 cases (44.1 kHz x 25 ms = 1102.5, 22.05 kHz x 10 ms =
    220.5)."""
    from a2m import _native as N
    w, h, n = ctypes.c_int32(), ctypes.c_int32(), ctypes.c_int32()
    rates = [8000, 11025, 16000, 22050, 24000, 32000, 44100, 48000, 96000]
    secs = [0.001, 0.0025, 0.005, 0.01, 0.015, 0.02, 0.025, 0.03, 0.032, 0.04, 0.05, 0.064,
            0.1, 0.128, 1 / 15, 1 / 30, 0.0125, 0.0375]
    seen_half = 0
    for sr in rates:
        for ws in secs:
            for hs in secs:
                rc = N.lib.a2m_logmel_geometry(sr, ws, hs, ctypes.byref(w), ctypes.byref(h), ctypes.byref(n))
                ew, eh = int(round(sr * ws)), int(round(sr * hs))
                if ew < 2 or eh < 1:
                    continue
                ef = 2 ** int(np.ceil(np.log(ew) / np.log(2.0)))
                if ef > 16384:
                    continue
                assert rc == 0, (sr, ws, hs)
                assert (w.value, h.value, n.value) == (ew, eh, ef), (sr, ws, hs)
                seen_half += (sr * ws) % 1 == 0.5
    assert seen_half > 0
    N.lib.a2m_logmel_geometry(44100, 0.025, 0.010, ctypes.byref(w), ctypes.byref(h), ctypes.byref(n))
    assert (w.value, h.value, n.value) == (1102, 441, 2048)
    N.lib.a2m_logmel_geometry(22050, 0.025, 0.010, ctypes.byref(w), ctypes.byref(h), ctypes.byref(n))
    assert (w.value, h.value, n.value) == (551, 220, 1024)


def _plan_arrays(sr, win, hop, nm, lo, hi):
    from a2m import _native as N
    nb = N.lib.a2m_logmel_plan_bytes(sr, win, hop, nm, lo, hi)
    buf = (ctypes.c_uint8 * nb)()
    assert N.lib.a2m_logmel_plan_build(sr, win, hop, nm, lo, hi, buf, nb) == 0
    raw = bytes(buf)
    hdr = np.frombuffer(raw[:48], dtype=np.int32)
    window, hopn, nfft, n_mels, n_bins, nnz = hdr[:6]
    o_win, o_tw, o_start, o_len, o_woff, o_w = hdr[6:12]
    start = np.frombuffer(raw[o_start:o_start + 4 * n_mels], dtype=np.int32)
    ln = np.frombuffer(raw[o_len:o_len + 4 * n_mels], dtype=np.int32)
    woff = np.frombuffer(raw[o_woff:o_woff + 4 * n_mels], dtype=np.int32)
    wts = np.frombuffer(raw[o_w:o_w + 4 * nnz], dtype=np.float32)
    dense = np.zeros((n_bins, n_mels), dtype=np.float32)
    for m in range(n_mels):
        dense[start[m]:start[m] + ln[m], m] = wts[woff[m]:woff[m] + ln[m]]
    hann = np.frombuffer(raw[o_win:o_win + 4 * window], dtype=np.float32)
    return dense, hann, nfft


def test_logmel_plan_matches_reference_filterbank():
    z = golden('mel.npz')
    dense, hann, nfft = _plan_arrays(16000, 0.128, 1 / 15, 128, 125.0, 7500.0)
    ref = z['mel_build_matrix']
    assert np.array_equal(dense, ref.astype(np.float32))
    assert (ref != 0).sum() == (dense != 0).sum()
    n = np.arange(2048)
    assert np.array_equal(hann, (0.5 - 0.5 * np.cos(2 * np.pi / 2048 * n)).astype(np.float32))


def test_logmel_plan_errors_match_reference_valueerror_text():
    from a2m import _native as N
    z = golden('mel.npz')
    cases = [(-1.0, 7500.0), (8000.0, 7000.0), (125.0, 9000.0)]
    for (lo, hi), msg in zip(cases, z['mel_errors']):
        buf = (ctypes.c_uint8 * 64)()
        rc = N.lib.a2m_logmel_plan_build(16000, 0.004, 0.001, 8, lo, hi, buf, 64)
        assert rc == N.A2M_EINVAL
        assert N.last_error() == msg


def test_state_dict_keys_match_reference():
    from a2m.real_motion_model import SelfAttention_D, SelfAttention_G
    keys = golden_keys()
    g = SelfAttention_G(p=0.0)
    d = SelfAttention_D(out_channels=64, p=0.0)
    for mod, ref in ((g, keys['G']), (d, keys['D'])):
        sd = mod.state_dict()
        assert sorted(sd) == sorted(ref)
        for k, shp in ref.items():
            assert list(sd[k].shape) == shp, k


def test_edge_template_checked_on_load():
    """A reference checkpoint's edge template loads; a different topology is refused."""
    import torch
    from a2m.real_motion_model import SelfAttention_G
    g = SelfAttention_G(p=0.0)
    sd = g.state_dict()
    g.load_state_dict(sd)
    bad = dict(sd)
    g.load_state_dict({**sd, 'body_edge_index_template': sd['body_edge_index_template'].flip(1)})
    bad['body_edge_index_template'] = sd['body_edge_index_template'].clone()
    bad['body_edge_index_template'][1, 0] = (bad['body_edge_index_template'][1, 0] + 3) % 10
    with pytest.raises(RuntimeError, match='edge template'):
        g.load_state_dict(bad)
    assert torch.equal(g.body_edge_index_template, sd['body_edge_index_template'])


def test_old_pyg_gat_keys_load():
    from a2m.graph_layers import GATConv
    m = GATConv(64, 64, heads=4, concat=False)
    sd = {k: v.clone() for k, v in m.state_dict().items()}
    w = sd.pop('lin.weight')
    sd['lin_src.weight'] = w + 1
    sd['lin_dst.weight'] = w + 1
    m.load_state_dict(sd)
    assert torch.equal(m.lin.weight, w + 1)


def test_skeleton_tables_match_reference():
    from a2m import skeleton as S
    z = golden('losses.npz')
    assert S.triples(10, 42) == [tuple(t) for t in z['hand_triples'].tolist()]
    assert S.triples(0, 10) == [tuple(t) for t in z['body_triples'].tolist()]
    assert S.edge_index(0, 10).shape == (2, 18)
    assert S.edge_index(10, 42).shape == (2, 80)
    ptr, idx = S.in_neighbour_csr(S.edge_index(10, 42), 42)
    assert ptr[-1] == 80 and int(ptr[1] - ptr[0]) == 5   # each hand root has 5 children


def test_encoder_live_columns():
    from a2m.model_layers import AudioEncoder
    enc = AudioEncoder()
    assert enc.live_columns(128) == [(9, 55), (5, 27), (3, 13), (4, 12), (7, 8)]


def test_ops_refuse_cpu_tensors():
    from a2m import functional as F
    x = torch.zeros(1, 4, 8)
    w = torch.zeros(4, 4, 3)
    with pytest.raises(RuntimeError, match='no CPU fallback'):
        F.conv1d(x, w)


def test_pats_window_index_geometry():
    """dataUtils.update_idx_list arithmetic (dataUtils.py:585-624; restated -- the reference
    loader does not import, so no reference run pins it): 4.3 s windows give 64 pose frames at
    15 fps and 64 audio frames from log_mel_512 at fs 89 with stride round(89/15) = 6."""
    from a2m.windowing import FS, window_index
    assert FS['audio/log_mel_512'] == 89 and FS['pose/data'] == 15
    s_p, w_p, i_p = window_index(1000, 'pose/data', 15, 4.3, 5)
    assert (w_p, i_p) == (64, 1) and s_p[1] - s_p[0] == 5 and s_p[-1] < 1000 - 64
    s_a, w_a, i_a = window_index(6000, 'audio/log_mel_512', 15, 4.3, 5)
    assert (w_a, i_a) == (382, 6) and s_a[1] - s_a[0] == 30 and len(range(0, w_a, i_a)) == 64
    s0, w0, _ = window_index(200, 'pose/data', 15, 4.3, 0)
    assert list(s0) == list(range(0, 200 - 64, 64))
    with pytest.raises(AssertionError):
        window_index(200, 'pose/data', 15, 4.3, 64)


def test_gemm_precision_switch():
    """fp32 by default; the context manager sets and restores; bad values raise like the ABI."""
    import a2m
    from a2m import _native as N
    assert N.lib.a2m_get_gemm_precision() == 0
    with a2m.gemm_precision('bf16'):
        assert N.lib.a2m_get_gemm_precision() == 1
    assert N.lib.a2m_get_gemm_precision() == 0
    assert N.lib.a2m_set_gemm_precision(7) == N.A2M_EINVAL
    with pytest.raises(ValueError):
        a2m.set_gemm_precision('fp16')
