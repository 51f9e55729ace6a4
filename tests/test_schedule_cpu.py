"""Host logic of the training schedule and the PATS windowing against the reference's own
code, run here through committed fixtures (oracle/make_fixtures_r2.py executes the reference's
DynamicGANTraining class and MiniData methods; these tests run a2m's on the same inputs).
No GPU."""
import json
import os

import numpy as np
import pytest

from conftest import GOLDEN, golden


@pytest.mark.parametrize('mode', ['plain', 'dynamic_smooth'])
def test_dynamic_gan_training_matches_reference(mode):
    """Every G/D frequency, learning rate, train-D branch, rolling mean and smoothed-label draw
    of version5_model_train.py:12-180 under the fixed loss sequence, bit for bit."""
    from a2m.training import DynamicGANTraining
    from oracle.drivers import DYN_LOSSES, run_schedule
    with open(os.path.join(GOLDEN, 'dyn_schedule.json')) as f:
        ref = json.load(f)
    assert [tuple(x) for x in ref['losses']] == DYN_LOSSES
    got = run_schedule(DynamicGANTraining, dynamic_smooth=(mode == 'dynamic_smooth'))
    want = ref[mode]
    for key in ('g_freq', 'd_freq', 'train_d'):
        assert got[key] == want[key], key
    for key in ('g_lr', 'd_lr', 'recent', 'labels_real', 'labels_fake'):
        assert np.array_equal(np.array(got[key]), np.array(want[key])), key
    # the sequence reaches every branch: both frequency moves, both LR moves, a skipped D step
    assert {False, True} <= set(want['train_d'])
    assert len(set(want['g_freq'])) >= 3 and len(set(want['d_freq'])) == 2
    assert min(want['g_lr']) < 5e-4 < max(want['g_lr'])


def _window_case(ci):
    z = golden('windowing.npz')
    from oracle.drivers import window_case_data
    lp, la, tm, hop, f0, f1 = z['cases'][ci]
    return z, (int(lp), int(la), float(tm), int(hop), (int(f0), int(f1))), window_case_data(ci, int(lp), int(la))


@pytest.mark.parametrize('ci', [0, 1, 2, 3])
def test_window_index_matches_reference(ci):
    """MiniData.update_idx_list / __len__ (dataUtils.py:585-626): starts, ends, interval, count
    for pose (fs 15) and log_mel_512 (fs 89) at the reference's own window/hop arithmetic."""
    from a2m.windowing import PatsClip, window_index
    z, (lp, la, tm, hop, fsn), _ = _window_case(ci)
    for mod, tag, L, fn in (('pose/data', 'p', lp, fsn[0]), ('audio/log_mel_512', 'a', la, fsn[1])):
        starts, window, interval = window_index(L, mod, fn, tm, hop)
        assert np.array_equal(starts, z[f'c{ci}_{tag}_starts'])
        assert np.array_equal(starts + window, z[f'c{ci}_{tag}_ends'])
        assert interval == int(z[f'c{ci}_{tag}_interval'])
    clip_len = min(len(window_index(lp, 'pose/data', fsn[0], tm, hop)[0]),
                   len(window_index(la, 'audio/log_mel_512', fsn[1], tm, hop)[0]))
    assert clip_len == int(z[f'c{ci}_len'])
    meta = PatsClip.window_times(window_index(lp, 'pose/data', fsn[0], tm, hop),
                                 window_index(la, 'audio/log_mel_512', fsn[1], tm, hop), fsn,
                                 z[f'c{ci}_picks'])
    for k in range(len(z[f'c{ci}_picks'])):
        assert np.allclose(meta[k], z[f'c{ci}_item{k}_meta'], rtol=0, atol=1e-12)


def test_window_slices_match_reference_host():
    """__getitem__'s slices data[start:end:interval] with the cached standardisation
    (x - mean) / where(std < 1e-7, 1, std) (dataUtils.py:646-663), restated on the host in
    float32 like the reference; the GPU gather is held to these same arrays in
    tests/test_gpu_eval.py."""
    from a2m.windowing import window_index
    z, (lp, la, tm, hop, fsn), (pose, audio, mean, std) = _window_case(0)
    sp, wp, ip = window_index(lp, 'pose/data', fsn[0], tm, hop)
    sa, wa, ia = window_index(la, 'audio/log_mel_512', fsn[1], tm, hop)
    sd = np.where(std < 1e-7, 1.0, std)
    for k, idx in enumerate(z['c0_picks']):
        p = (pose[sp[idx]:sp[idx] + wp:ip] - mean) / sd
        a = audio[sa[idx]:sa[idx] + wa:ia]
        assert np.array_equal(p, z[f'c0_item{k}_pose'])
        assert np.array_equal(a, z[f'c0_item{k}_audio'])
