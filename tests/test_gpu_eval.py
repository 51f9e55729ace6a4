"""GPU parity of the normalisation and PCK rows against the
reference's own outputs (tests/golden/eval_norm.npz, made by oracle/make_fixtures_eval.py)."""
import numpy as np
import pytest
import torch

from conftest import golden

pytestmark = pytest.mark.gpu


class _Loader:
    def __init__(self, batches):
        self.train = [{'pose/data': b} for b in batches]


@pytest.mark.parametrize('on_device', [False, True])
def test_mean_std_vs_reference(on_device):
    from a2m import normalization as NZ
    z = golden('eval_norm.npz')
    batches = [torch.from_numpy(z[f'batch{i}']) for i in range(int(z['n_batches']))]
    if on_device:
        batches = [b.cuda() for b in batches]
    for fn, tag in ((NZ.get_mean_std_necksub, 'necksub'), (NZ.get_mean_std, 'plain')):
        mean, std = fn(_Loader(batches))
        rm, rs = z[f'mean_{tag}'], z[f'std_{tag}']
        assert np.abs(mean.cpu().numpy() - rm).max() <= 1e-5 * np.abs(rm).max(), tag
        assert np.abs(std.cpu().numpy() - rs).max() <= 1e-5 * np.abs(rs).max(), tag


def test_normalize_denormalize():
    from a2m import normalization as NZ
    z = golden('eval_norm.npz')
    mean, std = torch.from_numpy(z['mean_necksub']).cuda(), torch.from_numpy(z['std_necksub']).cuda()
    pose = torch.from_numpy(z['batch0']).cuda()
    nrm = NZ.necksub_normalize(pose, mean, std)
    assert np.abs(nrm.cpu().numpy() - z['normalized0']).max() <= 1e-5
    assert np.abs(nrm.cpu().numpy()[..., [0, 52]]).max() <= 1e-6 * np.abs(z['mean_necksub']).max() + 1e-6
    den = NZ.denormalize(nrm, mean, std)
    assert np.abs(den.cpu().numpy() - z['denormalized0']).max() <= 1e-4


@pytest.mark.parametrize('K', [52, 48])
def test_pck_vs_reference(K):
    from a2m.evaluation import compute_pck
    z = golden('eval_norm.npz')
    for alpha, tag in ((0.2, 'a02'), (0.1, 'a01')):
        out = compute_pck(z[f'pck{K}_pred'], z[f'pck{K}_gt'], alpha)
        assert isinstance(out, np.ndarray) and np.array_equal(out, z[f'pck{K}_{tag}']), (K, tag)
    dev = compute_pck(torch.from_numpy(z[f'pck{K}_pred']).cuda(), torch.from_numpy(z[f'pck{K}_gt']).cuda())
    assert dev.is_cuda and np.array_equal(dev.cpu().numpy(), z[f'pck{K}_a02'])
    with pytest.raises(ValueError):
        compute_pck(z[f'pck{K}_pred'][:, :1], z[f'pck{K}_gt'][:, :1])


def test_inference_surface(tmp_path, g_state):
    """generate_motion_video.py's flow: Speech2Gesture_G, checkpoint round trip, generate with
    de-normalisation == generator output * std + mean."""
    from a2m import inference
    from a2m.real_motion_model import SelfAttention_G, Speech2Gesture_G
    assert Speech2Gesture_G is SelfAttention_G
    g = Speech2Gesture_G(p=0.0)
    g.load_state_dict(g_state, strict=False)
    path = tmp_path / 'gen.pth'
    torch.save(g.state_dict(), path)
    g2 = inference.load_generator(str(path), p=0.0)
    z = golden('g_eval_b2t64.npz')
    audio = torch.from_numpy(z['audio']).cuda()
    raw = inference.generate(g2, audio)
    assert np.abs(raw.cpu().numpy() - z['pose']).max() <= 1e-4 * np.abs(z['pose']).max()
    zn = golden('eval_norm.npz')
    mean, std = torch.from_numpy(zn['mean_necksub']), torch.from_numpy(zn['std_necksub'])
    den = inference.generate(g2, audio, mean, std)
    ref = z['pose'].astype(np.float64) * zn['std_necksub'] + zn['mean_necksub']
    assert np.abs(den.cpu().numpy() - ref).max() <= 1e-4 * np.abs(ref).max()
    assert tuple(inference.planar_frames(den).shape) == (2, 64, 2, 52)


def test_window_gather_matches_slicing():
    """gather_windows == data[start:start+window:interval] (dataUtils.py:646-665), with and
    without the loader's cached standardisation (std < 1e-7 -> 1)."""
    from a2m.windowing import PatsClip, gather_windows, window_index
    g = torch.Generator().manual_seed(5)
    mel = torch.randn(2000, 128, generator=g)
    pose = torch.randn(330, 104, generator=g)
    starts, window, interval = window_index(mel.shape[0], 'audio/log_mel_512', 15, 4.3, 5)
    out = gather_windows(mel.cuda(), starts, window, interval)
    ref = np.stack([mel.numpy()[s:s + window:interval] for s in starts])
    assert out.shape == ref.shape == (len(starts), 64, 128) and np.array_equal(out.cpu().numpy(), ref)
    mean, std = torch.randn(104, generator=g), torch.rand(104, generator=g) + 0.5
    std[3] = 0.0
    clip = PatsClip({'pose/data': pose.cuda(), 'audio/log_mel_512': mel.cuda()}, (15, 15), 4.3, 5,
                    norm_stats={'pose/data': (mean.cuda(), std.cuda())})
    n = len(clip)
    assert n == min(len(window_index(330, 'pose/data', 15, 4.3, 5)[0]), len(starts))
    b = clip.batch(np.arange(n))
    sp = window_index(330, 'pose/data', 15, 4.3, 5)[0][:n]
    sd = np.where(std.numpy() < 1e-7, 1.0, std.numpy())
    ref_p = np.stack([(pose.numpy()[s:s + 64] - mean.numpy()) / sd for s in sp]).astype(np.float32)
    assert np.abs(b['pose/data'].cpu().numpy() - ref_p).max() <= 1e-6 * np.abs(ref_p).max()
    assert b['audio/log_mel_512'].shape == (n, 64, 128)


def test_window_batches_match_reference_getitem():
    """PatsClip.batch / meta against the reference's own MiniData.__getitem__ outputs
    (tests/golden/windowing.npz, oracle/make_fixtures_r2.py): the gathered windows with the
    cached pose standardisation, and the start / end seconds."""
    from a2m.windowing import PatsClip
    from oracle.drivers import window_case_data
    z = golden('windowing.npz')
    lp, la, tm, hop, f0, f1 = z['cases'][0]
    pose, audio, mean, std = window_case_data(0, int(lp), int(la))
    clip = PatsClip({'pose/data': torch.from_numpy(pose).cuda(), 'audio/log_mel_512': torch.from_numpy(audio).cuda()},
                    (int(f0), int(f1)), float(tm), int(hop),
                    norm_stats={'pose/data': (torch.from_numpy(mean).cuda(), torch.from_numpy(std).cuda())})
    assert len(clip) == int(z['c0_len'])
    picks = z['c0_picks']
    b = clip.batch(picks)
    for k in range(len(picks)):
        ref_p = z[f'c0_item{k}_pose']
        assert np.abs(b['pose/data'][k].cpu().numpy() - ref_p).max() <= 1e-6 * np.abs(ref_p).max()
        assert np.array_equal(b['audio/log_mel_512'][k].cpu().numpy(), z[f'c0_item{k}_audio'])
    assert np.allclose(clip.meta(picks), np.stack([z[f'c0_item{k}_meta'] for k in range(len(picks))]),
                       rtol=0, atol=1e-12)


def test_graphed_generator_matches_eager(g_state):
    """a2m.inference.GraphedGenerator (trunk / body / hand / losses graphs on two streams)
    replays exactly the eager eval forward: same kernels, same order per output -> bitwise."""
    import torch
    from a2m.inference import GraphedGenerator
    from a2m.real_motion_model import SelfAttention_G
    g = SelfAttention_G(p=0.0)
    g.load_state_dict(g_state, strict=False)
    g = g.to('cuda').eval()
    torch.manual_seed(0)
    audio = torch.randn(4, 64, 128, device='cuda')
    with torch.no_grad():
        ref, ref_losses = g(audio)
        src = torch.empty_like(audio)
        runner = GraphedGenerator(g, lambda: src)
        for seed in (1, 2):
            src.copy_(audio if seed == 1 else audio.flip(0))
            out, losses = runner()
            want, want_l = (ref, ref_losses) if seed == 1 else g(audio.flip(0))
            assert torch.equal(out, want)
            assert torch.equal(losses[0], want_l[0])
