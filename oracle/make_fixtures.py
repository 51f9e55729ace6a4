"""Generate tests/golden/* by running the REFERENCE itself in this container.

Run:  python -m oracle.make_fixtures      (needs /root/reference; never runs on the GPU box)

The reference's import chain is broken as committed; this harness
  * imports model_layers first (transformers is present, only BertModel is imported),
  * registers empty stubs for h5py / librosa / webrtcvad / nltk.corpus and a top-level
    `common` with no-op Modality / MissingData (data plumbing, off the hot path),
  * loads pats/data_loading/skeleton.py by file path and exposes it as
    pats.data_loading.Skeleton2D (it reads ../data/cmu_intervals_df.csv relative to the
    CWD, so the harness runs from a temp dir holding a 2-column stand-in CSV),
  * provides torch_geometric from oracle/pyg_restatement.py (PyG absent -> GNN parity is
    pinned only against that restatement: "parity unpinned" vs real PyG),
  * applies the one shape fix the reference needs to run at all:
    unet.up_attention = SelfAttention(input_channels*8)  (model_layers.py:339 vs :364-365).
Nothing of the reference is copied: only inputs and outputs are written.
"""
import importlib.util
import json
import os
import sys
import tempfile
import types
import zlib

import numpy as np
import torch

REF = os.environ.get('A2M_REFERENCE', '/root/reference')
HERE = os.path.dirname(os.path.abspath(__file__))
REPO = os.path.dirname(HERE)
GOLDEN = os.path.join(REPO, 'tests', 'golden')
sys.path.insert(0, REPO)

from oracle import pyg_restatement, synth, weights  # noqa: E402


def _stub(name, **attrs):
    m = types.ModuleType(name)
    for k, v in attrs.items():
        setattr(m, k, v)
    sys.modules[name] = m
    return m


def load_reference():
    sys.path.insert(0, REF)
    import model_layers  # noqa: F401  (real transformers)
    from pose_video import mel_features
    for n in ('h5py', 'librosa', 'webrtcvad', 'nltk'):
        _stub(n)
    _stub('nltk.corpus', stopwords=None)

    class Modality:
        def __init__(self, *a, **k):
            pass

    class MissingData:
        def __init__(self, *a, **k):
            pass

    _stub('common', Modality=Modality, MissingData=MissingData)
    spec = importlib.util.spec_from_file_location(
        'ref_skeleton', os.path.join(REF, 'pats', 'data_loading', 'skeleton.py'))
    skel = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(skel)
    pats = _stub('pats')
    dl = _stub('pats.data_loading', Skeleton2D=skel.Skeleton2D)
    pats.data_loading = dl
    tg = _stub('torch_geometric')
    tg.nn = _stub('torch_geometric.nn', GATConv=pyg_restatement.GATConv,
                  GraphConv=pyg_restatement.GraphConv)
    tg.data = _stub('torch_geometric.data', Data=pyg_restatement.Data,
                    Batch=pyg_restatement.Batch)
    import real_motion_model
    return mel_features, model_layers, real_motion_model


def in_tmp_cwd():
    d = tempfile.mkdtemp(prefix='a2m_ref_')
    os.makedirs(os.path.join(d, 'data'))
    os.makedirs(os.path.join(d, 'run'))
    with open(os.path.join(d, 'data', 'cmu_intervals_df.csv'), 'w') as f:
        f.write('delta_time,interval_id\n1.0,0\n')
    os.chdir(os.path.join(d, 'run'))


def build_models(model_layers, rmm, p=0.0, seed=1234):
    g = rmm.SelfAttention_G(p=p)
    g.unet.up_attention = model_layers.SelfAttention(g.unet.up_attention.query_conv.in_channels * 2)
    d = rmm.SelfAttention_D(out_channels=64, p=p)
    weights.load_into(g, seed)
    weights.load_into(d, seed + 1)
    return g, d


def grad_summary(module, prefix, nsamp=16):
    names, sums, sqs, idxs, vals = [], [], [], [], []
    for name, prm in module.named_parameters():
        if prm.grad is None:
            continue
        g = prm.grad.detach().double().reshape(-1)
        rng = np.random.default_rng(zlib.crc32(name.encode()))
        k = min(nsamp, g.numel())
        ix = np.sort(rng.choice(g.numel(), k, replace=False))
        ix = np.pad(ix, (0, nsamp - k), constant_values=-1)
        v = np.where(ix >= 0, g.numpy()[np.maximum(ix, 0)], 0.0)
        names.append(name)
        sums.append(g.sum().item())
        sqs.append((g * g).sum().item())
        idxs.append(ix)
        vals.append(v)
    return {f'{prefix}_names': np.array(names), f'{prefix}_sum': np.array(sums),
            f'{prefix}_sumsq': np.array(sqs), f'{prefix}_idx': np.array(idxs),
            f'{prefix}_val': np.array(vals)}


def main():
    os.makedirs(GOLDEN, exist_ok=True)
    cwd = os.getcwd()
    in_tmp_cwd()
    mf, ml, rmm = load_reference()
    torch.manual_seed(0)
    out = {}

    # ---------------- log-mel front end (mel_features.py:192-223) ----------------
    B, T = 2, 64
    wav = synth.speech_like(B, synth.samples_for_frames(T), seed=7)
    build = dict(audio_sample_rate=16000, log_offset=0.01, window_length_secs=0.128,
                 hop_length_secs=1.0 / 15, num_mel_bins=128, lower_edge_hertz=125.0,
                 upper_edge_hertz=7500.0)
    mel = np.stack([mf.log_mel_spectrogram(w.astype(np.float64), **build) for w in wav])
    out['mel_build_wave'] = wav
    out['mel_build_out'] = mel
    out['mel_build_matrix'] = mf.spectrogram_to_mel_matrix(
        num_mel_bins=128, num_spectrogram_bins=1025, audio_sample_rate=16000,
        lower_edge_hertz=125.0, upper_edge_hertz=7500.0)
    w1 = synth.speech_like(1, 16000, seed=8)[0]
    out['mel_repr_wave'] = w1
    out['mel_repr_out'] = mf.log_mel_spectrogram(
        w1.astype(np.float64), audio_sample_rate=16000, log_offset=0.01,
        window_length_secs=0.025, hop_length_secs=0.010, num_mel_bins=64,
        lower_edge_hertz=125, upper_edge_hertz=7500)
    w2 = synth.speech_like(1, 8000, seed=9)[0]
    out['mel_default_wave'] = w2
    out['mel_default_out'] = mf.log_mel_spectrogram(w2.astype(np.float64))
    w3 = synth.speech_like(1, 2048, seed=10)[0]
    out['mel_oneframe_wave'] = w3
    out['mel_oneframe_out'] = mf.log_mel_spectrogram(w3.astype(np.float64), **build)
    out['mel_empty_out'] = mf.log_mel_spectrogram(w3[:2047].astype(np.float64), **build)
    errs = []
    for kw in (dict(lower_edge_hertz=-1.0), dict(lower_edge_hertz=8000.0, upper_edge_hertz=7000.0),
               dict(upper_edge_hertz=9000.0)):
        try:
            mf.spectrogram_to_mel_matrix(num_mel_bins=8, num_spectrogram_bins=33,
                                         audio_sample_rate=16000, **{**dict(lower_edge_hertz=125.0,
                                                                            upper_edge_hertz=7500.0), **kw})
            errs.append('')
        except ValueError as e:
            errs.append(str(e))
    out['mel_errors'] = np.array(errs)
    np.savez_compressed(os.path.join(GOLDEN, 'mel.npz'), **out)

    # ---------------- generator / discriminator, eval mode ----------------
    g, d = build_models(ml, rmm, p=0.0)
    g.eval()
    d.eval()
    audio = torch.from_numpy(mel.astype(np.float32))
    pose = torch.from_numpy(synth.pose_targets(B, T, seed=11))
    acts = {}
    hook_names = ['audio_encoder', 'unet', 'body_decoder_pre', 'hand_decoder_pre',
                  'body_gcn1', 'body_gcn2', 'hand_gcn1', 'hand_gcn2', 'body_proj_in', 'body_norm',
                  'hand_norm', 'body_decoder_post', 'hand_decoder_post', 'body_logits', 'hand_logits',
                  'unet.bottleneck_attention', 'unet.up_attention']
    mods = dict(g.named_modules())
    hs = [mods[n].register_forward_hook(
        (lambda n: lambda m, i, o: acts.__setitem__(n, o.detach().clone()))(n)) for n in hook_names]
    with torch.no_grad():
        gout, glosses = g(audio, real_pose=pose)
        dout, _ = d(torch.diff(pose, dim=1))
    for h in hs:
        h.remove()
    ev = {'audio': audio.numpy(), 'real_pose': pose.numpy(), 'pose': gout.numpy(),
          'bone': glosses[0].numpy(), 'angle': glosses[1].numpy(), 'd_real': dout.numpy()}
    for n, a in acts.items():
        ev['act/' + n] = a.numpy()
    np.savez_compressed(os.path.join(GOLDEN, 'g_eval_b2t64.npz'), **ev)
    keys = {'G': {k: list(v.shape) for k, v in g.state_dict().items()},
            'D': {k: list(v.shape) for k, v in d.state_dict().items()}}
    with open(os.path.join(GOLDEN, 'state_dict_keys.json'), 'w') as f:
        json.dump(keys, f, indent=0)

    # long-form: B=1, T=480 (C4)
    wl = synth.speech_like(1, synth.samples_for_frames(480), seed=12)[0]
    mel_l = mf.log_mel_spectrogram(wl.astype(np.float64), **build).astype(np.float32)
    with torch.no_grad():
        gl, ll = g(torch.from_numpy(mel_l)[None])
    np.savez_compressed(os.path.join(GOLDEN, 'g_eval_b1t480.npz'), audio=mel_l[None],
                        pose=gl.numpy(), angle=ll[0].numpy())

    # ---------------- small loss fixtures (real_motion_model.py:307-461) ----------------
    pz = torch.from_numpy(np.random.default_rng(13).standard_normal((3, 8, 104)).astype(np.float32))
    pr = torch.from_numpy(np.random.default_rng(14).standard_normal((3, 8, 104)).astype(np.float32))
    np.savez_compressed(os.path.join(GOLDEN, 'losses.npz'), gen=pz.numpy(), real=pr.numpy(),
                        bone=g.compute_bone_length_loss(pr, pz).numpy(),
                        hand=g.compute_hand_joint_angle_loss(pz).numpy(),
                        body=g.compute_body_joint_angle_loss(pz).numpy(),
                        angle=g.compute_comprehensive_angle_loss(pz).numpy(),
                        hand_triples=np.array(g.hand_triples), body_triples=np.array(g.body_triples))

    # ---------------- one training iteration, train mode, p=0 (version5_model_train.py:342-405) ----
    sys.path.insert(0, REF)
    g, d = build_models(ml, rmm, p=0.0)
    g.train()
    d.train()
    valid = torch.full((B, 4), 0.93)
    fake = torch.full((B, 4), 0.07)
    real_motion = torch.diff(pose, dim=1)
    fake_pose, internal = g(audio, real_pose=pose)
    fake_motion = torch.diff(fake_pose, dim=1)
    fake_d, _ = d(fake_motion)
    acc = fake_motion[:, 1:] - fake_motion[:, :-1]
    jerk = acc[:, 1:] - acc[:, :-1]
    l1 = torch.nn.L1Loss()(real_motion, fake_motion)
    adv = torch.nn.MSELoss()(fake_d, valid)
    smooth = torch.mean(torch.norm(acc, dim=-1))
    jk = torch.mean(torch.norm(jerk, dim=-1))
    G_loss = l1 + adv + 0.1 * smooth + 0.05 * jk + internal[0] + internal[1]
    G_loss.backward()
    tr = {'fake_pose': fake_pose.detach().numpy(), 'fake_d': fake_d.detach().numpy(),
          'G_loss': G_loss.detach().numpy(),
          'parts': np.array([l1.item(), adv.item(), smooth.item(), jk.item(),
                             internal[0].item(), internal[1].item()])}
    tr.update(grad_summary(g, 'gG'))
    tr['bn_rm/unet.bottleneck.norm'] = g.unet.bottleneck.norm.running_mean.numpy().copy()
    tr['bn_rv/unet.bottleneck.norm'] = g.unet.bottleneck.norm.running_var.numpy().copy()
    d.zero_grad()
    with torch.no_grad():
        fp2, _ = g(audio)
        fm2 = torch.diff(fp2, dim=1)
    fd2, _ = d(fm2.detach())
    rd2, _ = d(real_motion)
    D_loss = torch.nn.MSELoss()(rd2, valid) + torch.nn.MSELoss()(fd2, fake)
    D_loss.backward()
    tr['D_loss'] = D_loss.detach().numpy()
    tr['d_fake'] = fd2.detach().numpy()
    tr['d_real'] = rd2.detach().numpy()
    tr.update(grad_summary(d, 'gD'))
    np.savez_compressed(os.path.join(GOLDEN, 'train_step_b2t64.npz'), **tr)
    os.chdir(cwd)
    print('fixtures written to', GOLDEN)


if __name__ == '__main__':
    main()
