"""The data-parallel training path over RCCL on one MI355X (version5_model_train.py:350-405;
VERDICT r03 item 8).

A fresh child process initialises a one-rank `nccl` (= RCCL) process group before anything
touches the GPU, then runs the real GANTrainer with `force_collectives=True`, so the bucketed
gradient all-reduces are launched by RCCL from the autograd post-accumulate hooks during the
backward, and SyncBN's statistics all-reduces run, exactly as on N ranks:

  local     -- no collectives (the single-device step)
  dp_fp32   -- bucketed RCCL all-reduce, fp32 on the wire
  dp_bf16   -- the same with bf16 on the wire (configs[4]'s grad_reduce_dtype)
  dp_syncbn -- fp32 wire + SyncBN (every train-mode BatchNorm's statistics all-reduced)

each two G-steps (D frozen) and two D-steps at B = 8, lr = 0, p = 0, fixed labels, several
buckets (the second step of each launches buckets from the hooks during its backward).
With one rank a SUM all-reduce is the identity, so:
  - dp_fp32 gradients equal the local step's bit for bit;
  - dp_bf16 gradients equal the local gradients rounded to bf16, bit for bit;
  - dp_syncbn equals the local step to fp32 rounding (SyncBN runs its statistics through the
    split stats / all-reduce / apply path instead of the fused kernel).
"""
import json
import os
import socket
import subprocess
import sys

import pytest

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
pytestmark = pytest.mark.gpu


def _child(out):
    import torch
    import torch.distributed as dist
    sys.path[:0] = [REPO, os.path.join(REPO, 'audio-to-motion-generation_amd'), os.path.join(REPO, 'tests')]
    dev = torch.device('cuda', 0)
    # the process group first, before any GPU call (RCCL binds the device here)
    dist.init_process_group('nccl', rank=0, world_size=1, device_id=dev)
    torch.cuda.set_device(dev)
    from a2m import autograd as AG
    from a2m.training import GANTrainer
    from oracle import synth
    from test_gpu_configs import _models
    gen = torch.Generator().manual_seed(31)
    B = 8
    audio = (torch.randn(B, 64, 128, generator=gen) * 2.0 - 3.0).to(dev)
    pose = torch.from_numpy(synth.pose_targets(B, 64, seed=32)).to(dev)
    res = {}
    for mode in ('local', 'local_again', 'dp_fp32', 'dp_bf16', 'dp_syncbn'):
        g, d = _models(dev)
        tr = GANTrainer(g, d, lr=0.0, fixed_labels=(0.93, 0.07), bucket_mb=8.0,
                        force_collectives=mode != 'local', sync_bn=mode == 'dp_syncbn',
                        grad_reduce_dtype=torch.bfloat16 if mode == 'dp_bf16' else None)
        valid, fake = tr._labels(0, B, dev)
        for p_ in d.parameters():
            p_.requires_grad_(False)
        with tr.sync_bn_scope():
            # two steps each (lr = 0: the same parameters): the first learns which parameters
            # receive gradients, the second launches its buckets from the hooks during backward
            for _ in range(2):
                gl = tr.g_step(audio, pose, valid)
            for p_ in d.parameters():
                p_.requires_grad_(True)
            gg = tr.opt_G.flat_grad.detach().clone()
            gnamed = {n: p_.grad.detach().clone() for n, p_ in g.named_parameters() if p_.grad is not None}
            for _ in range(2):
                dl = tr.d_step(audio, AG.pos_to_motion(pose), valid, fake)
            dg = tr.opt_D.flat_grad.detach().clone()
        torch.cuda.synchronize()
        res[mode] = dict(gl=gl.item(), dl=dl.item(), gg=gg, dg=dg, gnamed=gnamed,
                         buckets=(len(tr.red_G.buckets), len(tr.red_D.buckets)),
                         in_backward=(tr.red_G.in_backward, tr.red_D.in_backward),
                         sync_bn=tr.sync_bn)
    loc = res['local']
    rep = {'backend': dist.get_backend(), 'world': dist.get_world_size()}
    for mode in ('local_again', 'dp_fp32', 'dp_bf16', 'dp_syncbn'):
        r = res[mode]
        ref_g, ref_d = loc['gg'], loc['dg']
        diff = sorted(((n, ((r['gnamed'][n] - v).abs().max() / v.abs().max().clamp_min(1e-30)).item())
                       for n, v in loc['gnamed'].items()), key=lambda kv: -kv[1])
        if mode == 'dp_bf16':
            ref_g, ref_d = ref_g.bfloat16().float(), ref_d.bfloat16().float()

        def rel(a, b):
            return ((a - b).abs().max() / b.abs().max()).item()
        rep[mode] = dict(g_equal=bool(torch.equal(r['gg'], ref_g)), d_equal=bool(torch.equal(r['dg'], ref_d)),
                         g_rel=rel(r['gg'], ref_g), d_rel=rel(r['dg'], ref_d),
                         gl_rel=abs(r['gl'] - loc['gl']) / abs(loc['gl']),
                         dl_rel=abs(r['dl'] - loc['dl']) / abs(loc['dl']),
                         buckets=r['buckets'], in_backward=r['in_backward'], sync_bn=r['sync_bn'],
                         g_worst=[(n, v) for n, v in diff[:6] if v > 0])
    dist.destroy_process_group()
    with open(out, 'w') as f:
        json.dump(rep, f)


def test_rccl_dp_step_one_rank(tmp_path):
    out = str(tmp_path / 'rccl.json')
    with socket.socket() as sk:
        sk.bind(('127.0.0.1', 0))
        port = sk.getsockname()[1]
    env = dict(os.environ, MASTER_ADDR='127.0.0.1', MASTER_PORT=str(port), RANK='0', WORLD_SIZE='1',
               LOCAL_RANK='0')
    p = subprocess.run([sys.executable, os.path.abspath(__file__), '--child', out], env=env,
                       capture_output=True, text=True, timeout=300)
    assert p.returncode == 0, p.stderr[-4000:]
    rep = json.load(open(out))
    print(json.dumps(rep))
    assert rep['backend'] == 'nccl' and rep['world'] == 1
    assert rep['local_again']['g_equal'] and rep['local_again']['d_equal'], rep['local_again']
    for mode in ('dp_fp32', 'dp_bf16', 'dp_syncbn'):
        r = rep[mode]
        # several buckets, and some of them launched from the gradient hooks during the backward
        assert r['buckets'][0] > 1 and r['in_backward'][0] >= 1, r
    assert rep['dp_fp32']['g_equal'] and rep['dp_fp32']['d_equal'], rep['dp_fp32']
    assert rep['dp_bf16']['g_equal'] and rep['dp_bf16']['d_equal'], rep['dp_bf16']
    s = rep['dp_syncbn']
    assert s['sync_bn']
    assert s['gl_rel'] < 1e-5 and s['dl_rel'] < 1e-5, s
    # gradients: the train step amplifies forward rounding ~200x, so a few ulps
    # of difference in the statistics may show at ~1e-5 here
    assert s['g_rel'] < 1e-3 and s['d_rel'] < 1e-3, s


def _child_graph(out):
    """GANTrainer(graphs=True) over the one-rank RCCL group: the G-step and D-step bodies are
    captured with their bucket all-reduces (launched from the gradient hooks during the captured
    backward) and replayed; the replayed gradients equal the local eager step's bit for bit."""
    import torch
    import torch.distributed as dist
    sys.path[:0] = [REPO, os.path.join(REPO, 'audio-to-motion-generation_amd'), os.path.join(REPO, 'tests')]
    dev = torch.device('cuda', 0)
    dist.init_process_group('nccl', rank=0, world_size=1, device_id=dev)
    torch.cuda.set_device(dev)
    from a2m import autograd as AG
    from a2m.training import GANTrainer
    from oracle import synth
    from test_gpu_configs import _models
    gen = torch.Generator().manual_seed(31)
    B = 8
    audio = (torch.randn(B, 64, 128, generator=gen) * 2.0 - 3.0).to(dev)
    pose = torch.from_numpy(synth.pose_targets(B, 64, seed=32)).to(dev)
    res = {}
    for mode in ('local', 'dp_graph'):
        g, d = _models(dev)
        tr = GANTrainer(g, d, lr=0.0, fixed_labels=(0.93, 0.07), bucket_mb=8.0,
                        force_collectives=mode != 'local', graphs=mode == 'dp_graph')
        valid, fake = tr._labels(0, B, dev)
        for p_ in d.parameters():
            p_.requires_grad_(False)
        gls = [tr.g_step(audio, pose, valid).item() for _ in range(4)]
        for p_ in d.parameters():
            p_.requires_grad_(True)
        gg = tr.opt_G.flat_grad.detach().clone()
        dls = [tr.d_step(audio, AG.pos_to_motion(pose), valid, fake).item() for _ in range(4)]
        dg = tr.opt_D.flat_grad.detach().clone()
        torch.cuda.synchronize()
        res[mode] = dict(gls=gls, dls=dls, gg=gg, dg=dg, buckets=(len(tr.red_G.buckets), len(tr.red_D.buckets)),
                         captured=(tr._captured['g'] is not None, tr._captured['d'] is not None))
    loc, r = res['local'], res['dp_graph']
    rep = {'backend': dist.get_backend(), 'world': dist.get_world_size(),
           'g_equal': bool(torch.equal(r['gg'], loc['gg'])), 'd_equal': bool(torch.equal(r['dg'], loc['dg'])),
           'losses_equal': r['gls'] == loc['gls'] and r['dls'] == loc['dls'],
           'gls': r['gls'], 'gls_local': loc['gls'], 'buckets': r['buckets'], 'captured': r['captured']}
    dist.destroy_process_group()
    with open(out, 'w') as f:
        json.dump(rep, f)


def test_rccl_dp_graph_one_rank(tmp_path):
    out = str(tmp_path / 'rccl_graph.json')
    with socket.socket() as sk:
        sk.bind(('127.0.0.1', 0))
        port = sk.getsockname()[1]
    env = dict(os.environ, MASTER_ADDR='127.0.0.1', MASTER_PORT=str(port), RANK='0', WORLD_SIZE='1',
               LOCAL_RANK='0')
    p = subprocess.run([sys.executable, os.path.abspath(__file__), '--child-graph', out], env=env,
                       capture_output=True, text=True, timeout=240)
    assert p.returncode == 0, p.stderr[-4000:]
    rep = json.load(open(out))
    print(json.dumps(rep))
    assert rep['backend'] == 'nccl' and rep['captured'] == [True, True], rep
    assert rep['buckets'][0] > 1, rep
    assert rep['g_equal'] and rep['d_equal'] and rep['losses_equal'], rep


if __name__ == '__main__':
    if len(sys.argv) == 3 and sys.argv[1] == '--child':
        _child(sys.argv[2])
    elif len(sys.argv) == 3 and sys.argv[1] == '--child-graph':
        _child_graph(sys.argv[2])
    else:
        sys.exit('usage: test_gpu_rccl.py --child OUT.json (run by pytest)')
