"""End-to-end SyncBN check over real process groups:
  python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 \
         --master-port 29511 tools/syncbn_check.py [--backend gloo|nccl]
Every rank holds half of B=8 clips.  One training step's G+D gradients (G's own terms, D's MSE
on real motion; p = 0) are all-reduced and compared with the single-process whole-batch step
that rank 0 also runs, once with SyncBN and once with per-rank BatchNorm statistics.  With gloo
both ranks may share one GPU.  Prints one JSON line from rank 0."""
import argparse
import json
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
for p in (REPO, os.path.join(REPO, 'audio-to-motion-generation_amd'), os.path.join(REPO, 'tests')):
    sys.path.insert(0, p)
import torch  # noqa: E402
import torch.distributed as dist  # noqa: E402

B = 8


def step(dev, audio, pose, sync_group, world):
    from conftest import golden_keys
    from a2m import autograd as AG
    from a2m import functional as F
    from a2m.real_motion_model import SelfAttention_D, SelfAttention_G
    from oracle import weights
    keys = golden_keys()
    g = SelfAttention_G(p=0.0)
    g.load_state_dict(weights.make_state_dict(keys['G'], seed=1234), strict=False)
    d = SelfAttention_D(out_channels=64, p=0.0)
    d.load_state_dict(weights.make_state_dict(keys['D'], seed=1235), strict=False)
    g, d = g.to(dev).train(), d.to(dev).train()
    prev = F.set_sync_bn_group(sync_group)
    try:
        fake, internal = g(audio, real_pose=pose)
        terms = AG.motion_terms(fake, pose)
        loss = terms[0] + 0.1 * terms[1] + 0.05 * terms[2] + internal[0]
        loss.backward()
        rd, _ = d(AG.pos_to_motion(pose))
        AG.mse_loss(rd, torch.full((rd.shape[0], 4), 0.93, device=dev)).backward()
    finally:
        F.set_sync_bn_group(prev)
    flat = torch.cat([p.grad.reshape(-1) for m in (g, d) for p in m.parameters() if p.grad is not None])
    if world > 1:
        dist.all_reduce(flat)
        flat /= world
    run = torch.cat([b.reshape(-1).float() for m in (g, d) for n, b in m.named_buffers() if 'running' in n])
    return flat, run, fake.detach()


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument('--backend', default='gloo')
    args = ap.parse_args()
    rank, world = int(os.environ['RANK']), int(os.environ['WORLD_SIZE'])
    local = int(os.environ.get('LOCAL_RANK', '0'))
    dev = torch.device('cuda', local if args.backend == 'nccl' else 0)
    torch.cuda.set_device(dev)
    dist.init_process_group(args.backend, rank=rank, world_size=world)
    from oracle import synth
    gen = torch.Generator().manual_seed(7)
    audio = torch.randn(B, 64, 128, generator=gen) * 2.0 - 3.0
    pose = torch.from_numpy(synth.pose_targets(B, 64, seed=8))
    sl = slice(rank * B // world, (rank + 1) * B // world)
    a, p = audio[sl].to(dev), pose[sl].to(dev)
    g_sync, r_sync, f_sync = step(dev, a, p, dist.group.WORLD, world)
    g_loc, r_loc, f_loc = step(dev, a, p, None, world)
    if rank == 0:
        g_one, r_one, f_one = step(dev, audio.to(dev), pose.to(dev), None, 1)

        def rel(x, y):
            return ((x - y).abs().max() / y.abs().max()).item()
        res = {'check': 'SyncBN DP step vs single-process whole batch', 'backend': args.backend,
               'world': world, 'clips': B,
               'sync': {'fake': rel(f_sync, f_one[sl]), 'grad': rel(g_sync, g_one), 'running': rel(r_sync, r_one)},
               'per_rank_bn': {'fake': rel(f_loc, f_one[sl]), 'grad': rel(g_loc, g_one), 'running': rel(r_loc, r_one)}}
        # grad bound: fp32 summation-order spread of this step (0.2-0.5 %)
        res['pass'] = bool(res['sync']['fake'] < 1e-4 and res['sync']['running'] < 1e-4 and
                           res['sync']['grad'] < 5e-3 and res['per_rank_bn']['fake'] > 10 * res['sync']['fake'] and
                           res['per_rank_bn']['grad'] > 10 * res['sync']['grad'])
        print(json.dumps(res), flush=True)
    dist.barrier()
    dist.destroy_process_group()


if __name__ == '__main__':
    main()
