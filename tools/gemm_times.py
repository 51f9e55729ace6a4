"""Per-launch GEMM-engine times (HIP events on each launch's stream) for one eager inference
step and one training iteration at B=64, T=64.  Run with A2M_GEMM_LOG=2: the library prints one
'a2m gemm-time ...' line per launch to stderr; this script prints a summary table grouped by
shape/plan, sorted by total time.  Diagnostic only (tools/)."""
import os
import re
import subprocess
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def child(mode):
    sys.path.insert(0, os.path.join(REPO, 'audio-to-motion-generation_amd'))
    import torch
    from a2m import functional as F
    from a2m import real_motion_model as RM
    from a2m.real_motion_model import SelfAttention_D, SelfAttention_G
    dev = torch.device('cuda:0')
    torch.manual_seed(0)
    RM._BRANCH_STREAMS = False
    g = SelfAttention_G(p=0.2).to(dev)
    audio = torch.randn(64, 64, 128, device=dev)
    if mode == 'infer':
        g.eval()
        with torch.no_grad():
            g(audio)
            torch.cuda.synchronize()
            with F.gemm_timing() as t:
                g(audio)
                torch.cuda.synchronize()
    else:
        from a2m.training import GANTrainer
        d = SelfAttention_D(out_channels=64).to(dev).train()
        tr = GANTrainer(g.train(), d, lr=1e-3)
        pose = torch.randn(64, 64, 104, device=dev)
        tr.iteration(audio, pose, epoch=0, g_freq=3, d_freq=1)
        torch.cuda.synchronize()
        with F.gemm_timing() as t:
            tr.iteration(audio, pose, epoch=1, g_freq=3, d_freq=1)
            torch.cuda.synchronize()
    print(f'{mode}: {t.launches} launches, tile {t.ms_tile:.3f} ms, reduce {t.ms_reduce:.3f} ms, '
          f'{t.flops / 1e9:.1f} GFLOP', flush=True)


def main():
    pat = re.compile(r'a2m gemm-time (.*) tile ([\d.]+) us reduce ([\d.]+) us ([\d.]+) TF')
    for mode in os.environ.get('GT_MODES', 'infer,train').split(','):
        env = dict(os.environ, A2M_GEMM_LOG='2')
        r = subprocess.run([sys.executable, __file__, '--child', mode], env=env, capture_output=True,
                           text=True, timeout=300)
        print(r.stdout.strip())
        os.makedirs(os.path.join(REPO, 'gpurun_out'), exist_ok=True)
        with open(os.path.join(REPO, 'gpurun_out', f'gemm_times_{mode}.err'), 'w') as f:
            f.write(r.stderr)
        if r.returncode != 0:
            print(r.stderr[-3000:])
            sys.exit(r.returncode)
        groups = {}
        for line in r.stderr.splitlines():
            m = pat.search(line)
            if not m:
                continue
            g = groups.setdefault(m.group(1), [0, 0.0, 0.0, 0.0])
            g[0] += 1
            g[1] += float(m.group(2))
            g[2] += float(m.group(3))
            g[3] += float(m.group(4)) * float(m.group(2))
        rows = sorted(groups.items(), key=lambda kv: -(kv[1][1] + kv[1][2]))
        tot = sum(v[1] + v[2] for _, v in rows)
        print(f'{mode}: {len(rows)} distinct plans, {tot:.0f} us')
        print(f'{"plan":60s} {"n":>4s} {"tile_us":>9s} {"red_us":>8s} {"TF":>6s}')
        for k, (n, tu, ru, tfw) in rows[:40]:
            print(f'{k:60s} {n:4d} {tu:9.1f} {ru:8.1f} {tfw / max(tu, 1e-9):6.1f}')


if __name__ == '__main__':
    if len(sys.argv) > 2 and sys.argv[1] == '--child':
        child(sys.argv[2])
    else:
        main()
