"""Per-shape GEMM times of one training iteration (bench.py --mode train, B=64): every engine
launch timed with events (a2m_gemm_timing_*), aggregated by (modes, M, N, K, plan).
usage: A2M_GEMM_LOG=2 python tools/train_gemm_times.py 2> log; python tools/train_gemm_times.py --summarise log"""
import collections
import os
import re
import sys

if len(sys.argv) > 2 and sys.argv[1] == '--summarise':
    agg = collections.defaultdict(lambda: [0, 0.0, 0.0])
    for line in open(sys.argv[2]):
        m = re.match(r'a2m gemm-time (.*) tile ([\d.]+) us (?:\(all-XCD span [\d.]+\) )?reduce ([\d.]+) us', line)
        if m:
            a = agg[m.group(1)]
            a[0] += 1
            a[1] += float(m.group(2))
            a[2] += float(m.group(3))
    tot = sum(v[1] + v[2] for v in agg.values())
    print(f'total {tot / 1e3:.2f} ms of engine time in one iteration')
    for k, (n, t, r) in sorted(agg.items(), key=lambda kv: -(kv[1][1] + kv[1][2]))[:40]:
        print(f'{(t + r) / 1e3:7.3f} ms {n:4d} x  {k}  (reduce {r / 1e3:.3f} ms)')
    sys.exit(0)

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, 'audio-to-motion-generation_amd'))
import torch  # noqa: E402

from a2m import functional as F  # noqa: E402
from a2m.real_motion_model import SelfAttention_D, SelfAttention_G  # noqa: E402
from a2m.training import GANTrainer  # noqa: E402

dev = torch.device('cuda')
torch.manual_seed(1234)
g = SelfAttention_G(time_steps=64, p=0.2).to(dev).train()
d = SelfAttention_D(out_channels=64).to(dev).train()
tr = GANTrainer(g, d, lr=10e-4, label_seed=7)
gen = torch.Generator().manual_seed(100)
audio = torch.randn(64, 64, 128, generator=gen).to(dev)
pose = torch.randn(64, 64, 104, generator=gen).to(dev)
for i in range(2):
    tr.iteration(audio, pose, epoch=i, g_freq=3, d_freq=1)
torch.cuda.synchronize()
with F.gemm_timing() as t:
    tr.iteration(audio, pose, epoch=2, g_freq=3, d_freq=1)
    torch.cuda.synchronize()
print(f'engine: {t.launches} launches, {t.ms_tile:.2f} ms tiles + {t.ms_reduce:.2f} ms reduces')
