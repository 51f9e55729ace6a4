"""Which Python lines issue device copies (aten::copy_) in one eval forward of the bench step."""
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)
sys.path.insert(0, os.path.join(REPO, 'audio-to-motion-generation_amd'))
import collections  # noqa: E402
import traceback  # noqa: E402

import torch  # noqa: E402

import bench  # noqa: E402
from a2m.mel_features import log_mel_batch  # noqa: E402
from a2m.real_motion_model import SelfAttention_G  # noqa: E402

dev = torch.device('cuda')
g = SelfAttention_G(p=0.2).to(dev).eval()
wave = bench.synth_wave(64, (64 - 1) * bench.HOP + bench.WIN, seed=0, device=dev)
with torch.no_grad():
    g(log_mel_batch(wave))
    torch.cuda.synchronize()
    sites = collections.Counter()
    orig_copy = torch.Tensor.copy_
    orig_contig = torch.Tensor.contiguous

    def where():
        st = [f for f in traceback.extract_stack()[:-2] if 'a2m' in f.filename or 'bench' in f.filename]
        return ' <- '.join(f'{os.path.basename(f.filename)}:{f.lineno}' for f in st[-3:])

    def copy_(self, src, *a, **k):
        sites['copy_ ' + where()] += 1
        return orig_copy(self, src, *a, **k)

    def contiguous(self, *a, **k):
        if not self.is_contiguous(*a, **k):
            sites['contiguous ' + where()] += 1
        return orig_contig(self, *a, **k)

    torch.Tensor.copy_ = copy_
    torch.Tensor.contiguous = contiguous
    with torch.profiler.profile(activities=[torch.profiler.ProfilerActivity.CUDA]) as prof:
        g(log_mel_batch(wave))
        torch.cuda.synchronize()
    torch.Tensor.copy_ = orig_copy
    torch.Tensor.contiguous = orig_contig
for k, v in sites.most_common(30):
    print(v, k)
print(prof.key_averages().table(sort_by='cuda_time_total', row_limit=12))
