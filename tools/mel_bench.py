"""Times the log-mel kernel alone at the bench workload (B=64 clips x 64 frames) and at the
long-form size (8 x 480 frames), graph-replayed so host launch cost is excluded."""
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)
sys.path.insert(0, os.path.join(REPO, 'audio-to-motion-generation_amd'))
import torch  # noqa: E402

import bench  # noqa: E402
from oracle import synth  # noqa: E402

dev = torch.device('cuda:0')
CFGS = ((64, 64), (8, 480), (256, 64))
if len(sys.argv) > 1:
    CFGS = CFGS[:int(sys.argv[1])]
for B, T in CFGS:
    wave = torch.from_numpy(synth.speech_like(B, synth.samples_for_frames(T), seed=1)).to(dev)
    ms, nbytes = bench.run_mel_kernel(dev, wave)
    print(f'logmel B={B} T={T}: {ms * 1e3:.2f} us/launch, {nbytes / ms / 1e6:.1f} GB/s '
          f'({nbytes / ms / 1e6 / 8000:.3f} of 8 TB/s), {B * T / ms * 1e3 / 1e6:.1f} M frames/s')
