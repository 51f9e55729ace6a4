"""AudioEncoder eval at B=64 x T=64, graph-replayed (diagnostic): run under rocprofv3
--kernel-trace to get every launch of the encoder; prints nothing itself."""
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, 'audio-to-motion-generation_amd'))
sys.path.insert(0, REPO)
import torch  # noqa: E402

from a2m.real_motion_model import SelfAttention_G  # noqa: E402
from tools.conv_ab import graph_time  # noqa: E402

torch.manual_seed(0)
enc = SelfAttention_G(p=0.2).cuda().eval().audio_encoder
x = torch.randn(64, 64, 128, device='cuda')
with torch.no_grad():
    print(f'encoder graph {graph_time(lambda: enc(x), iters=10, reps=2):.1f} us', flush=True)
