"""conv2d weight-gradient timing (graph-replayed) and a bit-level checksum at the training
encoder's shapes (B=64 x 64 frames, full columns); run once per library (A2M_LIB) to compare.
Diagnostic (tools/)."""
import hashlib
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, 'audio-to-motion-generation_amd'))
sys.path.insert(0, REPO)
import torch  # noqa: E402

from a2m import functional as F  # noqa: E402
from tools.conv_ab import graph_time  # noqa: E402

# (Ci, Co, H, W, kh, kw, stride, pad) of the AudioEncoder's conv layers (model_layers.py:254-263)
SHAPES = [(64, 128, 32, 64, 4, 4, 2, (1, 1)), (128, 256, 16, 32, 4, 4, 2, (1, 1)),
          (256, 512, 8, 16, 3, 3, 1, (1, 1)), (512, 256, 8, 16, 3, 8, 1, (1, 3))]
g = torch.Generator(device='cuda').manual_seed(0)
for Ci, Co, H, W, kh, kw, s, p in SHAPES:
    Ho, Wo = (H + 2 * p[0] - kh) // s + 1, (W + 2 * p[1] - kw) // s + 1
    x = torch.randn(64, Ci, H, W, device='cuda', generator=g)
    dy = torch.randn(64, Co, Ho, Wo, device='cuda', generator=g)
    dw = F.conv_wgrad(dy, x, (Co, Ci, kh, kw), s, p)
    torch.cuda.synchronize()
    h = hashlib.sha1(dw.cpu().numpy().tobytes()).hexdigest()[:12]
    t = graph_time(lambda: F.conv_wgrad(dy, x, (Co, Ci, kh, kw), s, p))
    fl = 2.0 * Co * Ci * kh * kw * 64 * Ho * Wo
    print(f'wgrad Ci={Ci} Co={Co} k=({kh},{kw}) Wo={Wo}: {t:8.1f} us {fl / t / 1e6:6.1f} TF  sha1 {h}', flush=True)
