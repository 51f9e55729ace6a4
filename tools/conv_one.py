"""One decoder tap conv1d (k3, Co = 256) launched R times eagerly (for PMC passes):
    python tools/conv_one.py B Ci [R]"""
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, 'audio-to-motion-generation_amd'))
import torch  # noqa: E402

from a2m import functional as F  # noqa: E402

B, Ci = int(sys.argv[1]), int(sys.argv[2])
R = int(sys.argv[3]) if len(sys.argv) > 3 else 10
dev = torch.device('cuda')
x = torch.randn(B, Ci, 64, device=dev)
w = torch.randn(256, Ci, 3, device=dev) * 0.05
b = torch.randn(256, device=dev)
cache = {}
for _ in range(R):
    F.conv1d(x, w, b, 1, 1, cache=cache)
torch.cuda.synchronize()
print('done')
