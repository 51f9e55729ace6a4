"""AudioEncoder eval forward alone (B=64, T=64), repeated: for rocprofv3 kernel traces / PMC
passes of the encoder's launches (tools/pmc_cmd.sh TAG FILTER tools/encoder_probe.py)."""
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, 'audio-to-motion-generation_amd'))
import torch  # noqa: E402

from a2m.model_layers import AudioEncoder  # noqa: E402

dev = torch.device('cuda')
torch.manual_seed(0)
enc = AudioEncoder().to(dev).eval()
x = torch.randn(64, 64, 128, device=dev)
with torch.no_grad():
    for _ in range(int(os.environ.get('REPS', '10'))):
        enc(x)
torch.cuda.synchronize()
print('ok')
