"""Times the decoders' SelfAttention(256) eval call (B=64, T=64: attn_fused_eval_kernel),
graph-replayed.   python tools/attn_eval_probe.py"""
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, 'audio-to-motion-generation_amd'))
import torch  # noqa: E402

from a2m import functional as F  # noqa: E402

dev = torch.device('cuda')
B, C, T = 64, 256, 64
x = torch.randn(B, C, T, device=dev)
wq, wk = torch.randn(C // 8, C, 1, device=dev) * 0.05, torch.randn(C // 8, C, 1, device=dev) * 0.05
wv = torch.randn(C, C, 1, device=dev) * 0.05
bq, bk, bv = torch.randn(C // 8, device=dev), torch.randn(C // 8, device=dev), torch.randn(C, device=dev)
g = torch.full((1,), 0.3, device=dev)
cache = {}
out = torch.empty_like(x)
run = lambda: F.self_attention(x, wq, bq, wk, bk, wv, bv, g, out=out, cache=cache)  # noqa: E731
run()
s = torch.cuda.Stream()
s.wait_stream(torch.cuda.current_stream())
iters = 50
with torch.cuda.stream(s):
    gr = torch.cuda.CUDAGraph()
    with torch.cuda.graph(gr, stream=s):
        for _ in range(iters):
            run()
    gr.replay()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record(s)
    for _ in range(5):
        gr.replay()
    e1.record(s)
e1.synchronize()
print(f'attention eval B={B} C={C} T={T}: {e0.elapsed_time(e1) * 1e3 / (5 * iters):.2f} us/launch', flush=True)
