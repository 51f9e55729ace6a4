"""Probe: a2m timing marks / GEMM timing events inside a torch HIP-graph capture."""
import os
import sys
import traceback
REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, 'audio-to-motion-generation_amd'))
import torch  # noqa: E402
from a2m import functional as F  # noqa: E402

dev = torch.device('cuda:0')
x = torch.randn(256, 256, device=dev)


def attempt(name, pre, body):
    try:
        pre()
        s = torch.cuda.Stream(dev)
        s.wait_stream(torch.cuda.current_stream(dev))
        with torch.cuda.stream(s):
            g = torch.cuda.CUDAGraph()
            with torch.cuda.graph(g, stream=s):
                body()
        torch.cuda.synchronize()
        g.replay()
        torch.cuda.synchronize()
        print(name, 'OK', F.timing_mark_elapsed(0, 1))
    except Exception as e:
        print(name, 'FAIL', repr(e)[:200])
        traceback.print_exc(limit=3)


def body():
    F.timing_mark(0)
    y = torch.empty(256, 256, device=dev)
    y.copy_(x * 2)
    F.timing_mark(1)


def body_nomark():
    y = torch.empty(256, 256, device=dev)
    y.copy_(x * 2)


def body_late():
    y = torch.empty(256, 256, device=dev)
    F.timing_mark(0)
    y.copy_(x * 2)
    F.timing_mark(1)
    z = torch.empty(512, 256, device=dev)
    z.zero_()


def body_kernel_first():
    y = torch.empty(256, 256, device=dev)
    y.zero_()
    F.timing_mark(0)
    y.copy_(x * 2)
    F.timing_mark(1)


mode = sys.argv[1]
if mode == 'c':
    attempt('no marks', lambda: None, body_nomark)
if mode == 'd':
    attempt('alloc before mark, alloc after', lambda: None, body_late)
if mode == 'e':
    attempt('kernel before first mark', lambda: None, body_kernel_first)
if mode == 'a':
    attempt('lazy-create marks', lambda: None, body)
elif mode == 'b':
    attempt('pre-created marks', lambda: (F.timing_mark(0), F.timing_mark(1), torch.cuda.synchronize()), body)
