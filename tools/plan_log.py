"""Prints every engine launch of one eager bench step with its plan (A2M_GEMM_LOG=1 lines on
stderr): shape, tile, splits, operand modes, and whether the pipelined tile ran.
    A2M_GEMM_LOG=1 python tools/plan_log.py [bf16] 2> plans.txt"""
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)
sys.path.insert(0, os.path.join(REPO, 'audio-to-motion-generation_amd'))
import torch  # noqa: E402

import bench  # noqa: E402

dev = torch.device('cuda:0')
import a2m  # noqa: E402
a2m.set_gemm_precision('bf16' if 'bf16' in sys.argv[1:] else 'fp32')
g, wave = bench.build_infer(64, 64, 0, dev)
with torch.no_grad():
    step = bench.infer_step(g, wave)
    step()
    torch.cuda.synchronize()
    print('--- second step', file=sys.stderr, flush=True)
    step()
    torch.cuda.synchronize()
