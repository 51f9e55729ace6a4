"""Runs exactly the bench step (bench.py configs[1]: HIP log-mel + SelfAttention_G eval over
B synthetic clips, captured in one HIP graph) and nothing else, for PMC passes whose per-launch
averages must describe the benched code: the two eager warm-up steps of bench.capture_step and
the capture, then one marker kernel (torch.cuda._sleep), then R graph replays.  The tools that
read the output (replay_filter.py) keep only the dispatches after the marker, i.e. the
replayed steps: no first-call repacks, no eager-step copies.

    rocprofv3 --pmc FETCH_SIZE -d DIR -- python tools/step_pmc.py [R] [--dtype bf16]
        [--engine-json F] [--stamps F] [--sync] [--batch B]
--stamps also records the engine launches' own span stamps in every replay (a device sync after
each replay), so the kernel trace and the stamps describe the same dispatches
(tools/stamp_vs_trace.py).
"""
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)
sys.path.insert(0, os.path.join(REPO, 'audio-to-motion-generation_amd'))
import torch  # noqa: E402

import bench  # noqa: E402


def main():
    argv = sys.argv[1:]
    ejson = None
    if '--engine-json' in argv:
        i = argv.index('--engine-json')
        ejson = argv[i + 1]
        del argv[i:i + 2]
    sjson = None
    if '--stamps' in argv:   # also record the engine's span stamps of every replay (tools/stamp_vs_trace.py)
        i = argv.index('--stamps')
        sjson = argv[i + 1]
        del argv[i:i + 2]
    # --sync: a device sync after every replay.  Free-running replays under --kernel-trace ran the
    # step 11 % slower than unprofiled (2.97 vs 2.67 ms, r04j) and lengthened every traced kernel
    # with it (engine 2628 us/step against 2345 us with a sync per replay, the stamps' 2265 us of
    # spans + 2.2 us per launch); unprofiled, synced and free-running replays take the same time
    # (tools/branch_probe.py: 2.672 vs 2.661 ms)
    B = 64
    if '--batch' in argv:
        i = argv.index('--batch')
        B = int(argv[i + 1])
        del argv[i:i + 2]
    sync = '--sync' in argv
    args = [a for a in argv if not a.startswith('--') and a != 'bf16']
    reps = int(args[0]) if args else 3
    dev = torch.device('cuda:0')
    import a2m
    a2m.set_gemm_precision('bf16' if '--dtype' in sys.argv and 'bf16' in sys.argv else 'fp32')
    from a2m.real_motion_model import SelfAttention_G
    T = 64
    torch.manual_seed(1234)
    g = SelfAttention_G(time_steps=T, p=0.2)
    for m in g.modules():
        if hasattr(m, 'gamma'):
            torch.nn.init.constant_(m.gamma, 0.3)
    g = g.to(dev).eval()
    wave = bench.synth_wave(B, (T - 1) * bench.HOP + bench.WIN, seed=0, device=dev)
    import contextlib
    from a2m import functional as F
    with torch.no_grad():
        with (F.gemm_timing(keep=True) if sjson else contextlib.nullcontext()) as tm:
            graph, out = bench.capture_step(dev, bench.infer_step(g, wave))
        graph.replay()
        torch.cuda.synchronize()
        if ejson:
            # the engine's algorithmic FLOPs per step (one eager step with the timing hook),
            # for tools/replay_breakdown.py's roofline figure
            gt = bench.gemm_engine_timing(bench.infer_step(g, wave))
            import json
            with open(ejson, 'w') as f:
                json.dump({'launches': gt.launches, 'gflop': gt.flops / 1e9}, f)
        torch.cuda._sleep(1000)             # the marker dispatch
        torch.cuda.synchronize()
        stamps = []
        if sjson:
            tm.spans()   # re-arm after the pre-marker replay
        for _ in range(reps):
            graph.replay()
            if sync:
                torch.cuda.synchronize()
            if sjson:
                stamps.append([sp for sp in tm.spans(ready=True) if sp[1] >= 0])
    torch.cuda.synchronize()
    if sjson:
        tm.release()
        import json
        with open(sjson, 'w') as f:
            json.dump({'replays': stamps}, f)
    print(f'step_pmc: 2 eager + 1 graph step, marker, then {reps} replayed steps, out {tuple(out.shape)}')


if __name__ == '__main__':
    main()
