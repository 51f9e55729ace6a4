"""Benchmark: pose-frames/sec on batch-64 x 64-frame clips (BASELINE.json metric, configs[1]).

One step = HIP log-mel front end over B synthetic 16 kHz waveforms (69,269 samples -> 64
frames each) + SelfAttention_G forward (eval) -> [B, 64, 104] poses, fp32, inputs resident
in HBM.  The step is captured once in a HIP graph and replayed.  N GPUs = N independent
replicas (inference does not shard further: "replicas only", weak scaling), launched one
process per GPU by torch.distributed.run; max-over-ranks time.

Printed JSON adds `roofline` (the dominant kernel family -- the implicit-GEMM engine's
gemm_kernel, ~65 % of kernel time -- every launch of the replayed step graph timed by its own
span stamps (first block start to last wave end on the GPU wall clock, the interval rocprof's
kernel trace reports), algorithmic FLOPs 2*M*N*K per launch, against the fp32 MFMA peak;
`traffic` from the committed PMC pass, profiles/traffic_latest.json), `mel_roofline`
(log-mel kernel vs HBM peak), `path_roofline` (the whole G forward's useful FLOPs) and
`cpu_baseline` (the torch-CPU oracle port on a bounded sample, rank 0 at N=1 only).
"""
import argparse
import json
import os
import sys
import time

REPO = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(REPO, 'audio-to-motion-generation_amd'))

import torch  # noqa: E402
import torch.distributed as dist  # noqa: E402

FP32_MFMA_PEAK_TFLOPS = 157.3     # MI355X_MICROARCH.md, chip-level parameters
BF16_MFMA_PEAK_TFLOPS = 2516.6  # dense bf16 MFMA (MI355X_MICROARCH.md; = 16 x the fp32 rate)
HBM_PEAK_GBS = 8000.0
SR, WIN, HOP = 16000, 2048, 1067


def synth_wave(B, n, seed, device):
    g = torch.Generator(device='cpu').manual_seed(seed)
    t = torch.arange(n, dtype=torch.float64) / SR
    f0 = 90 + 160 * torch.rand(B, 1, generator=g, dtype=torch.float64)
    env = 0.5 * (1 + torch.sin(2 * torch.pi * 4.0 * t))
    v = sum(a * torch.sin(2 * torch.pi * f0 * (h + 1) * t) for h, a in enumerate((0.3, 0.15, 0.08)))
    w = (v * env + 0.1 * torch.randn(B, n, generator=g, dtype=torch.float64)).clamp(-1, 1)
    return w.float().to(device)


def infer_step(g, wave):
    """One bench step: HIP log-mel over the resident waveforms + SelfAttention_G forward."""
    from a2m.mel_features import log_mel_batch

    def step():
        mel = log_mel_batch(wave)
        out, _ = g(mel)
        return out
    return step


def capture_step(dev, step):
    """Warm the step up on a side stream, then capture it in one HIP graph (the decoder
    branches' fork/join streams are recorded with it).  Returns (graph, static output)."""
    step()
    torch.cuda.synchronize()
    s = torch.cuda.Stream(dev)
    s.wait_stream(torch.cuda.current_stream(dev))
    with torch.cuda.stream(s):
        step()
    torch.cuda.current_stream(dev).wait_stream(s)
    graph = torch.cuda.CUDAGraph()
    with torch.cuda.graph(graph):
        static_out = step()
    return graph, static_out


def g_forward_flops(B, T, C=256):
    """Useful FLOPs of one G forward: 2*MACs of every conv/linear/bmm,
    encoder counted over live columns only."""
    f = 0

    def conv(co, ci, k, L):
        return 2 * co * ci * k * L
    # encoder, live columns (9..54, 5..26, 3..12, 4..11, 7)
    f += conv(64, 1, 16, T // 2 * 46) + conv(128, 64, 16, T // 4 * 22) + conv(256, 128, 16, T // 8 * 10)
    f += conv(512, 256, 9, T // 8 * 8) + conv(256, 512, 24, T // 8 * 1)

    def attn(c, t):
        return conv(c // 4 + c, c, 1, t) + 2 * t * t * (c // 8) + 2 * c * t * t
    f += conv(2 * C, C, 3, T) + conv(2 * C, 2 * C, 4, T // 2) + conv(4 * C, 2 * C, 3, T // 2)
    f += conv(4 * C, 4 * C, 4, T // 4) + conv(8 * C, 4 * C, 3, T // 4) + attn(8 * C, T // 4)
    f += conv(4 * C, 8 * C, 3, T // 4) + attn(8 * C, T // 2)   # convT 2048->1024 (Tin=T/4, 3 taps)
    f += conv(4 * C, 8 * C, 3, T // 2) + conv(2 * C, 4 * C, 3, T // 2) + conv(2 * C, 4 * C, 3, T)
    f += conv(C, 2 * C, 1, T)
    for J, post_ca in ((10, 0), (42, 1)):
        f += 2 * (2 * conv(C, C, 3, T) + attn(C, T)) + 2 * conv(C, C, 3, T) + 2 * attn(C, T)
        f += conv(J * 64, C, 1, T) * 2                              # proj_in + proj_out
        f += 3 * (J * T * 2 * 64 * 256) + 2 * (J * T * 2 * 64 * 128)  # 3 GAT + 2 GraphConv
    f += conv(104, C, 1, T)
    return f * B


def encoder_flops(B, T):
    """Useful FLOPs of the AudioEncoder over its live columns."""
    def conv(co, ci, k, L):
        return 2 * co * ci * k * L
    f = conv(64, 1, 16, T // 2 * 46) + conv(128, 64, 16, T // 4 * 22) + conv(256, 128, 16, T // 8 * 10)
    f += conv(512, 256, 9, T // 8 * 8) + conv(256, 512, 24, T // 8 * 1)
    return f * B


def run_graphed(dev, fn, iters=20, reps=5):
    """Average duration of fn() over `iters` launches captured in one HIP graph."""
    s = torch.cuda.Stream(dev)
    s.wait_stream(torch.cuda.current_stream(dev))
    with torch.cuda.stream(s):
        fn()
        g = torch.cuda.CUDAGraph()
        with torch.cuda.graph(g, stream=s):
            for _ in range(iters):
                fn()
        g.replay()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record(s)
        for _ in range(reps):
            g.replay()
        e1.record(s)
    e1.synchronize()
    return e0.elapsed_time(e1) / (iters * reps)


def mel_encoder_roofline(dev, g, wave, mel_ms, mel_bytes, peak):
    """north_star's mel + encoder path: the log-mel kernel (HBM-bound: wav in + mel out) and
    the AudioEncoder (MFMA-bound: live-column FLOPs; its minimum HBM traffic, mel in + features
    out + weights, is far below its FLOPs / ridge), each against its own roof, and the path as
    sum_k max(F_k / P_flop, B_k / P_bw) / measured time."""
    from a2m.mel_features import log_mel_batch
    mel = log_mel_batch(wave)
    B, T = mel.shape[0], mel.shape[1]
    with torch.no_grad():
        enc_ms = run_graphed(dev, lambda: g.audio_encoder(mel))
    ef = encoder_flops(B, T)
    wbytes = sum(p.numel() * 4 for p in g.audio_encoder.parameters())
    eb = mel.numel() * 4 + B * 256 * T * 4 + wbytes
    ideal_ms = mel_bytes / (HBM_PEAK_GBS * 1e9) * 1e3 + max(ef / (peak * 1e12), eb / (HBM_PEAK_GBS * 1e9)) * 1e3
    return {'mel_ms': round(mel_ms, 4), 'encoder_ms': round(enc_ms, 4),
            'encoder_achieved_tflops': round(ef / (enc_ms * 1e-3) / 1e12, 2), 'encoder_peak_tflops': peak,
            'encoder_frac': round(ef / (enc_ms * 1e-3) / 1e12 / peak, 4),
            'encoder_gflop': round(ef / 1e9, 2),
            'path_roofline_ms': round(ideal_ms, 4),
            'path_frac': round(ideal_ms / (mel_ms + enc_ms), 4)}


def gemm_engine_timing(step):
    """Run one eager step with every implicit-GEMM launch timed by its span stamps
    (a2m_gemm_timing_*): the engine's launches/step, algorithmic FLOPs (2*M*N*K) and summed
    tile-kernel / split-K-reduce time.  The generator's decoder branches run serialised for this
    pass, so no launch's duration includes a concurrent one's (`roofline.serialised_eager`: each
    launch alone on the chip)."""
    from a2m import functional as F
    from a2m import real_motion_model as RM
    torch.cuda.synchronize()
    branch, RM._BRANCH_STREAMS = RM._BRANCH_STREAMS, False
    try:
        with F.gemm_timing() as t:
            step()
            torch.cuda.synchronize()
    finally:
        RM._BRANCH_STREAMS = branch
    return t


def instep_timing(dev, g, wave, reps=20, warm=None, marks=(0,), gemm=True, enc_last=None):
    """The bench step captured once more with the engine's span stamps on (every implicit-GEMM
    launch stamps its own first-block start / last-wave end; nothing is added between kernels,
    so the two decoder branches overlap exactly as in the timed graph) and wall-clock mark
    kernels (step start, after the encoder); the graph is replayed
    `reps` times and each replay read back; `warm` (three replays of the timed bench graph) runs
    right before each of those replays, so that each timed replay follows back-to-back work as
    in the timed loop instead of an idle, clocked-down GPU after the previous read's sync.
    `marks` selects the mark kernels (0 before the log-mel, 1 after it, 2 after the encoder).
    The mel + encoder interval runs from mark 0 to the last block end of the encoder's final
    engine launch (record `enc_last`: conv4's tile kernel or its resample reduce, from the
    engine's own stamps), so no measurement kernel sits inside or after it; the in-step log-mel
    (0 -> 1) comes from a second capture (`gemm=False`: no engine stamps).
    Returns per-step means: the engine's launches /
    FLOPs / tile ms / reduce ms / queued ms (each launch from its ready mark -- a one-thread
    kernel the engine enqueues right before the tile kernel while timing -- to its last block
    end: its dispatch plus any wait for free CUs behind the other decoder branch, the extent a
    kernel trace gives a kernel), and the step's log-mel and log-mel + encoder phases (ms).
    This is the basis of `roofline` and of `mel_encoder_roofline.path_frac_instep`;
    tools/step_pmc.sh's rocprof kernel trace of the replayed bench graph is its cross-check
    (profiles/)."""
    import contextlib
    from a2m import functional as F
    from a2m.mel_features import log_mel_batch
    hook = (g.audio_encoder.register_forward_hook(lambda m, i, o: F.timing_mark(2))
            if 2 in marks else None)

    def step():
        F.timing_mark(0)
        mel = log_mel_batch(wave)
        if 1 in marks:
            F.timing_mark(1)
        return g(mel)[0]
    if not gemm:   # the mark buffer lives with the engine's stamp buffer: allocate it
        with F.gemm_timing():
            pass
    try:
        s = torch.cuda.Stream(dev)
        s.wait_stream(torch.cuda.current_stream(dev))
        with torch.cuda.stream(s):
            graph = torch.cuda.CUDAGraph()
            with (F.gemm_timing(keep=True) if gemm else contextlib.nullcontext()) as t:
                with torch.cuda.graph(graph, stream=s):
                    step()
        torch.cuda.current_stream(dev).wait_stream(s)
    finally:
        if hook is not None:
            hook.remove()
    acc = {'launches': 0, 'reduces': 0, 'flops': 0.0, 'ms_tile': 0.0, 'ms_reduce': 0.0, 'ms_queued': 0.0,
           'mel_ms': 0.0, 'mel_enc_ms': 0.0}
    try:
        graph.replay()
        torch.cuda.synchronize()
        if gemm:
            t.read()                 # discard the warm-up replay's stamps (re-arms them)
        for _ in range(reps):
            if warm is not None:
                warm()
            graph.replay()
            torch.cuda.synchronize()
            if gemm and enc_last is not None and 2 not in marks:
                # before t.read() re-arms the stamps
                acc['mel_enc_ms'] += F.timing_mark_to_launch_end(0, enc_last)
            if gemm:
                t.read()
                acc['launches'] += t.launches
                acc['reduces'] += t.reduces
                acc['flops'] += t.flops
                acc['ms_tile'] += t.ms_tile
                acc['ms_reduce'] += t.ms_reduce
                acc['ms_queued'] += t.ms_queued
            if 1 in marks:
                acc['mel_ms'] += F.timing_mark_elapsed(0, 1)
            if 2 in marks:
                acc['mel_enc_ms'] += F.timing_mark_elapsed(0, 2)

    finally:
        if gemm:
            t.release()
        del graph
    out = {k: v / reps for k, v in acc.items()}
    out['launches'] = int(round(out['launches']))
    out['reduces'] = int(round(out['reduces']))
    return out


def dispatch_overhead_ms(dev, n=48, reps=10):
    """Per-launch dispatch overhead that a kernel trace attributes to each kernel beyond its own
    execution span: a graph of n back-to-back one-block engine launches on one stream is
    replayed; the median gap from one launch's last block end to the next launch's first block
    start (span stamps) is what rocprof's back-to-back begin/end timestamps add to every kernel.
    `roofline.frac` charges it to each engine launch, so the line is comparable with the
    committed rocprof trace; `frac_execution` is the stamps alone."""
    from a2m import functional as F
    x = torch.randn(32, 32, device=dev)
    w = torch.randn(32, 32, device=dev)
    y = torch.empty(32, 32, device=dev)
    F.linear(x, w, out=y)
    torch.cuda.synchronize()
    s = torch.cuda.Stream(dev)
    s.wait_stream(torch.cuda.current_stream(dev))
    gaps = []
    with torch.cuda.stream(s):
        graph = torch.cuda.CUDAGraph()
        with F.gemm_timing(keep=True) as t:
            with torch.cuda.graph(graph, stream=s):
                for _ in range(n):
                    F.linear(x, w, out=y)
        try:
            graph.replay()
            t.spans()
            for _ in range(reps):
                graph.replay()
                sp = t.spans()
                gaps += [sp[i + 1][0] - sp[i][1] for i in range(len(sp) - 1)]
        finally:
            t.release()
    torch.cuda.current_stream(dev).wait_stream(s)
    gaps.sort()
    return gaps[len(gaps) // 2] / 1e3


def load_traffic(name):
    """HBM bytes per launch for a kernel family, from the committed PMC pass
    (tools/pmc_traffic.py -> profiles/traffic_latest.json), or None."""
    path = os.path.join(REPO, 'profiles', 'traffic_latest.json')
    try:
        with open(path) as f:
            return json.load(f).get(name)
    except (OSError, ValueError):
        return None


def run_mel_kernel(dev, wave, iters=50):
    """Average log-mel kernel duration: `iters` launches captured in one HIP graph (so host
    launch overhead is not in the number), replayed 5 times, timed with events on the replay
    stream."""
    from a2m.mel_features import log_mel_batch
    out = log_mel_batch(wave)
    s = torch.cuda.Stream(dev)
    s.wait_stream(torch.cuda.current_stream(dev))
    with torch.cuda.stream(s):
        log_mel_batch(wave, out=out)
        g = torch.cuda.CUDAGraph()
        with torch.cuda.graph(g, stream=s):
            for _ in range(iters):
                log_mel_batch(wave, out=out)
        g.replay()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        reps = 5
        e0.record(s)
        for _ in range(reps):
            g.replay()
        e1.record(s)
    e1.synchronize()
    ms = e0.elapsed_time(e1) / (iters * reps)
    nbytes = wave.numel() * 4 + out.numel() * 4       # algorithmic: wav in + mel out
    return ms, nbytes


def cgroup_cpus():
    """CPUs this job is granted by its cgroup's CPU quota (cgroup v2 cpu.max "quota period", or
    v1 cfs_quota_us / cfs_period_us), as (cpus or None, the raw quota string)."""
    for path in ('/sys/fs/cgroup/cpu.max',):
        try:
            with open(path) as f:
                raw = f.read().strip()
            q, per = raw.split()[:2]
            return (None if q == 'max' else max(1, -(-int(q) // int(per)))), f'{path}: {raw}'
        except (OSError, ValueError):
            pass
    try:
        with open('/sys/fs/cgroup/cpu/cpu.cfs_quota_us') as f:
            q = int(f.read())
        with open('/sys/fs/cgroup/cpu/cpu.cfs_period_us') as f:
            per = int(f.read())
        return (None if q <= 0 else max(1, -(-q // per))), f'cfs_quota_us {q} / cfs_period_us {per}'
    except (OSError, ValueError):
        return None, 'no cgroup CPU quota found'


def host_cpu():
    """CPU model, physical cores, CPUs in the affinity mask, and the cgroup-granted CPUs."""
    model = 'unknown'
    try:
        with open('/proc/cpuinfo') as f:
            for line in f:
                if line.startswith('model name'):
                    model = line.split(':', 1)[1].strip()
                    break
    except OSError:
        pass
    try:
        import psutil
        phys = psutil.cpu_count(logical=False)
    except Exception:
        phys = None
    try:
        avail = len(os.sched_getaffinity(0))
    except AttributeError:
        avail = os.cpu_count()
    granted, quota = cgroup_cpus()
    return model, phys, avail, granted, quota


def cpu_baseline(B=64, T=64, max_s=40.0):
    """torch-CPU fp32 oracle port (numpy float64 mel + functional G) on the bench's own
    workload shape (B clips x T frames), timed on this host's cores (all the
    cores the job may use -- the affinity mask capped by the cgroup CPU quota): two warm-up
    runs, then the median of up to 5 runs within max_s."""
    sys.path.insert(0, REPO)
    import numpy as np
    from oracle import mel as omel, model as omodel, synth, weights
    from a2m.real_motion_model import SelfAttention_G
    model_name, phys, avail, granted, quota = host_cpu()
    threads = min(avail, granted) if granted else avail
    prev_threads = torch.get_num_threads()
    torch.set_num_threads(threads)
    shapes = {k: tuple(v.shape) for k, v in SelfAttention_G(p=0.0).state_dict().items()}
    sd = weights.make_state_dict(shapes, seed=7)
    wav = synth.speech_like(B, synth.samples_for_frames(T), seed=1)

    def step():
        mel = np.stack([omel.log_mel(w, **omel.BUILD_CFG) for w in wav]).astype(np.float32)
        with torch.no_grad():
            omodel.generator(sd, torch.from_numpy(mel))
    try:
        for _ in range(2):
            step()
        times, t_all = [], time.perf_counter()
        while len(times) < 5 and time.perf_counter() - t_all < max_s:
            t0 = time.perf_counter()
            step()
            times.append(time.perf_counter() - t0)
    finally:
        torch.set_num_threads(prev_threads)
    med = sorted(times)[len(times) // 2]
    return {'value': round(B * T / med, 1), 'unit': 'pose-frames/s', 'cores': threads, 'kind': 'port',
            'cpu_model': model_name, 'host_physical_cores': phys, 'host_cpus_available': avail,
            'cgroup_cpus': granted, 'cgroup_quota': quota,
            'sample': f'{B} clips x {T} frames, the bench workload (numpy fp64 log-mel + torch-CPU fp32 '
                      f'G forward), 2 warm-up runs, median of {len(times)} runs, {threads} torch threads '
                      f'(affinity {avail} CPUs, cgroup quota {granted or "none"})'}


# dense FLOPs of one training iteration at T=64 measured with torch's
# FlopCounter on the reference modules: 3 G-steps x 891.7 GF + 1 D-step x 382.8 GF per 64 clips.
TRAIN_GFLOP_PER_CLIP_T64 = (3 * 891.7 + 382.8) / 64


def run_train(args, world, rank, dev):
    """configs[2]: one version5_model_train.py iteration (3 G-steps + 1 D-step, Adam) over a
    global batch split across ranks (strong scaling), DP gradient all-reduce over RCCL."""
    from a2m.real_motion_model import SelfAttention_D, SelfAttention_G
    from a2m.training import GANTrainer
    Bg, T = args.batch, args.frames
    assert Bg % world == 0, 'global batch must divide by the number of GPUs'
    B = Bg // world
    torch.manual_seed(1234)                           # identical initial weights on every rank
    g = SelfAttention_G(time_steps=T, p=0.2).to(dev).train()
    d = SelfAttention_D(out_channels=64).to(dev).train()
    graphs = not args.no_graph and (world == 1 or dist.get_backend() == 'nccl')
    tr = GANTrainer(g, d, lr=10e-4, sync_bn=args.sync_bn, bucket_mb=args.bucket_mb, label_seed=7,
                    grad_reduce_dtype=torch.bfloat16 if args.dtype == 'bf16' else None, graphs=graphs)
    gen = torch.Generator(device='cpu').manual_seed(100 + rank)
    audio = torch.randn(B, T, 128, generator=gen).to(dev)
    pose = torch.randn(B, T, 104, generator=gen).to(dev)

    def step(epoch):
        tr.iteration(audio, pose, epoch=epoch, g_freq=3, d_freq=1)

    for i in range(args.warmup):
        step(i)
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for i in range(args.steps):
        step(args.warmup + i)
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    elapsed = time.perf_counter() - t0
    if world > 1:
        t = torch.tensor([elapsed], device=dev, dtype=torch.float64)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        elapsed = t.item()
    tr.flush()   # the ranks agree that every step's gradients followed the bucket plan
    ms = elapsed / args.steps * 1e3
    flops = TRAIN_GFLOP_PER_CLIP_T64 * 1e9 * B * T / 64           # per rank
    tf = flops * world / (ms * 1e-3) / 1e12
    peak = mfma_peak(args.dtype)
    cfg = ('configs[2]' if args.dtype == 'fp32' else
           'configs[4] (bf16 GEMM operands, fp32 master weights / accumulation)')
    result = {
        'metric': 'pose-frames/sec (whole node), PATS 64-frame clips batch 64, training iteration',
        'value': round(Bg * T / (ms * 1e-3), 1), 'unit': 'pose-frames/s', 'n_gpus': world,
        'steps': args.steps, 'warmup': args.warmup, 'ms_per_step': round(ms, 3), 'higher_is_better': True,
        'scaling': 'strong', 'vs_baseline': None, 'dtype': dtype_label(args.dtype),
        'data': 'synthetic mel/pose tensors, random-init weights',
        'config': {'workload': cfg + ': version5_model_train.py iteration (G x3 + D x1, Adam, '
                               'smoothed noisy labels), DP over ranks',
                   'batchnorm': 'sync' if tr.sync_bn else 'per-rank statistics',
                   'hip_graph': ('G-step and D-step bodies captured, replayed per step' if graphs else 'none'),
                   'grad_allreduce': (f'{len(tr.red_G.buckets)} G / {len(tr.red_D.buckets)} D buckets '
                                      f'(each closed once >= {args.bucket_mb:g} MB), overlapped with backward, '
                                      f'{"bf16" if args.dtype == "bf16" else "fp32"} on the wire'),
                   'global_batch': Bg, 'seq_len': T, 'parallelism': f'dp{world}'},
        'path_roofline': {'bound': 'mfma', 'achieved': round(tf, 2), 'peak': peak,
                          'unit': 'TFLOP/s', 'frac': round(tf / peak / world, 4),
                          'gflop_per_iteration': round(flops * world / 1e9, 1),
                          'flop_source': 'SURVEY.md 8(d) FlopCounter count, dense'},
    }
    if args.rehearsal:
        result['rehearsal'] = args.rehearsal
    if rank == 0:
        print(json.dumps(result), flush=True)
    if world > 1:
        dist.destroy_process_group()


def dtype_label(dtype):
    """Arithmetic type of the GEMMs: f32; bf16 (bf16 operands, f32 accumulation)."""
    return {'fp32': 'f32', 'bf16': 'bf16'}[dtype]


def mfma_peak(dtype):
    return {'fp32': FP32_MFMA_PEAK_TFLOPS, 'bf16': BF16_MFMA_PEAK_TFLOPS}[dtype]


def roofline_entry(it, gt, peak=None, dispatch_ms=0.0, tr=None):
    """`roofline` for the dominant family, the implicit-GEMM engine: every tile-kernel launch
    (gemm_kernel / gemm_pipe_kernel / gemm_pipe_bf16_kernel) AND every split-K reduce of one step.  `achieved` =
    algorithmic FLOPs per step (2*M*N*K summed over the step's engine launches) / the family's
    summed kernel-trace durations per step (`traced_family`: rocprofv3 --kernel-trace of the
    replayed bench graph, the figure a kernel-trace breakdown gives); without a trace, the span
    stamps plus the measured per-launch dispatch overhead.  `frac_execution`: the stamps alone
    (first block start .. last block end over all XCDs, tile kernels + reduces)."""
    peak = peak or FP32_MFMA_PEAK_TFLOPS
    n_tile = max(it['launches'], 1)
    n_all = n_tile + it.get('reduces', 0)
    ms_exec = it['ms_tile'] + it['ms_reduce']
    ms_disp = ms_exec + n_all * dispatch_ms
    tf_exec = it['flops'] / (ms_exec * 1e-3) / 1e12
    tf_disp = it['flops'] / (ms_disp * 1e-3) / 1e12
    tf_ser = gt.flops / ((gt.ms_tile + gt.ms_reduce) * 1e-3) / 1e12
    traffic = load_traffic('gemm_engine') if peak == FP32_MFMA_PEAK_TFLOPS else None
    if tr:
        ms_fam = tr['family_us'] / 1e3
        tf = it['flops'] / (ms_fam * 1e-3) / 1e12
        basis = (f'kernel trace: rocprofv3 --kernel-trace of the replayed bench graph ({tr["reps"]} replays '
                 f'after a marker kernel, each followed by a device sync; bench.py --trace-child), the summed '
                 f'durations of every engine tile kernel and split-K reduce per step; FLOPs = 2*M*N*K over the '
                 f'step\'s engine launches')
    else:
        ms_fam = ms_disp
        tf = tf_disp
        basis = ('span stamps (no kernel trace available): first block start .. last block end of every engine '
                 'tile kernel and split-K reduce in the replayed step graph, plus the measured per-launch '
                 'dispatch overhead')
    return {'bound': 'mfma',
            'kernel': 'implicit-GEMM engine family (gemm_kernel, gemm_pipe_kernel, gemm_pipe_bf16_kernel, splitk_reduce*): every launch of one step',
            'achieved': round(tf, 2), 'peak': peak, 'unit': 'TFLOP/s',
            'frac': round(tf / peak, 4),
            'traffic': traffic['bytes_per_launch'] if traffic else None,
            'traffic_unit': 'HBM bytes per engine tile launch (the family\'s bytes per step / its tile launches)',
            'traffic_bytes_per_step': traffic.get('bytes_per_step') if traffic else None,
            'traffic_over_dense_operands': traffic.get('traffic_over_dense') if traffic else None,
            'traffic_source': traffic['source'] if traffic else None,
            'basis': basis,
            'family_ms_per_step': round(ms_fam, 4),
            'launches_per_step': it['launches'], 'reduces_per_step': it.get('reduces', 0),
            'gflop_per_step': round(it['flops'] / 1e9, 2),
            'trace_launches_per_step': round(tr['launches'], 1) if tr else None,
            'trace_reduce_ms_per_step': round(tr['reduce_us'] / 1e3, 4) if tr else None,
            'frac_execution': round(tf_exec / peak, 4),
            'frac_stamps_dispatch': round(tf_disp / peak, 4),
            'dispatch_ms_per_launch': round(dispatch_ms, 4),
            'stamps_ms_tile_per_step': round(it['ms_tile'], 4),
            'stamps_ms_reduce_per_step': round(it['ms_reduce'], 4),
            'serialised_eager': {'achieved': round(tf_ser, 2), 'frac': round(tf_ser / peak, 4),
                                 'ms_per_step': round(gt.ms_tile + gt.ms_reduce, 4)}}


GEMM_FAMILY = ('gemm_kernel', 'gemm_pipe_kernel', 'gemm_pipe_bf16_kernel', 'splitk_reduce')   # the engine's kernels


def under_profiler():
    """True when this process already runs under rocprofv3 (its preload library and ROCPROF_*
    settings are inherited): a nested traced child would stack a second profiler, so the line
    then keeps the span-stamp basis (roofline.basis says which)."""
    pre = os.environ.get('LD_PRELOAD', '')
    return 'librocprofiler-sdk-tool' in pre or 'ROCPROF_OUTPUT_PATH' in os.environ


def trace_child(args):
    """`--trace-child R` (run by traced_family under rocprofv3 --kernel-trace): the bench step
    exactly as the timed run builds it (rank 0's seeds), captured in one graph, one replay, a
    marker kernel (torch.cuda._sleep), then R replays each followed by a device sync (free-running
    replays run ~11 % slower under the kernel trace than unprofiled: DESIGN.md 6)."""
    dev = torch.device('cuda', 0)
    torch.cuda.set_device(dev)
    import a2m
    a2m.set_gemm_precision(args.dtype)
    g, wave = build_infer(args.batch, args.frames, 0, dev)
    with torch.no_grad():
        graph, _ = capture_step(dev, infer_step(g, wave))
        graph.replay()
        torch.cuda.synchronize()
        torch.cuda._sleep(1000)          # the marker dispatch: everything after it is a replayed step
        torch.cuda.synchronize()
        for _ in range(args.trace_child):
            graph.replay()
            torch.cuda.synchronize()


def _is_marker(name):
    n = name.lower()
    return ('sleep' in n or 'spin_kernel' in n) and 'a2m' not in n


def traced_family(args, flops_per_step, reps=10, keep_dir=None):
    """rocprofv3 --kernel-trace of the replayed bench step (a child process running
    `bench.py --trace-child`): per step, the summed durations of the engine's kernel family --
    tile kernels AND split-K reduces -- the figure `roofline.frac` is computed from, plus the
    trace's log-mel start .. encoder end interval and a per-kernel breakdown.  The trace CSV and
    breakdown are kept in keep_dir (A2M_BENCH_TRACE_DIR) when given.  None if rocprofv3 is
    unavailable or the child fails."""
    import csv
    import glob
    import shutil
    import subprocess
    import tempfile
    prof = shutil.which('rocprofv3')
    if prof is None:
        return None
    tmp = tempfile.mkdtemp(prefix='a2m_trace_')
    cmd = [prof, '--kernel-trace', '--output-format', 'csv', '-d', tmp, '-o', 'run', '--',
           sys.executable, os.path.abspath(__file__), '--trace-child', str(reps), '--batch', str(args.batch),
           '--frames', str(args.frames), '--dtype', args.dtype]
    env = dict(os.environ, TMPDIR=os.environ.get('TMPDIR', '/tmp'))
    env.pop('WORLD_SIZE', None)
    try:
        r = subprocess.run(cmd, stdout=subprocess.PIPE, stderr=subprocess.STDOUT, timeout=240, env=env)
        files = glob.glob(os.path.join(tmp, '**', '*kernel_trace.csv'), recursive=True)
        if r.returncode != 0 or not files:
            sys.stderr.write(f'bench.py: kernel-trace child failed (rc {r.returncode})\n' +
                             r.stdout.decode(errors='replace')[-2000:])
            return None
        rows = []
        for fn in files:
            with open(fn, newline='') as f:
                rows.extend(csv.DictReader(f))
        did = lambda row: int(row.get('Dispatch_Id') or row.get('Correlation_Id'))  # noqa: E731
        marks = [did(x) for x in rows if _is_marker(x.get('Kernel_Name', ''))]
        if not marks:
            return None
        rows = sorted((x for x in rows if did(x) > max(marks)), key=lambda x: int(x['Start_Timestamp']))
        dur = lambda x: (int(x['End_Timestamp']) - int(x['Start_Timestamp'])) / 1e3  # noqa: E731  us
        name = lambda x: x['Kernel_Name'].split('(')[0].replace('void ', '')  # noqa: E731
        fam = [x for x in rows if any(k in name(x) for k in GEMM_FAMILY)]
        fam_us = sum(dur(x) for x in fam) / reps
        red_us = sum(dur(x) for x in fam if 'splitk_reduce' in name(x)) / reps
        # per step: the log-mel's start .. the end of the encoder's last engine launch (its fused
        # resample reduce) -- north_star's mel + encoder path in the step
        starts = [i for i, x in enumerate(rows) if 'logmel' in name(x)]
        mel_enc = []
        for i in starts:
            j = next((k for k in range(i, len(rows)) if 'splitk_reduce_interp' in name(rows[k])), None)
            if j is not None:
                mel_enc.append((int(rows[j]['End_Timestamp']) - int(rows[i]['Start_Timestamp'])) / 1e3)
        agg = {}
        for x in rows:
            a = agg.setdefault(name(x)[:90], [0, 0.0])
            a[0] += 1
            a[1] += dur(x)
        tot = sum(v[1] for v in agg.values()) / reps
        lines = [f'{len(rows)} dispatches after the marker = {reps} replayed steps (device sync after each); '
                 f'kernel-time sum {tot:.1f} us/step',
                 f'engine family (gemm_kernel + gemm_pipe_kernel / gemm_pipe_bf16_kernel + splitk_reduce*): {len(fam) / reps:.1f} launches/step, '
                 f'{fam_us:.1f} us/step ({red_us:.1f} us of split-K reduces)',
                 f'engine roofline: {flops_per_step / 1e9:.1f} GFLOP / {fam_us:.1f} us = '
                 f'{flops_per_step / (fam_us * 1e-6) / 1e12:.1f} TF']
        for k, (c, t) in sorted(agg.items(), key=lambda kv: -kv[1][1]):
            lines.append(f'{t / reps:9.1f} us/step {c / reps:6.1f} calls/step {t / c:8.1f} us/call  {k}')
        if keep_dir:
            os.makedirs(keep_dir, exist_ok=True)
            shutil.copy(files[0], os.path.join(keep_dir, 'step_trace_replayed_kernel_trace.csv'))
            with open(os.path.join(keep_dir, 'step_breakdown.txt'), 'w') as f:
                f.write('\n'.join(lines) + '\n')
        return {'family_us': fam_us, 'reduce_us': red_us, 'launches': len(fam) / reps, 'reps': reps,
                'mel_enc_us': sorted(mel_enc)[len(mel_enc) // 2] if mel_enc else None}
    except (OSError, subprocess.SubprocessError, ValueError, KeyError) as e:
        sys.stderr.write(f'bench.py: kernel-trace child failed: {e}\n')
        return None
    finally:
        shutil.rmtree(tmp, ignore_errors=True)


def build_infer(B, T, rank, dev):
    """The bench's generator (random init, attention gammas 0.3, eval) and synthetic waves."""
    from a2m.real_motion_model import SelfAttention_G
    n = (T - 1) * HOP + WIN
    torch.manual_seed(1234 + rank)
    g = SelfAttention_G(time_steps=T, p=0.2)
    for m in g.modules():
        if hasattr(m, 'gamma'):
            torch.nn.init.constant_(m.gamma, 0.3)
    g = g.to(dev).eval()
    return g, synth_wave(B, n, seed=rank, device=dev)



def spawn_ranks(n):
    """`bench.py --gpus N` without a launcher: start N ranks as fresh child processes of
    torch.distributed.run (one per GPU, rendezvous on 127.0.0.1) before anything touches the
    GPU, and exit with their status."""
    import socket
    import subprocess
    with socket.socket() as sk:
        sk.bind(('127.0.0.1', 0))
        port = sk.getsockname()[1]
    cmd = [sys.executable, '-m', 'torch.distributed.run', '--nnodes=1', f'--nproc-per-node={n}',
           '--master-addr', '127.0.0.1', f'--master-port={port}', os.path.abspath(__file__)] + sys.argv[1:]
    sys.exit(subprocess.call(cmd))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument('--gpus', type=int, default=1)
    # defaults: 200 timed steps after 20 warm-up steps for inference (a ~2.9 ms step: 20 steps
    # left the mean at the mercy of clock ramp-up and queue jitter), 20 / 5 for training
    ap.add_argument('--steps', type=int, default=None)
    ap.add_argument('--warmup', type=int, default=None)
    ap.add_argument('--batch', type=int, default=64)
    ap.add_argument('--frames', type=int, default=64)
    ap.add_argument('--no-graph', action='store_true')
    ap.add_argument('--branch-graphs', action='store_true',
                    help='replay a2m.inference.GraphedGenerator (one graph per decoder branch, '
                         'two streams) instead of one graph with the branches forked inside')
    ap.add_argument('--no-cpu-baseline', action='store_true')
    ap.add_argument('--mode', choices=('infer', 'train'), default='infer')
    ap.add_argument('--sync-bn', action='store_true',
                    help='train mode: SyncBN over the DP ranks (SURVEY 8(e)); default per-rank statistics')
    ap.add_argument('--bucket-mb', type=float, default=25.0,
                    help='train mode: gradient all-reduce bucket size (MB)')
    ap.add_argument('--dtype', choices=('fp32', 'bf16'), default='fp32',
                    help='GEMM operand precision (bf16: configs[4], fp32 accumulation/storage)')
    ap.add_argument('--trace-child', type=int, default=0, help=argparse.SUPPRESS)
    ap.add_argument('--no-trace', action='store_true',
                    help='skip the kernel-trace pass (roofline from the span stamps only)')
    args = ap.parse_args()
    if args.trace_child:
        return trace_child(args)
    if args.steps is None:
        args.steps = 200 if args.mode == 'infer' else 20
    if args.warmup is None:
        args.warmup = 20 if args.mode == 'infer' else 5

    if 'WORLD_SIZE' not in os.environ and args.gpus > 1:
        return spawn_ranks(args.gpus)
    world = int(os.environ.get('WORLD_SIZE', '1'))
    if world != args.gpus:
        sys.exit(f'bench.py: --gpus {args.gpus} but WORLD_SIZE={world}; launch one rank per GPU')
    rank = int(os.environ.get('RANK', '0'))
    local = int(os.environ.get('LOCAL_RANK', '0'))
    # A2M_BENCH_BACKEND=gloo rehearses the N>1 path (barriers, max-over-ranks timing, the DP
    # all-reduce) with several ranks sharing the GPUs of a smaller box; RCCL is the default
    backend = os.environ.get('A2M_BENCH_BACKEND', 'nccl')
    args.rehearsal = None if backend == 'nccl' else (
        f'{backend} rehearsal: {world} ranks share {torch.cuda.device_count()} GPU(s); '
        f'not an N-GPU throughput')
    if backend != 'nccl':
        local = local % torch.cuda.device_count()
    if world > 1:
        if backend == 'nccl':
            dist.init_process_group('nccl', device_id=torch.device('cuda', local))
        else:
            dist.init_process_group(backend)
    dev = torch.device('cuda', local)
    torch.cuda.set_device(dev)
    import a2m
    a2m.set_gemm_precision(args.dtype)
    if args.mode == 'train':
        return run_train(args, world, rank, dev)

    B, T = args.batch, args.frames
    g, wave = build_infer(B, T, rank, dev)

    step = infer_step(g, wave)
    with torch.no_grad():
        graph, static_out = None, None
        if args.no_graph:
            run = step
        elif args.branch_graphs:
            from a2m.inference import GraphedGenerator
            from a2m.mel_features import log_mel_batch
            graph = GraphedGenerator(g, lambda: log_mel_batch(wave))
            static_out = graph.static['out']
            run = graph
        else:
            graph, static_out = capture_step(dev, step)
            run = graph.replay
        for _ in range(args.warmup):
            run()
        torch.cuda.synchronize()
        if world > 1:
            dist.barrier()
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for _ in range(args.steps):
            run()
        torch.cuda.synchronize()
        if world > 1:
            dist.barrier()
        elapsed = time.perf_counter() - t0
        if world > 1:
            t = torch.tensor([elapsed], device=dev, dtype=torch.float64)
            dist.all_reduce(t, op=dist.ReduceOp.MAX)
            elapsed = t.item()
        out = static_out if graph is not None else step()
        assert torch.isfinite(out).all()

        ms_step = elapsed / args.steps * 1e3
        value = world * B * T / (elapsed / args.steps)
        gt = gemm_engine_timing(step)
        warm = None if graph is None else (lambda: [run() for _ in range(3)])
        from a2m import functional as AF
        from a2m.mel_features import log_mel_batch
        with AF.gemm_timing() as et:   # the encoder's engine launches come first in the step
            g.audio_encoder(log_mel_batch(wave))
        it = instep_timing(dev, g, wave, warm=warm, enc_last=et.launches - 1)
        it['mel_ms'] = instep_timing(dev, g, wave, warm=warm, marks=(0, 1), gemm=False)['mel_ms']
        disp_ms = dispatch_overhead_ms(dev)
        mel_ms, mel_bytes = run_mel_kernel(dev, wave)
        mel_enc = mel_encoder_roofline(dev, g, wave, mel_ms, mel_bytes, mfma_peak(args.dtype))
        mel_enc['instep_mel_ms'] = round(it['mel_ms'], 4)
        mel_enc['instep_mel_encoder_ms'] = round(it['mel_enc_ms'], 4)
        mel_enc['path_frac_instep'] = round(mel_enc['path_roofline_ms'] / it['mel_enc_ms'], 4)
        tr = None
        if world == 1 and not args.no_trace and graph is not None and not args.branch_graphs and \
                not under_profiler():
            tr = traced_family(args, it['flops'], keep_dir=os.environ.get('A2M_BENCH_TRACE_DIR'))
        if tr and tr['mel_enc_us']:
            mel_enc['instep_mel_encoder_ms_trace'] = round(tr['mel_enc_us'] / 1e3, 4)
            mel_enc['path_frac_instep_trace'] = round(mel_enc['path_roofline_ms'] / (tr['mel_enc_us'] / 1e3), 4)
    path_tf = g_forward_flops(B, T) / (ms_step * 1e-3) / 1e12
    peak = mfma_peak(args.dtype)
    if args.dtype == 'bf16':
        workload = (f'configs[4] (bf16 GEMM operands, fp32 accumulation): log-mel + SelfAttention_G '
                    f'forward (eval), batch-{B} x {T}-frame clips per GPU, replicas only')
    elif T != 64:
        workload = (f'configs[3] long-form: log-mel + SelfAttention_G forward (eval), batch-{B} x '
                    f'{T}-frame ({(T - 1) * HOP + WIN} samples) clips per GPU, replicas only')
    else:
        workload = (f'configs[1]: log-mel + SelfAttention_G forward (eval), batch-{B} x {T}-frame '
                    f'clips per GPU, replicas only')
    result = {
        'metric': 'pose-frames/sec (whole node), PATS 64-frame clips batch 64, 1/2/4/8 MI355X',
        'value': round(value, 1), 'unit': 'pose-frames/s', 'n_gpus': world, 'steps': args.steps,
        'warmup': args.warmup, 'ms_per_step': round(ms_step, 4), 'higher_is_better': True,
        'scaling': 'weak', 'vs_baseline': None, 'dtype': dtype_label(args.dtype),
        'data': 'synthetic 16 kHz speech-like audio, random-init weights',
        'config': {'workload': workload, 'global_batch': B * world, 'seq_len': T,
                   'parallelism': f'replicas{world}', 'hip_graph': 'none' if graph is None else ('per-branch graphs, two streams' if args.branch_graphs else 'one graph')},
        'roofline': roofline_entry(it, gt, peak, disp_ms, tr),
        'mel_roofline': {'bound': 'hbm', 'achieved': round(mel_bytes / (mel_ms * 1e-3) / 1e9, 1),
                         'peak': HBM_PEAK_GBS, 'unit': 'GB/s',
                         'frac': round(mel_bytes / (mel_ms * 1e-3) / 1e9 / HBM_PEAK_GBS, 4),
                         'ms_per_launch': round(mel_ms, 4),
                         'algorithmic_bytes': int(mel_bytes),
                         'traffic': (load_traffic('logmel2048_kernel') or {}).get('bytes_per_launch')
                         if (B, T) == (64, 64) else None,
                         'note': 'VALU-issue bound (DESIGN.md 4): ~732 VALU instructions per frame-wave'},
        'mel_encoder_roofline': mel_enc,
        'path_roofline': {'bound': 'mfma', 'achieved': round(path_tf, 2), 'peak': peak,
                          'unit': 'TFLOP/s', 'frac': round(path_tf / peak, 4),
                          'gflop_per_step': round(g_forward_flops(B, T) / 1e9, 1)},
    }
    if rank == 0 and world == 1 and not args.no_cpu_baseline:
        result['cpu_baseline'] = cpu_baseline()
    if args.rehearsal:
        result['rehearsal'] = args.rehearsal
    if rank == 0:
        print(json.dumps(result), flush=True)
    if world > 1:
        dist.destroy_process_group()


if __name__ == '__main__':
    main()
