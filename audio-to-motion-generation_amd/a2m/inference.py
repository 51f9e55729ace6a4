"""Inference surface of generate_motion_video.py, on the device.

  load_generator(path)      :237-238  construct + load_state_dict (weights_only) + eval
  generate(g, audio, ...)   :247-260  generator(audio) on normalised audio features, then the
                                      normalised poses mapped back: pose * std + mean
  planar_frames(pose)       :262-266  [B, T, 104] -> [B, T, 2, 52] (x row, y row) for plotting

  GraphedGenerator(g, ...)  HIP-graph replay of a fixed-shape eval forward (the serving loop
                            of :247-260 at a fixed batch): one graph per decoder branch, the
                            two branches on two streams joined by events

Plotting and ffmpeg (:23-207) stay host-side reference code (out of scope).
"""
import torch

from . import functional as F
from .normalization import denormalize
from .real_motion_model import SelfAttention_G


def load_generator(path, device='cuda', **kwargs):
    g = SelfAttention_G(**kwargs)
    g.load_state_dict(torch.load(path, map_location='cpu', weights_only=True))
    return g.to(device).eval()


@torch.no_grad()
def generate(generator, audio, pose_mean=None, pose_std=None):
    """audio [B, T, 128] (device) -> poses [B, T, 104]; de-normalised when mean/std are given."""
    pose, _ = generator(audio)
    if pose_mean is not None:
        pose = denormalize(pose, pose_mean.to(pose.device), pose_std.to(pose.device))
    return pose


def planar_frames(pose):
    B, T, _ = pose.shape
    return pose.reshape(B, T, 2, -1)


class GraphedGenerator:
    """Fixed-shape eval forward of SelfAttention_G as four HIP graphs replayed on two streams:

        trunk  (main):  prologue() -> audio encoder -> UNet -> feats
        body   (side):  body decoder branch -> out[..., :20]      } concurrent after the fork
        hand   (main):  hand decoder branch -> out[..., 20:]      }
        losses (main):  after the join, pose losses of out

    One graph with both branches inside leaves the second branch waiting: on ROCm 7 its
    first kernel started 350-500 us after the fork in every replay we traced (r02 step
    trace).  Separate single-stream graphs start both branches at the fork (traced), but at
    B = 64 the branches' kernels already fill the chip, so the bench step measured no faster
    (3.19 vs 3.14 ms; bench.py --branch-graphs): kept as the serving-loop API, not the bench
    default.

    `prologue` produces the [B, T, 128] generator input from static device buffers (e.g. the
    bench's HIP log-mel over resident waveforms); call() replays and returns the static
    [B, T, 104] output and the losses list (valid until the next call)."""

    def __init__(self, generator, prologue):
        g = generator
        assert not g.training, 'GraphedGenerator replays the eval forward'
        self.g, self.prologue = g, prologue
        dev = next(g.parameters()).device
        self.main = torch.cuda.Stream(dev)
        self.side = torch.cuda.Stream(dev)
        self.fork, self.join = torch.cuda.Event(), torch.cuda.Event()
        self.static = {}
        with torch.no_grad():
            # warm-up: every workspace / cache is created on the stream that will replay it
            for _ in range(2):
                self._trunk()
                self._branches(eager=True)
                self._losses()
            torch.cuda.synchronize(dev)
            # the main-stream graphs share one pool (they replay in capture order on one
            # stream); the body graph runs concurrently with the hand graph, so its
            # temporaries must not alias theirs: a pool of its own
            pool, side_pool = torch.cuda.graph_pool_handle(), torch.cuda.graph_pool_handle()
            self.graphs = {}
            for name, stream, fn, pl in (('trunk', self.main, self._trunk, pool),
                                         ('body', self.side, lambda: self._branch('body'), side_pool),
                                         ('hand', self.main, lambda: self._branch('hand'), pool),
                                         ('losses', self.main, self._losses, pool)):
                gr = torch.cuda.CUDAGraph()
                with torch.cuda.graph(gr, pool=pl, stream=stream):
                    fn()
                self.graphs[name] = gr
        torch.cuda.synchronize(dev)

    def _trunk(self):
        with torch.cuda.stream(self.main):
            x = self.prologue()
            B, T, _ = x.shape
            self.static['feats'] = self.g.unet(self.g.audio_encoder(x))
            if 'out' not in self.static:
                self.static['out'] = torch.empty(B, T, self.g.body_feats + self.g.hand_feats,
                                                 device=x.device)

    def _branch(self, part):
        stream = self.side if part == 'body' else self.main
        with torch.cuda.stream(stream):
            f0 = 0 if part == 'body' else self.g.body_feats
            self.g._branch(part, self.static['feats'], self.static['out'], f0)

    def _branches(self, eager):
        self.fork.record(self.main)
        self.side.wait_event(self.fork)
        self._branch('body')
        self._branch('hand')
        self.join.record(self.side)
        self.main.wait_event(self.join)

    def _losses(self):
        with torch.cuda.stream(self.main):
            self.static['losses'] = F.pose_losses(self.static['out'], None)

    def __call__(self):
        cur = torch.cuda.current_stream()
        self.main.wait_stream(cur)
        with torch.cuda.stream(self.main):
            self.graphs['trunk'].replay()
            self.fork.record(self.main)
        self.side.wait_event(self.fork)
        with torch.cuda.stream(self.side):
            self.graphs['body'].replay()
            self.join.record(self.side)
        with torch.cuda.stream(self.main):
            self.graphs['hand'].replay()
            self.main.wait_event(self.join)
            self.graphs['losses'].replay()
        cur.wait_stream(self.main)
        return self.static['out'], [self.static['losses'][1]]
