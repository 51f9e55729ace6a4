"""Per-phase time of graph_layer_bwd_kernel from the diagnostic stamp build
(tools/build_variant.sh gbst train_graph "-DA2M_GBWD_STAMPS"; run with A2M_LIB=_ab/gbst.so):
thread 0 of each workgroup stamps the wall clock (100 MHz) after every phase barrier.
Prints the mean over workgroups of each phase's length at the training shapes of
tools/graph_bwd_bench.py (hand GAT / GraphConv J = 42, body GAT J = 10, 4096 frames)."""
import ctypes
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, 'audio-to-motion-generation_amd'))
import numpy as np  # noqa: E402
import torch  # noqa: E402

from a2m import _native as N  # noqa: E402
from a2m import functional as F  # noqa: E402
from a2m import skeleton as S  # noqa: E402

NS, NBLK = 32, 4096
NAMES = {0: 'start', 1: 'tile+nbl', 2: 'rev+logits', 3: 'fwd recompute', 4: 'LN bwd', 25: 'dU+dx+red', 26: 'partials'}
for h in range(4):
    for k, nm in enumerate(('dY mfma', 'dalpha', 'softmax bwd', 'da_src', 'dx acc')):
        NAMES[5 + 5 * h + k] = f'h{h} {nm}'
GCONV = {5: 'dagg/droot mfma', 6: 'droot to lds'}

dev = torch.device('cuda')
FR = int(os.environ.get('FRAMES', 4096))
fn = N.lib.a2m_debug_gbwd_stamps
fn.argtypes = [ctypes.c_void_p, ctypes.c_size_t]
# GraphConv first: the stamp buffer starts zeroed and the GAT runs overwrite every slot it used
for name, J, lo, kind in (('hand gconv', 42, 10, 1), ('hand gat', 42, 10, 0), ('body gat', 10, 0, 0)):
    ptr, idx = [t.to(dev) for t in S.in_neighbour_csr(S.edge_index(lo, J), J)]
    x = torch.randn(FR * J, 64, device=dev)
    dy = torch.randn(FR * J, 64, device=dev)
    if kind == 0:
        w0, w1 = torch.randn(256, 64, device=dev) * 0.1, None
        a_s, a_d = torch.randn(1, 4, 64, device=dev) * 0.3, torch.randn(1, 4, 64, device=dev) * 0.3
    else:
        w0, w1 = torch.randn(64, 64, device=dev) * 0.1, torch.randn(64, 64, device=dev) * 0.1
        a_s = a_d = None
    b = torch.zeros(64, device=dev)
    lw, lb = torch.ones(64, device=dev), torch.zeros(64, device=dev)
    pre = None
    if os.environ.get('SAVED', '0') == '1':
        pre = torch.empty_like(x)
        F.graph_layer(x, J, kind, ptr, idx, w0, w1, a_s, a_d, b, lw, lb, pre_ln=pre)
    for _ in range(3):
        F.graph_layer_bwd(x, dy, J, kind, ptr, idx, w0, w1, a_s, a_d, b, lw, lb, pre_ln=pre)
    torch.cuda.synchronize()
    buf = np.zeros(NBLK * NS, dtype=np.uint64)
    N.check(fn(buf.ctypes.data, buf.size))
    blocks = -(-FR // (128 // J))
    st = buf.reshape(NBLK, NS)[:min(blocks, NBLK)].astype(np.int64)
    idxs = [i for i in sorted(NAMES) if (st[:, i] > 0).all()]
    t0 = st[:, 0]
    total = (st[:, idxs[-1]] - t0).mean() / 100.0
    span = (st[:, idxs[-1]].max() - t0.min()) / 100.0
    print(f'{name}: {blocks} workgroups, mean workgroup {total:.2f} us, kernel span {span:.1f} us', flush=True)
    prev = 0
    for i in idxs[1:]:
        d = (st[:, i] - st[:, prev]).mean() / 100.0
        lbl = GCONV.get(i, NAMES[i]) if kind == 1 else NAMES[i]
        print(f'  {lbl:18s} {d:7.2f} us', flush=True)
        prev = i
