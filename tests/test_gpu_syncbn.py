"""SyncBatchNorm phases (include/a2m.h a2m_bn_sync_*): a batch split into two
"ranks", each running the stats phase on its half, the float64 sums added (the all-reduce), and
the apply phases run per half, must reproduce the fused single-batch BatchNorm forward (outputs,
saved mean / rstd, running stats) and backward (dx, dgamma / dbeta summed over the halves, the
conv-bias gradient).  The end-to-end DP check over real process groups is
tools/syncbn_check.py (torchrun, two gloo ranks; results in profiles/)."""
import pytest
import torch

from conftest import rel_err

pytestmark = pytest.mark.gpu
DEV = 'cuda'


@pytest.mark.parametrize('mode,act,p', [(0, 2, 0.0), (0, 1, 0.0), (0, 0, 0.0), (3, 2, 0.0)])
def test_sync_phases_match_fused_batch(mode, act, p):
    from a2m import _native as N
    from a2m import functional as F
    g = torch.Generator().manual_seed(mode * 10 + act)
    Bt, C, L = 8, 48, 37
    x = (torch.randn(Bt, C, L, generator=g) * 1.5 + 0.3).to(DEV)
    gamma = (torch.rand(C, generator=g) + 0.5).to(DEV)
    beta = (torch.randn(C, generator=g) * 0.1).to(DEV)
    rm0, rv0 = torch.zeros(C, device=DEV), torch.ones(C, device=DEV)
    seed = 1234
    # fused, whole batch
    rm, rv = rm0.clone(), rv0.clone()
    y, mean, rstd = F.bn_train(x, gamma, beta, rm, rv, 0.1, 1e-5, p, mode, seed, act)
    dy = torch.randn(Bt, C, L, generator=g).to(DEV)
    dx, dg, db, dbias = F.bn_train_bwd(dy, x, gamma, beta, mean, rstd, p, mode, seed, act)

    # two ranks: halves of the batch (p = 0: the dropout masks are per-rank hashes)
    halves = [x[:Bt // 2].contiguous(), x[Bt // 2:].contiguous()]
    sums = []
    for h in halves:
        s = torch.empty(C, 2, device=DEV, dtype=torch.float64)
        F._with_ws(DEV, lambda wp, wn: N.lib.a2m_bn_sync_stats_f32(
            F._p(h), h.stride(0), h.stride(1), Bt // 2, C, L, p, mode, seed, F._p(s), wp, wn, F._stream()))
        sums.append(s)
    tot = sums[0] + sums[1]
    ys, means, rstds, rms = [], [], [], []
    for h in halves:
        rmh, rvh = rm0.clone(), rv0.clone()
        yh = torch.empty_like(h)
        mh, sh = torch.empty(C, device=DEV), torch.empty(C, device=DEV)
        N.check(N.lib.a2m_bn_sync_apply_f32(
            F._p(h), h.stride(0), h.stride(1), Bt // 2, C, L, F._p(tot), Bt * L, F._p(gamma), F._p(beta),
            F._p(rmh), F._p(rvh), 0.1, 1e-5, p, mode, seed, act, 0.2, F._p(yh), yh.stride(0), yh.stride(1),
            F._p(mh), F._p(sh), F._stream()))
        ys.append(yh); means.append(mh); rstds.append(sh); rms.append((rmh, rvh))
    assert rel_err(torch.cat(ys).cpu(), y.cpu()) < 1e-5
    for mh, sh, (rmh, rvh) in zip(means, rstds, rms):
        assert rel_err(mh.cpu(), mean.cpu()) < 1e-6 and rel_err(sh.cpu(), rstd.cpu()) < 1e-6
        assert rel_err(rmh.cpu(), rm.cpu()) < 1e-6 and rel_err(rvh.cpu(), rv.cpu()) < 1e-6
    dys = [dy[:Bt // 2].contiguous(), dy[Bt // 2:].contiguous()]
    bsums, dgs, dbs = [], [], []
    for h, d in zip(halves, dys):
        s = torch.empty(C, 2, device=DEV, dtype=torch.float64)
        dgh, dbh = torch.empty(C, device=DEV), torch.empty(C, device=DEV)
        F._with_ws(DEV, lambda wp, wn: N.lib.a2m_bn_sync_bwd_stats_f32(
            F._p(d), d.stride(0), d.stride(1), F._p(h), h.stride(0), h.stride(1), Bt // 2, C, L, F._p(gamma),
            F._p(beta), F._p(mean), F._p(rstd), p, mode, seed, act, 0.2, F._p(s), F._p(dgh), F._p(dbh),
            wp, wn, F._stream()))
        bsums.append(s); dgs.append(dgh); dbs.append(dbh)
    btot = bsums[0] + bsums[1]
    dxs, dbiases = [], []
    for h, d in zip(halves, dys):
        dxh = torch.empty_like(h)
        dbh = torch.empty(C, device=DEV)
        F._with_ws(DEV, lambda wp, wn: N.lib.a2m_bn_sync_bwd_apply_f32(
            F._p(d), d.stride(0), d.stride(1), F._p(h), h.stride(0), h.stride(1), Bt // 2, C, L, F._p(gamma),
            F._p(beta), F._p(mean), F._p(rstd), p, mode, seed, act, 0.2, F._p(btot), Bt * L, F._p(dxh),
            F._p(dbh), wp, wn, F._stream()))
        dxs.append(dxh); dbiases.append(dbh)
    assert rel_err(torch.cat(dxs).cpu(), dx.cpu()) < 1e-5
    assert rel_err((dgs[0] + dgs[1]).cpu(), dg.cpu()) < 1e-5
    assert rel_err((dbs[0] + dbs[1]).cpu(), db.cpu()) < 1e-5
    # the conv-bias gradient through train-mode BN is zero in exact arithmetic: the halves carry
    # large opposite parts, so compare the sum on the halves' scale
    scale = max(dbiases[0].abs().max().item(), 1e-30)
    assert ((dbiases[0] + dbiases[1]) - dbias).abs().max().item() < 1e-5 * scale

