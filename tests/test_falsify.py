"""Residual falsifier (heavy sampling + lattice local search) — every hit is a true violation,
and on SAT toy partitions the local search finds one from few samples."""
import itertools

import numpy as np
import pytest
import torch

from fairify_amd.engine import exact
from fairify_amd.engine.falsify import residual_falsify
from fairify_amd.models.mlp import random_mlp
from fairify_amd.ops.backend import Backend
from fairify_amd.spec import Domain, Feature, Query

DOM = Domain("toy", tuple(Feature(f"f{i}", 0, w) for i, w in enumerate([6, 7, 1, 5, 6])))


def _brute_sat(m, q, lo, hi):
    pts = np.array(list(itertools.product(*[range(a, b + 1) for a, b in zip(lo, hi)])))
    s = dict(zip(map(tuple, pts), exact.exact_signs(m, pts)))
    for x in pts:
        for v in range(lo[2], hi[2] + 1):
            if v == x[2]:
                continue
            xp = x.copy()
            xp[2] = v
            if s[tuple(x)] * s[tuple(xp)] < 0:
                return True
    return False


@pytest.mark.parametrize("pa,ra,tau", [(("f2",), (), 0), (("f2",), ("f1",), 1)])
def test_residual_falsifier_hits_are_true_violations(pa, ra, tau):
    q = Query(pa=pa, ra=ra, tau=tau).resolve(DOM)
    lo = np.zeros(5, np.int64)
    hi = np.array([6, 7, 1, 5, 6])
    found_any = 0
    sat_cases = 0
    for seed in range(16):
        m = random_mlp(5, [8, 6], seed=100 + seed, bias_scale=0.5)
        be = Backend(m, "cpu")
        values = torch.tensor([[0], [1]])
        pairs = torch.tensor([[0, 1], [1, 0]])
        fr = residual_falsify(be, q, torch.tensor(lo[None]).float(), torch.tensor(hi[None]).float(),
                              torch.tensor([seed]), values, pairs, seed=seed, n_samples=32, k_starts=4, iters=30)
        if not q.relaxed:
            sat_cases += _brute_sat(m, q, lo, hi)
        if bool(fr.found[0]):
            found_any += 1
            X = fr.wit_x.numpy().round().astype(np.int64)
            XP = fr.wit_xp.numpy().round().astype(np.int64)
            assert exact.check_pair_constraints(X, XP, lo[None], hi[None], q.pa_idx, q.ra_idx, tau)[0]
            assert exact.is_violation(m, X, XP)[0]
    assert found_any > 0
    if not q.relaxed:
        assert found_any >= max(1, sat_cases // 2)   # local search recovers most SAT toy boxes


@pytest.mark.gpu
def test_ascent_kernel_matches_torch_loop(cuda, monkeypatch):
    """fa_ascent_kernel (one launch for all rounds) finds the same partitions as the PyTorch
    round loop it replaces, and every witness is an exact violation inside its box."""
    from fairify_amd.engine import falsify as F
    from fairify_amd.ops import hip

    q = Query(pa=("f2",)).resolve(DOM)
    g = torch.Generator().manual_seed(0)
    P = 300
    lo = torch.stack([torch.randint(0, max(1, w - 2), (P,), generator=g) for w in (6, 7, 1, 5, 6)], 1).float()
    hi = torch.minimum(lo + torch.randint(1, 4, (P, 5), generator=g).float(), torch.tensor([6., 7., 1., 5., 6.]))
    lo[:, 2], hi[:, 2] = 0, 1
    pids = torch.arange(P)
    values = torch.tensor([[0], [1]], device=cuda)
    pairs = torch.tensor([[0, 1], [1, 0]], device=cuda)
    calls = {"n": 0}
    real = hip.ascent

    def counted(*a, **k):
        calls["n"] += 1
        return real(*a, **k)

    for seed in range(4):
        m = random_mlp(5, [16, 8], seed=300 + seed, bias_scale=0.5)
        be = Backend(m, cuda)
        args = (be, q, lo.to(cuda), hi.to(cuda), pids.to(cuda), values, pairs)
        monkeypatch.setattr(hip, "ascent", counted)
        a = F._local_search(*args, seed=seed, n_samples=16, k_starts=4, iters=12, sub=128)
        monkeypatch.setattr(hip, "ascent", lambda *x, **k: None)
        b = F._local_search(*args, seed=seed, n_samples=16, k_starts=4, iters=12, sub=128)
        assert torch.equal(a.found, b.found)
        idx = torch.nonzero(a.found).flatten().cpu().numpy()
        if idx.size:
            X = a.wit_x.cpu().numpy()[idx].round().astype(np.int64)
            XP = a.wit_xp.cpu().numpy()[idx].round().astype(np.int64)
            lo_n, hi_n = lo.numpy()[idx].astype(np.int64), hi.numpy()[idx].astype(np.int64)
            assert exact.check_pair_constraints(X, XP, lo_n, hi_n, q.pa_idx, q.ra_idx, 0).all()
            assert exact.is_violation(m, X, XP).all()
    assert calls["n"] >= 4   # the kernel path ran
