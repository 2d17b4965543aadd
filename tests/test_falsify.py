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
