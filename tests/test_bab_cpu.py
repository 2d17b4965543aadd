"""Branch-and-bound decision vs brute-force enumeration (CPU reference path)."""
import itertools

import numpy as np
import pytest

from fairify_amd.engine import exact
from fairify_amd.engine.bab import SAT, UNSAT, BaBConfig, BaBSolver
from fairify_amd.models.mlp import random_mlp
from fairify_amd.ops.backend import Backend
from fairify_amd.spec import Domain, Feature, Query

DOM = Domain("toy", tuple(Feature(f"f{i}", 0, w) for i, w in enumerate([3, 4, 2, 4, 5])))


def brute(m, q, lo, hi):
    pts = np.array(list(itertools.product(*[range(a, b + 1) for a, b in zip(lo, hi)])))
    s = dict(zip(map(tuple, pts), exact.exact_signs(m, pts)))
    for x in pts:
        rngs = []
        for i in range(len(lo)):
            if i in q.pa_idx:
                rngs.append([v for v in range(lo[i], hi[i] + 1) if v != x[i]])
            elif i in q.ra_idx:
                rngs.append(range(x[i] - q.tau, x[i] + q.tau + 1))
            else:
                rngs.append([x[i]])
        xps = np.array(list(itertools.product(*rngs)))
        if len(xps) and np.any(s[tuple(x)] * exact.exact_signs(m, xps) < 0):
            return SAT
    return UNSAT


@pytest.mark.parametrize("pa,ra,tau", [(("f2",), (), 0), (("f2", "f0"), (), 0), (("f2",), ("f3",), 1),
                                       (("f2",), ("f1", "f4"), 2)])
def test_bab_matches_bruteforce(pa, ra, tau):
    q = Query(pa=pa, ra=ra, tau=tau).resolve(DOM)
    lo = np.zeros(5, int)
    hi = np.array([3, 4, 2, 4, 5])
    for seed in range(10):
        m = random_mlp(5, [6, 4], seed=300 + seed, bias_scale=1.0 if seed % 3 else 0.0)
        res = BaBSolver(Backend(m), q, BaBConfig(node_budget=10 ** 6)).solve(lo[None], hi[None], m)
        assert res.status[0] == brute(m, q, lo, hi), seed
        if res.status[0] == SAT:
            assert exact.check_pair_constraints(res.cex_x, res.cex_xp, lo[None], hi[None], q.pa_idx, q.ra_idx, tau)[0]
            assert exact.is_violation(m, res.cex_x, res.cex_xp)[0]


def test_single_pa_value_is_unsat():
    q = Query(pa=("f2",)).resolve(DOM)
    m = random_mlp(5, [4], seed=1)
    lo = np.zeros((1, 5), int)
    hi = np.array([[3, 4, 0, 4, 5]])
    assert BaBSolver(Backend(m), q, BaBConfig()).solve(lo, hi, m).status[0] == UNSAT


def test_budget_gives_unknown_not_wrong():
    q = Query(pa=("f2",)).resolve(DOM)
    lo = np.zeros(5, int)
    hi = np.array([3, 4, 2, 4, 5])
    for seed in range(6):
        m = random_mlp(5, [8, 8], seed=400 + seed, bias_scale=0.5)
        res = BaBSolver(Backend(m), q, BaBConfig(node_budget=2)).solve(lo[None], hi[None], m)
        if res.status[0] != 0:
            assert res.status[0] == brute(m, q, lo, hi)


def test_exact_signs_fraction_fallback():
    m = random_mlp(3, [4], seed=0)
    m.biases = [np.zeros_like(b) for b in m.biases]
    x = np.zeros((2, 3), dtype=np.int64)
    assert np.all(exact.exact_signs(m, x) == 0)


def test_escalated_pass_is_sound_and_monotone():
    """The escalated second BaB pass (VerifyConfig.escalate_budget) only turns UNKNOWN into
    verdicts that agree with brute force, and never decides fewer partitions than one pass."""
    from fairify_amd.engine.pipeline import VerifyConfig, verify_chunk
    from fairify_amd.partition import Grid

    q = Query(pa=("f2",)).resolve(DOM)
    grid = Grid.reference(DOM, 3)
    ids = np.arange(len(grid))
    lo_all, hi_all = grid.decode(ids)
    for seed in range(3):
        m = random_mlp(5, [8, 6], seed=500 + seed, bias_scale=0.3)
        be = Backend(m)
        base = dict(sim_size=16, node_budget=2, heuristic=False, residual_samples=0, smt_backend="none")
        one = verify_chunk(be, m, q, grid, ids, VerifyConfig(**base))
        two = verify_chunk(be, m, q, grid, ids, VerifyConfig(escalate_budget=10 ** 5, **base))
        v1 = one.cols["verdict"]
        v2 = two.cols["verdict"]
        assert (v2 != "unknown").sum() >= (v1 != "unknown").sum()
        assert np.all((v1 == "unknown") | (v1 == v2))
        for k in np.nonzero(v2 != "unknown")[0]:
            want = "sat" if brute(m, q, lo_all[k], hi_all[k]) == SAT else "unsat"
            assert v2[k] == want, (seed, k)
