"""Native (C++/HIP) branch-and-bound vs brute-force lattice enumeration on a real MI355X."""
import itertools

import numpy as np
import pytest
import torch

from fairify_amd.engine import exact
from fairify_amd.engine.bab import SAT, UNSAT, BaBConfig, BaBSolver
from fairify_amd.models.mlp import random_mlp
from fairify_amd.ops.backend import Backend
from fairify_amd.spec import Domain, Feature, Query

pytestmark = pytest.mark.gpu

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


@pytest.mark.parametrize("pa,ra,tau", [(("f2",), (), 0), (("f2", "f0"), (), 0), (("f2",), ("f3",), 1)])
def test_native_bab_matches_bruteforce(cuda, pa, ra, tau):
    q = Query(pa=pa, ra=ra, tau=tau).resolve(DOM)
    lo = np.zeros(5, int)
    hi = np.array([3, 4, 2, 4, 5])
    bad = 0
    for seed in range(12):
        m = random_mlp(5, [6, 4], seed=200 + seed, bias_scale=1.0 if seed % 3 else 0.0)
        be = Backend(m, cuda)
        assert be.hip
        solver = BaBSolver(be, q, BaBConfig(node_budget=10 ** 6, batch_nodes=512, max_pool=1 << 16))
        res = solver.solve(lo[None], hi[None], m)
        truth = brute(m, q, lo, hi)
        if res.status[0] != truth:
            bad += 1
        if res.status[0] == SAT:
            assert exact.check_pair_constraints(res.cex_x, res.cex_xp, lo[None], hi[None], q.pa_idx, q.ra_idx, tau)[0]
            assert exact.is_violation(m, res.cex_x, res.cex_xp)[0]
    assert bad == 0


def test_native_matches_torch_bab_on_adult(cuda):
    import os

    from fairify_amd import presets
    from fairify_amd.models.zoo import get_model
    from fairify_amd.partition import processing_order

    pre = presets.get("src/AC-sex")
    grid = pre.grid()
    q = pre.resolved()
    ids = processing_order(grid, 0)[:256]
    lo, hi = grid.decode(ids)
    m = get_model("AC-3")
    be = Backend(m, cuda)
    nat = BaBSolver(be, q, BaBConfig(node_budget=4096)).solve(lo, hi, m)
    os.environ["FAIRIFY_TORCH_BAB"] = "1"
    try:
        tor = BaBSolver(be, q, BaBConfig(node_budget=4096)).solve(lo, hi, m)
    finally:
        del os.environ["FAIRIFY_TORCH_BAB"]
    decided = (nat.status != 0) & (tor.status != 0)
    assert np.array_equal(nat.status[decided], tor.status[decided])
    assert decided.mean() > 0.9


def test_open_left_reported_only_for_unknown(cuda):
    """The native BaB reports, for partitions it leaves UNKNOWN at the node budget, the open
    frontier they left (the escalation filter's predictor); decided partitions report 0."""
    q = Query(pa=("f2",)).resolve(DOM)
    lo = np.zeros((6, 5), int)
    hi = np.tile(np.array([3, 4, 2, 4, 5]), (6, 1))
    for seed in range(4):
        m = random_mlp(5, [12, 12], seed=700 + seed, bias_scale=0.3)
        res = BaBSolver(Backend(m, cuda), q, BaBConfig(node_budget=4)).solve(lo, hi, m)
        assert res.open_left is not None and res.open_left.shape == (6,)
        assert np.all(res.open_left[res.status != 0] == 0)
        assert np.all(res.open_left >= 0)
        if np.any(res.status == 0):
            assert np.all(res.open_left[res.status == 0] > 0)


@pytest.mark.parametrize("name", ["AC-7", "AC-8", "AC-12"])
def test_escalation_steps_only_stop_earlier(cuda, name):
    """Stepped inline escalation (fa_settle_kernel: budget -> 2048 -> 4096 -> 8192 with frontier
    limits) follows the same per-partition search tree as the one-step schedule and only stops
    partitions earlier: every partition it decides has the one-step verdict, and it decides no
    partition the one-step schedule leaves UNKNOWN."""
    from fairify_amd import presets
    from fairify_amd.models.zoo import get_model
    from fairify_amd.partition import processing_order

    pre = presets.get("src/AC-sex")
    grid, q = pre.grid(), pre.resolved()
    lo, hi = grid.decode(processing_order(grid, 0)[:512])
    m = get_model(name, weights="random", seed=0)
    be = Backend(m, cuda)
    base = dict(node_budget=512, escalate_budget=8192, escalate_max_w=384)
    one = BaBSolver(be, q, BaBConfig(**base)).solve(lo, hi, m)
    steps = BaBSolver(be, q, BaBConfig(**base, escalate_steps=((2048, 768), (4096, 1024)))).solve(lo, hi, m)
    dec = steps.status != 0
    assert np.array_equal(steps.status[dec], one.status[dec])
    assert not np.any(dec & (one.status == 0))
    assert (one.status != 0).sum() >= dec.sum()


@pytest.mark.parametrize("name", ["AC-7", "AC-12", "AC-4"])
def test_fused_settle_matches_separate_launch(cuda, name):
    """The level end fused into the last split launch (its last workgroup settles every partition,
    csrc/bab.hip fa_split_kernel tail) gives exactly the per-partition verdicts and node counts of
    the separate fa_settle_kernel launch, inline escalation steps included."""
    from fairify_amd import presets
    from fairify_amd.models.zoo import get_model
    from fairify_amd.partition import processing_order

    pre = presets.get("src/AC-sex")
    grid, q = pre.grid(), pre.resolved()
    lo, hi = grid.decode(processing_order(grid, 0)[:1024])
    m = get_model(name, weights="random", seed=0)
    be = Backend(m, cuda)
    base = dict(node_budget=512, escalate_budget=8192, escalate_max_w=384, escalate_steps=((2048, 768), (4096, 1024)))
    out = {}
    for fused in (False, True):
        r = BaBSolver(be, q, BaBConfig(**base, fuse_settle=fused)).solve(lo, hi, m)
        out[fused] = r
    assert np.array_equal(out[True].status, out[False].status)
    assert np.array_equal(out[True].nodes, out[False].nodes)
