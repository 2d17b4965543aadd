"""Host MILP back-end (HiGHS via SciPy) against brute-force lattice enumeration (exact signs)."""
import itertools

import numpy as np
import pytest
import torch

from fairify_amd.engine import exact
from fairify_amd.models.mlp import random_mlp
from fairify_amd.ops.backend import Backend
from fairify_amd.smt import milp
from fairify_amd.spec import Domain, Feature, Query

pytestmark = pytest.mark.skipif(not milp.available(), reason="scipy.optimize.milp missing")

DOM = Domain("toy", tuple(Feature(f"f{i}", 0, w) for i, w in enumerate([6, 7, 1, 5, 6])))


def _brute(m, q, lo, hi):
    """Exact: does some lattice pair violate fairness?"""
    pts = np.array(list(itertools.product(*[range(a, b + 1) for a, b in zip(lo, hi)])))
    s = dict(zip(map(tuple, pts), exact.exact_signs(m, pts)))
    pa = q.pa_idx[0]
    for x in pts:
        for v in range(lo[pa], hi[pa] + 1):
            if v == x[pa]:
                continue
            base = x.copy()
            base[pa] = v
            cands = [base]
            if q.relaxed:
                cands = []
                r = q.ra_idx[0]
                for dlt in range(-int(q.tau), int(q.tau) + 1):
                    c = base.copy()
                    c[r] = x[r] + dlt
                    cands.append(c)
            for xp in cands:
                sp = exact.exact_signs(m, xp[None])[0] if tuple(xp) not in s else s[tuple(xp)]
                if s[tuple(x)] * sp < 0:
                    return True
    return False


@pytest.mark.parametrize("relaxed", [False, True])
def test_milp_matches_bruteforce(relaxed):
    q = (Query(pa=("f2",), ra=("f1",), tau=1) if relaxed else Query(pa=("f2",))).resolve(DOM)
    lo = np.array([0, 0, 0, 0, 0])
    hi = np.array([6, 7, 1, 5, 6])
    values = q.pa_values(lo, hi)
    pairs = q.pa_pairs(values)
    decided = sat = 0
    for seed in range(12):
        m = random_mlp(5, [8, 6], seed=500 + seed, bias_scale=0.5)
        be = Backend(m, "cpu")
        lbs, ubs = milp.layer_bounds_rows(be, lo[None], hi[None], q, values, widen_ra=False)
        plbs, pubs = milp.layer_bounds_rows(be, lo[None], hi[None], q, values, widen_ra=True)
        rb = {v: ([l[0, v] for l in lbs], [u[0, v] for u in ubs]) for v in range(len(values))}
        pb = {v: ([l[0, v] for l in plbs], [u[0, v] for u in pubs]) for v in range(len(values))}
        verdict, pair = milp.solve_partition(m.weights, m.biases, lo, hi, q.pa_idx, values, pairs, q.ra_idx,
                                             float(q.tau), rb, pb, time_limit=30.0)
        truth = _brute(m, q, lo, hi)
        if verdict == "sat":
            X, XP = np.array([pair[0]]), np.array([pair[1]])
            assert exact.check_pair_constraints(X, XP, lo[None], hi[None], q.pa_idx, q.ra_idx, q.tau)[0]
            assert exact.is_violation(m, X, XP)[0], "MILP candidate is not a violation"
            assert truth
            sat += 1
        elif verdict == "unsat":
            assert not truth, "MILP claimed UNSAT on a SAT partition"
        decided += verdict != "unknown"
    assert decided >= 10 and sat >= 1


def test_output_bound_brackets_exact_extremes():
    q = Query(pa=("f2",)).resolve(DOM)
    lo = np.array([0, 0, 0, 0, 0])
    hi = np.array([6, 7, 1, 5, 6])
    values = q.pa_values(lo, hi)
    for seed in range(4):
        m = random_mlp(5, [8, 6], seed=700 + seed, bias_scale=0.5)
        be = Backend(m, "cpu")
        lbs, ubs = milp.layer_bounds_rows(be, lo[None], hi[None], q, values, widen_ra=False)
        for v in range(len(values)):
            pts = np.array(list(itertools.product(*[range(a, b + 1) for a, b in zip(lo, hi)])))
            pts = pts[pts[:, 2] == values[v][0]]
            z = m.logits(pts)
            bnd = ([l[0, v] for l in lbs], [u[0, v] for u in ubs])
            mn = milp.output_bound(m.weights, m.biases, lo, hi, q.pa_idx, values[v], bnd, 1.0, 30.0)
            mx = milp.output_bound(m.weights, m.biases, lo, hi, q.pa_idx, values[v], bnd, -1.0, 30.0)
            assert mn <= z.min() + 1e-6 and mn >= z.min() - 1e-3 * (1 + abs(z.min()))
            assert mx >= z.max() - 1e-6 and mx <= z.max() + 1e-3 * (1 + abs(z.max()))
