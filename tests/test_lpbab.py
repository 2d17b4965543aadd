"""Verified-LP branch-and-bound (smt/lpbab.py, stage "lp"): verdicts against brute-force lattice
enumeration, and the rigour of the dual certificate (it never undercuts the true optimum, even
from perturbed or wrong multipliers)."""
import itertools

import numpy as np
import pytest

from fairify_amd import presets
from fairify_amd.engine import exact
from fairify_amd.models.mlp import random_mlp
from fairify_amd.ops import reference as ref
from fairify_amd.partition import processing_order

scipy = pytest.importorskip("scipy")


def _brute(m, lo, hi, pa):
    pts = np.array(list(itertools.product(*[range(a, b + 1) for a, b in zip(lo, hi)])))
    z0 = m.logits(np.where(np.arange(m.n_in) == pa, 0, pts))
    z1 = m.logits(np.where(np.arange(m.n_in) == pa, 1, pts))
    return bool((((z0 > 0) & (z1 < 0)) | ((z0 < 0) & (z1 > 0))).any())


def _row_bounds(m, lo, hi, q, values):
    import torch

    out = {}
    for v in range(len(values)):
        rl = lo.astype(np.float32).copy()
        rh = hi.astype(np.float32).copy()
        rl[list(q.pa_idx)] = values[v]
        rh[list(q.pa_idx)] = values[v]
        ws = [torch.from_numpy(np.asarray(w, np.float32)) for w in m.weights]
        bs = [torch.from_numpy(np.asarray(b, np.float32)) for b in m.biases]
        r = ref.bounds(ws, bs, torch.from_numpy(rl[None]), torch.from_numpy(rh[None]), mode="symbolic",
                       keep_layers=True)
        out[v] = ([t[0].double().numpy() for t in r.layer_lb], [t[0].double().numpy() for t in r.layer_ub])
    return out


@pytest.mark.parametrize("seed", [3, 4, 5])
def test_lpbab_matches_bruteforce(seed):
    from fairify_amd.smt import lpbab

    pre = presets.get("src/AC-sex")
    grid, q = pre.grid(), pre.resolved()
    ids = processing_order(grid, 0)[:24]
    lo, hi = grid.decode(ids)
    hi = np.minimum(hi, lo + 1)                  # <= 2 values per free dim: enumerable
    m = random_mlp(13, [6, 5], seed=seed, bias_scale=0.5)
    from fairify_amd.engine.bab import _pa_table

    values, pairs = _pa_table(q, lo[:1], hi[:1])
    pa = q.pa_idx[0]
    decided = 0
    for k in range(len(ids)):
        rb = _row_bounds(m, lo[k], hi[k], q, values)

        def confirm(xs, xps):
            ok = exact.check_pair_constraints(xs[None], xps[None], lo[k:k + 1], hi[k:k + 1], q.pa_idx, q.ra_idx, q.tau)
            return bool(ok[0] and exact.is_violation(m, xs[None], xps[None])[0])

        st, wit, nodes = lpbab.solve_partition(m.weights, m.biases, lo[k], hi[k], q.pa_idx, values, pairs, rb,
                                               4096, 60.0, confirm)
        truth = _brute(m, lo[k], hi[k], pa)
        if st == "sat":
            assert truth, k
            assert exact.is_violation(m, np.asarray(wit[0])[None], np.asarray(wit[1])[None])[0]
        elif st == "unsat":
            assert not truth, k
        decided += st != "unknown"
    assert decided == len(ids)                   # complete within the budget on these boxes


def test_certified_bound_never_undercuts_the_optimum():
    """Weak duality with rounding terms: any multipliers (optimal, perturbed, random) give a bound
    >= the LP optimum."""
    from scipy.optimize import linprog
    from scipy.sparse import csr_matrix

    from fairify_amd.smt.lpbab import certified_bound

    rng = np.random.default_rng(0)
    for trial in range(20):
        n, m = 8, 12
        A = rng.normal(size=(m, n))
        b = rng.uniform(1, 3, size=m)
        c = rng.normal(size=n)
        lb, ub = -rng.uniform(0.5, 2, n), rng.uniform(0.5, 2, n)
        res = linprog(-c, A_ub=A, b_ub=b, bounds=np.stack([lb, ub], 1), method="highs")
        assert res.status == 0
        opt = -res.fun
        y = np.maximum(-res.ineqlin.marginals, 0)
        A_s = csr_matrix(A)
        empty = csr_matrix((0, n))
        tight = certified_bound(c, A_s, b, empty, np.zeros(0), y, np.zeros(0), lb, ub)
        assert tight >= opt - 1e-12 and tight <= opt + 1e-6
        for yy in (y * (1 + 0.1 * rng.normal(size=m)), rng.uniform(0, 1, m), np.zeros(m)):
            assert certified_bound(c, A_s, b, empty, np.zeros(0), yy, np.zeros(0), lb, ub) >= opt - 1e-12


def test_certified_bound_rows_any_sign_never_undercuts():
    """Two-sided rows, multipliers of either sign (optimal, flipped, random): the bound is never
    below the LP optimum, and tight for the optimal ones."""
    from scipy.optimize import linprog
    from scipy.sparse import csr_matrix

    from fairify_amd.smt.lpbab import certified_bound_rows

    rng = np.random.default_rng(1)
    for trial in range(20):
        n, m = 8, 10
        A = rng.normal(size=(m, n))
        rlo = np.where(rng.uniform(size=m) < 0.3, -np.inf, -rng.uniform(1, 3, size=m))
        rhi = rng.uniform(1, 3, size=m)
        d = rng.normal(size=n)
        lb, ub = -rng.uniform(0.5, 2, n), rng.uniform(0.5, 2, n)
        fin = np.isfinite(rlo)
        A_ub = np.concatenate([A, -A[fin]])
        b_ub = np.concatenate([rhi, -rlo[fin]])
        res = linprog(-d, A_ub=A_ub, b_ub=b_ub, bounds=np.stack([lb, ub], 1), method="highs")
        assert res.status == 0
        opt = -res.fun
        y = -res.ineqlin.marginals
        lam = y[:m].copy()
        lam[fin] -= y[m:]
        A_s = csr_matrix(A)
        tight = certified_bound_rows(d, A_s, rlo, rhi, lam, lb, ub)
        assert opt - 1e-12 <= tight <= opt + 1e-6
        for ll in (-lam, rng.normal(size=m), np.zeros(m)):
            assert certified_bound_rows(d, A_s, rlo, rhi, ll, lb, ub) >= opt - 1e-12


def test_lp_infeasible_node_needs_a_certificate():
    """A phase pattern no point of the box satisfies: the warm-started LP reports it infeasible
    and the elastic phase-1 certificate proves it (bound -inf); both phases of that neuron
    together cover the box, so exactly one child is provably empty."""
    from fairify_amd.smt import lpbab

    W0 = np.array([[1.0], [0.0]])            # z = x0 + 0.5 on x0 in [0, 3]: always active
    b0 = np.array([0.5])
    W1 = np.array([[1.0]])
    b1 = np.array([-1.0])
    lo = np.array([0.0, 0.0])
    hi = np.array([3.0, 1.0])
    rb = ([np.array([-0.5])], [np.array([3.5])])   # loose bounds keep the neuron "unstable"
    lp = lpbab._LP([W0, W1], [b0, b1], lo, hi, [1], [0.0], [1.0], rb, rb)
    a = lp.a_vars[0][0]
    lb, ub = lp.lb.copy(), lp.ub.copy()
    lb[a] = ub[a] = 0.0                            # inactive: z <= 0 impossible
    t0, cert0, v0, _ = lp.solve(lb, ub)
    assert v0 is None and cert0 == -np.inf
    lb[a] = ub[a] = 1.0
    t1, cert1, v1, _ = lp.solve(lb, ub)
    assert v1 is not None and np.isfinite(cert1)


def test_lp_model_runs_after_other_highs_users():
    """HiGHS keeps a process-global thread scheduler: a model configured with its own thread
    count after SciPy's MILP / linprog had started it failed every solve (every node stayed open).
    The LP stage's models must keep working in a process where other HiGHS users ran first."""
    from scipy.optimize import LinearConstraint, milp

    from fairify_amd.smt import lpbab

    milp(c=np.array([1.0, 1.0]), constraints=LinearConstraint(np.array([[1.0, 2.0]]), 1.0, np.inf),
         integrality=np.array([1, 1]))
    W0 = np.array([[1.0], [0.0]])
    b0 = np.array([0.5])
    W1 = np.array([[1.0]])
    b1 = np.array([-1.0])
    rb = ([np.array([0.5])], [np.array([3.5])])
    lp = lpbab._LP([W0, W1], [b0, b1], np.array([0.0, 0.0]), np.array([3.0, 1.0]), [1], [0.0], [1.0], rb, rb)
    t, cert, v, basis = lp.solve(lp.lb, lp.ub)
    assert v is not None and np.isfinite(cert) and basis is not None


@pytest.mark.parametrize("seed", [7, 8])
def test_lpbab_multivalued_pa_with_sign_pretests(seed):
    """Race (5 values, 20 ordered pairs): the per-value single-copy sign tests that close whole
    rows / columns of the pair table keep the verdicts equal to brute force."""
    from fairify_amd.engine.bab import _pa_table
    from fairify_amd.smt import lpbab

    pre = presets.get("src/AC-race")
    grid, q = pre.grid(), pre.resolved()
    ids = processing_order(grid, 0)[:10]
    lo, hi = grid.decode(ids)
    pa = q.pa_idx[0]
    hi_full = hi.copy()
    hi = np.minimum(hi, lo + 1)
    hi[:, pa] = hi_full[:, pa]                     # all 5 race values, <= 2 values elsewhere
    m = random_mlp(13, [6, 5], seed=seed, bias_scale=0.5)
    values, pairs = _pa_table(q, lo[:1], hi[:1])
    assert len(pairs) > 2
    for k in range(len(ids)):
        rb = _row_bounds(m, lo[k], hi[k], q, values)

        def confirm(xs, xps):
            ok = exact.check_pair_constraints(xs[None], xps[None], lo[k:k + 1], hi[k:k + 1], q.pa_idx, q.ra_idx, q.tau)
            return bool(ok[0] and exact.is_violation(m, xs[None], xps[None])[0])

        def exact_sign(xs):
            return int(exact.exact_signs(m, xs[None])[0])

        st, wit, nodes = lpbab.solve_partition(m.weights, m.biases, lo[k], hi[k], q.pa_idx, values, pairs, rb,
                                               4096, 60.0, confirm, exact_sign)
        pts = np.array(list(itertools.product(*[range(a, b + 1) for a, b in zip(lo[k], hi[k])])))
        zs = [m.logits(np.where(np.arange(m.n_in) == pa, values[v][0], pts)) for v in range(len(values))]
        truth = any(((zs[i] < 0) & (zs[j] > 0)).any() for i, j in pairs)
        assert st != "unknown", k
        assert (st == "sat") == truth, k
        if st == "sat":
            assert exact.is_violation(m, np.asarray(wit[0])[None], np.asarray(wit[1])[None])[0]


def _row_bounds_box(m, lo, hi, q, values):
    return _row_bounds(m, lo, hi, q, values)


@pytest.mark.parametrize("seed,tau,race", [(11, 2, False), (12, 3, False), (13, 2, True)])
def test_lpbab_relaxed_matches_bruteforce(seed, tau, race):
    """Relaxed queries (|x_r - x'_r| <= tau on RA = age, x' NOT clipped to the box; reference
    relaxed/BM/Verify-BM.py:53-54, utils/verif_utils.py:879-887): both orientations, x' bounds over
    the widened box; verdicts equal enumeration of every (x, x') pair."""
    from fairify_amd.engine.bab import _pa_table
    from fairify_amd.smt import lpbab
    from fairify_amd.spec import ADULT, Query

    q = Query(pa=("race",) if race else ("sex",), ra=("age",), tau=tau).resolve(ADULT)
    grid = presets.get("src/AC-race" if race else "src/AC-sex").grid()
    ids = processing_order(grid, 0)[:12]
    lo, hi = grid.decode(ids)
    pa, ra = q.pa_idx[0], q.ra_idx[0]
    keep = hi.copy()
    hi = np.minimum(hi, lo + 1)
    if race:
        hi[:, pa] = np.minimum(keep[:, pa], lo[:, pa] + 2)      # 3 race values: 6 ordered pairs
    m = random_mlp(13, [6, 5], seed=seed, bias_scale=0.5)
    decided = 0
    for k in range(len(ids)):
        values, pairs = _pa_table(q, lo[k:k + 1], hi[k:k + 1])
        rb = _row_bounds(m, lo[k], hi[k], q, values)
        lw, hw = lo[k].copy(), hi[k].copy()
        lw[ra] -= tau
        hw[ra] += tau
        rbp = _row_bounds(m, lw, hw, q, values)

        def confirm(xs, xps):
            ok = exact.check_pair_constraints(xs[None], xps[None], lo[k:k + 1], hi[k:k + 1], q.pa_idx, q.ra_idx, q.tau)
            return bool(ok[0] and exact.is_violation(m, xs[None], xps[None])[0])

        def exact_sign(xs):
            return int(exact.exact_signs(m, xs[None])[0])

        st, wit, nodes = lpbab.solve_partition(m.weights, m.biases, lo[k], hi[k], q.pa_idx, values, pairs, rb,
                                               8192, 60.0, confirm, exact_sign, ra_idx=q.ra_idx, tau=float(tau),
                                               row_bounds_p=rbp)
        pts = np.array(list(itertools.product(*[range(a, b + 1) for a, b in zip(lo[k], hi[k])])))
        truth = False
        for vi, vj in pairs:
            x = pts.copy()
            x[:, pa] = values[vi][0]
            z = m.logits(x)
            for d in range(-tau, tau + 1):
                xp = x.copy()
                xp[:, pa] = values[vj][0]
                xp[:, ra] += d
                zp = m.logits(xp)
                if (((z < 0) & (zp > 0)) | ((z > 0) & (zp < 0))).any():
                    truth = True
                    break
            if truth:
                break
        if st == "sat":
            assert truth, k
            assert confirm(np.asarray(wit[0]), np.asarray(wit[1]))
        elif st == "unsat":
            assert not truth, k
        decided += st != "unknown"
    assert decided == len(ids)
