"""beta-CROWN ReLU-phase branch-and-bound (ops/beta.py, engine/beta_bab.py, stage "beta") on CPU:
the rigorous bound against brute-force lattice enumeration on the phase regions, the monotone warm
start of the children, verdicts against enumeration, and the trained AC-7 residue the round-4
stages could not close (profiles/r4/lp_tree_sizes_ac7_trained.jsonl)."""
import itertools

import numpy as np
import pytest
import torch

from fairify_amd import presets
from fairify_amd.engine import exact
from fairify_amd.engine.bab import SAT, UNKNOWN, UNSAT
from fairify_amd.engine.beta_bab import BetaBaBSolver, BetaConfig
from fairify_amd.models.mlp import random_mlp
from fairify_amd.models.zoo import get_model
from fairify_amd.ops import beta as B
from fairify_amd.ops import reference as ref
from fairify_amd.ops.backend import Backend
from fairify_amd.partition import processing_order


def _lattice(lo, hi):
    return np.array(list(itertools.product(*[range(int(a), int(b) + 1) for a, b in zip(lo, hi)])), dtype=np.float64)


def _setup(seed, widths=(6, 5, 4), n0=4, R=6, fix=0.3):
    g = np.random.default_rng(seed)
    m = random_mlp(n0, list(widths), seed=seed, bias_scale=0.5)
    ws = [torch.tensor(np.asarray(w), dtype=torch.float32) for w in m.weights]
    bs = [torch.tensor(np.asarray(b), dtype=torch.float32).reshape(-1) for b in m.biases]
    pa = [1]
    lo = np.tile(np.array([0, 0, 1, -2], np.float32)[:n0], (R, 1))
    hi = lo + g.integers(1, 3, size=(R, n0)).astype(np.float32)
    lo[:, pa] = 0
    hi[:, pa] = 1
    va = np.zeros((R, 1), np.float32)
    vb = np.ones((R, 1), np.float32)
    # partition bounds of each copy: the reference's rigorous symbolic bounds
    be = Backend(m)
    NH = be.n_hidden
    out = []
    for v in (va, vb):
        rl, rh = lo.copy(), hi.copy()
        rl[:, pa] = v
        rh[:, pa] = v
        res = be.bounds(torch.from_numpy(rl), torch.from_numpy(rh), keep_layers=True)
        out.append((torch.cat(res.layer_lb, 1)[:, :NH].float(), torch.cat(res.layer_ub, 1)[:, :NH].float()))
    ph = []
    for c in range(2):
        p = g.integers(-1, 2, size=(R, NH)) * (g.random((R, NH)) < fix)
        ph.append(torch.from_numpy(p.astype(np.int8)))
    return m, ws, bs, pa, torch.from_numpy(lo), torch.from_numpy(hi), torch.from_numpy(va), torch.from_numpy(vb), out, ph


def _true_min(m, lo, hi, pa, va, vb, phA, phB, t, widths):
    """min over lattice points of the box satisfying both copies' phases of t N(x,va) - (1-t) N(x,vb)
    (exact enough in fp64 for these small integer boxes), or +inf when none does."""
    X = _lattice(lo, hi)
    ok = np.ones(len(X), bool)
    outs = []
    for v, ph in ((va, phA), (vb, phB)):
        h = X.copy()
        h[:, pa] = v
        o = 0
        for l, (W, b) in enumerate(zip(m.weights, m.biases)):
            z = h @ np.asarray(W, np.float64) + np.asarray(b, np.float64)
            if l < len(m.weights) - 1:
                p = ph[o:o + z.shape[1]]
                ok &= ((p[None] * z) >= 0).all(1)
                o += z.shape[1]
                h = np.maximum(z, 0)
            else:
                h = z
        outs.append(h[:, 0])
    f = t * outs[0] - (1 - t) * outs[1]
    return f[ok].min() if ok.any() else np.inf


@pytest.mark.parametrize("seed", [0, 1, 2])
@pytest.mark.parametrize("neg_beta", [False, True])
def test_rigorous_bound_below_every_phase_feasible_point(seed, neg_beta):
    m, ws, bs, pa, lo, hi, va, vb, bnd, ph = _setup(seed)
    R = lo.shape[0]
    widths = [w.shape[1] for w in ws[:-1]]
    NH = sum(widths)
    g = torch.Generator().manual_seed(seed)
    al = [torch.rand(R, NH, generator=g) for _ in range(2)]
    be_ = [torch.rand(R, NH, generator=g) * (2 if neg_beta else 1) - (1 if neg_beta else 0) for _ in range(2)]
    t = torch.rand(R, generator=g)
    lev = B.level_ref(ws, bs, widths, lo, hi, pa, va, vb, bnd[0][0], bnd[0][1], bnd[1][0], bnd[1][1], ph[0], ph[1],
                      al[0], al[1], be_[0], be_[1], t, iters=0, lr_a=0.1, lr_b=0.5, lr_t=0.1)
    for r in range(R):
        tm = _true_min(m, lo[r].numpy(), hi[r].numpy(), pa, va[r].numpy(), vb[r].numpy(), ph[0][r].numpy(),
                       ph[1][r].numpy(), float(t[r]), widths)
        assert float(lev.bound[r]) <= tm, (r, float(lev.bound[r]), tm)


@pytest.mark.parametrize("seed", [0, 1])
def test_orientation_sign_equals_negated_network(seed):
    """osg = -1 (the reverse orientation of a row) bounds exactly what the network with its logit
    negated bounds with osg = +1 -- the merged-orientation search replaces the second solve on the
    negated net -- and the bound stays below every phase-feasible point of that orientation."""
    from fairify_amd.engine.relu_bab import negated

    m, ws, bs, pa, lo, hi, va, vb, bnd, ph = _setup(seed)
    R = lo.shape[0]
    widths = [w.shape[1] for w in ws[:-1]]
    NH = sum(widths)
    g = torch.Generator().manual_seed(seed)
    al = [torch.rand(R, NH, generator=g) for _ in range(2)]
    be_ = [torch.rand(R, NH, generator=g) for _ in range(2)]
    t = torch.rand(R, generator=g)
    mn = negated(m)
    wsn = [torch.tensor(np.asarray(w), dtype=torch.float32) for w in mn.weights]
    bsn = [torch.tensor(np.asarray(b), dtype=torch.float32).reshape(-1) for b in mn.biases]
    args = (lo, hi, pa, va, vb, bnd[0][0], bnd[0][1], bnd[1][0], bnd[1][1], ph[0], ph[1])
    cp = lambda: [x.clone() for x in (al[0], al[1], be_[0], be_[1], t)]  # noqa: E731
    neg = B.level_ref(ws, bs, widths, *args, *cp(), iters=0, lr_a=0.1, lr_b=0.5, lr_t=0.1,
                      osg=torch.full((R,), -1, dtype=torch.int8))
    ref_ = B.level_ref(wsn, bsn, widths, *args, *cp(), iters=0, lr_a=0.1, lr_b=0.5, lr_t=0.1)
    assert torch.equal(neg.bound, ref_.bound)
    assert torch.equal(neg.split, ref_.split)
    for r in range(R):
        tm = _true_min(mn, lo[r].numpy(), hi[r].numpy(), pa, va[r].numpy(), vb[r].numpy(), ph[0][r].numpy(),
                       ph[1][r].numpy(), float(t[r]), widths)
        assert float(neg.bound[r]) <= tm


@pytest.mark.parametrize("seed", [3, 4])
def test_optimised_bound_sound_and_not_worse(seed):
    m, ws, bs, pa, lo, hi, va, vb, bnd, ph = _setup(seed, fix=0.15)
    R = lo.shape[0]
    widths = [w.shape[1] for w in ws[:-1]]
    NH = sum(widths)
    mk = lambda: ([torch.full((R, NH), 0.5) for _ in range(2)], [torch.zeros(R, NH) for _ in range(2)],  # noqa: E731
                  torch.full((R,), 0.5))
    al0, be0, t0 = mk()
    l0 = B.level_ref(ws, bs, widths, lo, hi, pa, va, vb, bnd[0][0], bnd[0][1], bnd[1][0], bnd[1][1], ph[0], ph[1],
                     al0[0], al0[1], be0[0], be0[1], t0, iters=0, lr_a=0.1, lr_b=0.5, lr_t=0.1)
    al1, be1, t1 = mk()
    l1 = B.level_ref(ws, bs, widths, lo, hi, pa, va, vb, bnd[0][0], bnd[0][1], bnd[1][0], bnd[1][1], ph[0], ph[1],
                     al1[0], al1[1], be1[0], be1[1], t1, iters=60, lr_a=0.1, lr_b=0.5, lr_t=0.1)
    fin = torch.isfinite(l0.bound)
    assert bool((l1.bound[fin] >= l0.bound[fin] - 1e-5 * (1 + l0.bound[fin].abs())).all())
    assert bool((l1.bound[fin] > l0.bound[fin] + 1e-3).any())          # the optimiser does something
    for r in range(R):
        tm = _true_min(m, lo[r].numpy(), hi[r].numpy(), pa, va[r].numpy(), vb[r].numpy(), ph[0][r].numpy(),
                       ph[1][r].numpy(), float(t1[r]), widths)
        assert float(l1.bound[r]) <= tm


def test_children_start_at_parent_bound():
    """binit reproduces the parent's relaxation of the split neuron: each child's bound at the
    parent's parameters equals the parent's bound (warm starts never lose bound)."""
    m, ws, bs, pa, lo, hi, va, vb, bnd, ph = _setup(5, fix=0.0)
    R = lo.shape[0]
    widths = [w.shape[1] for w in ws[:-1]]
    NH = sum(widths)
    al = [torch.full((R, NH), 0.5) for _ in range(2)]
    be_ = [torch.zeros(R, NH) for _ in range(2)]
    t = torch.full((R,), 0.5)
    lev = B.level_ref(ws, bs, widths, lo, hi, pa, va, vb, bnd[0][0], bnd[0][1], bnd[1][0], bnd[1][1], ph[0], ph[1],
                      al[0], al[1], be_[0], be_[1], t, iters=30, lr_a=0.1, lr_b=0.5, lr_t=0.1)
    nd = {"phA": ph[0], "phB": ph[1], "alA": al[0], "alB": al[1], "beA": be_[0], "beB": be_[1], "t": t,
          "lo": lo, "hi": hi, "va": va, "vb": vb, "LBA": bnd[0][0], "UBA": bnd[0][1], "LBB": bnd[1][0],
          "UBB": bnd[1][1], "part": torch.arange(R), "root": torch.ones(R, dtype=torch.bool)}
    sel = torch.nonzero(lev.split >= 0).flatten()
    assert sel.numel() > 0
    kid = BetaBaBSolver._children({k: v[sel] for k, v in nd.items()}, lev.split[sel], lev.binit[sel], NH, lo.shape[1])
    lk = B.level_ref(ws, bs, widths, kid["lo"], kid["hi"], pa, kid["va"], kid["vb"], kid["LBA"], kid["UBA"],
                     kid["LBB"], kid["UBB"], kid["phA"], kid["phB"], kid["alA"], kid["alB"], kid["beA"], kid["beB"],
                     kid["t"], iters=0, lr_a=0.1, lr_b=0.5, lr_t=0.1)
    par = lev.bound[sel].repeat_interleave(2)
    fin = torch.isfinite(lk.bound)
    # equal up to the fp32 rounding of the stored multiplier
    assert bool((lk.bound[fin] >= par[fin] - 1e-6 * (1 + par[fin].abs())).all())


def _brute_pair(m, lo, hi, pa):
    X = _lattice(lo, hi)
    a = X.copy()
    b = X.copy()
    a[:, pa] = 0
    b[:, pa] = 1
    z0, z1 = m.logits(a), m.logits(b)
    return bool((((z0 > 0) & (z1 < 0)) | ((z0 < 0) & (z1 > 0))).any())


@pytest.mark.parametrize("seed,input_every,branch", [(3, 0, "kernel"), (6, 0, "kernel"), (3, 2, "kernel"),
                                                     (3, 0, "pgap"), (6, 0, "pgap")])
def test_beta_bab_matches_bruteforce(seed, input_every, branch):
    """Decided verdicts equal lattice enumeration (input_every > 0: the experimental forced input
    splits of BetaConfig; branch "pgap": the primal-gap rule at the averaged primal iterate)."""
    pre = presets.get("src/AC-sex")
    grid, q = pre.grid(), pre.resolved()
    ids = processing_order(grid, 0)[:24]
    lo, hi = grid.decode(ids)
    hi = np.minimum(hi, lo + 1)
    m = random_mlp(13, [8, 6, 4], seed=seed, bias_scale=0.5)
    cfg = BetaConfig(node_budget=256, iters=20, root_iters=40, input_every=input_every, branch=branch)
    res = BetaBaBSolver(Backend(m), q, cfg).solve(lo, hi, m)
    pa = q.pa_idx[0]
    assert (res.status != UNKNOWN).mean() > 0.5
    for k in range(len(ids)):
        if res.status[k] == UNKNOWN:
            continue
        assert (res.status[k] == SAT) == _brute_pair(m, lo[k], hi[k], pa), k
    sat = np.nonzero(res.status == SAT)[0]
    if sat.size:
        assert exact.is_violation(m, res.cex_x[sat], res.cex_xp[sat]).all()


@pytest.mark.slow
def test_beta_closes_trained_ac7_residue():
    """Trained AC-7 partitions the input-split and interval ReLU-phase stages leave open and the
    verified LP needs 21-5 000 nodes for (profiles/r4/lp_tree_sizes_ac7_trained.jsonl): the beta
    stage proves them within a few dozen nodes."""
    pre = presets.get("src/AC-sex")
    grid, q = pre.grid(), pre.resolved()
    m = get_model("AC-7", weights="zoo", seed=0)
    ids = np.array([12596, 4387, 6769, 6543, 4330, 13901])
    lo, hi = grid.decode(ids)
    res = BetaBaBSolver(Backend(m), q, BetaConfig(node_budget=200)).solve(lo, hi, m)
    assert (res.status == UNSAT).sum() >= 5, res.status


def _relaxed_truth(m, lo, hi, pa, ra, tau):
    pts = _lattice(lo, hi)
    for s1 in (0, 1):
        x = pts.copy()
        x[:, pa] = s1
        z = m.logits(x)
        for d in range(-tau, tau + 1):
            xp = x.copy()
            xp[:, pa] = 1 - s1
            xp[:, ra] += d
            zp = m.logits(xp)
            if (((z < 0) & (zp > 0)) | ((z > 0) & (zp < 0))).any():
                return True
    return False


def test_primal_gap_scores_rule():
    """The LP rule's score: max(mean h - relu(mean z), 0) on unfixed neurons unstable over the node's
    bounds, 0 on fixed / stable ones and on rows that took no optimisation step."""
    z = torch.tensor([[2.0, -4.0, 1.0, 3.0], [1.0, 1.0, 1.0, 1.0]])
    h = torch.tensor([[3.0, 1.0, 0.0, 5.0], [2.0, 2.0, 2.0, 2.0]])
    n = torch.tensor([2.0, 0.0])
    lb = torch.tensor([[-1.0, -1.0, -1.0, 0.5], [-1.0] * 4])
    ub = torch.ones(2, 4)
    ph = torch.tensor([[0, 0, 1, 0], [0, 0, 0, 0]], dtype=torch.int8)
    s = B.primal_gap_scores(z, h, n, lb, ub, ph)
    assert torch.allclose(s[0], torch.tensor([0.5, 0.5, 0.0, 0.0]))    # fixed (ph) / stable (lb > 0): 0
    assert bool((s[1] == 0).all())


@pytest.mark.parametrize("seed,tau,merge", [(21, 2, True), (24, 3, True), (21, 2, False)])
def test_beta_bab_relaxed_matches_bruteforce(seed, tau, merge):
    """Relaxed queries (|x_r - x'_r| <= tau on RA = age, x' unclipped): nodes carry x''s box on the
    RA dims (split like input dims), the second orientation runs on the negated network; every
    decided verdict equals enumeration of all (x, x') pairs, every SAT pair is exactly confirmed."""
    from fairify_amd.spec import ADULT, Query

    q = Query(pa=("sex",), ra=("age",), tau=tau).resolve(ADULT)
    grid = presets.get("src/AC-sex").grid()
    ids = processing_order(grid, 0)[:16]
    lo, hi = grid.decode(ids)
    hi = np.minimum(hi, lo + 1)
    pa, ra = q.pa_idx[0], q.ra_idx[0]
    m = random_mlp(13, [8, 6, 4], seed=seed, bias_scale=0.5)
    res = BetaBaBSolver(Backend(m), q, BetaConfig(node_budget=512, iters=20, root_iters=40,
                                                  merge_orient=merge)).solve(lo, hi, m)
    decided = 0
    for k in range(len(ids)):
        pts = _lattice(lo[k], hi[k])
        truth = False
        for s1 in (0, 1):
            x = pts.copy()
            x[:, pa] = s1
            z = m.logits(x)
            for d in range(-tau, tau + 1):
                xp = x.copy()
                xp[:, pa] = 1 - s1
                xp[:, ra] += d
                zp = m.logits(xp)
                if (((z < 0) & (zp > 0)) | ((z > 0) & (zp < 0))).any():
                    truth = True
        if res.status[k] == SAT:
            assert truth, k
            ok = exact.check_pair_constraints(res.cex_x[k:k + 1], res.cex_xp[k:k + 1], lo[k:k + 1], hi[k:k + 1],
                                              q.pa_idx, q.ra_idx, q.tau)
            assert ok[0] and exact.is_violation(m, res.cex_x[k:k + 1], res.cex_xp[k:k + 1])[0]
        elif res.status[k] == UNSAT:
            assert not truth, k
        decided += res.status[k] != UNKNOWN
    assert decided >= 0.5 * len(ids)


@pytest.mark.parametrize("relaxed", [False, True])
def test_sign_pruned_roots_match_bruteforce(relaxed):
    """Race (5 values: 20 ordered pairs, x 2 orientations when relaxed): the per-value logit sign tests
    close many trees before their roots are bounded; the verdicts stay those of enumeration and of the
    unpruned search."""
    from fairify_amd.spec import ADULT, Query

    q = Query(pa=("race",), ra=("age",) if relaxed else (), tau=2 if relaxed else 0).resolve(ADULT)
    grid = presets.get("src/AC-race").grid()
    ids = processing_order(grid, 0)[:12]
    lo, hi = grid.decode(ids)
    hi = np.minimum(hi, lo + 1)
    hi[:, q.pa_idx[0]] = np.maximum(hi[:, q.pa_idx[0]], lo[:, q.pa_idx[0]])
    m = random_mlp(13, [8, 6, 4], seed=5, bias_scale=0.5)
    be = Backend(m)
    sols = {sp: BetaBaBSolver(be, q, BetaConfig(node_budget=256, iters=20, root_iters=40, sign_prune=sp))
            for sp in (True, False)}
    res = {sp: s.solve(lo, hi, m).status for sp, s in sols.items()}
    assert sols[True].stats.get("sign_pruned", 0) > 0
    both = (res[True] != UNKNOWN) & (res[False] != UNKNOWN)
    assert bool((res[True][both] == res[False][both]).all())
    assert (res[True] != UNKNOWN).sum() >= (res[False] != UNKNOWN).sum()
    pa, ra = q.pa_idx[0], (q.ra_idx[0] if relaxed else None)
    for k in np.nonzero(res[True] != UNKNOWN)[0]:
        pts = _lattice(lo[k], hi[k])
        vals = range(int(lo[k, pa]), int(hi[k, pa]) + 1)
        truth = False
        for v1 in vals:
            x = pts.copy()
            x[:, pa] = v1
            z = m.logits(x)
            for v2 in vals:
                if v2 == v1:
                    continue
                for d in (range(-2, 3) if relaxed else (0,)):
                    xp = x.copy()
                    xp[:, pa] = v2
                    if relaxed:
                        xp[:, ra] += d
                    zp = m.logits(xp)
                    truth = truth or bool((((z < 0) & (zp > 0)) | ((z > 0) & (zp < 0))).any())
        assert (res[True][k] == SAT) == truth, k


def test_probe_verdicts_do_not_depend_on_grouping():
    """With the probe on, each partition's verdict is its own: solving the partitions together, in
    two halves, or one by one gives the same statuses (the product runner re-shards residues over
    ranks, tests/test_dist_gloo.py::test_residual_redistribution_matches_one_rank)."""
    pre = presets.get("src/AC-sex")
    grid, q = pre.grid(), pre.resolved()
    ids = processing_order(grid, 0)[:12]
    lo, hi = grid.decode(ids)
    m = random_mlp(13, [24, 12, 6], seed=5, bias_scale=0.5)
    cfg = BetaConfig(node_budget=48, iters=10, root_iters=20, probe_levels=1)
    be = Backend(m)
    whole = BetaBaBSolver(be, q, cfg).solve(lo, hi, m).status
    halves = np.concatenate([BetaBaBSolver(be, q, cfg).solve(lo[s], hi[s], m).status
                             for s in (slice(0, 5), slice(5, 12))])
    single = np.array([BetaBaBSolver(be, q, cfg).solve(lo[k:k + 1], hi[k:k + 1], m).status[0]
                       for k in range(len(ids))])
    assert np.array_equal(whole, halves) and np.array_equal(whole, single)


def test_crossed_bounds_without_a_fixed_phase_give_no_bound():
    """A node whose pre-activation bounds cross (lb > ub) proves its region empty only through a fixed
    phase.  With none fixed the bounds are not sound bounds of the (non-empty) box: the node gets no
    bound (NaN) -- never +inf, which would close its tree -- in the reference and in the BaB loop."""
    m, ws, bs, pa, lo, hi, va, vb, bnd, ph = _setup(3, fix=0.0)
    R = lo.shape[0]
    NH = bnd[0][0].shape[1]
    LBA, UBA = bnd[0][0].clone(), bnd[0][1].clone()
    LBA[0, 2] = UBA[0, 2] + 1.0            # row 0: crossed, no phase fixed
    ph1 = [p.clone() for p in ph]
    LBA[1, 3] = UBA[1, 3] + 1.0            # row 1: crossed on a neuron fixed inactive -> empty (inf)
    ph1[0][1, 3] = 1
    g = torch.Generator().manual_seed(0)
    al = [torch.rand(R, NH, generator=g) for _ in range(2)]
    be_ = [torch.zeros(R, NH) for _ in range(2)]
    t = torch.full((R,), 0.5)
    lev = B.level_ref(ws, bs, [x.shape[1] for x in ws[:-1]], lo, hi, pa, va, vb, LBA, UBA, bnd[1][0], bnd[1][1],
                      ph1[0], ph1[1], al[0], al[1], be_[0], be_[1], t, iters=0, lr_a=0.1, lr_b=0.5, lr_t=0.1)
    assert torch.isnan(lev.bound[0])
    assert float(lev.bound[1]) == float("inf")
    assert bool(torch.isfinite(lev.bound[2:]).all())


def test_beta_transposed_weights_are_built_once_under_concurrency():
    """The runner's worker threads share one Backend per model; the native beta runtime keeps the device
    pointer of the transposed weights (ops/hip.py:_beta_wt).  Racing first calls must all get the SAME
    tensor -- a second copy published over the first freed the memory a runtime still read (whole chunks
    of beta roots bounded with freed weights)."""
    import threading

    from fairify_amd.ops import hip

    for trial in range(5):
        be = Backend(random_mlp(6, [40, 30], seed=trial), device="cpu")
        bar = threading.Barrier(12)
        got = []

        def one():
            bar.wait()
            got.append(hip._beta_wt(be))

        th = [threading.Thread(target=one) for _ in range(12)]
        for t in th:
            t.start()
        for t in th:
            t.join()
        assert len(got) == 12 and all(g is got[0] for g in got)
