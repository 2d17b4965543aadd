"""ReLU-phase branch-and-bound (engine/relu_bab.py, stage "relu") on CPU: verdicts against
brute-force lattice enumeration, the residue the input-split BaB cannot close, and the soundness
of the phase-fixed bounds / exact-zero backward concretisation it relies on."""
import itertools
import json
import os

import numpy as np
import pytest
import torch

from fairify_amd import presets
from fairify_amd.engine.bab import SAT, UNKNOWN, UNSAT
from fairify_amd.engine.relu_bab import ReluBaBSolver, ReluConfig
from fairify_amd.models.mlp import random_mlp
from fairify_amd.models.zoo import get_model
from fairify_amd.ops import reference as ref
from fairify_amd.ops.backend import Backend
from fairify_amd.partition import processing_order

HERE = os.path.dirname(os.path.abspath(__file__))


def _brute(m, lo, hi, pa):
    pts = np.array(list(itertools.product(*[range(a, b + 1) for a, b in zip(lo, hi)])))
    z0 = m.logits(np.where(np.arange(m.n_in) == pa, 0, pts))
    z1 = m.logits(np.where(np.arange(m.n_in) == pa, 1, pts))
    return bool((((z0 > 0) & (z1 < 0)) | ((z0 < 0) & (z1 > 0))).any())


@pytest.mark.parametrize("name", ["AC-8", "AC-12", "AC-9"])
def test_relu_bab_matches_bruteforce(name):
    pre = presets.get("src/AC-sex")
    grid, q = pre.grid(), pre.resolved()
    m = get_model(name, weights="random", seed=1)
    ids = processing_order(grid, 0)[:48]
    lo, hi = grid.decode(ids)
    hi = np.minimum(hi, lo + 1)         # <= 2 values per free dim: enumerable
    res = ReluBaBSolver(Backend(m), q, ReluConfig(node_budget=4096)).solve(lo, hi, m)
    pa = q.pa_idx[0]
    assert (res.status != UNKNOWN).mean() > 0.9
    for k in range(len(ids)):
        v = _brute(m, lo[k], hi[k], pa)
        if res.status[k] == SAT:
            assert v, k
        elif res.status[k] == UNSAT:
            assert not v, k


def test_relu_bab_matches_bruteforce_biased_nets():
    """Non-zero biases (trained-like nets): no exact-zero structure, the coupled certificate and
    input splits do the work."""
    pre = presets.get("src/AC-sex")
    grid, q = pre.grid(), pre.resolved()
    ids = processing_order(grid, 0)[:32]
    lo, hi = grid.decode(ids)
    hi = np.minimum(hi, lo + 1)
    pa = q.pa_idx[0]
    for seed in (3, 4):
        m = random_mlp(13, [6, 6], seed=seed, bias_scale=0.5)
        res = ReluBaBSolver(Backend(m), q, ReluConfig(node_budget=4096)).solve(lo, hi, m)
        for k in range(len(ids)):
            v = _brute(m, lo[k], hi[k], pa)
            if res.status[k] != UNKNOWN:
                assert (res.status[k] == SAT) == v, (seed, k)
        sat = np.nonzero(res.status == SAT)[0]
        from fairify_amd.engine import exact

        if sat.size:
            assert exact.is_violation(m, res.cex_x[sat], res.cex_xp[sat]).all()


@pytest.mark.parametrize("name,min_closed", [("AC-8", 20), ("AC-12", 22)])
def test_relu_bab_closes_input_split_residue(name, min_closed):
    """The partitions the bench's input-split BaB left UNKNOWN on the GPU (tests/data/relu_residue.json):
    the ReLU-phase stage proves most of them UNSAT with a few dozen nodes (measured: AC-8 22/24,
    AC-12 24/24)."""
    ids = np.asarray(json.load(open(os.path.join(HERE, "data", "relu_residue.json")))[name])
    pre = presets.get("src/AC-sex")
    grid, q = pre.grid(), pre.resolved()
    lo, hi = grid.decode(ids)
    m = get_model(name, weights="random", seed=0)
    res = ReluBaBSolver(Backend(m), q, ReluConfig(node_budget=1024)).solve(lo, hi, m)
    assert int((res.status == UNSAT).sum()) >= min_closed, res.status
    assert np.median(res.nodes[res.status == UNSAT]) <= 64


@pytest.mark.parametrize("hidden,bias", [([5, 5], 0.0), ([5] * 6, 0.0), ([8, 6, 4], 0.4)])
def test_phase_bounds_sound_on_branch_region(hidden, bias):
    """Forward bounds and the every-layer backward bounds with random fixed phases enclose the
    network on every lattice point of the branch region (points whose activations match the
    fixed phases); infeasible flags only on empty regions."""
    g = np.random.default_rng(7)
    n0 = 6
    m = random_mlp(n0, hidden, seed=5, bias_scale=bias)
    ws = [torch.from_numpy(w) for w in m.weights]
    bs = [torch.from_numpy(b) for b in m.biases]
    Nh = sum(hidden)
    for trial in range(40):
        lo = g.integers(-3, 3, size=(1, n0))
        hi = lo + g.integers(0, 3, size=(1, n0))
        ph = np.zeros((1, Nh), np.int8)
        sel = g.choice(Nh, size=3, replace=False)
        ph[0, sel] = g.choice([-1, 1], size=3)
        pts = np.array(list(itertools.product(*[range(a, b + 1) for a, b in zip(lo[0], hi[0])])))
        acts = m.layer_outputs(pts)
        pre_act = []
        h = pts.astype(np.float64)
        for W, b in zip(m.weights, m.biases):
            zz = h @ W.astype(np.float64) + b
            pre_act.append(zz)
            h = np.maximum(zz, 0)
        zh = np.concatenate(pre_act[:-1], axis=1)
        inreg = np.all(np.where(ph[0] < 0, zh <= 0, True) & np.where(ph[0] > 0, zh >= 0, True), axis=1)
        z = m.logits(pts)
        L, H = torch.tensor(lo, dtype=torch.float32), torch.tensor(hi, dtype=torch.float32)
        res = ref.bounds(ws, bs, L, H, keep_layers=True, phase=torch.from_numpy(ph))
        pc, forms = ref.crown_phase(ws, bs, L, H, res, torch.from_numpy(ph))
        if bool(res.infeasible[0]):
            assert not inreg.any(), trial
            continue
        if not inreg.any():
            continue
        zr = z[inreg]
        assert float(res.out_lb[0]) <= zr.min() and float(res.out_ub[0]) >= zr.max(), trial
        assert float(pc.low[0, 0]) <= zr.min(), trial
        assert -float(pc.low[0, 1]) >= zr.max(), trial
        for sg, k in ((1.0, 0), (-1.0, 1)):
            lam, c, err, low = forms[sg]
            lin = pts[inreg] @ lam[0].double().numpy() + float(c[0]) - float(err[0])
            assert np.all(sg * zr >= lin - 1e-9), trial
        del acts


def test_exact_zero_survives_rounding():
    """Zero-bias net whose only positive output path is closed by a fixed-inactive neuron: the
    backward bound of N is EXACTLY 0 (not 0 + rounding), so the strict query closes."""
    W1 = np.array([[1.0, -1.0], [0.5, 2.0]], np.float32)
    W2 = np.array([[0.7], [-0.3]], np.float32)
    from fairify_amd.models.mlp import MLP

    m = MLP([W1, W2], [np.zeros(2, np.float32), np.zeros(1, np.float32)])
    ws = [torch.from_numpy(w) for w in m.weights]
    bs = [torch.from_numpy(b) for b in m.biases]
    L = torch.tensor([[-3.0, -2.0]])
    H = torch.tensor([[4.0, 5.0]])
    ph = torch.tensor([[-1, 0]], dtype=torch.int8)     # neuron 0 (the positive path) off
    res = ref.bounds(ws, bs, L, H, keep_layers=True, phase=ph)
    pc, _ = ref.crown_phase(ws, bs, L, H, res, ph)
    assert -float(pc.low[0, 1]) == 0.0 or float(res.out_ub[0]) == 0.0


def test_pipeline_relu_stage_and_anytime_rounds():
    """verify_chunk: the relu stage decides the input-split residue (stage "relu"); in anytime mode
    relu rounds with growing budgets run for networks outside the width gate too; verdicts agree
    with the plain input-split ones wherever both decided, every SAT pair is exact."""
    from fairify_amd.engine import exact
    from fairify_amd.engine.pipeline import VerifyConfig, verify_chunk

    pre = presets.get("src/AC-sex")
    grid, q = pre.grid(), pre.resolved()
    m = get_model("AC-8", weights="random", seed=0)
    ids = processing_order(grid, 0)[:64]
    be = Backend(m)
    base = dict(sim_size=200, node_budget=64, heuristic=False, smt_backend="none")
    off = verify_chunk(be, m, q, grid, ids, VerifyConfig(relu_budget=0, **base))
    on = verify_chunk(be, m, q, grid, ids, VerifyConfig(relu_budget=256, **base))
    # (anytime_beta=0: the beta rounds, first in every anytime round, would take the relu rounds' share of
    # the wall budget on a loaded host)
    wide = verify_chunk(be, m, q, grid, ids, VerifyConfig(relu_budget=256, relu_max_width=1, anytime_seconds=90,
                                                          anytime_beta=0, **base))
    for r in (on, wide):
        assert (r.cols["stage"] == "relu").sum() > 10
        assert (r.cols["verdict"] != "unknown").sum() > (off.cols["verdict"] != "unknown").sum()
        both = (off.cols["verdict"] != "unknown") & (r.cols["verdict"] != "unknown")
        assert (off.cols["verdict"][both] == r.cols["verdict"][both]).all()
        sat = np.nonzero(r.cols["verdict"] == "sat")[0]
        lo, hi = grid.decode(ids[sat])
        X, XP = r.cols["cex_x"][sat], r.cols["cex_xp"][sat]
        assert exact.check_pair_constraints(X, XP, lo, hi, q.pa_idx, q.ra_idx, q.tau).all()
        assert exact.is_violation(m, X, XP).all()


def test_relu_bab_two_protected_attributes_matches_bruteforce():
    """Two PA dims (race, sex): the pair certificate folds both PA coordinates into the constants;
    its rounding margin takes the folded products' magnitudes (their sum can cancel).  Every PA must
    differ (src/GC/Verify-GC.py:135-141): verdicts equal enumeration of all (x, x') pairs."""
    from fairify_amd.spec import ADULT, Query

    q = Query(pa=("race", "sex")).resolve(ADULT)
    pre = presets.get("src/AC-sex")
    grid = pre.grid()
    ids = processing_order(grid, 0)[:24]
    lo, hi = grid.decode(ids)
    hi = np.minimum(hi, lo + 1)
    ri, si = q.pa_idx
    for seed in (5, 6):
        m = random_mlp(13, [6, 6], seed=seed, bias_scale=0.5)
        res = ReluBaBSolver(Backend(m), q, ReluConfig(node_budget=4096)).solve(lo, hi, m)
        for k in range(len(ids)):
            rv = range(int(lo[k, ri]), int(hi[k, ri]) + 1)
            free = [range(a, b + 1) for a, b in zip(lo[k], hi[k])]
            pts = np.array(list(itertools.product(*free)))
            viol = False
            for r1, r2 in itertools.product(rv, rv):
                if r1 == r2:
                    continue
                for s1 in (0, 1):
                    x = pts.copy(); x[:, ri] = r1; x[:, si] = s1
                    xp = pts.copy(); xp[:, ri] = r2; xp[:, si] = 1 - s1
                    z, zp = m.logits(x), m.logits(xp)
                    if (((z > 0) & (zp < 0)) | ((z < 0) & (zp > 0))).any():
                        viol = True
                        break
                if viol:
                    break
            if res.status[k] != UNKNOWN:
                assert (res.status[k] == SAT) == viol, (seed, k)


@pytest.mark.parametrize("seed,tau", [(21, 2), (22, 3), (23, 2)])
def test_relu_bab_relaxed_matches_bruteforce(seed, tau):
    """Relaxed queries (|x_r - x'_r| <= tau on RA = age, x' unclipped): the nodes carry an x' box on
    the RA dims, the second orientation runs on the negated network; every decided verdict equals
    enumeration of all (x, x') pairs, and every SAT pair is exactly confirmed."""
    from fairify_amd.engine import exact
    from fairify_amd.spec import ADULT, Query

    q = Query(pa=("sex",), ra=("age",), tau=tau).resolve(ADULT)
    grid = presets.get("src/AC-sex").grid()
    ids = processing_order(grid, 0)[:16]
    lo, hi = grid.decode(ids)
    hi = np.minimum(hi, lo + 1)
    pa, ra = q.pa_idx[0], q.ra_idx[0]
    m = random_mlp(13, [6, 6], seed=seed, bias_scale=0.0 if seed % 2 else 0.5)
    res = ReluBaBSolver(Backend(m), q, ReluConfig(node_budget=8192)).solve(lo, hi, m)
    decided = 0
    for k in range(len(ids)):
        pts = np.array(list(itertools.product(*[range(a, b + 1) for a, b in zip(lo[k], hi[k])])))
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
    assert decided >= 0.9 * len(ids)


def test_anytime_lp_overlaps_gpu_stages_and_agrees():
    """Anytime mode with the verified LP: the LP searches start with each round and run in the host
    workers while the BaB / relu stages work on the same residue; a partition decided by both keeps
    one verdict, LP verdicts agree with the plain input-split ones, and LP SAT pairs are exact."""
    from fairify_amd.engine import exact
    from fairify_amd.engine.pipeline import VerifyConfig, _lp_available, verify_chunk

    if not _lp_available():
        pytest.skip("SciPy HiGHS bindings not available")
    pre = presets.get("src/AC-sex")
    grid, q = pre.grid(), pre.resolved()
    m = get_model("AC-8", weights="random", seed=0)
    ids = processing_order(grid, 0)[:48]
    be = Backend(m)
    base = dict(sim_size=200, node_budget=32, heuristic=False, relu_budget=0)
    off = verify_chunk(be, m, q, grid, ids, VerifyConfig(smt_backend="none", **base))
    r = verify_chunk(be, m, q, grid, ids, VerifyConfig(smt_backend="auto", anytime_seconds=20, lp_budget=256,
                                                       smt_workers=2, **base))
    assert (r.cols["verdict"] != "unknown").sum() >= (off.cols["verdict"] != "unknown").sum()
    both = (off.cols["verdict"] != "unknown") & (r.cols["verdict"] != "unknown")
    assert (off.cols["verdict"][both] == r.cols["verdict"][both]).all()
    sat = np.nonzero(r.cols["verdict"] == "sat")[0]
    lo, hi = grid.decode(ids[sat])
    X, XP = r.cols["cex_x"][sat], r.cols["cex_xp"][sat]
    assert exact.check_pair_constraints(X, XP, lo, hi, q.pa_idx, q.ra_idx, q.tau).all()
    assert exact.is_violation(m, X, XP).all()
