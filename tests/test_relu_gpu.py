"""ReLU-phase branch-and-bound on the MI355X: fa_crown_phase_kernel vs ops/reference.py:crown_phase,
phase-aware forward kernels vs ref.bounds, and the native runtime (csrc/relu_runtime.cpp) against
brute-force enumeration and on the input-split residue."""
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

pytestmark = pytest.mark.gpu
HERE = os.path.dirname(os.path.abspath(__file__))


def _rows(n0, hidden, R, seed, bias):
    g = np.random.default_rng(seed)
    m = random_mlp(n0, hidden, seed=seed, bias_scale=bias)
    lo = g.integers(0, 12, size=(R, n0)).astype(np.float32)
    hi = lo + g.integers(0, 6, size=(R, n0)).astype(np.float32)
    Nh = sum(hidden)
    ph = np.zeros((R, Nh), np.int8)
    for r in range(R):
        k = g.integers(0, 4)
        sel = g.choice(Nh, size=k, replace=False)
        ph[r, sel] = g.choice([-1, 1], size=k)
    return m, torch.from_numpy(lo), torch.from_numpy(hi), torch.from_numpy(ph)


@pytest.mark.parametrize("n0,hidden,bias", [(13, [5, 5], 0.0), (13, [5] * 9, 0.0), (13, [64, 32, 16, 8, 4], 0.0),
                                            (13, [16, 8], 0.5), (20, [50], 0.3), (6, [3, 3, 3], 0.0)])
def test_phase_bounds_and_crown_phase_match_reference(cuda, n0, hidden, bias):
    m, lo, hi, ph = _rows(n0, hidden, 300, 11, bias)
    cpu = Backend(m, "cpu")
    gpu = Backend(m, cuda)
    rc = cpu.bounds(lo, hi, keep_layers=True, phase=ph)
    pcc, forms = cpu.crown_phase(lo, hi, rc, ph)
    rg = gpu.bounds(lo.to(cuda), hi.to(cuda), keep_layers=True, phase=ph.to(cuda))
    # forward pass with phases
    scale = float(((rc.out_ub - rc.out_lb).abs() + rc.out_ub.abs()).max() + 1e-3)
    assert torch.allclose(rg.out_lb.cpu(), rc.out_lb, rtol=1e-4, atol=1e-4 * scale)
    assert torch.allclose(rg.out_ub.cpu(), rc.out_ub, rtol=1e-4, atol=1e-4 * scale)
    agree = (rg.infeasible.cpu() == rc.infeasible).float().mean()
    assert agree > 0.98
    inf = rc.infeasible & rg.infeasible.cpu()
    pcg, _ = gpu.crown_phase(lo.to(cuda), hi.to(cuda), rg, ph.to(cuda))
    ok = ~(rc.infeasible | rg.infeasible.cpu())
    for k in range(2):
        a, b = pcg.low[:, k].cpu()[ok], pcc.low[:, k][ok].float()
        assert torch.allclose(a, b, rtol=1e-3, atol=1e-3 * scale), (k, (a - b).abs().max())
        # exact zeros are structural: the kernel reproduces the reference's exactly-zero bounds
        z = b == 0
        if int(z.sum()) >= 5:
            assert float((a[z] == 0).float().mean()) > 0.9
    # in-place refinement: logit bounds intersected, infeasible rows (+inf, -inf)
    olb = torch.maximum(rc.out_lb, pcc.low[:, 0].float())
    oub = torch.minimum(rc.out_ub, -pcc.low[:, 1].float())
    assert torch.allclose(rg.out_lb.cpu()[ok], olb[ok], rtol=1e-3, atol=1e-3 * scale)
    assert torch.allclose(rg.out_ub.cpu()[ok], oub[ok], rtol=1e-3, atol=1e-3 * scale)
    if bool(inf.any()):
        assert torch.isinf(rg.out_lb.cpu()[inf]).all()


@pytest.mark.parametrize("n0,hidden,bias", [(6, [5, 5], 0.0), (6, [4, 4, 4], 0.3), (5, [8, 6], 0.0)])
def test_crown_phase_kernel_sound_on_branch_region(cuda, n0, hidden, bias):
    """Kernel bounds enclose the exact logits of every lattice point of each row's branch region."""
    m, lo, hi, ph = _rows(n0, hidden, 64, 5, bias)
    hi = torch.minimum(hi, lo + 2)
    gpu = Backend(m, cuda)
    rg = gpu.bounds(lo.to(cuda), hi.to(cuda), keep_layers=True, phase=ph.to(cuda))
    gpu.crown_phase(lo.to(cuda), hi.to(cuda), rg, ph.to(cuda))
    olb, oub = rg.out_lb.cpu().double().numpy(), rg.out_ub.cpu().double().numpy()
    for r in range(lo.shape[0]):
        pts = np.array(list(itertools.product(*[range(int(a), int(b) + 1) for a, b in zip(lo[r], hi[r])])))
        h = pts.astype(np.float64)
        pre = []
        for W, b in zip(m.weights, m.biases):
            zz = h @ W.astype(np.float64) + b
            pre.append(zz)
            h = np.maximum(zz, 0)
        zh = np.concatenate(pre[:-1], axis=1)
        p = ph[r].numpy()
        inreg = np.all(np.where(p < 0, zh <= 0, True) & np.where(p > 0, zh >= 0, True), axis=1)
        if not inreg.any():
            continue
        z = pre[-1][inreg, 0]
        assert olb[r] <= z.min() and oub[r] >= z.max(), r
        Lf = pts[inreg] @ rg.Lc[r].double().cpu().numpy() + float(rg.L0[r]) - float(rg.Le[r])
        Uf = pts[inreg] @ rg.Uc[r].double().cpu().numpy() + float(rg.U0[r]) + float(rg.Ue[r])
        assert np.all(z >= Lf - 1e-9) and np.all(z <= Uf + 1e-9), r


def _brute(m, lo, hi, pa):
    pts = np.array(list(itertools.product(*[range(a, b + 1) for a, b in zip(lo, hi)])))
    z0 = m.logits(np.where(np.arange(m.n_in) == pa, 0, pts))
    z1 = m.logits(np.where(np.arange(m.n_in) == pa, 1, pts))
    return bool((((z0 > 0) & (z1 < 0)) | ((z0 < 0) & (z1 > 0))).any())


@pytest.mark.parametrize("name,seed,bias", [("AC-8", 1, None), ("AC-12", 1, None), ("AC-9", 1, None),
                                            ("mlp", 3, 0.5)])
def test_native_relu_bab_matches_bruteforce(cuda, name, seed, bias):
    pre = presets.get("src/AC-sex")
    grid, q = pre.grid(), pre.resolved()
    m = get_model(name, weights="random", seed=seed) if bias is None else random_mlp(13, [6, 6], seed=seed,
                                                                                      bias_scale=bias)
    ids = processing_order(grid, 0)[:64]
    lo, hi = grid.decode(ids)
    hi = np.minimum(hi, lo + 1)
    res = ReluBaBSolver(Backend(m, cuda), q, ReluConfig(node_budget=4096)).solve(lo, hi, m)
    pa = q.pa_idx[0]
    assert (res.status != UNKNOWN).mean() > 0.9
    for k in range(len(ids)):
        v = _brute(m, lo[k], hi[k], pa)
        if res.status[k] == SAT:
            assert v, k
        elif res.status[k] == UNSAT:
            assert not v, k


@pytest.mark.parametrize("name,min_closed", [("AC-8", 20), ("AC-12", 22)])
def test_native_relu_closes_residue(cuda, name, min_closed):
    ids = np.asarray(json.load(open(os.path.join(HERE, "data", "relu_residue.json")))[name])
    pre = presets.get("src/AC-sex")
    grid, q = pre.grid(), pre.resolved()
    lo, hi = grid.decode(ids)
    m = get_model(name, weights="random", seed=0)
    nat = ReluBaBSolver(Backend(m, cuda), q, ReluConfig(node_budget=1024)).solve(lo, hi, m)
    assert int((nat.status == UNSAT).sum()) >= min_closed, nat.status
    tor = ReluBaBSolver(Backend(m, "cpu"), q, ReluConfig(node_budget=1024)).solve(lo, hi, m)
    both = (nat.status != UNKNOWN) & (tor.status != UNKNOWN)
    assert np.array_equal(nat.status[both], tor.status[both])


@pytest.mark.parametrize("seed,tau", [(21, 2), (22, 3), (23, 2)])
def test_native_relu_relaxed_matches_bruteforce_and_torch(cuda, seed, tau):
    """Relaxed queries on the native runtime (x' RA box per node in csrc/relu_runtime.cpp, the
    certificate concretising the copies' RA dims separately, x' RA splits; the second orientation on
    the negated network): every decided verdict equals enumeration of all (x, x') pairs, every SAT
    pair is exactly confirmed, and the verdicts agree with the torch orchestration where both
    decide (FAIRIFY_TORCH_BAB=1)."""
    from fairify_amd.engine import exact
    from fairify_amd.spec import ADULT, Query

    q = Query(pa=("sex",), ra=("age",), tau=tau).resolve(ADULT)
    grid = presets.get("src/AC-sex").grid()
    ids = processing_order(grid, 0)[:16]
    lo, hi = grid.decode(ids)
    hi = np.minimum(hi, lo + 1)
    pa, ra = q.pa_idx[0], q.ra_idx[0]
    m = random_mlp(13, [6, 6], seed=seed, bias_scale=0.0 if seed % 2 else 0.5)
    res = ReluBaBSolver(Backend(m, cuda), q, ReluConfig(node_budget=8192)).solve(lo, hi, m)
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
    os.environ["FAIRIFY_TORCH_BAB"] = "1"
    try:
        tor = ReluBaBSolver(Backend(m, cuda), q, ReluConfig(node_budget=8192)).solve(lo, hi, m)
    finally:
        del os.environ["FAIRIFY_TORCH_BAB"]
    both = (res.status != UNKNOWN) & (tor.status != UNKNOWN)
    assert np.array_equal(res.status[both], tor.status[both])


def test_native_relu_relaxed_wide_boxes_decide_like_torch(cuda):
    """Wider boxes with a node budget that binds: copy B's rows follow x's input splits on the shared
    dims (only the RA dims read x''s own box), so the native runtime decides about as many partitions
    as the torch orchestration and agrees with it wherever both decide."""
    from fairify_amd.spec import ADULT, Query

    q = Query(pa=("sex",), ra=("age",), tau=2).resolve(ADULT)
    grid = presets.get("src/AC-sex").grid()
    ids = processing_order(grid, 0)[:64]
    lo, hi = grid.decode(ids)
    hi = np.minimum(hi, lo + 4)
    m = random_mlp(13, [8, 6], seed=31, bias_scale=0.5)
    nat = ReluBaBSolver(Backend(m, cuda), q, ReluConfig(node_budget=128)).solve(lo, hi, m)
    os.environ["FAIRIFY_TORCH_BAB"] = "1"
    try:
        tor = ReluBaBSolver(Backend(m, cuda), q, ReluConfig(node_budget=128)).solve(lo, hi, m)
    finally:
        del os.environ["FAIRIFY_TORCH_BAB"]
    both = (nat.status != UNKNOWN) & (tor.status != UNKNOWN)
    assert np.array_equal(nat.status[both], tor.status[both])
    dn, dt = int((nat.status != UNKNOWN).sum()), int((tor.status != UNKNOWN).sum())
    assert dt > 0 and dn >= dt - max(2, dt // 10), (dn, dt)
