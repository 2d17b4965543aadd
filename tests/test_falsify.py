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


@pytest.mark.gpu
@pytest.mark.parametrize("model", ["AC-1", "AC-4", "AC-7"])
def test_fused_falsifier_matches_sim_and_is_sound(cuda, monkeypatch, model):
    """fa_falsify_kernel (sampling + boundary walk + ascent in one launch) against the unfused
    path it replaces (simulation kernel + PyTorch boundary walk + fa_ascent_kernel):
    * every witness is an exact violation inside its box;
    * the sampling phase reports the simulation kernel's first flip with the identical witness,
      except where one of the two witnesses has a logit whose rigorous fp32 bound straddles 0
      (the two kernels sum the MFMA products in different orders);
    * it decides at least 98 % of what the unfused path decides."""
    from fairify_amd import presets
    from fairify_amd.engine import falsify as F
    from fairify_amd.engine.bab import _pa_table
    from fairify_amd.models.zoo import get_model
    from fairify_amd.ops import hip
    from fairify_amd.partition import processing_order

    pre = presets.get("src/AC-sex")
    grid, q = pre.grid(), pre.resolved()
    ids = processing_order(grid, seed=0)[:768]
    lo_np, hi_np = grid.decode(ids)
    m = get_model(model, weights="random", seed=0)
    be = Backend(m, cuda)
    v_np, p_np = _pa_table(q, lo_np, hi_np)
    values, pairs = torch.from_numpy(v_np).to(cuda), torch.from_numpy(p_np).to(cuda)
    lo, hi = torch.from_numpy(lo_np).to(cuda).float(), torch.from_numpy(hi_np).to(cuda).float()
    pids = torch.from_numpy(ids).to(cuda)
    fused = F.residual_falsify(be, q, lo, hi, pids, values, pairs, 0, n_samples=2048, k_starts=16, iters=12)
    assert fused.how is not None, "fused kernel did not run"
    monkeypatch.setenv("FAIRIFY_FUSED_FALSIFY", "0")
    legacy = F.residual_falsify(be, q, lo, hi, pids, values, pairs, 0, n_samples=2048, k_starts=16, iters=12)
    sim = hip.simulate(be, q, lo, hi, pids, 2048, (0 ^ 0x6A09E667) & 0xFFFFFFFF, values, pairs, 0, 0)
    f = fused.found.cpu().numpy()
    how = fused.how.cpu().numpy()
    idx = np.nonzero(f)[0]
    X = fused.wit_x.cpu().numpy()[idx].round().astype(np.int64)
    XP = fused.wit_xp.cpu().numpy()[idx].round().astype(np.int64)
    assert exact.check_pair_constraints(X, XP, lo_np[idx], hi_np[idx], q.pa_idx, q.ra_idx, 0).all()
    assert exact.is_violation(m, X, XP).all()
    s_found = sim.found.cpu().numpy()
    sx, sxp = sim.wit_x.cpu().numpy(), sim.wit_xp.cpu().numpy()
    fx, fxp = fused.wit_x.cpu().numpy(), fused.wit_xp.cpu().numpy()
    bad = [i for i in range(len(ids)) if s_found[i] != (how[i] == 1) or
           (s_found[i] and not (np.array_equal(sx[i], fx[i]) and np.array_equal(sxp[i], fxp[i])))]
    if bad:
        pts = torch.from_numpy(np.concatenate([sx[bad], sxp[bad], fx[bad], fxp[bad]])).to(cuda)
        lb, ub = be.point_bounds(pts)
        amb = ((lb <= 0) & (ub >= 0)).view(4, len(bad)).any(dim=0).cpu().numpy()
        assert amb.all(), f"{int((~amb).sum())} sampling-phase mismatches outside the rounding margin"
    assert f.sum() >= 0.98 * legacy.found.cpu().numpy().sum()


@pytest.mark.gpu
@pytest.mark.parametrize("preset,model", [("relaxed/BM", "BM-1"), ("relaxed/BM", "BM-8"), ("relaxed/AC", "AC-3")])
def test_fused_falsifier_relaxed_is_sound_and_matches_torch(cuda, monkeypatch, preset, model):
    """Relaxed queries through fa_falsify_kernel (x' offsets on the RA dims, both orientations):
    every witness satisfies the pair constraints (|x_r - x'_r| <= tau, x' unclipped) and flips the
    exact network, and the kernel decides at least 95 % of what the PyTorch local search decides."""
    from fairify_amd import presets
    from fairify_amd.engine import falsify as F
    from fairify_amd.engine.bab import _pa_table
    from fairify_amd.models.zoo import get_model
    from fairify_amd.partition import processing_order

    pre = presets.get(preset)
    grid, q = pre.grid(), pre.resolved()
    assert q.relaxed
    ids = processing_order(grid, seed=0)[:512]
    lo_np, hi_np = grid.decode(ids)
    m = get_model(model, weights="random", seed=0)
    be = Backend(m, cuda)
    v_np, p_np = _pa_table(q, lo_np, hi_np)
    values, pairs = torch.from_numpy(v_np).to(cuda), torch.from_numpy(p_np).to(cuda)
    lo, hi = torch.from_numpy(lo_np).to(cuda).float(), torch.from_numpy(hi_np).to(cuda).float()
    pids = torch.from_numpy(ids).to(cuda)
    fused = F.residual_falsify(be, q, lo, hi, pids, values, pairs, 0, n_samples=1024, k_starts=16, iters=12)
    assert fused.how is not None, "fused kernel did not run"
    f = fused.found.cpu().numpy()
    idx = np.nonzero(f)[0]
    X = fused.wit_x.cpu().numpy()[idx].round().astype(np.int64)
    XP = fused.wit_xp.cpu().numpy()[idx].round().astype(np.int64)
    assert exact.check_pair_constraints(X, XP, lo_np[idx], hi_np[idx], q.pa_idx, q.ra_idx, q.tau).all()
    assert exact.is_violation(m, X, XP).all()
    monkeypatch.setenv("FAIRIFY_FUSED_FALSIFY", "0")
    legacy = F.residual_falsify(be, q, lo, hi, pids, values, pairs, 0, n_samples=1024, k_starts=16, iters=12)
    n_leg = int(legacy.found.cpu().numpy().sum())
    assert f.sum() >= 0.95 * n_leg and (n_leg == 0 or idx.size > 0), (int(f.sum()), n_leg)
