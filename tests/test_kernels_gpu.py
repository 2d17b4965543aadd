"""HIP kernels vs the PyTorch reference (fp32 CPU / fp64 oracle) — run on a real MI355X."""
import itertools

import numpy as np
import pytest
import torch

from fairify_amd.models.mlp import random_mlp
from fairify_amd.models.zoo import get_model
from fairify_amd.ops import reference as ref
from fairify_amd.ops.backend import Backend
from fairify_amd.spec import ADULT, Query

pytestmark = pytest.mark.gpu


def _boxes(n0, R, seed, span=6):
    g = np.random.default_rng(seed)
    lo = g.integers(-5, 20, size=(R, n0)).astype(np.float32)
    hi = lo + g.integers(0, span, size=(R, n0)).astype(np.float32)
    return torch.from_numpy(lo), torch.from_numpy(hi)


NETS = [(13, [16, 8]), (16, [150, 100, 50]), (30, [16, 16, 16]), (6, [3]), (20, [64, 32, 16, 8, 4]), (13, [100, 100])]


@pytest.mark.parametrize("n0,hidden", NETS)
@pytest.mark.parametrize("mode", ["ibp", "symbolic"])
def test_bounds_match_reference(cuda, n0, hidden, mode):
    m = random_mlp(n0, hidden, seed=n0 + len(hidden), bias_scale=0.3)
    lo, hi = _boxes(n0, 257, 1)
    cpu = Backend(m, "cpu")
    gpu = Backend(m, cuda)
    assert gpu.hip
    r_c = cpu.bounds(lo, hi, mode=mode, keep_layers=True)
    r_g = gpu.bounds(lo.to(cuda), hi.to(cuda), mode=mode, keep_layers=True)
    scale = (r_c.out_ub - r_c.out_lb).abs() + r_c.out_ub.abs() + 1e-3
    assert torch.allclose(r_g.out_lb.cpu(), r_c.out_lb, rtol=1e-4, atol=1e-4 * float(scale.max()))
    assert torch.allclose(r_g.out_ub.cpu(), r_c.out_ub, rtol=1e-4, atol=1e-4 * float(scale.max()))
    for a, b in zip(r_g.layer_ub, r_c.layer_ub):
        assert torch.allclose(a.cpu(), b, rtol=1e-4, atol=1e-3 * float(b.abs().max() + 1))
    if mode == "symbolic":
        # output forms: equal to the reference's up to rounding, except rows where a hidden
        # neuron's relaxation choice (chord / identity, lambda) flipped on a bound within
        # rounding of its threshold -- at most 1 % of the rows, and those rows' GPU forms must
        # still bound the network pointwise on the box's lattice points
        def close(g, c):
            tol = 1e-4 * (c.abs().max(dim=-1).values if c.dim() == 2 else c.abs()) + 1e-4 * (float(c.abs().max()) + 1)
            d = (g - c).abs()
            return (d <= tol[:, None]).all(dim=1) if d.dim() == 2 else d <= tol
        ok = torch.ones(lo.shape[0], dtype=torch.bool)
        for g_, c_ in ((r_g.Lc.cpu(), r_c.Lc), (r_g.Uc.cpu(), r_c.Uc), (r_g.L0.cpu(), r_c.L0), (r_g.U0.cpu(), r_c.U0)):
            ok &= close(g_, c_)
        bad = torch.nonzero(~ok).flatten()
        assert bad.numel() <= max(1, lo.shape[0] // 100), bad.numel()
        g = np.random.default_rng(0)
        for r in bad.tolist():
            pts = g.integers(lo[r].numpy().astype(np.int64), hi[r].numpy().astype(np.int64) + 1, size=(256, n0))
            z = m.logits(pts)
            X = torch.from_numpy(pts).double()
            up = X @ r_g.Uc[r].cpu().double() + float(r_g.U0[r]) + float(r_g.Ue[r])
            dn = X @ r_g.Lc[r].cpu().double() + float(r_g.L0[r]) - float(r_g.Le[r])
            assert (up.numpy() >= z - 1e-9).all() and (dn.numpy() <= z + 1e-9).all(), r


@pytest.mark.parametrize("n0,hidden", NETS[:4])
def test_bounds_sound_vs_bruteforce(cuda, n0, hidden):
    m = random_mlp(n0, hidden, seed=7, bias_scale=0.5)
    g = np.random.default_rng(3)
    gpu = Backend(m, cuda)
    for mode in ("ibp", "symbolic"):
        for _ in range(4):
            lo = g.integers(0, 5, size=(1, n0))
            hi = lo.copy()
            dims = g.choice(n0, size=min(n0, 4), replace=False)
            hi[0, dims] += g.integers(1, 3, size=dims.size)
            pts = np.array(list(itertools.product(*[range(a, b + 1) for a, b in zip(lo[0], hi[0])])))
            z = m.logits(pts)
            r = gpu.bounds(torch.tensor(lo, dtype=torch.float32, device=cuda),
                           torch.tensor(hi, dtype=torch.float32, device=cuda), mode=mode)
            assert float(r.out_lb[0]) <= z.min() + 1e-9
            assert float(r.out_ub[0]) >= z.max() - 1e-9


def test_forward_matches(cuda):
    for n0, hidden in NETS:
        m = random_mlp(n0, hidden, seed=11)
        x = torch.randint(-3, 30, (1000, n0)).float()
        z_ref = torch.from_numpy(m.logits(x.numpy().astype(np.float64))).float()
        be = Backend(m, cuda)
        z = be.forward(x.to(cuda)).cpu()
        err = be.forward_error(x.to(cuda)).cpu()
        assert torch.all((z - z_ref).abs() <= err + 1e-6)
        # dead mask
        dead = torch.rand(1000, m.n_neurons - 1) < 0.3
        zd = be.forward(x.to(cuda), dead.to(cuda)).cpu()
        zr = ref.forward([w.cpu() for w in be.ws], [b.cpu() for b in be.bs], x, dead)
        assert torch.allclose(zd, zr, rtol=1e-4, atol=1e-3)


def test_sim_kernel_matches_reference(cuda):
    """fa_sim_kernel against exact (fp64) evaluation of the same counter-hash samples.

    Activation counts may differ from the exact counts only by the number of samples whose
    pre-activation has a rigorous fp32 interval containing 0; the first flip (found + witness)
    must be the exact first flip unless a sample at or before it has an ambiguous logit sign."""
    from fairify_amd.engine.sim import simulate
    from fairify_amd.partition import Grid

    q = Query(("race",)).resolve(ADULT)
    grid = Grid.reference(ADULT, 10)
    ids = np.arange(0, 16000, 97)[:128]
    lo, hi = grid.decode(ids)
    values = q.pa_values(lo[0], hi[0])
    pairs = q.pa_pairs(values)
    m = get_model("AC-3")
    gpu = Backend(m, cuda)
    S, seed = 300, 5
    lo_t, hi_t, pid = torch.from_numpy(lo).float(), torch.from_numpy(hi).float(), torch.from_numpy(ids)
    b = simulate(gpu, q, lo_t.to(cuda), hi_t.to(cuda), pid.to(cuda), S, seed, torch.from_numpy(values).to(cuda),
                 torch.from_numpy(pairs).to(cuda), 0, 0)
    X = ref.sample_points(lo_t, hi_t, pid, S, seed)                       # [P, S, n0]
    P, n0 = lo.shape
    Xf = X.reshape(-1, n0)
    # exact activation counts and rigorous per-neuron pre-activation intervals
    acts = m.layer_outputs(Xf.numpy().astype(np.float64))               # per layer [R, w], post-ReLU, fp64
    iv = gpu.bounds(Xf.to(cuda), Xf.to(cuda), mode="ibp", keep_layers=True)
    cnt_b = b.counts.cpu().numpy()
    off = 0
    for l, w in enumerate(m.widths[:-1]):
        exact = (acts[l] > 0).reshape(P, S, w).sum(1)
        amb = ((iv.layer_lb[l] <= 0) & (iv.layer_ub[l] >= 0)).cpu().numpy().reshape(P, S, w).sum(1)
        assert (np.abs(cnt_b[:, off:off + w] - exact) <= amb).all()
        off += w
    # exact first flip per partition vs the kernel's
    V = len(values)
    XV = np.repeat(X.numpy()[:, :, None, :], V, axis=2)
    XV[:, :, :, list(q.pa_idx)] = values[None, None]
    XVf = XV.reshape(-1, n0)
    z = m.logits(XVf.astype(np.float64)).reshape(P, S, V)
    lb, ub = gpu.point_bounds(torch.from_numpy(XVf).float().to(cuda))
    amb = ((lb <= 0) & (ub >= 0)).cpu().numpy().reshape(P, S, V).any(axis=2)
    zi, zj = z[:, :, pairs[:, 0]], z[:, :, pairs[:, 1]]
    flip = ((zi < 0) & (zj > 0)) | ((zi > 0) & (zj < 0))                 # [P, S, Pp]
    found_b = b.found.cpu().numpy()
    wx, wxp = b.wit_x.cpu().numpy(), b.wit_xp.cpu().numpy()
    checked = 0
    for p in range(P):
        fl = np.nonzero(flip[p].reshape(-1))[0]
        key = int(fl[0]) if fl.size else S * len(pairs)
        s_key = key // len(pairs)
        if amb[p, :min(S, s_key + 1)].any():
            continue                                                    # sign ambiguous before the flip
        checked += 1
        assert bool(found_b[p]) == bool(fl.size)
        if fl.size:
            s, qi = divmod(key, len(pairs))
            assert np.array_equal(wx[p], XV[p, s, pairs[qi, 0]]) and np.array_equal(wxp[p], XV[p, s, pairs[qi, 1]])
    assert checked >= 0.9 * P


@pytest.mark.parametrize("relaxed", [False, True])
@pytest.mark.parametrize("bisect", [(0, 0), (16, 12)])
def test_sim_split_identical(cuda, monkeypatch, relaxed, bisect):
    """Sample tiles spread over several workgroups per partition (``fa_sim_kernel`` split +
    ``fa_sim_finalize_kernel``) give bit-identical counts, flags and witnesses, also with the
    boundary walk on (every split workgroup writes its own tiles of z0, which the walk reads)."""
    from fairify_amd.engine.sim import simulate
    from fairify_amd.ops import hip
    from fairify_amd.partition import Grid

    q = (Query(("sex",), ("age",), 2) if relaxed else Query(("race",))).resolve(ADULT)
    grid = Grid.reference(ADULT, 10)
    ids = np.arange(0, 16000, 401)[:37]
    lo, hi = grid.decode(ids)
    values = torch.from_numpy(q.pa_values(lo[0], hi[0])).to(cuda)
    pairs = torch.from_numpy(q.pa_pairs(values.cpu().numpy())).to(cuda)
    gpu = Backend(get_model("AC-3"), cuda)
    lo_t, hi_t = torch.from_numpy(lo).float().to(cuda), torch.from_numpy(hi).float().to(cuda)
    pid = torch.from_numpy(ids).to(cuda)
    monkeypatch.setattr(hip, "_SIM_BLOCKS_ENV", "dynamic")
    monkeypatch.setenv("FAIRIFY_SIM_BLOCKS", "2048")
    assert hip._sim_split(37, 4000) > 1
    out = []
    for flag in ("0", "2048"):
        monkeypatch.setenv("FAIRIFY_SIM_BLOCKS", flag)
        out.append(simulate(gpu, q, lo_t, hi_t, pid, 4000, 9, values, pairs, *bisect))
    a, b = out
    assert torch.equal(a.counts, b.counts)
    assert torch.equal(a.found, b.found)
    assert torch.equal(a.wit_x[a.found], b.wit_x[b.found])
    assert torch.equal(a.wit_xp[a.found], b.wit_xp[b.found])


def test_certify_matches_reference(cuda):
    from fairify_amd.engine.bab import BaBSolver, BaBConfig

    q = Query(("sex",), ("age",), 2).resolve(ADULT)
    m = get_model("AC-1")
    values = torch.tensor([[0], [1]])
    pairs = torch.from_numpy(q.pa_pairs(values.numpy()))
    lo, hi = _boxes(13, 64, 9, span=4)
    lo[:, 8] = 0
    hi[:, 8] = 1
    plo, phi = lo.clone(), hi.clone()
    plo[:, 0] -= 2
    phi[:, 0] += 2
    shared = torch.ones(13, dtype=torch.bool)
    shared[0] = False
    pa = torch.tensor([8])
    outs = []
    for dev in ("cpu", cuda):
        be = Backend(m, dev)
        rows = BaBSolver(be, q, BaBConfig())._rows
        rl, rh = rows(lo.to(dev), hi.to(dev), values.to(dev))
        pl, ph = rows(plo.to(dev), phi.to(dev), values.to(dev))
        rx = be.bounds(rl, rh)
        rxp = be.bounds(pl, ph)
        outs.append(be.pair_certify(rx, rxp, lo.to(dev), hi.to(dev), plo.to(dev), phi.to(dev), pairs.to(dev),
                                    values.to(dev), pa.to(dev), shared.to(dev), True))
    a, b = outs
    # the two sides round the symbolic forms differently (fp32, different summation orders):
    # scores agree to rounding, and open/closed may differ only where the score is ~0
    tol = 1e-3 * (a.score.abs() + 1)
    assert bool(((a.score - b.score.cpu()).abs() <= tol).all())
    differ = a.open_ != b.open_.cpu()
    assert bool((a.score[differ].abs() <= tol[differ]).all())


@pytest.mark.parametrize("model,relaxed", [("AC-3", True), ("AC-7", True), ("AC-3", False), ("AC-7", False),
                                           ("wide", True), ("wide", False)])
def test_sim_reg_kernel_relaxed_matches_tile_kernel(cuda, monkeypatch, model, relaxed):
    """The register-resident simulation kernel against the 64-row tile kernel, relaxed queries
    (x' rows with the tile kernel's RA offsets) and a plain multi-valued PA (race): activation
    counts equal up to rounding-ambiguous samples (compared in total), every witness is an exact
    violation within the pair constraints, and the found sets agree on >= 99 % of the
    partitions."""
    from fairify_amd.engine import exact
    from fairify_amd.engine.sim import simulate
    from fairify_amd.partition import Grid

    q = (Query(("sex",), ("age",), 5) if relaxed else Query(("race",))).resolve(ADULT)
    grid = Grid.reference(ADULT, 10)
    ids = np.arange(0, 16000, 37)[:256]
    lo, hi = grid.decode(ids)
    values = torch.from_numpy(q.pa_values(lo[0], hi[0])).to(cuda)
    pairs = torch.from_numpy(q.pa_pairs(values.cpu().numpy())).to(cuda)
    # "wide": a 150-100-50 net (BM-4's hidden shape, the 10-tile register kernel)
    m = random_mlp(13, [150, 100, 50], seed=0) if model == "wide" else get_model(model, weights="random", seed=0)
    gpu = Backend(m, cuda)
    lo_t, hi_t = torch.from_numpy(lo).float().to(cuda), torch.from_numpy(hi).float().to(cuda)
    pid = torch.from_numpy(ids).to(cuda)
    out = {}
    for flag in ("1", "0"):
        monkeypatch.setenv("FAIRIFY_SIM_REG", flag)
        out[flag] = simulate(gpu, q, lo_t, hi_t, pid, 1000, 3, values, pairs, 0, 0)
    a, b = out["1"], out["0"]
    ca, cb = a.counts.cpu().numpy().astype(np.int64), b.counts.cpu().numpy().astype(np.int64)
    assert np.abs(ca - cb).sum() <= 1e-3 * max(1, cb.sum())
    fa, fb = a.found.cpu().numpy(), b.found.cpu().numpy()
    assert (fa == fb).mean() >= 0.99
    idx = np.nonzero(fa)[0]
    X = a.wit_x.cpu().numpy()[idx].round().astype(np.int64)
    XP = a.wit_xp.cpu().numpy()[idx].round().astype(np.int64)
    assert exact.check_pair_constraints(X, XP, lo[idx], hi[idx], q.pa_idx, q.ra_idx, q.tau).all()
    assert exact.is_violation(m, X, XP).all()
