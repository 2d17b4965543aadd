"""fa_beta_kernel (csrc/beta.hip) against the PyTorch reference of the same op (ops/beta.py:level_ref)
and against brute-force lattice enumeration; the beta BaB stage on the device."""
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
from fairify_amd.ops import hip
from fairify_amd.ops.backend import Backend
from fairify_amd.partition import processing_order

from test_beta_bab import _brute_pair, _setup, _true_min

pytestmark = pytest.mark.gpu


def _params(R, NH, seed, neg):
    g = torch.Generator().manual_seed(seed)
    al = [torch.rand(R, NH, generator=g) for _ in range(2)]
    be_ = [torch.rand(R, NH, generator=g) * (2 if neg else 1) - (1 if neg else 0) for _ in range(2)]
    t = torch.rand(R, generator=g)
    return al, be_, t


def _both(cuda, seed, iters, neg=False, lookahead=0, fix=0.3, widths=(6, 5, 4), pgap=False):
    m, ws, bs, pa, lo, hi, va, vb, bnd, ph = _setup(seed, widths=widths, fix=fix)
    R = lo.shape[0]
    w = [x.shape[1] for x in ws[:-1]]
    NH = sum(w)
    al, be_, t = _params(R, NH, seed, neg)
    lr = dict(lr_a=0.1, lr_b=0.5, lr_t=0.1)
    cpu = [x.clone() for x in (al[0], al[1], be_[0], be_[1], t)]
    lr_ = B.level_ref(ws, bs, w, lo, hi, pa, va, vb, bnd[0][0], bnd[0][1], bnd[1][0], bnd[1][1], ph[0], ph[1], *cpu,
                      iters=iters, lookahead=lookahead, beta_pos=not neg, pgap=pgap, **lr)
    gb = Backend(m, cuda)
    d = lambda x: x.to(cuda).contiguous()  # noqa: E731
    gpu = [d(x.clone()) for x in (al[0], al[1], be_[0], be_[1], t)]
    lg = hip.beta_level(gb, d(lo), d(hi), pa, d(va), d(vb), d(bnd[0][0]), d(bnd[0][1]), d(bnd[1][0]), d(bnd[1][1]),
                        d(ph[0]), d(ph[1]), *gpu, iters=iters, lookahead=lookahead, beta_pos=not neg, pgap=pgap,
                        **lr)
    torch.cuda.synchronize()
    return m, w, (lo, hi, va, vb, ph, pa), lr_, lg, cpu, [x.cpu() for x in gpu]


@pytest.mark.parametrize("seed", [0, 1, 2])
@pytest.mark.parametrize("neg", [False, True])
def test_beta_kernel_rigorous_bound_matches_reference(cuda, seed, neg):
    """iters = 0: both evaluate the same parameters -- the fp64 bounds agree to rounding-term
    size, and the kernel's bound is below every phase-feasible lattice point."""
    m, w, (lo, hi, va, vb, ph, pa), lr_, lg, _, gp = _both(cuda, seed, 0, neg)
    bg = lg.bound.cpu()
    fin = torch.isfinite(lr_.bound)
    assert bool((torch.isfinite(bg) == fin).all())
    assert torch.allclose(bg[fin], lr_.bound[fin], rtol=1e-9, atol=1e-9)
    assert torch.equal(lg.xstar.cpu()[fin], lr_.xstar[fin])
    t = gp[4]
    for r in range(lo.shape[0]):
        tm = _true_min(m, lo[r].numpy(), hi[r].numpy(), pa, va[r].numpy(), vb[r].numpy(), ph[0][r].numpy(),
                       ph[1][r].numpy(), float(t[r]), w)
        assert float(bg[r]) <= tm


@pytest.mark.parametrize("seed", [3, 4, 5])
def test_beta_kernel_split_and_binit_match_reference(cuda, seed):
    """iters = 0, no look-ahead: the kernel branches on a neuron the reference scores (within
    fp32-vs-fp64 rounding) as best, or both split the same input dim; the child multipliers match."""
    m, w, _, lr_, lg, _, _ = _both(cuda, seed, 0, fix=0.1)
    sg, sr = lg.split.cpu(), lr_.split
    sc = lr_.scores
    for r in range(sg.numel()):
        if not torch.isfinite(lr_.bound[r]) or lr_.bound[r] >= 0:
            # closed (an empty region, or the bound proves it): never branched, the kernel skips
            # scores and look-ahead and returns LEAF
            assert float(lg.bound[r].cpu()) >= 0
            continue
        if sr[r] >= 0:
            assert sg[r] >= 0, (r, int(sg[r]), int(sr[r]))
            best = float(sc[r].max())
            assert float(sc[r, sg[r]]) >= best * (1 - 1e-4) - 1e-9, (r, int(sg[r]), int(sr[r]),
                                                                     float(sc[r, sg[r]]), best)
        else:
            assert int(sg[r]) == int(sr[r]), (r, int(sg[r]), int(sr[r]))
    nb = (sg == sr) & (sr >= 0) & (lr_.bound < 0)
    assert torch.allclose(lg.binit.cpu()[nb], lr_.binit[nb], rtol=1e-4, atol=1e-6)


@pytest.mark.parametrize("seed", [5, 8, 12])      # seeds with open nodes the reference splits on a neuron
def test_beta_kernel_primal_gap_split_matches_reference(cuda, seed):
    """pgap, a few optimisation steps (fp32 trajectories still agree): the kernel splits a neuron the
    reference's primal-gap scores rank best (within fp32 summation noise), or both split the same
    input dim; the rigorous bounds agree and the child multipliers reproduce the node's relaxation."""
    m, w, _, lr_, lg, _, _ = _both(cuda, seed, 3, fix=0.1, pgap=True)
    sg, sr, sc = lg.split.cpu(), lr_.split, lr_.scores
    fin = torch.isfinite(lr_.bound)
    assert torch.allclose(lg.bound.cpu()[fin], lr_.bound[fin], rtol=1e-5, atol=1e-5)
    n_neu = 0
    for r in range(sg.numel()):
        if not torch.isfinite(lr_.bound[r]) or lr_.bound[r] >= 0:
            continue
        if sr[r] >= 0:
            n_neu += 1
            assert sg[r] >= 0, (r, int(sg[r]), int(sr[r]))
            best = float(sc[r].max())
            assert float(sc[r, sg[r]]) >= best * (1 - 1e-3) - 1e-5, (r, int(sg[r]), int(sr[r]))
        else:
            assert int(sg[r]) == int(sr[r]), (r, int(sg[r]), int(sr[r]))
    assert n_neu > 0


@pytest.mark.parametrize("seed", [3, 4])
@pytest.mark.parametrize("look", [0, 4])
def test_beta_kernel_optimises_soundly(cuda, seed, look):
    m, w, (lo, hi, va, vb, ph, pa), lr_, lg, _, gp = _both(cuda, seed, 60, lookahead=look, fix=0.15)
    m0, _, _, lr0, lg0, _, _ = _both(cuda, seed, 0, lookahead=look, fix=0.15)
    bg, b0 = lg.bound.cpu(), lg0.bound.cpu()
    fin = torch.isfinite(b0)
    # the start parameters here are random: 60 steps never end below them and usually well above
    assert bool((bg[fin] >= b0[fin] - 1e-5 * (1 + b0[fin].abs())).all())
    assert bool((bg[fin] > b0[fin] + 1e-3).any())
    # fp32 trajectories differ from the reference's only by summation order: same ball-park
    assert float((bg[fin] - lr_.bound[fin]).abs().max()) < 0.05 * (1 + float(lr_.bound[fin].abs().max()))
    t = gp[4]
    for r in range(lo.shape[0]):
        tm = _true_min(m, lo[r].numpy(), hi[r].numpy(), pa, va[r].numpy(), vb[r].numpy(), ph[0][r].numpy(),
                       ph[1][r].numpy(), float(t[r]), w)
        assert float(bg[r]) <= tm


def test_beta_kernel_wide_layers(cuda):
    """Layers wider than a wave (lanes loop over neurons) and deeper nets."""
    m, w, (lo, hi, va, vb, ph, pa), lr_, lg, _, gp = _both(cuda, 7, 0, widths=(100, 70, 3))
    fin = torch.isfinite(lr_.bound)
    assert torch.allclose(lg.bound.cpu()[fin], lr_.bound[fin], rtol=1e-9, atol=1e-9)


@pytest.mark.parametrize("widths", [(6, 5, 4), (150, 100, 50)])
def test_beta_kernel_weight_placement_is_bitwise_neutral(cuda, monkeypatch, widths):
    """The three weight placements (both copies in LDS, forward copy in LDS, both read from L2 --
    BM-4's 150-wide layer runs the last) run the same arithmetic: optimised parameters, rigorous
    bounds, splits and vertices are bitwise equal."""
    outs = []
    # (both copies of the wide net's weights do not fit in LDS together)
    for wm in (("1", "0", "2") if max(widths) < 100 else ("0", "2")):
        monkeypatch.setenv("FAIRIFY_BETA_WM", wm)
        _, _, _, _, lg, _, gp = _both(cuda, 9, 20, fix=0.2, widths=widths, pgap=True)
        outs.append((lg, gp))
    monkeypatch.delenv("FAIRIFY_BETA_WM")
    (l0, g0) = outs[0]
    for lg, gp in outs[1:]:
        assert torch.equal(lg.bound.cpu(), l0.bound.cpu())
        assert torch.equal(lg.split.cpu(), l0.split.cpu())
        assert torch.equal(lg.xstar.cpu(), l0.xstar.cpu())
        for a, b in zip(gp, g0):
            assert torch.equal(a, b)


@pytest.mark.parametrize("seed,branch,native", [(3, "kernel", True), (6, "kernel", True), (3, "pgap", True),
                                                (6, "pgap", True), (3, "kernel", False), (6, "pgap", False)])
def test_beta_bab_gpu_matches_bruteforce(cuda, seed, branch, native):
    """Decided verdicts equal lattice enumeration: the native level loop (csrc/beta_runtime.cpp) and the
    torch loop over the same kernel."""
    pre = presets.get("src/AC-sex")
    grid, q = pre.grid(), pre.resolved()
    ids = processing_order(grid, 0)[:24]
    lo, hi = grid.decode(ids)
    hi = np.minimum(hi, lo + 1)
    m = random_mlp(13, [8, 6, 4], seed=seed, bias_scale=0.5)
    sol = BetaBaBSolver(Backend(m, cuda), q, BetaConfig(node_budget=256, iters=20, root_iters=40, branch=branch,
                                                        native=native))
    res = sol.solve(lo, hi, m)
    assert bool(sol.stats.get("native")) == native
    pa = q.pa_idx[0]
    assert (res.status != UNKNOWN).mean() > 0.5
    for k in range(len(ids)):
        if res.status[k] != UNKNOWN:
            assert (res.status[k] == SAT) == _brute_pair(m, lo[k], hi[k], pa), k
    sat = np.nonzero(res.status == SAT)[0]
    if sat.size:
        assert exact.is_violation(m, res.cex_x[sat], res.cex_xp[sat]).all()


def test_beta_gpu_closes_trained_ac7_residue(cuda):
    pre = presets.get("src/AC-sex")
    grid, q = pre.grid(), pre.resolved()
    m = get_model("AC-7", weights="zoo", seed=0)
    ids = np.array([12596, 4387, 6769, 6543, 4330, 13901, 956, 7121, 4516, 5716, 5527, 14939])
    lo, hi = grid.decode(ids)
    res = BetaBaBSolver(Backend(m, cuda), q, BetaConfig(node_budget=400)).solve(lo, hi, m)
    assert (res.status == UNSAT).sum() >= 10, res.status
    assert (res.status == SAT).sum() == 0              # the verified LP proves all 12 UNSAT


def _true_min_rx(m, lo, hi, plo, phi, pa, ra, va, vb, phA, phB, t, tau=None):
    """min of t N(x, va) - (1 - t) N(x', vb) over lattice x in the box and x' = x except its RA dims,
    which range over [plo, phi] independently (the bound drops the tau tie, so it must hold on this
    superset), restricted to points satisfying both copies' phases."""
    import itertools

    X = np.array(list(itertools.product(*[range(int(a), int(b) + 1) for a, b in zip(lo, hi)])), dtype=np.float64)
    D = np.array(list(itertools.product(*[range(int(plo[r]), int(phi[r]) + 1) for r in ra])), dtype=np.float64)

    def run(h, ph):
        ok = np.ones(len(h), bool)
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
        return h[:, 0], ok

    xa = X.copy()
    xa[:, pa] = va
    fa, oka = run(xa, phA)
    best = np.inf
    for dv in D:
        xb = X.copy()
        xb[:, pa] = vb
        xb[:, ra] = dv
        fb, okb = run(xb, phB)
        ok = oka & okb
        if tau is not None:         # the tie |x_r - x'_r| <= tau (a bound using its multipliers)
            ok &= (np.abs(X[:, ra] - dv[None]) <= tau).all(1)
        if ok.any():
            best = min(best, float((t * fa - (1 - t) * fb)[ok].min()))
    return best


@pytest.mark.parametrize("seed,tie", [(0, False), (2, False), (0, True), (3, True)])
def test_beta_kernel_relaxed_matches_reference_and_is_sound(cuda, seed, tie):
    m, ws, bs, pa, lo, hi, va, vb, bnd, ph = _setup(seed)
    R, n0 = lo.shape
    w = [x.shape[1] for x in ws[:-1]]
    NH = sum(w)
    ra = [2]
    ram = torch.zeros(n0, dtype=torch.bool)
    ram[ra] = True
    plo, phi = lo.clone(), hi.clone()
    plo[:, ra] -= 1
    phi[:, ra] += 1
    # copy B's partition bounds over x''s box (RA dims widened), as the solver supplies them
    rl, rh = plo.clone(), phi.clone()
    rl[:, pa] = vb
    rh[:, pa] = vb
    rb = Backend(m).bounds(rl, rh, keep_layers=True)
    bnd = [bnd[0], (torch.cat(rb.layer_lb, 1)[:, :NH].float(), torch.cat(rb.layer_ub, 1)[:, :NH].float())]
    al, be_, t = _params(R, NH, seed, False)
    lr = dict(lr_a=0.1, lr_b=0.5, lr_t=0.1)
    cpu = [x.clone() for x in (al[0], al[1], be_[0], be_[1], t)]
    tau = 1.0
    g = torch.Generator().manual_seed(seed + 100)
    gP = torch.rand(R, n0, generator=g) * ram.float()
    gM = torch.rand(R, n0, generator=g) * ram.float()
    rxc = (ram, plo, phi, tau, gP.clone(), gM.clone()) if tie else (ram, plo, phi)
    lr_ = B.level_ref(ws, bs, w, lo, hi, pa, va, vb, bnd[0][0], bnd[0][1], bnd[1][0], bnd[1][1], ph[0], ph[1], *cpu,
                      iters=0, rx=rxc, **lr)
    d = lambda x: x.to(cuda).contiguous()  # noqa: E731
    gpu = [d(x.clone()) for x in (al[0], al[1], be_[0], be_[1], t)]
    rxg = (ram, d(plo), d(phi), tau, d(gP), d(gM)) if tie else (ram, d(plo), d(phi))
    lg = hip.beta_level(Backend(m, cuda), d(lo), d(hi), pa, d(va), d(vb), d(bnd[0][0]), d(bnd[0][1]), d(bnd[1][0]),
                        d(bnd[1][1]), d(ph[0]), d(ph[1]), *gpu, iters=0, rx=rxg, **lr)
    torch.cuda.synchronize()
    bg = lg.bound.cpu()
    fin = torch.isfinite(lr_.bound)
    assert torch.allclose(bg[fin], lr_.bound[fin], rtol=1e-9, atol=1e-9)
    assert torch.equal(lg.xpstar.cpu()[fin][:, ra], lr_.xpstar[fin][:, ra])
    for r in range(R):
        tm = _true_min_rx(m, lo[r].numpy(), hi[r].numpy(), plo[r].numpy(), phi[r].numpy(), pa, ra, va[r].numpy(),
                          vb[r].numpy(), ph[0][r].numpy(), ph[1][r].numpy(), float(t[r]), tau if tie else None)
        assert float(bg[r]) <= tm, (r, float(bg[r]), tm)


@pytest.mark.parametrize("seed,tau,branch,native", [(21, 2, "kernel", True), (24, 3, "kernel", True),
                                                    (21, 2, "pgap", True), (21, 2, "kernel", False)])
def test_beta_bab_gpu_relaxed_matches_bruteforce(cuda, seed, tau, branch, native):
    """GPU twin of test_beta_bab.py::test_beta_bab_relaxed_matches_bruteforce: relaxed queries through
    the HIP kernel (x' RA boxes, tie multipliers, both orientations, exact confirmation); every
    decided verdict equals enumeration of all (x, x') pairs."""
    from fairify_amd.spec import ADULT, Query
    from test_beta_bab import _relaxed_truth

    q = Query(pa=("sex",), ra=("age",), tau=tau).resolve(ADULT)
    grid = presets.get("src/AC-sex").grid()
    ids = processing_order(grid, 0)[:16]
    lo, hi = grid.decode(ids)
    hi = np.minimum(hi, lo + 1)
    pa, ra = q.pa_idx[0], q.ra_idx[0]
    m = random_mlp(13, [8, 6, 4], seed=seed, bias_scale=0.5)
    sol = BetaBaBSolver(Backend(m, cuda), q, BetaConfig(node_budget=512, iters=20, root_iters=40, branch=branch,
                                                        native=native))
    res = sol.solve(lo, hi, m)
    assert bool(sol.stats.get("native")) == native
    decided = 0
    for k in range(len(ids)):
        if res.status[k] == UNKNOWN:
            continue
        decided += 1
        truth = _relaxed_truth(m, lo[k], hi[k], pa, ra, tau)
        assert (res.status[k] == SAT) == truth, k
        if res.status[k] == SAT:
            ok = exact.check_pair_constraints(res.cex_x[k:k + 1], res.cex_xp[k:k + 1], lo[k:k + 1], hi[k:k + 1],
                                              q.pa_idx, q.ra_idx, q.tau)
            assert ok[0] and exact.is_violation(m, res.cex_x[k:k + 1], res.cex_xp[k:k + 1])[0]
    assert decided >= 0.5 * len(ids)


@pytest.mark.parametrize("seed", [0, 2])
def test_beta_kernel_orientation_sign_matches_reference(cuda, seed):
    """osg = -1 rows through the kernel: the rigorous bounds equal the reference's (which equal the
    negated network's, tests/test_beta_bab.py::test_orientation_sign_equals_negated_network)."""
    m, ws, bs, pa, lo, hi, va, vb, bnd, ph = _setup(seed)
    R = lo.shape[0]
    w = [x.shape[1] for x in ws[:-1]]
    NH = sum(w)
    al, be_, t = _params(R, NH, seed, False)
    osg = torch.tensor([1, -1] * (R // 2) + [1] * (R % 2), dtype=torch.int8)
    lr = dict(lr_a=0.1, lr_b=0.5, lr_t=0.1)
    cpu = [x.clone() for x in (al[0], al[1], be_[0], be_[1], t)]
    lr_ = B.level_ref(ws, bs, w, lo, hi, pa, va, vb, bnd[0][0], bnd[0][1], bnd[1][0], bnd[1][1], ph[0], ph[1], *cpu,
                      iters=0, osg=osg, **lr)
    d = lambda x: x.to(cuda).contiguous()  # noqa: E731
    gpu = [d(x.clone()) for x in (al[0], al[1], be_[0], be_[1], t)]
    lg = hip.beta_level(Backend(m, cuda), d(lo), d(hi), pa, d(va), d(vb), d(bnd[0][0]), d(bnd[0][1]), d(bnd[1][0]),
                        d(bnd[1][1]), d(ph[0]), d(ph[1]), *gpu, iters=0, osg=d(osg), **lr)
    torch.cuda.synchronize()
    fin = torch.isfinite(lr_.bound)
    assert torch.allclose(lg.bound.cpu()[fin], lr_.bound[fin], rtol=1e-9, atol=1e-9)


@pytest.mark.parametrize("relaxed", [False, True])
def test_beta_native_agrees_with_torch_loop(cuda, relaxed):
    """The native runtime and the torch loop run the same kernel on the same trees: wherever both
    decide a partition they agree, and neither decides much less than the other (their level / budget
    granularity differs: whole BFS levels vs FIFO batches)."""
    from fairify_amd.spec import ADULT, Query

    pre = presets.get("src/AC-sex")
    grid = pre.grid()
    q = Query(pa=("sex",), ra=("age",), tau=2).resolve(ADULT) if relaxed else pre.resolved()
    ids = processing_order(grid, 0)[:48]
    lo, hi = grid.decode(ids)
    hi = np.minimum(hi, lo + 2)
    m = random_mlp(13, [16, 8, 4], seed=9, bias_scale=0.5)
    be = Backend(m, cuda)
    out = {}
    for native in (True, False):
        sol = BetaBaBSolver(be, q, BetaConfig(node_budget=256, iters=24, root_iters=48, native=native))
        out[native] = sol.solve(lo, hi, m).status
        assert bool(sol.stats.get("native")) == native
    a, b = out[True], out[False]
    both = (a != UNKNOWN) & (b != UNKNOWN)
    assert both.sum() >= 0.5 * len(ids)
    assert bool((a[both] == b[both]).all())
    assert abs(int((a != UNKNOWN).sum()) - int((b != UNKNOWN).sum())) <= 0.1 * len(ids)


def test_beta_kernel_crossed_bounds_without_fixed_phase_give_no_bound(cuda):
    """Kernel twin of test_beta_bab.py::test_crossed_bounds_without_a_fixed_phase_give_no_bound: crossed
    bounds with no fixed phase -> NaN (the native loop stops the partition), through a fixed phase ->
    +inf (empty region)."""
    m, ws, bs, pa, lo, hi, va, vb, bnd, ph = _setup(3, fix=0.0)
    R = lo.shape[0]
    NH = bnd[0][0].shape[1]
    LBA, UBA = bnd[0][0].clone(), bnd[0][1].clone()
    LBA[0, 2] = UBA[0, 2] + 1.0
    phA = ph[0].clone()
    LBA[1, 3] = UBA[1, 3] + 1.0
    phA[1, 3] = 1
    gb = Backend(m, cuda)
    d = lambda x: x.to(cuda).contiguous()  # noqa: E731
    g = torch.Generator().manual_seed(0)
    al = [d(torch.rand(R, NH, generator=g)) for _ in range(2)]
    be_ = [d(torch.zeros(R, NH)) for _ in range(2)]
    lg = hip.beta_level(gb, d(lo), d(hi), pa, d(va), d(vb), d(LBA), d(UBA), d(bnd[1][0]), d(bnd[1][1]), d(phA),
                        d(ph[1]), al[0], al[1], be_[0], be_[1], d(torch.full((R,), 0.5)), iters=0, lr_a=0.1,
                        lr_b=0.5, lr_t=0.1)
    b = lg.bound.cpu()
    assert torch.isnan(b[0])
    assert float(b[1]) == float("inf")
    assert bool(torch.isfinite(b[2:]).all())
