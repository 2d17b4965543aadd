"""Register-resident symbolic bound kernel (csrc/symbolic.hip) vs the PyTorch reference.

Covers every template shape the dispatcher can pick (column tiles NT = 1..3, row tiles
TM = 1..10), folded degenerate input dims (the node-row expansion of the BaB runtime), forced
dead neurons, and soundness against brute-force enumeration.  Run on a real MI355X.
"""
import itertools

import numpy as np
import pytest
import torch

from fairify_amd.models.mlp import random_mlp
from fairify_amd.ops.backend import Backend

pytestmark = pytest.mark.gpu

# (n0, hidden, folded dims): NT = ceil((n0 - |fold| + 4) / 16), TM = ceil(max width / 16)
SHAPES = [
    (13, [100, 100], (8,)),            # AC-4 with PA folded: NT=1, TM=7
    (13, [64, 32, 16, 8, 4], (8,)),    # AC-7: NT=1, TM=4
    (13, [50], (7,)),                  # AC-3: NT=1, TM=4
    (13, [5] * 9, (8,)),               # AC-12: NT=1, TM=1
    (13, [16, 8], ()),                 # no fold: NT=2, TM=1
    (20, [50], (11,)),                 # GC-1: NT=2, TM=4
    (16, [64, 16], (0,)),              # BM-1: NT=2, TM=4
    (30, [16, 16, 16], (20,)),         # DF: NT=3, TM=2
    (6, [16, 8], (3,)),                # CP-1: NT=1, TM=1
    (12, [32, 32], (3, 4)),            # two folded dims
    (16, [150, 100, 50], (0,)),        # BM-4: NT=2, TM=10 (scratch-backed operand tiles)
    (13, [150, 20], (8,)),             # NT=1, TM=10
    # packed narrow networks (PG boxes per MFMA tile, block-diagonal weights)
    (13, [3, 3, 3, 3], (8,)),          # AC-9: PG=5
    (13, [5, 5], (7,)),                # AC-8: PG=3
    (6, [4, 4, 4], (3,)),              # PG=4
    (13, [8, 8, 8], (8,)),             # PG=2
    (13, [5, 1, 5], (8,)),             # PG=3 with a 1-wide hidden layer
]


def _boxes(n0, R, seed, fold, span=6):
    g = np.random.default_rng(seed)
    lo = g.integers(-5, 20, size=(R, n0)).astype(np.float32)
    hi = lo + g.integers(0, span, size=(R, n0)).astype(np.float32)
    for d in fold:
        hi[:, d] = lo[:, d]
    return torch.from_numpy(lo), torch.from_numpy(hi)


@pytest.mark.parametrize("n0,hidden,fold", SHAPES)
def test_symbolic_kernel_matches_reference(cuda, n0, hidden, fold):
    m = random_mlp(n0, hidden, seed=n0 + 3 * len(hidden), bias_scale=0.3)
    lo, hi = _boxes(n0, 300, 5, fold)
    cpu = Backend(m, "cpu")
    gpu = Backend(m, cuda)
    assert gpu.hip
    rc = cpu.bounds(lo, hi, mode="symbolic", keep_layers=True)
    rg = gpu.bounds(lo.to(cuda), hi.to(cuda), mode="symbolic", keep_layers=True, fold=fold)
    scale = float(((rc.out_ub - rc.out_lb).abs() + rc.out_ub.abs()).max() + 1e-3)
    assert torch.allclose(rg.out_lb.cpu(), rc.out_lb, rtol=1e-4, atol=1e-4 * scale)
    assert torch.allclose(rg.out_ub.cpu(), rc.out_ub, rtol=1e-4, atol=1e-4 * scale)
    for a, b in zip(rg.layer_ub, rc.layer_ub):
        assert torch.allclose(a.cpu(), b, rtol=1e-4, atol=1e-3 * float(b.abs().max() + 1))
    for a, b in zip(rg.layer_lb, rc.layer_lb):
        assert torch.allclose(a.cpu(), b, rtol=1e-4, atol=1e-3 * float(b.abs().max() + 1))
    # folded dims move into the constant: compare the forms evaluated on the folded value
    keep = [d for d in range(n0) if d not in fold]
    for C_g, c_g, C_c, c_c in ((rg.Lc, rg.L0, rc.Lc, rc.L0), (rg.Uc, rg.U0, rc.Uc, rc.U0)):
        C_g, c_g = C_g.cpu(), c_g.cpu()
        tol = 1e-4 * float(C_c.abs().max() + 1)
        assert torch.allclose(C_g[:, keep], C_c[:, keep], rtol=1e-4, atol=tol)
        if fold:
            assert float(C_g[:, list(fold)].abs().max()) == 0.0
        folded_c = c_c + (C_c[:, list(fold)] * lo[:, list(fold)]).sum(1) if fold else c_c
        assert torch.allclose(c_g, folded_c, rtol=1e-4, atol=1e-4 * float(folded_c.abs().max() + 1))
    # dead flags agree except on neurons whose bound is within rounding of 0
    assert rg.dead is not None


@pytest.mark.parametrize("n0,hidden,fold,dead", [
    (13, [64, 32, 16, 8, 4], (8,), False), (13, [64, 32, 16, 8, 4], (8,), True),    # AC-7
    (13, [64, 32, 16, 8, 4], (), False),                                            # AC-7, NT=2
    (16, [64, 32, 16, 8, 4], (0,), False), (16, [64, 32, 16, 8, 4], (0,), True),    # BM-8
    (13, [64, 64], (8,), False), (13, [50], (7,), False),                           # AC-5, AC-3
    (13, [100, 100], (8,), False), (13, [100, 100], (8,), True), (13, [100], (8,), False)])   # AC-4, AC-2
def test_shaped_symbolic_kernel_is_bitwise_the_generic_one(cuda, monkeypatch, n0, hidden, fold, dead):
    """The compile-time-shape instances (csrc/symbolic.hip SymShape: layer loop unrolled, widths
    constant) run the generic kernel's arithmetic: every output is bitwise equal."""
    m = random_mlp(n0, hidden, seed=n0 + len(hidden), bias_scale=0.3)
    lo, hi = _boxes(n0, 700, 9, fold)
    dm = (torch.rand(700, m.n_neurons - 1, generator=torch.Generator().manual_seed(1)) < 0.2).to(cuda) if dead else None
    be = Backend(m, cuda)
    outs = []
    for shaped in ("1", "0"):
        monkeypatch.setenv("FAIRIFY_SYM_SHAPED", shaped)
        outs.append(be.bounds(lo.to(cuda), hi.to(cuda), mode="symbolic", keep_layers=True, fold=fold, dead=dm))
    a, b = outs
    for x, y in [(a.out_lb, b.out_lb), (a.out_ub, b.out_ub), (a.Lc, b.Lc), (a.Uc, b.Uc), (a.L0, b.L0), (a.U0, b.U0),
                 (a.Le, b.Le), (a.Ue, b.Ue)] + \
            list(zip(a.layer_lb, b.layer_lb)) + list(zip(a.layer_ub, b.layer_ub)):
        assert torch.equal(x.cpu(), y.cpu())
    if a.dead is not None:
        assert torch.equal(a.dead.cpu(), b.dead.cpu())


@pytest.mark.parametrize("n0,hidden,fold", [SHAPES[0], SHAPES[3], SHAPES[5], SHAPES[7], SHAPES[12]])
def test_symbolic_kernel_forced_dead(cuda, n0, hidden, fold):
    m = random_mlp(n0, hidden, seed=11, bias_scale=0.3)
    lo, hi = _boxes(n0, 128, 7, fold)
    dead = torch.rand(128, m.n_neurons - 1, generator=torch.Generator().manual_seed(0)) < 0.3
    rc = Backend(m, "cpu").bounds(lo, hi, mode="symbolic", dead=dead)
    rg = Backend(m, cuda).bounds(lo.to(cuda), hi.to(cuda), mode="symbolic", dead=dead.to(cuda), fold=fold)
    scale = float(((rc.out_ub - rc.out_lb).abs() + rc.out_ub.abs()).max() + 1e-3)
    assert torch.allclose(rg.out_lb.cpu(), rc.out_lb, rtol=1e-4, atol=1e-4 * scale)
    assert torch.allclose(rg.out_ub.cpu(), rc.out_ub, rtol=1e-4, atol=1e-4 * scale)


@pytest.mark.parametrize("n0,hidden", [(13, [100, 100]), (13, [16, 8]), (20, [50]), (6, [16, 8]), (13, [5, 5, 5]),
                                       (6, [3, 3])])
def test_symbolic_kernel_sound_vs_bruteforce(cuda, n0, hidden):
    m = random_mlp(n0, hidden, seed=3, bias_scale=0.5)
    g = np.random.default_rng(4)
    be = Backend(m, cuda)
    pa = n0 // 2
    for _ in range(6):
        lo = g.integers(0, 5, size=(1, n0))
        hi = lo.copy()
        dims = [d for d in g.choice(n0, size=min(n0, 5), replace=False) if d != pa]
        hi[0, dims] += g.integers(1, 3, size=len(dims))
        pts = np.array(list(itertools.product(*[range(a, b + 1) for a, b in zip(lo[0], hi[0])])))
        z = m.logits(pts)
        r = be.bounds(torch.tensor(lo, dtype=torch.float32, device=cuda),
                      torch.tensor(hi, dtype=torch.float32, device=cuda), mode="symbolic", fold=(pa,))
        assert float(r.out_lb[0]) <= z.min() + 1e-9
        assert float(r.out_ub[0]) >= z.max() - 1e-9


def test_native_bab_agrees_with_torch_bab_ac4(cuda):
    """AC-4 (the TM=7 shape) through the native BaB runtime (node-row expansion, PA folded) vs
    the tensor BaB (explicit rows, nothing folded): decided verdicts must agree."""
    import os

    from fairify_amd import presets
    from fairify_amd.engine.bab import BaBConfig, BaBSolver
    from fairify_amd.models.zoo import get_model
    from fairify_amd.partition import processing_order

    pre = presets.get("src/AC-sex")
    grid = pre.grid()
    q = pre.resolved()
    ids = processing_order(grid, 0)[:192]
    lo, hi = grid.decode(ids)
    m = get_model("AC-4", weights="random", seed=0)
    be = Backend(m, cuda)
    nat = BaBSolver(be, q, BaBConfig(node_budget=1024)).solve(lo, hi, m)
    os.environ["FAIRIFY_TORCH_BAB"] = "1"
    try:
        tor = BaBSolver(be, q, BaBConfig(node_budget=1024)).solve(lo, hi, m)
    finally:
        del os.environ["FAIRIFY_TORCH_BAB"]
    decided = (nat.status != 0) & (tor.status != 0)
    assert np.array_equal(nat.status[decided], tor.status[decided])
    assert decided.mean() > 0.5


@pytest.mark.parametrize("n0,hidden", [(13, [100, 100]), (13, [64, 32, 16, 8, 4]), (6, [16, 8]), (20, [50]),
                                       (16, [150, 100, 50])])
def test_point_kernel_matches_reference(cuda, n0, hidden):
    from fairify_amd.ops import reference as ref

    m = random_mlp(n0, hidden, seed=n0, bias_scale=0.5)
    x = torch.randint(-3, 40, (1000, n0)).float()
    dead = torch.rand(1000, m.n_neurons - 1, generator=torch.Generator().manual_seed(1)) < 0.2
    be = Backend(m, cuda)
    for d in (None, dead):
        lb, ub = be.point_bounds(x.to(cuda), None if d is None else d.to(cuda))
        rl, ru = ref.point_bounds([torch.from_numpy(w) for w in m.weights], [torch.from_numpy(b) for b in m.biases],
                                  x, d)
        z = ref.forward([torch.from_numpy(w).double() for w in m.weights],
                        [torch.from_numpy(b).double() for b in m.biases], x.double(), d)
        assert torch.all(lb.cpu().double() <= z) and torch.all(z <= ub.cpu().double())
        # every width up to 160 (BM-4's 150 included) runs the point kernel, the reference's arithmetic
        tol = 1e-4 * (1 + float(z.abs().max()))
        assert torch.allclose(lb.cpu(), rl, atol=tol) and torch.allclose(ub.cpu(), ru, atol=tol)


CROWN_SHAPES = [(13, [100, 100]), (13, [64, 32, 16, 8, 4]), (13, [5] * 9), (16, [150, 100, 50]), (20, [50]),
                (30, [16, 16, 16]), (6, [3])]


@pytest.mark.parametrize("n0,hidden", CROWN_SHAPES)
def test_crown_kernel_matches_reference(cuda, n0, hidden):
    """csrc/crown.hip vs ops/reference.py:crown_output on the same forward-pass layer bounds."""
    from fairify_amd.ops import reference as ref

    m = random_mlp(n0, hidden, seed=11 + n0 + len(hidden), bias_scale=0.3)
    lo, hi = _boxes(n0, 257, 9, ())
    cpu = Backend(m, "cpu")
    gpu = Backend(m, cuda)
    rc = cpu.bounds(lo, hi, mode="symbolic", crown=True)
    rg = gpu.bounds(lo.to(cuda), hi.to(cuda), mode="symbolic", crown=True)
    scale = float(((rc.out_ub - rc.out_lb).abs() + rc.out_ub.abs()).max() + 1e-3)
    assert torch.allclose(rg.out_lb.cpu(), rc.out_lb, rtol=1e-3, atol=1e-3 * scale)
    assert torch.allclose(rg.out_ub.cpu(), rc.out_ub, rtol=1e-3, atol=1e-3 * scale)
    # the backward bounds never loosen the forward ones
    rf = gpu.bounds(lo.to(cuda), hi.to(cuda), mode="symbolic")
    assert bool((rg.out_lb >= rf.out_lb).all()) and bool((rg.out_ub <= rf.out_ub).all())


@pytest.mark.parametrize("n0,hidden", CROWN_SHAPES[:3] + [(5, [8, 8, 8])])
def test_crown_kernel_sound_vs_bruteforce(cuda, n0, hidden):
    m = random_mlp(n0, hidden, seed=3 + len(hidden), bias_scale=0.0 if len(hidden) > 2 else 0.5)
    g = np.random.default_rng(4)
    gpu = Backend(m, cuda)
    for _ in range(6):
        lo = g.integers(0, 5, size=(1, n0))
        hi = lo.copy()
        dims = g.choice(n0, size=min(n0, 4), replace=False)
        hi[0, dims] += g.integers(1, 3, size=dims.size)
        pts = np.array(list(itertools.product(*[range(a, b + 1) for a, b in zip(lo[0], hi[0])])))
        z = m.logits(pts)
        r = gpu.bounds(torch.tensor(lo, dtype=torch.float32, device=cuda),
                       torch.tensor(hi, dtype=torch.float32, device=cuda), mode="symbolic", crown=True)
        Lf = pts @ r.Lc[0].double().cpu().numpy() + float(r.L0[0]) - float(r.Le[0])
        Uf = pts @ r.Uc[0].double().cpu().numpy() + float(r.U0[0]) + float(r.Ue[0])
        assert np.all(z >= Lf - 1e-9) and np.all(z <= Uf + 1e-9)
        assert z.min() >= float(r.out_lb[0]) and z.max() <= float(r.out_ub[0])


@pytest.mark.parametrize("name", ["AC-8", "AC-12", "AC-9"])
def test_packed_native_bab_matches_bruteforce(cuda, name):
    """Narrow nets through the native BaB (packed symbolic kernel, node-row expansion): every
    decided verdict equals exhaustive enumeration of the partition's lattice points."""
    from fairify_amd import presets
    from fairify_amd.engine.bab import SAT, UNSAT, BaBConfig, BaBSolver
    from fairify_amd.models.zoo import get_model
    from fairify_amd.partition import processing_order

    pre = presets.get("src/AC-sex")
    grid, q = pre.grid(), pre.resolved()
    m = get_model(name, weights="random", seed=1)
    be = Backend(m, cuda)
    ids = processing_order(grid, 0)[:64]
    lo, hi = grid.decode(ids)
    # shrink the boxes so enumeration stays cheap (<= 2 values per free dim)
    hi = np.minimum(hi, lo + 1)
    res = BaBSolver(be, q, BaBConfig(node_budget=4096)).solve(lo, hi, m)
    pa = q.pa_idx[0]
    for k in range(len(ids)):
        pts = np.array(list(itertools.product(*[range(a, b + 1) for a, b in zip(lo[k], hi[k])])))
        pts = pts[pts[:, pa] == lo[k, pa]] if lo[k, pa] == hi[k, pa] else pts
        z0 = m.logits(np.where(np.arange(m.n_in) == pa, 0, pts))
        z1 = m.logits(np.where(np.arange(m.n_in) == pa, 1, pts))
        # the query's post-condition: strictly opposite logit signs (an exact 0 is neither)
        viol = bool((((z0 > 0) & (z1 < 0)) | ((z0 < 0) & (z1 > 0))).any())
        if res.status[k] == SAT:
            assert viol, k
        elif res.status[k] == UNSAT:
            assert not viol, k


@pytest.mark.parametrize("hidden2", [False, True])
def test_cr_kernel_error_slack_only_on_error_columns(cuda, hidden2):
    """Centre/radius multi-tile kernel (DF shape: 30 inputs, PA SEX_2 folded -> NT=3, TM=2).

    Round-2 advisor finding: the 2 gamma |Q| recombination slack meant for the error columns 1 / 3
    also landed on coefficient columns 17 / 19 of the second column tile, moving a zero upper
    coefficient by +e.  cdim[13] = BILL_AMT6 has a negative domain (-339 603 ..), so e * |x|
    pulled the upper form below the network.  The net is built so that the logit's upper form has
    an exactly zero coefficient on dim 13 next to a large radius: hidden neuron 0 is unstable with
    the lambda = 0 lower relaxation, the next weight is -1.  Bounds must enclose the brute-force
    logits of every lattice point of the box."""
    from fairify_amd.models.mlp import MLP

    n0 = 30
    W1 = np.zeros((n0, 16), np.float32)
    b1 = np.zeros(16, np.float32)
    W1[13, 0], b1[0] = 1.0, 339543.0            # z1 in [-60, 40] over the box: lambda = 0, s = 0.4
    if hidden2:
        W2 = np.zeros((16, 16), np.float32)
        b2 = np.zeros(16, np.float32)
        W2[0, 0], b2[0] = -1.0, 10.0             # z2 = 10 - relu(z1) in [-30, 10]
        W3 = np.zeros((16, 1), np.float32)
        W3[0, 0] = 1.0
        m = MLP([W1, W2, W3], [b1, b2, np.zeros(1, np.float32)], name="cr-probe2")
    else:
        W2 = np.zeros((16, 1), np.float32)
        W2[0, 0] = -1.0
        m = MLP([W1, W2], [b1, np.zeros(1, np.float32)], name="cr-probe")
    lo = np.zeros((4, n0), np.float32)
    hi = np.zeros((4, n0), np.float32)
    lo[:, 13], hi[:, 13] = -339603.0, -339503.0
    lo[:, 20] = hi[:, 20] = np.array([0, 1, 0, 1], np.float32)
    be = Backend(m, cuda)
    r = be.bounds(torch.from_numpy(lo).to(cuda), torch.from_numpy(hi).to(cuda), mode="symbolic", fold=(20,))
    pts = np.zeros((101, n0))
    pts[:, 13] = np.arange(-339603, -339502)
    z = m.logits(pts)
    assert float(r.out_ub.max()) >= z.max() and float(r.out_lb.min()) <= z.min()
    for k in range(4):
        Lf = pts @ r.Lc[k].double().cpu().numpy() + float(r.L0[k]) - float(r.Le[k])
        Uf = pts @ r.Uc[k].double().cpu().numpy() + float(r.U0[k]) + float(r.Ue[k])
        assert np.all(z >= Lf - 1e-9) and np.all(z <= Uf + 1e-9), k
