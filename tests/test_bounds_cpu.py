"""Reference bound propagation: soundness vs brute force, exact zeros, fp64 tightness."""
import itertools

import numpy as np
import pytest
import torch

from fairify_amd.models.mlp import random_mlp
from fairify_amd.ops import reference as ref
from fairify_amd.ops.backend import Backend


def _brute(m, lo, hi):
    pts = np.array(list(itertools.product(*[range(a, b + 1) for a, b in zip(lo, hi)])))
    return m.layer_outputs(pts)


@pytest.mark.parametrize("mode", ["ibp", "symbolic"])
@pytest.mark.parametrize("seed", range(6))
def test_bounds_sound(mode, seed):
    m = random_mlp(5, [8, 6, 4], seed=seed, bias_scale=0.5 if seed % 2 else 0.0)
    be = Backend(m)
    g = np.random.default_rng(seed)
    lo = g.integers(-3, 5, (6, 5))
    hi = lo + g.integers(0, 4, (6, 5))
    r = be.bounds(torch.tensor(lo).float(), torch.tensor(hi).float(), mode=mode, keep_layers=True)
    for k in range(6):
        outs = _brute(m, lo[k], hi[k])
        for l, o in enumerate(outs):
            pre = o if l == len(outs) - 1 else None
            if pre is not None:
                assert float(r.out_lb[k]) <= o[:, 0].min() and float(r.out_ub[k]) >= o[:, 0].max()
        # hidden post-activations are within relu(bounds)
        for l, o in enumerate(outs[:-1]):
            assert np.all(o <= np.maximum(r.layer_ub[l][k].numpy(), 0) + 1e-6)


def test_symbolic_tighter_than_ibp_on_average():
    m = random_mlp(13, [50, 50], seed=4, bias_scale=0.2)
    be = Backend(m)
    g = np.random.default_rng(1)
    lo = g.integers(0, 20, (64, 13))
    hi = lo + 3
    a = be.bounds(torch.tensor(lo).float(), torch.tensor(hi).float(), mode="ibp")
    b = be.bounds(torch.tensor(lo).float(), torch.tensor(hi).float(), mode="symbolic")
    assert float((b.out_ub - b.out_lb).mean()) < float((a.out_ub - a.out_lb).mean())
    assert torch.all(b.out_ub - b.out_lb <= a.out_ub - a.out_lb + 1e-4)


def test_exact_zero_kept_exact():
    # zero biases + non-positive output weights: N <= 0 exactly everywhere
    m = random_mlp(4, [6, 5], seed=2)
    m.weights[-1] = -np.abs(m.weights[-1])
    be = Backend(m)
    lo = torch.zeros(3, 4)
    hi = torch.full((3, 4), 7.0)
    r = be.bounds(lo, hi, mode="symbolic")
    assert torch.all(r.out_ub <= 0)


def test_fp64_matches_fp32_within_margin():
    m = random_mlp(6, [16, 8], seed=9, bias_scale=0.3)
    g = np.random.default_rng(2)
    lo = torch.tensor(g.integers(0, 50, (32, 6))).float()
    hi = lo + 5
    r32 = Backend(m).bounds(lo, hi)
    r64 = Backend(m, dtype=torch.float64).bounds(lo.double(), hi.double())
    assert torch.all(r32.out_lb <= r64.out_lb.float() + 1e-3)
    assert torch.all(r32.out_ub >= r64.out_ub.float() - 1e-3)


def test_rng_stream_is_stable():
    lo = torch.zeros(2, 3)
    hi = torch.tensor([[5.0, 9.0, 1.0], [100.0, 3.0, 7.0]])
    a = ref.sample_points(lo, hi, torch.tensor([3, 4]), 50, seed=11)
    b = ref.sample_points(lo, hi, torch.tensor([3, 4]), 50, seed=11)
    assert torch.equal(a, b)
    assert torch.all(a >= lo[:, None]) and torch.all(a <= hi[:, None])
    c = ref.sample_points_at(lo, hi, torch.tensor([3, 4]), torch.tensor([[7, 8], [0, 49]]), seed=11)
    assert torch.equal(c[0], a[0, 7:9]) and torch.equal(c[1, 1], a[1, 49])


def test_point_bounds_contain_exact_logits():
    """ops.reference.point_bounds (= csrc/points.hip arithmetic) brackets the exact logit and
    keeps exact zeros: a neuron provably dead at the point contributes exactly nothing."""
    import numpy as np
    import torch

    from fairify_amd.engine import exact
    from fairify_amd.models.mlp import random_mlp
    from fairify_amd.ops import reference as ref

    for seed, (n0, hidden) in enumerate([(13, [100, 100]), (6, [16, 8]), (20, [64, 32, 16, 8, 4])]):
        m = random_mlp(n0, hidden, seed=seed, bias_scale=0.5)
        x = torch.randint(-3, 40, (500, n0)).float()
        lb, ub = ref.point_bounds([torch.from_numpy(w) for w in m.weights], [torch.from_numpy(b) for b in m.biases], x)
        z = m.logits(x.numpy().astype(np.float64))
        assert np.all(lb.numpy() <= z) and np.all(z <= ub.numpy())
        assert float((ub - lb).max()) < 1e-2 * (1 + float(np.abs(z).max()))
        s = exact.exact_signs(m, x.numpy().astype(np.int64))
        assert np.all(s[lb.numpy() > 0] == 1) and np.all(s[ub.numpy() < 0] == -1)


@pytest.mark.parametrize("crown", [False, True])
def test_output_forms_pointwise_sound(crown):
    """The logit's linear forms (not only their concretisation) bound every lattice point:
    L(x) - eL <= N(x) <= U(x) + eU.  Regression: an unstable neuron whose upper form stays >= 0
    on the box must keep the identity upper relaxation (a chord from the form's minimum cut
    below relu(z)); the pair certificate evaluates the forms themselves."""
    import itertools

    from fairify_amd.models.mlp import random_mlp
    from fairify_amd.ops.backend import Backend

    g = np.random.default_rng(4)
    for seed in range(24):
        n0 = 13 if seed % 2 else 6
        hidden = [[64, 32, 16, 8, 4], [8, 8, 8], [5] * 6, [16, 8]][seed % 4]
        m = random_mlp(n0, hidden, seed=seed, bias_scale=0.0 if seed % 3 == 0 else 0.4)
        be = Backend(m, "cpu")
        lo = g.integers(0, 5, size=(1, n0))
        hi = lo.copy()
        dims = g.choice(n0, size=min(n0, 4), replace=False)
        hi[0, dims] += g.integers(1, 3, size=dims.size)
        pts = np.array(list(itertools.product(*[range(a, b + 1) for a, b in zip(lo[0], hi[0])])))
        z = m.logits(pts)
        r = be.bounds(torch.tensor(lo, dtype=torch.float32), torch.tensor(hi, dtype=torch.float32), mode="symbolic",
                      crown=crown)
        Lf = pts @ r.Lc[0].double().numpy() + float(r.L0[0]) - float(r.Le[0])
        Uf = pts @ r.Uc[0].double().numpy() + float(r.U0[0]) + float(r.Ue[0])
        assert np.all(z >= Lf - 1e-9), (seed, float((z - Lf).min()))
        assert np.all(z <= Uf + 1e-9), (seed, float((Uf - z).min()))
        assert z.min() >= float(r.out_lb[0]) and z.max() <= float(r.out_ub[0])


def _pre_activations(m, x):
    """Pre-activation of every layer at points x (fp64)."""
    h = np.asarray(x, dtype=np.float64)
    out = []
    for l, (w, b) in enumerate(zip(m.weights, m.biases)):
        z = h @ w.astype(np.float64) + b.astype(np.float64)
        out.append(z)
        h = np.maximum(z, 0)
    return out


@pytest.mark.parametrize("seed", range(8))
def test_refined_layer_bounds_sound_and_tighter(seed):
    """ref.crown_refine: every lattice point's hidden pre-activations lie inside the refined bounds,
    which are never looser than the forward ones; the output forms computed on them stay sound."""
    import itertools

    from fairify_amd.models.mlp import random_mlp
    from fairify_amd.ops import reference as ref
    from fairify_amd.ops.backend import Backend

    g = np.random.default_rng(100 + seed)
    n0 = 13 if seed % 2 else 6
    hidden = [[64, 32, 16, 8, 4], [10, 10, 10, 10], [16, 16, 16], [8, 8, 8]][seed % 4]
    m = random_mlp(n0, hidden, seed=seed, bias_scale=0.0 if seed % 3 == 0 else 0.4)
    be = Backend(m, "cpu")
    lo = g.integers(0, 5, size=(1, n0))
    hi = lo.copy()
    dims = g.choice(n0, size=min(n0, 4), replace=False)
    hi[0, dims] += g.integers(1, 4, size=dims.size)
    pts = np.array(list(itertools.product(*[range(a, b + 1) for a, b in zip(lo[0], hi[0])])))
    L_, H_ = torch.tensor(lo, dtype=torch.float32), torch.tensor(hi, dtype=torch.float32)
    fw = ref.bounds(be.ws, be.bs, L_, H_, mode="symbolic", keep_layers=True, unit=be.unit)
    rf = ref.crown_refine(be.ws, be.bs, L_, H_, fw, unit=be.unit)
    z = _pre_activations(m, pts)
    for k in range(len(hidden)):
        lb, ub = rf.layer_lb[k][0].double().numpy(), rf.layer_ub[k][0].double().numpy()
        assert np.all(z[k] >= lb - 1e-9) and np.all(z[k] <= ub + 1e-9), (seed, k)
        assert np.all(lb >= fw.layer_lb[k][0].double().numpy()) and np.all(ub <= fw.layer_ub[k][0].double().numpy())
    r = be.bounds(L_, H_, mode="symbolic", crown=True, refine=True)
    zl = m.logits(pts)
    Lf = pts @ r.Lc[0].double().numpy() + float(r.L0[0]) - float(r.Le[0])
    Uf = pts @ r.Uc[0].double().numpy() + float(r.U0[0]) + float(r.Ue[0])
    assert np.all(zl >= Lf - 1e-9) and np.all(zl <= Uf + 1e-9)
    assert zl.min() >= float(r.out_lb[0]) and zl.max() <= float(r.out_ub[0])


def test_refine_tightens_deep_net():
    """On the deep AC-7 shape the back-substituted bounds are strictly tighter somewhere."""
    from fairify_amd.models.mlp import random_mlp
    from fairify_amd.ops import reference as ref
    from fairify_amd.ops.backend import Backend

    m = random_mlp(13, [64, 32, 16, 8, 4], seed=7)
    be = Backend(m, "cpu")
    g = np.random.default_rng(3)
    lo = g.integers(0, 30, size=(32, 13)).astype(np.float32)
    hi = lo + g.integers(0, 10, size=(32, 13)).astype(np.float32)
    fw = ref.bounds(be.ws, be.bs, torch.from_numpy(lo), torch.from_numpy(hi), mode="symbolic", keep_layers=True)
    rf = ref.crown_refine(be.ws, be.bs, torch.from_numpy(lo), torch.from_numpy(hi), fw)
    gain = sum(float((rf.layer_ub[k] - rf.layer_lb[k]).sum()) for k in range(1, 5))
    base = sum(float((fw.layer_ub[k] - fw.layer_lb[k]).sum()) for k in range(1, 5))
    assert gain < 0.9 * base


@pytest.mark.parametrize("seed", range(6))
def test_backward_bounds_sound(seed):
    """ref.backward_bounds (no forward pass): sound on every lattice point (hidden pre-activations,
    forms, logit bounds).  (Not always as tight as forward + refine + output pass: the forward forms
    sometimes win at the output.)"""
    import itertools

    from fairify_amd.models.mlp import random_mlp
    from fairify_amd.ops import reference as ref
    from fairify_amd.ops.backend import Backend

    g = np.random.default_rng(200 + seed)
    n0 = 13 if seed % 2 else 6
    hidden = [[64, 32, 16, 8, 4], [10, 10, 10, 10], [16, 16, 16]][seed % 3]
    m = random_mlp(n0, hidden, seed=seed, bias_scale=0.0 if seed % 3 == 0 else 0.4)
    be = Backend(m, "cpu")
    lo = g.integers(0, 5, size=(1, n0))
    hi = lo.copy()
    dims = g.choice(n0, size=min(n0, 4), replace=False)
    hi[0, dims] += g.integers(1, 4, size=dims.size)
    pts = np.array(list(itertools.product(*[range(a, b + 1) for a, b in zip(lo[0], hi[0])])))
    L_, H_ = torch.tensor(lo, dtype=torch.float32), torch.tensor(hi, dtype=torch.float32)
    r = ref.backward_bounds(be.ws, be.bs, L_, H_, unit=be.unit)
    z = _pre_activations(m, pts)
    for k in range(len(hidden)):
        assert np.all(z[k] >= r.layer_lb[k][0].double().numpy() - 1e-9)
        assert np.all(z[k] <= r.layer_ub[k][0].double().numpy() + 1e-9)
    zl = m.logits(pts)
    Lf = pts @ r.Lc[0].double().numpy() + float(r.L0[0]) - float(r.Le[0])
    Uf = pts @ r.Uc[0].double().numpy() + float(r.U0[0]) + float(r.Ue[0])
    assert np.all(zl >= Lf - 1e-9) and np.all(zl <= Uf + 1e-9)
    assert zl.min() >= float(r.out_lb[0]) and zl.max() <= float(r.out_ub[0])
