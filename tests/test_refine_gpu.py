"""Back-substituted hidden-layer bounds on the MI355X: csrc/refine.hip vs ops/reference.py:crown_refine
on the same forward-pass bounds, soundness against lattice enumeration, and native-BaB verdicts with
the refined bounds against brute force."""
import itertools

import numpy as np
import pytest
import torch

from fairify_amd.models.mlp import random_mlp
from fairify_amd.ops import reference as ref
from fairify_amd.ops.backend import Backend

pytestmark = pytest.mark.gpu

SHAPES = [(13, [64, 32, 16, 8, 4]), (13, [10, 10, 10, 10]), (16, [150, 100, 50]), (30, [16, 16, 16]),
          (13, [5] * 9), (20, [100, 60, 30])]


def _boxes(n0, R, seed, span=6):
    g = np.random.default_rng(seed)
    lo = g.integers(-5, 20, size=(R, n0)).astype(np.float32)
    hi = lo + g.integers(0, span, size=(R, n0)).astype(np.float32)
    return torch.from_numpy(lo), torch.from_numpy(hi)


@pytest.mark.parametrize("n0,hidden", SHAPES)
def test_refine_kernel_matches_reference(cuda, n0, hidden):
    """Same forward bounds in (the GPU's), kernel vs fp64 reference out: the kernel's rounding terms
    are the reference's up to the GEMM gamma convention, so the bounds agree to ~1e-4 relative,
    and the kernel never loosens a forward bound."""
    m = random_mlp(n0, hidden, seed=5 + n0 + len(hidden), bias_scale=0.3)
    lo, hi = _boxes(n0, 301, 3)
    gpu = Backend(m, cuda)
    rg = gpu.bounds(lo.to(cuda), hi.to(cuda), mode="symbolic", keep_layers=True)
    fw_lb = [t.clone() for t in rg.layer_lb]
    fw_ub = [t.clone() for t in rg.layer_ub]
    # fp64 reference on the GPU's forward bounds
    fw = ref.BoundResult(out_lb=rg.out_lb.cpu().double(), out_ub=rg.out_ub.cpu().double(),
                         layer_lb=[t.cpu().double() for t in fw_lb], layer_ub=[t.cpu().double() for t in fw_ub])
    ws = [w.double() for w in Backend(m, "cpu").ws]
    bs = [b.double() for b in Backend(m, "cpu").bs]
    rr = ref.crown_refine(ws, bs, lo.double(), hi.double(), fw, unit=ref.FP32_UNIT)
    from fairify_amd.ops import hip as H

    H.refine(gpu, lo.to(cuda), hi.to(cuda), rg)
    torch.cuda.synchronize()
    for k in range(len(hidden)):
        glb, gub = rg.layer_lb[k].cpu().double(), rg.layer_ub[k].cpu().double()
        scale = float((fw.layer_ub[k] - fw.layer_lb[k]).abs().max() + fw.layer_ub[k].abs().max() + 1e-3)
        assert torch.allclose(glb, rr.layer_lb[k], rtol=1e-4, atol=1e-4 * scale), k
        assert torch.allclose(gub, rr.layer_ub[k], rtol=1e-4, atol=1e-4 * scale), k
        assert bool((glb >= fw_lb[k].cpu().double()).all()) and bool((gub <= fw_ub[k].cpu().double()).all())
    if len(hidden) >= 3:       # it does refine something on the deep shapes
        w0 = sum(float((fw_ub[k] - fw_lb[k]).sum()) for k in range(1, len(hidden)))
        w1 = sum(float((rg.layer_ub[k] - rg.layer_lb[k]).sum()) for k in range(1, len(hidden)))
        assert w1 < w0


@pytest.mark.parametrize("n0,hidden", [(13, [64, 32, 16, 8, 4]), (5, [8, 8, 8]), (6, [16, 16, 16, 16])])
def test_refine_kernel_sound_vs_bruteforce(cuda, n0, hidden):
    m = random_mlp(n0, hidden, seed=9 + len(hidden), bias_scale=0.0 if len(hidden) > 3 else 0.5)
    g = np.random.default_rng(8)
    gpu = Backend(m, cuda)
    for _ in range(6):
        lo = g.integers(0, 5, size=(1, n0))
        hi = lo.copy()
        dims = g.choice(n0, size=min(n0, 4), replace=False)
        hi[0, dims] += g.integers(1, 3, size=dims.size)
        pts = np.array(list(itertools.product(*[range(a, b + 1) for a, b in zip(lo[0], hi[0])])))
        L_ = torch.tensor(lo, dtype=torch.float32, device=cuda)
        H_ = torch.tensor(hi, dtype=torch.float32, device=cuda)
        r = gpu.bounds(L_, H_, mode="symbolic", crown=True, refine=True)
        h = pts.astype(np.float64)
        for k, (w, b) in enumerate(zip(m.weights[:-1], m.biases[:-1])):
            z = h @ w.astype(np.float64) + b.astype(np.float64)
            assert np.all(z >= r.layer_lb[k][0].double().cpu().numpy() - 1e-9)
            assert np.all(z <= r.layer_ub[k][0].double().cpu().numpy() + 1e-9)
            h = np.maximum(z, 0)
        zl = m.logits(pts)
        Lf = pts @ r.Lc[0].double().cpu().numpy() + float(r.L0[0]) - float(r.Le[0])
        Uf = pts @ r.Uc[0].double().cpu().numpy() + float(r.U0[0]) + float(r.Ue[0])
        assert np.all(zl >= Lf - 1e-9) and np.all(zl <= Uf + 1e-9)
        assert zl.min() >= float(r.out_lb[0]) and zl.max() <= float(r.out_ub[0])


@pytest.mark.parametrize("name", ["AC-7", "AC-11"])
def test_refined_native_bab_matches_bruteforce(cuda, name):
    """The native BaB with refined bounds (BaBConfig.refine='on'): every decided verdict equals
    exhaustive enumeration of the partition's lattice points."""
    from fairify_amd import presets
    from fairify_amd.engine.bab import SAT, UNSAT, BaBConfig, BaBSolver
    from fairify_amd.models.zoo import get_model
    from fairify_amd.partition import processing_order

    pre = presets.get("src/AC-sex")
    grid, q = pre.grid(), pre.resolved()
    m = get_model(name, weights="random", seed=1)
    be = Backend(m, cuda)
    ids = processing_order(grid, 0)[:96]
    lo, hi = grid.decode(ids)
    hi = np.minimum(hi, lo + 1)
    res = BaBSolver(be, q, BaBConfig(node_budget=4096, refine="on")).solve(lo, hi, m)
    pa = q.pa_idx[0]
    n_dec = 0
    for k in range(len(ids)):
        pts = np.array(list(itertools.product(*[range(a, b + 1) for a, b in zip(lo[k], hi[k])])))
        z0 = m.logits(np.where(np.arange(m.n_in) == pa, 0, pts))
        z1 = m.logits(np.where(np.arange(m.n_in) == pa, 1, pts))
        viol = bool((((z0 > 0) & (z1 < 0)) | ((z0 < 0) & (z1 > 0))).any())
        if res.status[k] == SAT:
            assert viol, k
            n_dec += 1
        elif res.status[k] == UNSAT:
            assert not viol, k
            n_dec += 1
    assert n_dec == len(ids)


def test_refine_cuts_bab_nodes_on_ac7(cuda):
    """The point of the stage: on full AC-7 partitions the refined bounds decide at least as many
    partitions with fewer BaB nodes than the forward bounds."""
    from fairify_amd import presets
    from fairify_amd.engine.bab import SAT, UNSAT, BaBConfig, BaBSolver
    from fairify_amd.models.zoo import get_model
    from fairify_amd.partition import processing_order

    pre = presets.get("src/AC-sex")
    grid, q = pre.grid(), pre.resolved()
    m = get_model("AC-7", weights="random", seed=0)
    be = Backend(m, cuda)
    ids = processing_order(grid, 0)[:2048]
    lo, hi = grid.decode(ids)
    out = {}
    for mode in ("off", "on"):
        r = BaBSolver(be, q, BaBConfig(node_budget=2048, refine=mode)).solve(lo, hi, m)
        out[mode] = (int(np.isin(r.status, (SAT, UNSAT)).sum()), int(r.nodes.sum()))
    assert out["on"][0] >= out["off"][0], out
    assert out["on"][1] < out["off"][1], out


@pytest.mark.parametrize("n0,hidden", SHAPES)
def test_backward_kernel_matches_reference_and_is_sound(cuda, n0, hidden):
    """Mode FULL (one launch, no forward pass) vs ref.backward_bounds in fp64 with fp32 error terms --
    the kernel charges the MFMA GEMM convention gamma(2n+1) where the reference charges gamma(n+1),
    and with no forward intervals to intersect the difference compounds over 5 layers (AC-7 shape:
    ~6e-4 on bounds of ~8), hence 1e-3 relative; sound against sampled lattice points (hidden
    pre-activations, logit forms, logit bounds)."""
    m = random_mlp(n0, hidden, seed=21 + n0 + len(hidden), bias_scale=0.3)
    lo, hi = _boxes(n0, 203, 7)
    gpu = Backend(m, cuda)
    rg = gpu.bounds(lo.to(cuda), hi.to(cuda), mode="backward")
    ws = [w.double() for w in Backend(m, "cpu").ws]
    bs = [b.double() for b in Backend(m, "cpu").bs]
    rr = ref.backward_bounds(ws, bs, lo.double(), hi.double(), unit=ref.FP32_UNIT)
    def close(a, b, scale):
        # >= 99 % of the entries within 1e-3 relative; the rest (a neuron whose stability differs
        # between fp32 and fp64 by a rounding hair switches its relaxation, and without forward
        # intervals the difference propagates) within 5 % of the layer's scale
        d = (a - b).abs()
        tol = 1e-3 * scale + 1e-3 * b.abs()
        return float((d <= tol).double().mean()) >= 0.99 and float(d.max()) <= 0.05 * scale

    for k in range(len(hidden)):
        scale = float((rr.layer_ub[k] - rr.layer_lb[k]).abs().max() + rr.layer_ub[k].abs().max() + 1e-3)
        assert close(rg.layer_lb[k].cpu().double(), rr.layer_lb[k], scale), k
        assert close(rg.layer_ub[k].cpu().double(), rr.layer_ub[k], scale), k
    scale = float((rr.out_ub - rr.out_lb).abs().max() + rr.out_ub.abs().max() + 1e-3)
    assert close(rg.out_lb.cpu().double(), rr.out_lb, scale)
    assert close(rg.out_ub.cpu().double(), rr.out_ub, scale)
    g = np.random.default_rng(5)
    X = (lo[:, None, :] + torch.from_numpy(g.random((lo.shape[0], 64, n0))).float()
         * (hi - lo + 1)[:, None, :]).floor().clamp(max=hi[:, None, :]).numpy().astype(np.float64)
    h = X
    for k, (w, b) in enumerate(zip(m.weights[:-1], m.biases[:-1])):
        z = h @ w.astype(np.float64) + b.astype(np.float64)
        assert np.all(z >= rg.layer_lb[k].double().cpu().numpy()[:, None, :] - 1e-9)
        assert np.all(z <= rg.layer_ub[k].double().cpu().numpy()[:, None, :] + 1e-9)
        h = np.maximum(z, 0)
    zl = m.logits(X.reshape(-1, n0)).reshape(X.shape[0], -1)
    Lf = np.einsum("rsn,rn->rs", X, rg.Lc.double().cpu().numpy()) + (rg.L0 - rg.Le).double().cpu().numpy()[:, None]
    Uf = np.einsum("rsn,rn->rs", X, rg.Uc.double().cpu().numpy()) + (rg.U0 + rg.Ue).double().cpu().numpy()[:, None]
    assert np.all(zl >= Lf - 1e-9) and np.all(zl <= Uf + 1e-9)
    assert np.all(zl >= rg.out_lb.double().cpu().numpy()[:, None]) and np.all(zl <= rg.out_ub.double().cpu().numpy()[:, None])


@pytest.mark.parametrize("name", ["AC-7", "AC-4"])
def test_backward_native_bab_matches_bruteforce(cuda, name):
    """The native BaB bounding with back-substitution alone (BaBConfig.refine='full') decides like
    exhaustive enumeration."""
    from fairify_amd import presets
    from fairify_amd.engine.bab import SAT, UNSAT, BaBConfig, BaBSolver
    from fairify_amd.models.zoo import get_model
    from fairify_amd.partition import processing_order

    pre = presets.get("src/AC-sex")
    grid, q = pre.grid(), pre.resolved()
    m = get_model(name, weights="random", seed=2)
    be = Backend(m, cuda)
    ids = processing_order(grid, 0)[:96]
    lo, hi = grid.decode(ids)
    hi = np.minimum(hi, lo + 1)
    res = BaBSolver(be, q, BaBConfig(node_budget=4096, refine="full")).solve(lo, hi, m)
    pa = q.pa_idx[0]
    for k in range(len(ids)):
        pts = np.array(list(itertools.product(*[range(a, b + 1) for a, b in zip(lo[k], hi[k])])))
        z0 = m.logits(np.where(np.arange(m.n_in) == pa, 0, pts))
        z1 = m.logits(np.where(np.arange(m.n_in) == pa, 1, pts))
        viol = bool((((z0 > 0) & (z1 < 0)) | ((z0 < 0) & (z1 > 0))).any())
        assert res.status[k] in (SAT, UNSAT), k
        assert (res.status[k] == SAT) == viol, k


@pytest.mark.parametrize("n0,hidden", [(13, [64, 32, 16, 8, 4]), (13, [10, 10, 10, 10]), (16, [150, 100, 50])])
def test_fused_refine_crown_equals_refine_then_crown(cuda, n0, hidden):
    """The runtime's one-launch refine + logit pass (refine_crown) gives the forms and logit bounds
    of the two launches it replaces (refine, then crown.hip), to rounding-order differences."""
    from fairify_amd.ops import ext
    from fairify_amd.ops import hip as H

    m = random_mlp(n0, hidden, seed=31 + len(hidden), bias_scale=0.3)
    lo, hi = _boxes(n0, 257, 11)
    gpu = Backend(m, cuda)
    L_, H_ = lo.to(cuda), hi.to(cuda)
    two = gpu.bounds(L_, H_, mode="symbolic", crown=True, refine=True)
    one = gpu.bounds(L_, H_, mode="symbolic", keep_layers=True)
    ext().refine_crown(H._net(gpu), gpu.flat.data_ptr(), L_.contiguous().data_ptr(), H_.contiguous().data_ptr(), 0,
                       L_.shape[0], one.out_lb.data_ptr(), one.out_ub.data_ptr(), one.Lc.data_ptr(), one.L0.data_ptr(),
                       one.Le.data_ptr(), one.Uc.data_ptr(), one.U0.data_ptr(), one.Ue.data_ptr(),
                       one.lay_lb_full.data_ptr(), one.lay_ub_full.data_ptr(), H._stream(cuda))
    torch.cuda.synchronize()
    scale = float((two.out_ub - two.out_lb).abs().max().cpu() + two.out_ub.abs().max().cpu() + 1e-3)
    assert torch.allclose(one.out_lb, two.out_lb, rtol=1e-4, atol=1e-4 * scale)
    assert torch.allclose(one.out_ub, two.out_ub, rtol=1e-4, atol=1e-4 * scale)


@pytest.mark.parametrize("seed", [0, 1, 2])
def test_phase_refine_sound_and_infeasibility_exact(cuda, seed):
    """Phase-aware refinement (ReLU-phase BaB rows): on every lattice point of the box whose
    activation pattern satisfies the row's fixed phases, each hidden pre-activation lies in the
    refined bounds; a row flagged infeasible has no such point."""
    from fairify_amd.ops import hip as H

    torch.manual_seed(seed)
    n0, hidden = 5, [12, 10, 8]
    m = random_mlp(n0, hidden, seed=seed)
    be = Backend(m, cuda)
    g = torch.Generator().manual_seed(seed)
    R = 48
    lo = torch.randint(0, 3, (R, n0), generator=g).float()
    hi = lo + torch.randint(0, 3, (R, n0), generator=g).float()
    Nh = sum(hidden)
    phase = torch.zeros(R, Nh, dtype=torch.int8)
    for r in range(R):          # fix a few neurons per row, either phase
        idx = torch.randperm(Nh, generator=g)[:4]
        phase[r, idx] = (torch.randint(0, 2, (4,), generator=g) * 2 - 1).to(torch.int8)
    lo_d, hi_d, ph_d = lo.to(cuda), hi.to(cuda), phase.to(cuda)
    res = H.bounds(be, lo_d, hi_d, mode="symbolic", keep_layers=True, phase=ph_d)
    res = H.refine(be, lo_d, hi_d, res, phase=ph_d)
    llb, lub = res.lay_lb_full.cpu().double(), res.lay_ub_full.cpu().double()
    infeas = res.infeasible.cpu()
    cpu = Backend(m, "cpu")
    W = [w.double() for w in cpu.ws]
    B = [b.double() for b in cpu.bs]
    n_feas_rows = 0
    for r in range(R):
        pts = torch.tensor(list(itertools.product(*[range(int(a), int(b) + 1) for a, b in zip(lo[r], hi[r])])),
                           dtype=torch.float64)
        h, zs = pts, []
        for l in range(len(hidden)):
            z = h @ W[l] + B[l]
            zs.append(z)
            h = torch.relu(z)
        Z = torch.cat(zs, 1)                                     # [pts, Nh]
        ph = phase[r].double()
        ok = torch.all(((ph > 0) & (Z < 0)).logical_not() & ((ph < 0) & (Z > 0)).logical_not(), dim=1)
        if infeas[r]:
            assert not ok.any(), r
            continue
        if not ok.any():
            continue
        n_feas_rows += 1
        Zf = Z[ok]
        # rigorous bounds: no slack beyond the fp64 evaluation of the lattice points themselves
        # (the kernel's fp32 rounding terms are ~1e-6 relative; fp64 noise here is ~1e-15)
        assert torch.all(Zf >= llb[r, :Nh] - 1e-9), r
        assert torch.all(Zf <= lub[r, :Nh] + 1e-9), r
    assert n_feas_rows > 0


def test_backward_kernel_with_dead_mask(cuda):
    """Mode FULL with a forced-dead mask (heuristically pruned nets): every neuron gets finite bounds
    that match ref.backward_bounds on the same mask, and the masked neurons are reported dead (the
    kernel used to leave them at -inf / +inf and alive)."""
    n0, hidden = 6, [16, 12, 8]
    m = random_mlp(n0, hidden, seed=77, bias_scale=0.3)
    lo, hi = _boxes(n0, 64, 3)
    R, NH = lo.shape[0], sum(hidden)
    g = torch.Generator().manual_seed(3)
    dead = (torch.rand(R, NH, generator=g) < 0.2).to(torch.uint8)
    gpu = Backend(m, cuda)
    rg = gpu.bounds(lo.to(cuda), hi.to(cuda), mode="backward", dead=dead.to(cuda))
    ws = [w.double() for w in Backend(m, "cpu").ws]
    bs = [b.double() for b in Backend(m, "cpu").bs]
    rr = ref.backward_bounds(ws, bs, lo.double(), hi.double(), dead=dead.bool(), unit=ref.FP32_UNIT)
    for k in range(len(hidden)):
        a, b = rg.layer_lb[k].cpu().double(), rr.layer_lb[k]
        assert torch.isfinite(a).all() and torch.isfinite(rg.layer_ub[k].cpu()).all(), k
        scale = float((rr.layer_ub[k] - b).abs().max() + rr.layer_ub[k].abs().max() + 1e-3)
        assert float((a - b).abs().max()) <= 0.05 * scale, k
    assert bool((rg.dead.cpu() | ~dead.bool()).all())           # masked -> dead
    assert bool((rr.dead | ~dead.bool()).all())
    assert float((rg.dead.cpu() == rr.dead).double().mean()) >= 0.99


@pytest.mark.parametrize("mode", ["refine", "refine_crown", "backward"])
def test_global_weight_refine_bitwise_equals_staged(cuda, monkeypatch, mode):
    """BM-4's shape (16-150-100-50): the back-substitution kernel reading W from the global
    backward-order block (8 box rows per workgroup) gives bitwise the bounds of the LDS-staged
    kernel (1 row per workgroup): same arithmetic, same order, per column."""
    from fairify_amd.ops import ext
    from fairify_amd.ops import hip as H

    m = random_mlp(16, [150, 100, 50], seed=41, bias_scale=0.3)
    lo, hi = _boxes(16, 203, 13)
    gpu = Backend(m, cuda)
    L_, H_ = lo.to(cuda), hi.to(cuda)
    outs = []
    for kb in ("64", "0"):                     # default (global weights) / never
        monkeypatch.setenv("FAIRIFY_REFINE_WG_KB", kb)
        if mode == "backward":
            r = gpu.bounds(L_, H_, mode="backward", keep_layers=True)
            outs.append([r.out_lb, r.out_ub, r.Lc, r.Uc, r.L0, r.U0, r.Le, r.Ue, torch.cat(r.layer_lb, 1),
                         torch.cat(r.layer_ub, 1)])
            continue
        r = gpu.bounds(L_, H_, mode="symbolic", keep_layers=True)
        if mode == "refine":
            H.refine(gpu, L_, H_, r)
        else:
            ext().refine_crown(H._net(gpu), gpu.flat.data_ptr(), L_.contiguous().data_ptr(),
                               H_.contiguous().data_ptr(), 0, L_.shape[0], r.out_lb.data_ptr(), r.out_ub.data_ptr(),
                               r.Lc.data_ptr(), r.L0.data_ptr(), r.Le.data_ptr(), r.Uc.data_ptr(), r.U0.data_ptr(),
                               r.Ue.data_ptr(), r.lay_lb_full.data_ptr(), r.lay_ub_full.data_ptr(), H._stream(cuda))
        torch.cuda.synchronize()
        outs.append([r.out_lb, r.out_ub, r.Lc, r.Uc, r.lay_lb_full, r.lay_ub_full])
    for a, b in zip(*outs):
        assert torch.equal(a, b)


@pytest.mark.parametrize("n0,hidden", [(13, [64, 32, 16, 8, 4]), (16, [64, 32, 16, 8, 4]), (13, [64, 64]),
                                       (13, [100, 100])])
def test_shaped_refine_kernel_is_bitwise_the_generic_one(cuda, monkeypatch, n0, hidden):
    """The compile-time-shape refine instances (common.h FaShape: the column body unrolled per layer,
    widths constant) run the generic kernel's arithmetic: REFINE, REFINE + logit (the runtime's
    fused launch) and FULL agree with it to rounding.  Not bitwise: the unrolled code contracts a
    different set of multiply-adds into FMAs (HIP's default fp-contract); each form is covered by the
    same rounding terms (the fp64 reference test above holds for the shaped kernels, the default)."""
    from fairify_amd.ops import ext
    from fairify_amd.ops import hip as H

    m = random_mlp(n0, hidden, seed=41 + n0 + len(hidden), bias_scale=0.3)
    lo, hi = _boxes(n0, 611, 13)
    gpu = Backend(m, cuda)
    L_, H_ = lo.to(cuda), hi.to(cuda)
    outs = []
    for shaped in ("1", "0"):
        monkeypatch.setenv("FAIRIFY_REFINE_SHAPED", shaped)
        a = gpu.bounds(L_, H_, mode="symbolic", crown=True, refine=True)
        f = gpu.bounds(L_, H_, mode="symbolic", keep_layers=True)
        ext().refine_crown(H._net(gpu), gpu.flat.data_ptr(), L_.contiguous().data_ptr(), H_.contiguous().data_ptr(),
                           0, L_.shape[0], f.out_lb.data_ptr(), f.out_ub.data_ptr(), f.Lc.data_ptr(),
                           f.L0.data_ptr(), f.Le.data_ptr(), f.Uc.data_ptr(), f.U0.data_ptr(), f.Ue.data_ptr(),
                           f.lay_lb_full.data_ptr(), f.lay_ub_full.data_ptr(), H._stream(cuda))
        b = gpu.bounds(L_, H_, mode="backward")
        torch.cuda.synchronize()
        outs.append((a, f, b))
    def close(p, q):
        p, q = p.cpu().double(), q.cpu().double()
        return torch.allclose(p, q, rtol=1e-5, atol=1e-5 * float(q.abs().max() + 1))

    for x, y in zip(outs[0], outs[1]):
        for fld in ("out_lb", "out_ub", "Lc", "Uc", "L0", "U0", "Le", "Ue"):
            if getattr(x, fld) is not None:
                assert close(getattr(x, fld), getattr(y, fld)), fld
        for p, q in zip(x.layer_lb or [], y.layer_lb or []):
            assert close(p, q)
        for p, q in zip(x.layer_ub or [], y.layer_ub or []):
            assert close(p, q)
