"""Beta-CROWN bounds of ReLU-phase branch-and-bound nodes (stage ``beta``; csrc/beta.hip).

The reference decides a partition with Z3, whose simplex case-splits every ReLU
``If(z >= 0, z, 0)`` (utils/verif_utils.py:525-528, solved at src/AC/Verify-AC.py:146-158): inside
a case split the phase is a LINEAR CONSTRAINT on the input region.  The round-4 GPU ReLU-phase
stage (engine/relu_bab.py) only clamped intervals with the phases and closed none of trained
AC-7's residue; the verified host LP (smt/lpbab.py) closed it, slowly, because its phase splits
are constraints.  This module bounds a node the way that LP does, by Lagrangian duality, on the
GPU:

* node = (input box, ordered PA pair (va, vb), phase in {-1, 0, +1} of every hidden neuron of the
  copies N(., va) and N(., vb)); both copies read the same x on the non-PA dims;
* violation needs N(x, va) < 0 < N(x, vb), so for any t in [0, 1]
  ``f_t(x) = t N(x, va) - (1 - t) N(x, vb) < 0``; a lower bound of f_t >= 0 over the node's
  region closes the node;
* the lower bound is a backward (CROWN) pass per copy with free lower slopes ``alpha`` in [0, 1]
  for unstable neurons, the chord as upper relaxation, fixed phases exact (active: identity,
  inactive: 0) and, for every fixed neuron, the Lagrangian term ``- beta_j s_j z_j`` (s_j z_j >= 0
  on the region: beta >= 0 uses the phase constraint; beta < 0 the neuron's interval side,
  ``- beta_j s_j z_j <= - beta_j s_j e_j`` with e = ub (active) / lb (inactive)) -- the split
  constraint acts on the whole region, not only on the neuron's interval.  A child's new multiplier
  starts where the parent's relaxation of that neuron is reproduced exactly (``binit``), so warm
  starts never lose bound;
* (alpha, beta, t) are optimised by projected Adam in fp32 (gradients in closed form: the bound is
  the linearised network evaluated at the concretising vertex x*, so d/d alpha_j = lam_j z_j(x*),
  d/d beta_j = -s_j (z_j(x*) - [beta_j < 0] e_j), d/dt = N_lin(x*, va) + N_lin(x*, vb)); children start from their
  parent's values (warm start);
* the bound that decides is re-evaluated in fp64 at the best parameters with rigorous rounding
  terms (Higham gamma_k on every product and sum, chord slopes rounded up), so any parameter values
  give a sound bound; intermediate (pre-activation) bounds are the rigorous fp32 bounds of the
  node's partition (the same ones the verified LP uses), clamped by the phases;
* branching: the unfixed unstable neuron (either copy) with the largest ``|lam_j| x`` relaxation
  gap at x* (what fixing its phase recovers at the current optimum); with none, an input split on
  the dim of largest |coefficient| x width; single lattice points are decided exactly.

CPU prototype and measurements: tools/exp/beta_bab.py (trained AC-7 residue partitions that the LP
closes in 40-5 000 nodes close here in ~9 per ordered pair).  This module is the reference
semantics (CPU tests); ``level`` dispatches to the HIP kernel on the GPU.
"""
from __future__ import annotations

from dataclasses import dataclass
from typing import List, Optional, Sequence

import torch

from . import reference as ref

U64 = ref.FP64_UNIT


@dataclass
class BetaLevel:
    bound: torch.Tensor       # [R] float64 rigorous lower bound of f_t over the node region (+inf: empty)
    split: torch.Tensor       # [R] int64: >= 0 neuron (copy A: j, copy B: NH + j); -1 - d: input dim d
    #                           (d >= n0: x''s RA dim d - n0); LEAF(n0): single lattice point
    xstar: torch.Tensor       # [R, n0] float32 concretising vertex (candidate pair's shared dims)
    binit: torch.Tensor       # [R, 2] float32 beta of the split neuron in the (inactive, active) child
    #                           that reproduces this node's relaxation of it (monotone warm start)
    xpstar: Optional[torch.Tensor] = None   # [R, n0] copy B's vertex (relaxed: its RA dims from x''s box)
    scores: Optional[torch.Tensor] = None   # [R, 2 NH] branching scores (reference only: tests)


def LEAF(n0: int) -> int:
    """Split code of a node with no input width left (x and, relaxed, x' RA dims): decided exactly."""
    return -(2 * n0 + 1)


def _layers(v: torch.Tensor, widths: Sequence[int]) -> List[torch.Tensor]:
    out, o = [], 0
    for w in widths:
        out.append(v[:, o:o + w])
        o += w
    return out


def _g(k: int) -> float:
    return ref.gamma(k, U64)


def _backward(ws, bs, LB, UB, ph, al, be, scale, hmax_in, rig: bool):
    """One copy's backward pass for rows R, objective ``scale * logit``.  LB / UB / ph / al / be:
    per hidden layer [R, w].  Returns (input coefficients [R, n0], constant [R], rounding error
    [R] (rig only, else zeros), per-layer records (lam, kind, s) for the gradient / scores).
    kind: 0 inactive, 1 active, 2 unstable with the alpha lower relaxation, 3 unstable chord."""
    L = len(ws)
    dt = scale.dtype
    lam = scale[:, None] * ws[L - 1][:, 0][None]
    c = scale * bs[L - 1][0]
    err = torch.zeros_like(c)
    if rig:
        err = err + U64 * (lam.abs() * UB[L - 2].clamp(min=0)).sum(1) + U64 * c.abs()
    rec = [None] * (L - 1)
    for l in range(L - 2, -1, -1):
        lb, ub, p = LB[l], UB[l], ph[l]
        pf = p.to(dt)
        dead = (ub <= 0) | (p < 0)
        act = ((lb >= 0) | (p > 0)) & ~dead
        un = ~(dead | act)
        low = un & (lam >= 0)
        upp = un & (lam < 0)
        one = torch.ones_like(ub)
        den = torch.where(un, ub - lb, one)
        s = torch.where(un, ub / den, torch.zeros_like(ub))
        if rig:
            s = s * (1 + 4 * U64)              # rounded up: a steeper chord is still an upper bound
        slope = torch.where(act, one, torch.where(low, al[l], torch.where(upp, s, torch.zeros_like(ub))))
        base = lam * slope
        kap = torch.where(upp, -base * lb, torch.zeros_like(ub))
        bet = be[l]
        mu = base - bet * pf
        # a negative multiplier of a fixed neuron uses the interval side of its region instead:
        # -beta s z <= -beta s e for s z in [0, s e] (e = ub active, lb inactive)
        kb = torch.where((p != 0) & (bet < 0), bet * pf * torch.where(p > 0, ub, lb), torch.zeros_like(ub))
        kap = kap + kb
        zmax = torch.maximum(lb.abs(), ub.abs())
        mb = mu * bs[l][None]
        if rig:
            e = torch.where(low, _g(1) * base.abs() * zmax, torch.zeros_like(ub))
            e = e + torch.where(upp, 3 * U64 * (2 * base.abs() * zmax + kap.abs()), torch.zeros_like(ub))
            e = e + torch.where(p != 0, _g(1) * (mu.abs() * zmax + kb.abs()), torch.zeros_like(ub))
            w = lb.shape[1]
            err = err + e.sum(1) + _g(2 * w + 1) * (c.abs() + mb.abs().sum(1) + kap.abs().sum(1))
        c = c + mb.sum(1) + kap.sum(1)
        kind = torch.where(dead, 0, torch.where(act, 1, torch.where(low, 2, 3)))
        rec[l] = (lam, kind, s, slope)
        W = ws[l]
        lam = mu @ W.T
        if rig:
            hm = UB[l - 1].clamp(min=0) if l > 0 else hmax_in
            err = err + (_g(W.shape[1]) * (mu.abs() @ W.abs().T) * hm).sum(1)
    return lam, c, err, rec


def _forward_lin(ws, bs, x, LB, rec, al, hs=None):
    """Pre-activations of the linearised network (each neuron's chosen relaxation) at x; logit.
    ``hs`` (a list): receives each layer's relaxation outputs h (the Lagrangian's primal iterate)."""
    h = x
    zs = []
    for l in range(len(ws) - 1):
        z = h @ ws[l] + bs[l][None]
        zs.append(z)
        lam, kind, s, _ = rec[l]
        h = torch.where(kind == 1, z, torch.where(kind == 2, al[l] * z,
                                                  torch.where(kind == 3, s * (z - LB[l]), torch.zeros_like(z))))
        if hs is not None:
            hs.append(h)
    return zs, (h @ ws[-1] + bs[-1][None])[:, 0]


def evaluate(ws, bs, lo, hi, pa, va, vb, bA, bB, phA, phB, alA, alB, beA, beB, t, rig: bool, need_lin: bool = True,
             rx=None, osg=None, obj: float = 1.0):
    """The coupled bound of rows R at the given parameters (per-layer lists), in the dtype of
    ``ws``.  ``rig``: fp64 with every rounding term subtracted (the sound bound).

    ``rx`` = (ra [n0] bool, plo, phi [R, n0][, tau, gP, gM]) for relaxed queries: copy B reads x'
    whose RA dims range over their own box [plo, phi] (unclipped, reference semantics); on those dims
    the two copies are concretised separately, and the tie |x_r - x'_r| <= tau enters through its
    own Lagrange multipliers gP, gM >= 0 [R, n0] (``f >= f + gP (x_r - x'_r - tau) + gM (x'_r - x_r -
    tau)`` on every admissible pair; all zero: the tie dropped, as the relu stage does).
    ``osg`` [R] (+1 / -1, default +1): the orientation of the violation a row rules out -- +1: N(x, va)
    < 0 < N(x', vb), objective t N_A - (1 - t) N_B; -1: N(x, va) > 0 > N(x', vb), the same objective
    negated (both orientations of a relaxed query as rows of one search; a PA-only query has x' = x
    off the PA dims, so its swapped ordered pair is the second orientation).
    Returns a dict: B [R], g (gradients), lin (per-copy records), xs (x*), xps (x'*), cA, cB."""
    dt = ws[0].dtype
    pa = list(pa)
    n0 = lo.shape[1]
    free = torch.ones(n0, dtype=torch.bool, device=lo.device)
    free[pa] = False
    lo_, hi_ = lo.to(dt), hi.to(dt)
    if rx is not None:
        ram = rx[0].to(lo.device)
        loB = torch.where(ram[None], rx[1].to(dt), lo_)
        hiB = torch.where(ram[None], rx[2].to(dt), hi_)
    else:
        ram = torch.zeros(n0, dtype=torch.bool, device=lo.device)
        loB, hiB = lo_, hi_
    hmA = torch.maximum(lo_.abs(), hi_.abs())
    hmB = torch.maximum(loB.abs(), hiB.abs())
    hmA[:, pa] = va.abs().to(dt)
    hmB[:, pa] = vb.abs().to(dt)
    og = (torch.ones_like(t) if osg is None else osg.to(t.dtype)) * obj    # obj = 0: constraints only
    cA, kA, eA, rA = _backward(ws, bs, bA[0], bA[1], phA, alA, beA, og * t, hmA, rig)
    cB, kB, eB, rB = _backward(ws, bs, bB[0], bB[1], phB, alB, beB, -og * (1 - t), hmB, rig)
    pA = cA[:, pa] * va.to(dt)
    pB = cB[:, pa] * vb.to(dt)
    shared = free & ~ram
    coef = torch.where(shared[None], cA + cB, torch.zeros_like(cA))
    xs = torch.where(coef >= 0, lo_, hi_)
    terms = coef * xs
    # the tau tie's multipliers move coefficient between the copies on the RA dims
    tie = rx is not None and len(rx) > 3 and rx[4] is not None
    if tie:
        tau = float(rx[3])
        gP = torch.where(ram[None], rx[4].to(dt), torch.zeros_like(cA))
        gM = torch.where(ram[None], rx[5].to(dt), torch.zeros_like(cA))
        cAe = cA + (gP - gM)
        cBe = cB + (gM - gP)
        ktie = -tau * (gP + gM).sum(1)
    else:
        cAe, cBe = cA, cB
        ktie = torch.zeros_like(kA)
    xA = torch.where(cAe >= 0, lo_, hi_)
    xB = torch.where(cBe >= 0, loB, hiB)
    tA = torch.where(ram[None], cAe * xA, torch.zeros_like(cA))
    tB = torch.where(ram[None], cBe * xB, torch.zeros_like(cB))
    xs = torch.where(ram[None], xA, xs)
    xps = torch.where(ram[None], xB, xs)
    B = terms.sum(1) + tA.sum(1) + tB.sum(1) + pA.sum(1) + pB.sum(1) + kA + kB + ktie
    if rig:
        mag = terms.abs().sum(1) + tA.abs().sum(1) + tB.abs().sum(1) + pA.abs().sum(1) + pB.abs().sum(1) + \
            kA.abs() + kB.abs() + ktie.abs()
        econ = U64 * (coef.abs() * torch.maximum(lo_.abs(), hi_.abs())).sum(1) + _g(2 * n0 + 4) * mag
        if tie:     # the RA coefficient sums cA + (gP - gM) etc. and tau (gP + gM); fl(gP - gM) is off by
            # u (gP + gM), charged on both copies' magnitudes (cA may cancel it: |cAe| alone does not cover it)
            econ = econ + 2 * U64 * torch.where(ram[None], cAe.abs() * hmA + cBe.abs() * hmB +
                                                (gP + gM) * (hmA + hmB), torch.zeros_like(cA)).sum(1) \
                + 2 * U64 * ktie.abs()
        B = B - (eA + eB + econ) * (1 + 1e-6)
    out = {"B": B, "xs": xs, "xps": xps, "cA": cAe, "cB": cBe, "coef": coef, "g": None, "lin": None}
    if not need_lin:
        return out
    xa, xb = xs.clone(), xps.clone()
    xa[:, pa] = va.to(dt)
    xb[:, pa] = vb.to(dt)
    hA, hB = [], []
    zA, oA = _forward_lin(ws, bs, xa, bA[0], rA, alA, hA)
    zB, oB = _forward_lin(ws, bs, xb, bB[0], rB, alB, hB)
    g = {"t": og * (oA + oB)}
    if tie:
        g["gP"] = torch.where(ram[None], xs - xps - tau, torch.zeros_like(xs))
        g["gM"] = torch.where(ram[None], xps - xs - tau, torch.zeros_like(xs))
    for nm, z, rec, ph, bet, bnd in (("A", zA, rA, phA, beA, bA), ("B", zB, rB, phB, beB, bB)):
        g["al" + nm] = [torch.where(r[1] == 2, r[0] * zz, torch.zeros_like(zz)) for zz, r in zip(z, rec)]
        g["be" + nm] = [torch.where(p == 0, torch.zeros_like(zz),
                                    -p.to(dt) * (zz - torch.where(be_ < 0, torch.where(p > 0, ub, lb), torch.zeros_like(zz))))
                        for zz, p, be_, lb, ub in zip(z, ph, bet, bnd[0], bnd[1])]
    out["g"] = g
    out["lin"] = ((zA, rA), (zB, rB))
    out["h"] = (hA, hB)
    return out


def _scores(bnd, lin, ph, al):
    LB = bnd[0]
    z, rec = lin
    out = []
    for l in range(len(z)):
        lam, kind, s, _ = rec[l]
        zz = z[l]
        gap = torch.where(kind == 2, torch.relu(zz) - al[l] * zz,
                          torch.where(kind == 3, s * (zz - LB[l]) - torch.relu(zz), torch.zeros_like(zz)))
        out.append(torch.where((kind >= 2) & (ph[l] == 0), lam.abs() * gap.abs(), torch.zeros_like(zz)))
    return torch.cat(out, 1)


def _intercepts(bnd, lin, ph):
    """BaBSR-style score: the constant the chord of an unfixed unstable neuron costs the bound."""
    LB = bnd[0]
    z, rec = lin
    out = []
    for l in range(len(z)):
        lam, kind, s, _ = rec[l]
        out.append(torch.where((kind == 3) & (ph[l] == 0), (lam * s * LB[l]).abs(), torch.zeros_like(lam)))
    return torch.cat(out, 1)


def _lookahead(ws32, bs32, widths, lo, hi, pa, va, vb, lbA, ubA, lbB, ubB, phA, phB, alA, alB, beA, beB, t, sc, lin,
               K: int, j0, rx=None, osg=None):
    """Filtered branching: the top-K neurons by relaxation-gap score and the top-K by chord intercept
    are each tried -- both children bounded at the node's parameters with the new multiplier at 0
    (one backward pass each) -- and the neuron whose worse child is best wins."""
    R, NH = phA.shape
    dev = lo.device
    d = torch.float64
    ic = torch.cat([_intercepts((_layers(lbA.to(d), widths), None), lin[0], _layers(phA, widths)),
                    _intercepts((_layers(lbB.to(d), widths), None), lin[1], _layers(phB, widths))], 1)
    k1 = min(K, sc.shape[1])
    v1, c1 = sc.topk(k1, dim=1)
    v2, c2 = ic.topk(k1, dim=1)
    cand = torch.cat([c1, c2], 1)                                  # [R, 2K]
    valid = torch.cat([v1 > 0, v2 > 0], 1)
    C = cand.shape[1]
    rows = torch.arange(R, device=dev).repeat_interleave(2 * C)
    cc = cand.repeat_interleave(2, dim=1).reshape(-1)
    sg = torch.tensor([-1, 1], dtype=torch.int8, device=dev).repeat(R * C)
    pA2, pB2 = phA[rows].clone(), phB[rows].clone()
    r_ = torch.arange(rows.numel(), device=dev)
    ia = cc < NH
    pA2[r_[ia], cc[ia]] = sg[ia]
    pB2[r_[~ia], cc[~ia] - NH] = sg[~ia]
    lA, uA, iA = clamp_bounds(lbA[rows], ubA[rows], pA2)
    lB, uB, iB = clamp_bounds(lbB[rows], ubB[rows], pB2)
    L = lambda v: _layers(v, widths)  # noqa: E731
    rxr = None if rx is None else ((rx[0], rx[1][rows], rx[2][rows]) if len(rx) <= 3 or rx[4] is None else
                                   (rx[0], rx[1][rows], rx[2][rows], rx[3], rx[4][rows], rx[5][rows]))
    Bc = evaluate(ws32, bs32, lo[rows], hi[rows], pa, va[rows], vb[rows], (L(lA), L(uA)), (L(lB), L(uB)),
                  L(pA2), L(pB2), L(alA[rows]), L(alB[rows]), L(beA[rows]), L(beB[rows]), t[rows],
                  rig=False, need_lin=False, rx=rxr, osg=None if osg is None else osg[rows])["B"]
    Bc = torch.where(iA | iB, torch.full_like(Bc, float("inf")), Bc.float())
    worst = Bc.reshape(R, C, 2).min(2).values
    worst = torch.where(valid, worst, torch.full_like(worst, -float("inf")))
    bw, bi = worst.max(1)
    pick = cand.gather(1, bi[:, None])[:, 0]
    return torch.where(torch.isfinite(bw) | (bw > 0), pick, j0), bw


def primal_gap_scores(zsum, hsum, n, lb, ub, ph):
    """[R, 2 NH] the LP-BaB branching score at the averaged primal point: for an unfixed neuron
    unstable over the node's (phase-clamped) bounds, ``max(h_bar - relu(z_bar), 0)`` with z_bar /
    h_bar the means of the linearised network's pre-activations / relaxation outputs over the ``n``
    optimisation steps (fp32 sums, the kernel's order: one step at a time); 0 elsewhere."""
    nn = n.clamp(min=1.0)[:, None]
    zb = zsum.float() / nn
    hb = hsum.float() / nn
    gap = (hb - torch.relu(zb)).clamp(min=0)
    un = (ph == 0) & (lb < 0) & (ub > 0)
    return torch.where(un & (n[:, None] > 0), gap, torch.zeros_like(gap))


def feasibility_ref(ws32, bs32, widths, lo, hi, pa, va, vb, lbA, ubA, lbB, ubB, phA, phB, alA, alB, t, iters: int,
                    lr_a: float, lr_b: float, lr_t: float, decay: float, rx, osg, run) -> torch.Tensor:
    """[R] bool: rows whose phase region is proven EMPTY (the kernel's ``feas`` pass).

    The Lagrangian of the fixed phases alone, ``min over the relaxed region of -sum_j beta_j s_j z_j``
    (plus the tau tie's multipliers on relaxed rows), is <= 0 whenever some point satisfies every
    phase; a rigorous value > 0 (Farkas) proves no point does -- the LP-BaB closes such nodes as
    infeasible after two or three phase splits, where the objective's Lagrangian (weight 1 on the
    logits) would need unboundedly large multipliers.  The value is positively homogeneous in the
    multipliers, so they live in [0, 1]; projected Adam from 0.5 on the fixed neurons, the slopes
    from the main pass's best, objective weight 0."""
    R = lo.shape[0]
    dev = lo.device
    L32 = lambda v: _layers(v, widths)  # noqa: E731
    bA32, bB32 = (L32(lbA), L32(ubA)), (L32(lbB), L32(ubB))
    pA, pB = L32(phA), L32(phB)
    half = torch.full_like(alA, 0.5)
    cur = {"alA": alA.clone(), "alB": alB.clone(), "beA": torch.where(phA != 0, half, torch.zeros_like(alA)),
           "beB": torch.where(phB != 0, half, torch.zeros_like(alB))}
    tie = rx is not None and len(rx) > 3 and rx[4] is not None
    if tie:
        cur["gP"] = torch.zeros_like(rx[4])
        cur["gM"] = torch.zeros_like(rx[5])
    rxc = lambda c: rx if not tie else (rx[0], rx[1], rx[2], rx[3], c["gP"], c["gM"])  # noqa: E731
    best = torch.full((R,), -float("inf"), dtype=torch.float32, device=dev)
    bestp = {k: v.clone() for k, v in cur.items()}
    m = {k: torch.zeros_like(v) for k, v in cur.items()}
    vv = {k: torch.zeros_like(v) for k, v in cur.items()}
    act = run.clone()
    b1, b2, eps = 0.9, 0.999, 1e-8
    for it in range(iters):
        ev = evaluate(ws32, bs32, lo, hi, pa, va, vb, bA32, bB32, pA, pB, L32(cur["alA"]), L32(cur["alB"]),
                      L32(cur["beA"]), L32(cur["beB"]), t, rig=False, rx=rxc(cur), osg=osg, obj=0.0)
        Bv, g = ev["B"], ev["g"]
        imp = act & (Bv > best)
        best = torch.where(imp, Bv, best)
        for k in cur:
            bestp[k] = torch.where(imp[:, None], cur[k], bestp[k])
        act = act & ~(best > 0)
        if not bool(act.any()):
            break
        c1 = 1 - b1 ** (it + 1)
        c2 = 1 - b2 ** (it + 1)
        dk = decay ** it
        for k in cur:
            gk = torch.cat(g[k], 1) if isinstance(g[k], list) else g[k]
            m[k] = b1 * m[k] + (1 - b1) * gk
            vv[k] = b2 * vv[k] + (1 - b2) * gk * gk
            lr = (lr_a if k.startswith("al") else (lr_t if k.startswith("g") else lr_b)) * dk
            x = cur[k] + lr * (m[k] / c1) / ((vv[k] / c2).sqrt() + eps)
            x = x.clamp(0, 1)
            cur[k] = torch.where(act[:, None], x, cur[k])
    fp = bestp if iters > 0 else cur
    d = torch.float64
    ws64 = [w.to(d) for w in ws32]
    bs64 = [b.to(d) for b in bs32]
    L64 = lambda v: _layers(v.to(d), widths)  # noqa: E731
    ev = evaluate(ws64, bs64, lo.to(d), hi.to(d), pa, va.to(d), vb.to(d), (L64(lbA), L64(ubA)), (L64(lbB), L64(ubB)),
                  pA, pB, L64(fp["alA"]), L64(fp["alB"]), L64(fp["beA"]), L64(fp["beB"]), t.to(d), rig=True,
                  need_lin=False, rx=rxc(fp), osg=osg, obj=0.0)
    return run & (ev["B"] > 0)


def clamp_bounds(LB: torch.Tensor, UB: torch.Tensor, ph: torch.Tensor):
    """Phase-clamped pre-activation bounds [R, NH] and the rows whose region they prove empty."""
    lb = torch.where(ph > 0, LB.clamp(min=0), LB)
    ub = torch.where(ph < 0, UB.clamp(max=0), UB)
    return lb, ub, (lb > ub).any(1)


def level_ref(ws32, bs32, widths, lo, hi, pa, va, vb, LBA, UBA, LBB, UBB, phA, phB, alA, alB, beA, beB, t,
              iters: int, lr_a: float, lr_b: float, lr_t: float, decay: float = 1.0,
              lookahead: int = 0, beta_pos: bool = True, rx=None, stall: bool = True, pgap: int = 0,
              osg=None, feas_iters: int = 0, feas_lr=None) -> BetaLevel:
    """One BaB level of rows R (the HIP kernel's semantics, csrc/beta.hip): ``iters`` projected-Adam
    steps in fp32 from the rows' current (alpha, beta, t) -- updated IN PLACE to the best iterate --
    then the rigorous fp64 bound, the branching decision and x* at those parameters.

    lo, hi [R, n0]; va, vb [R, npa]; LB*/UB* [R, NH] partition bounds (unclamped); ph* [R, NH] int8;
    al*/be* [R, NH] float32; t [R] float32.  ``rx`` = (ra [n0] bool, plo, phi [R, n0]): relaxed
    queries, copy B's RA dims over their own box (:func:`evaluate`); x' RA dims are split too
    (``split`` = -1 - (n0 + d)).  ``osg`` [R] int8: each row's orientation (:func:`evaluate`).

    ``pgap``: branch by the verified LP's rule (smt/lpbab.py:_lp_bab) at a primal point of the node's
    relaxation instead of at the vertex x*: the Lagrangian's primal iterates (x*, z, h of the
    linearised network) are averaged over the optimisation steps -- the ergodic average of a dual
    (sub)gradient method converges to a primal optimum of the LP it dualises -- and an unfixed
    unstable neuron scores its primal gap ``mean(h) - relu(mean(z))`` (look-ahead, when on, takes its
    first candidate list from these scores).  The iterates' weights: ``pgap`` 1 uniform, 2 ``it + 1``
    (later iterates count more), 3 the second half of the steps only."""
    R, n0 = lo.shape
    dev = lo.device
    lbA, ubA, infA = clamp_bounds(LBA, UBA, phA)
    lbB, ubB, infB = clamp_bounds(LBB, UBB, phB)
    infeas = infA | infB
    L32 = lambda v: _layers(v, widths)  # noqa: E731
    bA32, bB32 = (L32(lbA), L32(ubA)), (L32(lbB), L32(ubB))
    pA, pB = L32(phA), L32(phB)
    keys = ("alA", "alB", "beA", "beB")
    par = {"alA": alA, "alB": alB, "beA": beA, "beB": beB}
    tie = rx is not None and len(rx) > 3 and rx[4] is not None
    if tie:                     # the tau tie's multipliers (relaxed): optimised like beta, >= 0
        keys = keys + ("gP", "gM")
        par["gP"], par["gM"] = rx[4], rx[5]
    rxc = lambda c: rx if not tie else (rx[0], rx[1], rx[2], rx[3], c["gP"], c["gM"])  # noqa: E731
    best = torch.full((R,), -float("inf"), dtype=torch.float32, device=dev)
    bestp = {k: v.clone() for k, v in par.items()}
    best_t = t.clone()
    cur = {k: v.clone() for k, v in par.items()}
    ct = t.clone()
    m = {k: torch.zeros_like(v) for k, v in par.items()}
    vv = {k: torch.zeros_like(v) for k, v in par.items()}
    mt = torch.zeros_like(t)
    vt = torch.zeros_like(t)
    b1, b2, eps = 0.9, 0.999, 1e-8
    act = ~infeas
    zsum = hsum = None
    nsum = torch.zeros(R, dtype=torch.float32, device=dev)
    for it in range(iters):
        ev = evaluate(ws32, bs32, lo, hi, pa, va, vb, bA32, bB32, pA, pB, L32(cur["alA"]), L32(cur["alB"]),
                      L32(cur["beA"]), L32(cur["beB"]), ct, rig=False, rx=rxc(cur), osg=osg)
        B, g = ev["B"], ev["g"]
        wi = float(it + 1) if pgap == 2 else (float(2 * it >= iters) if pgap == 3 else 1.0)
        if pgap and wi > 0:   # the primal iterate of rows still optimising (the kernel's accumulators)
            zi = torch.cat([torch.cat(ev["lin"][0][0], 1), torch.cat(ev["lin"][1][0], 1)], 1)
            hi_ = torch.cat([torch.cat(ev["h"][0], 1), torch.cat(ev["h"][1], 1)], 1)
            a_ = act[:, None].to(zi.dtype) * wi
            zsum = zi * a_ if zsum is None else zsum + zi * a_
            hsum = hi_ * a_ if hsum is None else hsum + hi_ * a_
            nsum = nsum + act.to(torch.float32) * wi
        imp = act & (B > best)
        best = torch.where(imp, B, best)
        for k in keys:
            bestp[k] = torch.where(imp[:, None], cur[k], bestp[k])
        best_t = torch.where(imp, ct, best_t)
        act = act & ~(best > 0)
        if not bool(act.any()):
            break
        c1 = 1 - b1 ** (it + 1)
        c2 = 1 - b2 ** (it + 1)
        dk = decay ** it
        for k in keys:
            gk = torch.cat(g[k], 1) if isinstance(g[k], list) else g[k]
            m[k] = b1 * m[k] + (1 - b1) * gk
            vv[k] = b2 * vv[k] + (1 - b2) * gk * gk
            lr = (lr_a if k.startswith("al") else (lr_t if k.startswith("g") else lr_b)) * dk
            x = cur[k] + lr * (m[k] / c1) / ((vv[k] / c2).sqrt() + eps)
            if k.startswith("al"):
                x = x.clamp(0, 1)
            elif beta_pos or k.startswith("g"):
                x = x.clamp(min=0)
            cur[k] = torch.where(act[:, None], x, cur[k])
        mt = b1 * mt + (1 - b1) * g["t"]
        vt = b2 * vt + (1 - b2) * g["t"] * g["t"]
        xt = (ct + lr_t * dk * (mt / c1) / ((vt / c2).sqrt() + eps)).clamp(0, 1)
        ct = torch.where(act, xt, ct)
    if iters == 0:
        bestp = {k: v.clone() for k, v in par.items()}
        best_t = t.clone()
    for k in keys:
        par[k].copy_(bestp[k])
    t.copy_(best_t)
    # rigorous fp64 evaluation at the kept parameters
    d = torch.float64
    ws64 = [w.to(d) for w in ws32]
    bs64 = [b.to(d) for b in bs32]
    L64 = lambda v: _layers(v.to(d), widths)  # noqa: E731
    bA, bB = (L64(lbA), L64(ubA)), (L64(lbB), L64(ubB))
    alA64, alB64 = L64(alA), L64(alB)
    ev = evaluate(ws64, bs64, lo.to(d), hi.to(d), pa, va.to(d), vb.to(d), bA, bB, pA, pB, alA64, alB64, L64(beA),
                  L64(beB), t.to(d), rig=True, rx=rxc(par), osg=osg)
    B, lin, xs, coef = ev["B"], ev["lin"], ev["xs"], ev["coef"]
    B = torch.where(infeas, torch.full_like(B, float("inf")), B)
    # crossed bounds with no fixed phase are not sound bounds of a non-empty box: no bound (NaN), the
    # kernel's guard (csrc/beta.hip)
    nofix = ~((phA != 0).any(1) | (phB != 0).any(1))
    B = torch.where(infeas & nofix, torch.full_like(B, float("nan")), B)
    if feas_iters > 0:
        # the infeasibility pass (the kernel's second launch): nodes left open with a fixed phase
        fixed = (phA != 0).any(1) | (phB != 0).any(1)
        run = (B < 0) & fixed & ~infeas
        if bool(run.any()):
            emp = feasibility_ref(ws32, bs32, widths, lo, hi, pa, va, vb, lbA, ubA, lbB, ubB, phA, phB, alA, alB, t,
                                  feas_iters, *(feas_lr or (lr_a, lr_b, lr_t)), decay, rx, osg, run)
            B = torch.where(emp, torch.full_like(B, float("inf")), B)
    sc = torch.cat([_scores(bA, lin[0], pA, alA64), _scores(bB, lin[1], pB, alB64)], 1)
    if pgap and zsum is not None:
        sc = primal_gap_scores(zsum, hsum, nsum, torch.cat([lbA, lbB], 1), torch.cat([ubA, ubB], 1),
                               torch.cat([phA, phB], 1)).to(sc.dtype)
    mx, j = sc.max(1)
    if lookahead > 0:
        j, bw = _lookahead(ws32, bs32, widths, lo, hi, pa, va, vb, lbA, ubA, lbB, ubB, phA, phB, alA, alB, beA, beB,
                           t, sc, lin, lookahead, j, rx, osg)
        if stall:
            # no candidate's children beat this node: the relaxations are not what keeps it open
            # -- split the input box instead (as the verified LP does)
            mx = torch.where(bw.double() <= B, torch.zeros_like(mx), mx)
    free = torch.ones(n0, dtype=torch.bool, device=dev)
    free[list(pa)] = False
    # input split: |coefficient| x width over x's non-PA dims (RA dims: copy A's coefficient) and,
    # relaxed, x''s RA dims (copy B's); none left: a lattice leaf
    cx = torch.where(coef != 0, coef, ev["cA"])
    w = torch.where(free[None], (hi - lo).to(d), torch.zeros_like(coef))
    isc = torch.where(w > 0, cx.abs() * w + 1e-9 * w, torch.full_like(w, -1.0))
    if rx is not None:
        wp = torch.where(rx[0][None], (rx[2] - rx[1]).to(d), torch.zeros_like(coef))
        isc = torch.cat([isc, torch.where(wp > 0, ev["cB"].abs() * wp + 1e-9 * wp, torch.full_like(wp, -1.0))], 1)
    im, dd = isc.max(1)
    split = torch.where(mx > 0, j, torch.where(im > 0, -1 - dd, torch.full_like(dd, LEAF(n0))))
    # the split neuron's multipliers that make each child start from this node's relaxation of it
    lam = torch.cat([torch.cat([r[0] for r in lin[0][1]], 1), torch.cat([r[0] for r in lin[1][1]], 1)], 1)
    slope = torch.cat([torch.cat([r[3] for r in lin[0][1]], 1), torch.cat([r[3] for r in lin[1][1]], 1)], 1)
    jj = j.clamp(min=0)[:, None]
    lj, sj = lam.gather(1, jj)[:, 0], slope.gather(1, jj)[:, 0]
    binit = torch.stack([lj * sj, lj * (1 - sj)], 1).to(torch.float32)
    return BetaLevel(bound=B, split=split, xstar=xs.to(torch.float32), binit=binit,
                     xpstar=ev["xps"].to(torch.float32), scores=sc)
