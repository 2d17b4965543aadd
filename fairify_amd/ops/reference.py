"""PyTorch reference implementations of every hot op (CPU path + numerics oracle).

Each function here has a hand-written HIP/CDNA4 counterpart in ``fairify_amd/csrc`` with the
same arguments and the same arithmetic (fp32 accumulate in the same order where it matters
for soundness accounting).  On a GPU the engine calls the HIP versions (``ops/hip.py``) and
fails loudly if the extension is missing; these versions run on CPU (tests, tiny jobs) and
are what the kernel tests compare against.

Ops:
* K3/K8  :func:`sample_points` / :func:`forward` / :func:`activation_counts` — uniform integer
  simulation inside boxes with a counter-based hash RNG (identical stream on host and device),
  replacing ``simluate_data`` + ``candidate_dead_nodes`` (utils/prune.py:168-222).
* K2     :func:`bounds` with ``mode='ibp'`` — interval bound propagation, replacing
  ``neuron_bounds`` (utils/prune.py:105-164), in centre/radius-free [lo, hi] GEMM form.
* K4     :func:`bounds` with ``mode='symbolic'`` — forward symbolic (linear) bound propagation
  with chord/zero-or-identity ReLU relaxations.  It replaces the per-neuron Z3 "singular
  verification" (utils/prune.py:276-364) as the tighter sound pruner and is the bounding
  primitive of the branch-and-bound prover (K9).
* K9     :func:`pair_certify` — the fairness-pair LP certificate on a node (see docstring).

Soundness: every bound carries an additive error term that dominates fp rounding of the
GEMMs, concretisations and relaxations (``unit`` = 2^-24 for fp32, 2^-53 for fp64), so an
UNSAT certificate computed in fp32 holds for the exact rational network like Z3's.
"""
from __future__ import annotations

import math
from dataclasses import dataclass
from typing import List, Optional, Sequence, Tuple

import numpy as np
import torch

U32 = 0xFFFFFFFF
FP32_UNIT = 2.0 ** -24
FP64_UNIT = 2.0 ** -53


def gamma(k: int, unit: float) -> float:
    """Higham's gamma_k = k u / (1 - k u), padded by 2 extra operations for safety."""
    ku = (k + 2) * unit
    return ku / (1.0 - ku)


# ======================================================================================
# Counter-based RNG (same integer hash on host and device: lowbias32, Wellons)
# ======================================================================================

def hash32(x: torch.Tensor) -> torch.Tensor:
    x = x & U32
    x = x ^ (x >> 16)
    x = (x * 0x7FEB352D) & U32
    x = x ^ (x >> 15)
    x = (x * 0x846CA68B) & U32
    x = x ^ (x >> 16)
    return x


def rng_u32(seed: int, pid: torch.Tensor, sample: torch.Tensor, dim: torch.Tensor) -> torch.Tensor:
    """Uniform uint32 (as int64) keyed by (seed, partition id, sample index, feature index)."""
    h = hash32((sample.to(torch.int64) * 64 + dim.to(torch.int64)) ^ (seed & U32))
    h = hash32(h ^ (pid.to(torch.int64) & U32))
    h = hash32(h ^ ((pid.to(torch.int64) >> 32) & U32) ^ 0x5BD1E995)
    return h


def sample_points(lo: torch.Tensor, hi: torch.Tensor, pids: torch.Tensor, n_samples: int, seed: int,
                  sample_offset: int = 0) -> torch.Tensor:
    """Uniform integer points in each box: [B, S, n] (float32). ``lo,hi`` [B, n] integral."""
    B, n = lo.shape
    dev = lo.device
    s = torch.arange(sample_offset, sample_offset + n_samples, device=dev, dtype=torch.int64)
    d = torch.arange(n, device=dev, dtype=torch.int64)
    h = rng_u32(seed, pids.to(torch.int64)[:, None, None], s[None, :, None], d[None, None, :])
    width = (hi - lo).to(torch.int64) + 1
    off = h % width[:, None, :]
    return (lo.to(torch.int64)[:, None, :] + off).to(torch.float32)


def sample_points_at(lo: torch.Tensor, hi: torch.Tensor, pids: torch.Tensor, idx: torch.Tensor,
                     seed: int) -> torch.Tensor:
    """Samples with explicit indices ``idx`` [B, k] (same stream as :func:`sample_points`)."""
    B, n = lo.shape
    d = torch.arange(n, device=lo.device, dtype=torch.int64)
    h = rng_u32(seed, pids.to(torch.int64)[:, None, None], idx.to(torch.int64)[:, :, None], d[None, None, :])
    width = (hi - lo).to(torch.int64) + 1
    return (lo.to(torch.int64)[:, None, :] + h % width[:, None, :]).to(torch.float32)


# ======================================================================================
# Concrete forward
# ======================================================================================

def forward(ws: Sequence[torch.Tensor], bs: Sequence[torch.Tensor], x: torch.Tensor,
            dead: Optional[torch.Tensor] = None, return_acts: bool = False):
    """Logits of a ReLU MLP for rows ``x`` [..., n0]; optional per-row dead-neuron mask
    ``dead`` [..., N_hidden] (bool) forcing neurons to 0 (heuristically pruned networks)."""
    h = x
    acts = []
    off = 0
    L = len(ws)
    for l in range(L):
        h = h @ ws[l] + bs[l]
        if l < L - 1:
            h = torch.relu(h)
            if dead is not None:
                n = ws[l].shape[1]
                h = h.masked_fill(dead[..., off:off + n], 0.0)
                off += n
            if return_acts:
                acts.append(h)
    out = h[..., 0]
    return (out, acts) if return_acts else out


def activation_counts(ws, bs, x: torch.Tensor) -> torch.Tensor:
    """Per-neuron count of rows with non-zero post-activation, over axis -2 of ``x`` [B, S, n0]
    -> [B, N] int32 (all layers incl. the linear output, like ``candidate_dead_nodes``)."""
    h = x
    counts = []
    L = len(ws)
    for l in range(L):
        h = h @ ws[l] + bs[l]
        if l < L - 1:
            h = torch.relu(h)
        counts.append((h != 0).sum(dim=-2).to(torch.int32))
    return torch.cat(counts, dim=-1)


def forward_error_bound(ws, bs, x: torch.Tensor, unit: float = FP32_UNIT) -> torch.Tensor:
    """Rigorous bound on |fl(N(x)) - N(x)| for the fp32 forward: propagate magnitudes."""
    m = x.abs()
    e = torch.zeros_like(x)
    L = len(ws)
    for l in range(L):
        W = ws[l]
        g = gamma(W.shape[0] + 1, unit)
        aw = W.abs()
        e = (e + g * m) @ aw + g * bs[l].abs()
        m = m @ aw + bs[l].abs()
    return e[..., 0] * (1 + 1e-6) + 1e-30


def point_bounds(ws: Sequence[torch.Tensor], bs: Sequence[torch.Tensor], x: torch.Tensor,
                 dead: Optional[torch.Tensor] = None, unit: Optional[float] = None):
    """Rigorous logit interval at points ``x`` [R, n0] (csrc/points.hip, same arithmetic).

    Per layer: z = h W + b, d = (|W|^T (e + g|h|)) (1 + 2g) + g|b| + g1|z| bounds |v - z|;
    ReLU keeps exact zeros (z + d <= 0 or forced dead -> 0 with error 0)."""
    dt = x.dtype
    if unit is None:
        unit = FP64_UNIT if dt == torch.float64 else FP32_UNIT
    gi = gamma(1, unit)
    h = x
    L = len(ws)
    g0 = gamma(ws[0].shape[0] + 1, unit)
    eo = g0 * h.abs()
    off = 0
    for l in range(L):
        W = ws[l].to(dt)
        b = bs[l].to(dt)
        g = gamma(W.shape[0] + 1, unit)
        z = h @ W + b
        d = (eo @ W.abs()) * (1 + 2 * g) + g * b.abs() + gi * z.abs()
        if l == L - 1:
            return (z - d)[:, 0], (z + d)[:, 0]
        n = W.shape[1]
        zero = (z + d) <= 0
        if dead is not None:
            zero = zero | dead[:, off:off + n].bool()
        off += n
        h = torch.where(zero, torch.zeros_like(z), z.clamp(min=0))
        e = torch.where(zero, torch.zeros_like(d), d)
        gn = gamma(ws[l + 1].shape[0] + 1, unit)
        eo = e + gn * h
    raise AssertionError("unreachable")


# ======================================================================================
# Bound propagation (IBP and forward symbolic) with rigorous fp error terms
# ======================================================================================

@dataclass
class BoundResult:
    out_lb: torch.Tensor          # [R] sound lower bound of the logit
    out_ub: torch.Tensor          # [R] sound upper bound of the logit
    # output linear forms (symbolic mode): coef [R, n0], const [R], err [R]
    Lc: Optional[torch.Tensor] = None
    L0: Optional[torch.Tensor] = None
    Le: Optional[torch.Tensor] = None
    Uc: Optional[torch.Tensor] = None
    U0: Optional[torch.Tensor] = None
    Ue: Optional[torch.Tensor] = None
    layer_lb: Optional[List[torch.Tensor]] = None   # per layer [R, n_l] pre-activation bounds
    layer_ub: Optional[List[torch.Tensor]] = None
    dead: Optional[torch.Tensor] = None             # [R, N_hidden] stable-inactive (ub <= 0)
    active: Optional[torch.Tensor] = None           # [R, N_hidden] stable-active  (lb >= 0)
    # HIP path: the per-neuron bounds as one [R, N] tensor each (layer_lb/ub are views into it)
    # and the stable-inactive flags as the kernel's uint8 [R, N_hidden]
    lay_lb_full: Optional[torch.Tensor] = None
    lay_ub_full: Optional[torch.Tensor] = None
    dead_u8: Optional[torch.Tensor] = None
    # ReLU-phase rows (``phase`` given): the row's branch region is empty (a neuron fixed inactive
    # with lb > 0, or fixed active with ub < 0)
    infeasible: Optional[torch.Tensor] = None


def _concretize(E: torch.Tensor, lo: torch.Tensor, hi: torch.Tensor):
    """E [R, n0+1, n] (last row = constant) -> (min, max, magnitude) over the box, each [R, n]."""
    C = E[:, :-1, :]
    c0 = E[:, -1, :]
    lo_ = lo[:, :, None]
    hi_ = hi[:, :, None]
    a = C * lo_
    b = C * hi_
    mn = torch.minimum(a, b).sum(1) + c0
    mx = torch.maximum(a, b).sum(1) + c0
    m = torch.maximum(lo.abs(), hi.abs())[:, :, None]
    mag = (C.abs() * m).sum(1) + c0.abs()
    return mn, mx, mag


def bounds(ws: Sequence[torch.Tensor], bs: Sequence[torch.Tensor], lo: torch.Tensor, hi: torch.Tensor,
           mode: str = "symbolic", dead: Optional[torch.Tensor] = None, unit: Optional[float] = None,
           keep_layers: bool = False, lower_slope: str = "adaptive",
           phase: Optional[torch.Tensor] = None) -> BoundResult:
    """Sound bounds of every neuron and of the logit over boxes ``[lo, hi]`` [R, n0].

    Symbolic mode keeps linear forms ``E(x) = sum_i E_i x_i + E_c`` per neuron as matrices
    ``[R, n0+1, n]`` (upper U, lower L) with error terms ``eU, eL`` (``z <= U(x) + eU``,
    ``z >= L(x) - eL``), plus two *interval rows* (Ih, Il) that carry the tightest known
    concrete bounds of the previous layer's outputs.  A layer is one GEMM of all those rows
    against [W+; W-] (the HIP kernel runs it on f32 MFMA); the epilogue intersects the
    symbolic and interval bounds, applies the ReLU relaxation and re-seeds the interval rows
    with max(0, bound).  Interval rounding margins are proportional to the terms actually
    summed, so sign-structured sums (e.g. non-positive weights on non-negative ReLU outputs)
    keep exact zeros exact — essential under the strict ``N(x) < 0 < N(x')`` semantics.
    ``mode='ibp'`` keeps only the interval rows.

    ``phase`` [R, N_hidden] int8 (ReLU-split branch-and-bound, engine/relu_bab.py): -1 = the row's
    branch region has z <= 0 at that neuron (output 0, like a forced-dead neuron), +1 = z >= 0
    there (relu(z) = z: the upper relaxation is the identity instead of the chord; the lower one
    stays lambda * L, valid because z >= 0 on the region; the range of the output is still
    [max(lb, 0), max(ub, 0)]).  Every bound then holds on the branch region, which is all the
    search needs; a region proven empty (fixed inactive with lb > 0, fixed active with ub < 0) is
    flagged in ``infeasible``.
    """
    dt = lo.dtype
    if unit is None:
        unit = FP64_UNIT if dt == torch.float64 else FP32_UNIT
    R, n0 = lo.shape
    dev = lo.device
    sym = mode == "symbolic"
    if mode not in ("symbolic", "ibp"):
        raise ValueError(mode)
    if sym:
        eye = torch.zeros(n0 + 1, n0, dtype=dt, device=dev)
        eye[torch.arange(n0), torch.arange(n0)] = 1.0
        U = eye.expand(R, n0 + 1, n0).clone()
        L = U.clone()
        eU = torch.zeros(R, n0, dtype=dt, device=dev)
        eL = torch.zeros_like(eU)
        gc = gamma(n0 + 1, unit)
    Ih, Il = hi.clone(), lo.clone()          # rigorous interval of the layer inputs
    gi = gamma(1, unit)
    layer_lb, layer_ub, deads, actives = [], [], [], []
    off = 0
    infeas = None
    nL = len(ws)
    res = None
    for l in range(nL):
        W = ws[l].to(dt)
        b = bs[l].to(dt)
        Wp = W.clamp(min=0)
        Wn = W.clamp(max=0)
        g = gamma(2 * W.shape[0] + 1, unit)
        # ---- interval rows (errors proportional to the summed terms)
        Ihn = Ih @ Wp + Il @ Wn + b
        Iln = Il @ Wp + Ih @ Wn + b
        eIh = (g * Ih.abs()) @ Wp - (g * Il.abs()) @ Wn
        eIl = (g * Il.abs()) @ Wp - (g * Ih.abs()) @ Wn
        ub = Ihn + gi * Ihn.abs() + eIh * (1 + 2 * g) + g * b.abs()
        lb = Iln - gi * Iln.abs() - eIl * (1 + 2 * g) - g * b.abs()
        if sym:
            _, _, MU = _concretize(U, lo, hi)
            _, _, ML = _concretize(L, lo, hi)
            aU = eU + g * MU
            aL = eL + g * ML
            Un = U @ Wp + L @ Wn
            Ln = L @ Wp + U @ Wn
            Un[:, -1, :] += b
            Ln[:, -1, :] += b
            eUn = (aU @ Wp - aL @ Wn) * (1 + 2 * g) + g * b.abs()
            eLn = (aL @ Wp - aU @ Wn) * (1 + 2 * g) + g * b.abs()
            lbU, ubU, MUn = _concretize(Un, lo, hi)
            lbL, ubL, MLn = _concretize(Ln, lo, hi)
            ub = torch.minimum(ub, ubU + gc * MUn + eUn)
            lb = torch.maximum(lb, lbL - gc * MLn - eLn)
        if keep_layers:
            layer_lb.append(lb)
            layer_ub.append(ub)
        if l == nL - 1:
            res = BoundResult(out_lb=lb[:, 0], out_ub=ub[:, 0])
            if sym:
                res.Lc, res.L0, res.Le = Ln[:, :-1, 0], Ln[:, -1, 0], eLn[:, 0]
                res.Uc, res.U0, res.Ue = Un[:, :-1, 0], Un[:, -1, 0], eUn[:, 0]
            break
        # ---------------- ReLU
        n = W.shape[1]
        is_dead = ub <= 0
        is_act = lb >= 0
        if dead is not None:
            forced = dead[:, off:off + n].bool()
        else:
            forced = torch.zeros_like(is_dead)
        fact = torch.zeros_like(is_dead)
        if phase is not None:
            ph = phase[:, off:off + n]
            forced = forced | (ph < 0)
            fact = ph > 0
            bad = ((ph < 0) & (lb > 0)) | ((ph > 0) & (ub < 0))
            infeas = bad.any(dim=1) if infeas is None else (infeas | bad.any(dim=1))
        off += n
        deads.append(is_dead)
        actives.append(is_act)
        zero = is_dead | forced
        Ih = torch.where(zero, torch.zeros_like(ub), ub.clamp(min=0))
        Il = torch.where(zero, torch.zeros_like(lb), lb.clamp(min=0))
        if not sym:
            continue
        # upper: identity if stable active -- or if the upper form T = U + eU itself stays >= 0
        # on the box (then relu(z) <= relu(T) = T; a chord from (a, 0) would cut below T) --
        # zero if dead, else the chord over [a, bb] of T
        a = lbU - gc * MUn + eUn
        bb = ubU + gc * MUn + eUn
        identU = (is_act | (a >= 0) | fact) & ~zero
        cross = ~(zero | identU)
        denom = torch.where(cross, bb - a, torch.ones_like(bb))
        s = torch.where(cross, (bb / denom) * (1 + 4 * unit), torch.ones_like(bb))
        shift = torch.where(cross, eUn - a, torch.zeros_like(bb))
        Unew = Un * s[:, None, :]
        Unew[:, -1, :] += s * shift
        eUc = 4 * unit * s * (MUn + shift.abs()) * cross
        eUnew = torch.where(identU, eUn, eUc)
        Unew = torch.where(zero[:, None, :], torch.zeros_like(Unew), Unew)
        eUnew = torch.where(zero, torch.zeros_like(eUnew), eUnew)
        # lower: lambda * (L(x) - eL), lambda in {0, 1}
        aL_ = lbL - gc * MLn - eLn
        bL_ = ubL + gc * MLn - eLn
        if lower_slope == "zero":
            lam1 = is_act
        elif lower_slope == "one":
            lam1 = bL_ > 0
        else:
            lam1 = is_act | ((bL_ > 0) & (bL_ > -aL_))
        lam1 = lam1 & ~zero
        Lnew = torch.where(lam1[:, None, :], Ln, torch.zeros_like(Ln))
        eLnew = torch.where(lam1, eLn, torch.zeros_like(eLn))
        U, L, eU, eL = Unew, Lnew, eUnew, eLnew
    if deads:
        res.dead = torch.cat(deads, dim=1)
        res.active = torch.cat(actives, dim=1)
    if phase is not None:
        res.infeasible = infeas if infeas is not None else torch.zeros(R, dtype=torch.bool, device=dev)
    if keep_layers:
        res.layer_lb, res.layer_ub = layer_lb, layer_ub
    return res


def _backsub(ws, bs, lo: torch.Tensor, hi: torch.Tensor, lbs, ubs, lam: torch.Tensor, c: torch.Tensor, top: int,
             dead: Optional[torch.Tensor], unit: float):
    """Back-substitute the linear function ``lam . h_{top-1} + c`` (rows [R, dims[top]]) through the
    ReLU relaxations of layers top-1 .. 0 down to the input box, with rigorous error terms
    (csrc/crown.hip, csrc/refine.hip).  Returns (coef [R, n0], const [R], err [R], lower bound [R])
    with ``lam . h + c >= coef . x + const - err >= low`` on the box for the exact network."""
    dt = lo.dtype
    R, n0 = lo.shape
    L = len(ws)
    offs = [0]
    for l in range(L - 1):
        offs.append(offs[-1] + ws[l].shape[1])
    mx_in = torch.maximum(lo.abs(), hi.abs())
    err = torch.zeros(R, dtype=dt, device=lo.device)
    for l in range(top - 1, -1, -1):
        W = ws[l].to(dt)
        b = bs[l].to(dt)
        n = W.shape[1]
        lb, ub = lbs[l].to(dt), ubs[l].to(dt)
        dd = ub <= 0
        if dead is not None:
            dd = dd | dead[:, offs[l]:offs[l] + n].bool()
        act = (lb >= 0) & ~dd
        unst = ~(dd | act)
        alpha = (ub > -lb).to(dt)
        den = torch.where(unst, ub - lb, torch.ones_like(ub))
        s = torch.where(unst, (ub / den) * (1 + 4 * unit), torch.zeros_like(ub))
        neg = unst & (lam < 0)
        slope = torch.where(act, torch.ones_like(ub), torch.where(dd, torch.zeros_like(ub),
                            torch.where(lam >= 0, alpha, s)))
        mu = lam * slope
        t = torch.where(neg, -mu * lb, torch.zeros_like(ub))
        # only the chord multipliers mu = lambda * s and intercepts t = -mu l are rounded
        zmax = torch.maximum(lb.abs(), ub.abs())
        e_rel = torch.where(neg, 3 * unit * (mu.abs() * zmax + t.abs()), torch.zeros_like(ub))
        g_c = gamma(2 * n + 1, unit)
        csum = (mu * b[None]).sum(1) + t.sum(1)
        cmag = c.abs() + (mu * b[None]).abs().sum(1) + t.abs().sum(1)
        c = c + csum
        if l > 0:                       # |h| of the layer below: max(0, ub), 0 if forced dead
            hm = ubs[l - 1].to(dt).clamp(min=0)
            if dead is not None:
                hm = torch.where(dead[:, offs[l - 1]:offs[l - 1] + W.shape[0]].bool(), torch.zeros_like(hm), hm)
        else:
            hm = mx_in
        lam = mu @ W.T
        eps = gamma(n + 1, unit) * (mu.abs() @ W.abs().T)
        err = err + e_rel.sum(1) + (eps * hm).sum(1) + g_c * cmag
    a = lam * lo
    bb = lam * hi
    conc = torch.minimum(a, bb).sum(1) + c
    cmg = (lam.abs() * mx_in).sum(1) + c.abs()
    err = err * (1 + 2 * gamma(2 * sum(int(w.shape[1]) for w in ws) + 4 * L + 4, unit))
    low = conc - err - gamma(n0 + 1, unit) * cmg - gamma(1, unit) * conc.abs()
    return lam, c, err, low


def crown_refine(ws: Sequence[torch.Tensor], bs: Sequence[torch.Tensor], lo: torch.Tensor, hi: torch.Tensor,
                 res: BoundResult, dead: Optional[torch.Tensor] = None, unit: Optional[float] = None) -> BoundResult:
    """Tighten the per-neuron pre-activation bounds of hidden layers 2 .. L-2 by back-substitution
    (csrc/refine.hip, same arithmetic and error terms).

    The forward symbolic pass relaxes every layer with the forms it propagated forward, so on deep
    networks the intermediate bounds -- and through the relaxation intervals every later bound --
    degrade with depth.  Here, layer by layer, every neuron z_k[j] = W_k[:, j] . h_{k-1} + b_k[j]
    is bounded by back-substituting +-W_k[:, j] to the input box through the relaxations of the
    layers below (CROWN for intermediate neurons), whose intervals are the already refined bounds;
    each bound is intersected with the forward one.  The output forms are then computed by
    :func:`crown_output` on the refined intervals.  On the bench residue this closes AC-7's
    partitions with a median of ~800 nodes where the forward intervals needed > 32 768
    (tools/diag_open_nodes.py --bound fullcrown, profiles/r4/refine/)."""
    dt = lo.dtype
    if unit is None:
        unit = FP64_UNIT if dt == torch.float64 else FP32_UNIT
    R, n0 = lo.shape
    L = len(ws)
    lbs = [t.clone() for t in res.layer_lb]
    ubs = [t.clone() for t in res.layer_ub]
    # from hidden layer 2 on (the kernel's rule): a layer-1 neuron back-substituted through layer 0
    # gets the forward pass's own relaxation choice per weight sign -- the same bounds up to rounding
    for k in range(2, L - 1):
        n_k = ws[k].shape[1]
        Wt = ws[k].to(dt).T                                       # [n_k, dims[k]]
        rep = lambda t: t.repeat_interleave(n_k, dim=0)          # noqa: E731  rows x targets
        rl, rh = rep(lo), rep(hi)
        lb_r, ub_r = [rep(t.to(dt)) for t in lbs[:k]], [rep(t.to(dt)) for t in ubs[:k]]
        d_r = rep(dead) if dead is not None else None
        low = {}
        for sg in (1.0, -1.0):
            lam = (sg * Wt)[None].expand(R, -1, -1).reshape(R * n_k, -1).clone()
            c = (sg * bs[k].to(dt))[None].expand(R, -1).reshape(-1).clone()
            low[sg] = _backsub(ws, bs, rl, rh, lb_r, ub_r, lam, c, k, d_r, unit)[3].view(R, n_k)
        # only unstable neurons are refined (the kernel's column list): a stable neuron's relaxation
        # is exact, its interval only enters rounding terms
        unst = (lbs[k] < 0) & (ubs[k] > 0)
        if dead is not None:
            off = sum(int(w.shape[1]) for w in ws[:k])
            unst = unst & ~dead[:, off:off + n_k].bool()
        lbs[k] = torch.where(unst, torch.maximum(lbs[k], low[1.0].to(lbs[k].dtype)), lbs[k])
        ubs[k] = torch.where(unst, torch.minimum(ubs[k], (-low[-1.0]).to(ubs[k].dtype)), ubs[k])
    r = BoundResult(out_lb=res.out_lb, out_ub=res.out_ub, Lc=res.Lc, L0=res.L0, Le=res.Le, Uc=res.Uc, U0=res.U0,
                    Ue=res.Ue, layer_lb=lbs, layer_ub=ubs)
    Nh = sum(int(w.shape[1]) for w in ws[:-1])
    if Nh:
        r.dead = torch.cat([u <= 0 for u in ubs[:-1]], dim=1)
        r.active = torch.cat([l >= 0 for l in lbs[:-1]], dim=1)
    return r



def backward_bounds(ws: Sequence[torch.Tensor], bs: Sequence[torch.Tensor], lo: torch.Tensor, hi: torch.Tensor,
                    dead: Optional[torch.Tensor] = None, unit: Optional[float] = None) -> BoundResult:
    """Bounds of every neuron and the logit's linear forms by back-substitution alone (csrc/refine.hip,
    mode FULL): layer 0 from the box, each hidden layer k by back-substituting +-W_k[:, j] through the
    relaxations of the layers below, the logit's forms likewise -- no forward symbolic pass.  On the
    deep nets the forward intervals add nothing to these (the refined bounds close the same AC-7
    residue with or without them, tools/diag_open_nodes.py --bound fullcrown vs crown_refine), so the
    BaB bounds them with this one pass instead of forward + refine + output (3 launches -> 1)."""
    dt = lo.dtype
    if unit is None:
        unit = FP64_UNIT if dt == torch.float64 else FP32_UNIT
    R, n0 = lo.shape
    L = len(ws)
    lbs, ubs = [], []
    for k in range(L - 1):
        n_k = ws[k].shape[1]
        Wt = ws[k].to(dt).T
        rep = lambda t: t.repeat_interleave(n_k, dim=0)          # noqa: E731
        rl, rh = rep(lo), rep(hi)
        lb_r, ub_r = [rep(t) for t in lbs], [rep(t) for t in ubs]
        d_r = rep(dead) if dead is not None else None
        low = {}
        for sg in (1.0, -1.0):
            lam = (sg * Wt)[None].expand(R, -1, -1).reshape(R * n_k, -1).clone()
            c = (sg * bs[k].to(dt))[None].expand(R, -1).reshape(-1).clone()
            low[sg] = _backsub(ws, bs, rl, rh, lb_r, ub_r, lam, c, k, d_r, unit)[3].view(R, n_k)
        lbs.append(low[1.0])
        ubs.append(-low[-1.0])
    inf = torch.full((R,), float("inf"), dtype=dt, device=lo.device)
    base = BoundResult(out_lb=-inf, out_ub=inf, Lc=torch.zeros(R, n0, dtype=dt, device=lo.device),
                       L0=torch.zeros(R, dtype=dt, device=lo.device), Le=inf.clone(),
                       Uc=torch.zeros(R, n0, dtype=dt, device=lo.device), U0=torch.zeros(R, dtype=dt, device=lo.device),
                       Ue=inf.clone(), layer_lb=lbs + [-inf[:, None]], layer_ub=ubs + [inf[:, None]])
    r = crown_output(ws, bs, lo, hi, base, dead, unit=unit)
    r.layer_lb = lbs + [r.out_lb[:, None]]
    r.layer_ub = ubs + [r.out_ub[:, None]]
    if lbs:
        r.dead = torch.cat([u <= 0 for u in ubs], dim=1)
        if dead is not None:
            r.dead = r.dead | dead.bool()       # forced-zero neurons are dead whatever their bounds
        r.active = torch.cat([l >= 0 for l in lbs], dim=1) & ~r.dead
    return r


def crown_output(ws: Sequence[torch.Tensor], bs: Sequence[torch.Tensor], lo: torch.Tensor, hi: torch.Tensor,
                 res: BoundResult, dead: Optional[torch.Tensor] = None, unit: Optional[float] = None) -> BoundResult:
    """Backward (CROWN-style) linear bounds of the logit, replacing the forward-symbolic output
    forms of ``res`` where they are tighter (csrc/crown.hip, same arithmetic and error terms).

    The forward pass concretises each layer's forms before relaxing it, so the relaxation
    slack of every layer is propagated as a fixed interval term; back-substituting from the
    output instead picks, per neuron, the relaxation that the sign of its output multiplier
    needs (lower: h >= a z with a in {0, 1}; upper: the chord h <= s (z - l)).  The per-neuron
    pre-activation bounds ``res.layer_lb/layer_ub`` of the forward pass are the relaxation
    intervals.  On the deep AC shapes this halves the open BaB frontier (tools/diag_open_nodes.py).

    Rounding: every multiplier mu = lambda * slope, intercept t = -mu l, back-substituted
    coefficient lambda' = W mu and constant sum carries a gamma-bounded error, accumulated with
    the magnitudes of the layer's inputs (|x| on the box, max(0, ub) of hidden outputs) into the
    form's error term, so ``sigma * y >= lambda . x + c - err`` holds for the exact network.
    """
    dt = lo.dtype
    if unit is None:
        unit = FP64_UNIT if dt == torch.float64 else FP32_UNIT
    R, n0 = lo.shape
    L = len(ws)
    out = {}
    for sg in (1.0, -1.0):
        lam = (sg * ws[L - 1][:, 0].to(dt))[None].expand(R, -1).clone()
        c = torch.full((R,), sg * float(bs[L - 1][0]), dtype=dt, device=lo.device)
        out[sg] = _backsub(ws, bs, lo, hi, res.layer_lb, res.layer_ub, lam, c, L - 1, dead, unit)
    lamL, cL, eL, lowL = out[1.0]
    lamU, cU, eU, lowU = out[-1.0]
    r = BoundResult(out_lb=torch.maximum(res.out_lb, lowL.to(res.out_lb.dtype)),
                    out_ub=torch.minimum(res.out_ub, (-lowU).to(res.out_ub.dtype)))
    r.layer_lb, r.layer_ub, r.dead, r.active = res.layer_lb, res.layer_ub, res.dead, res.active
    # per row, keep the forward forms where they concretise tighter (both are sound)
    useL = (lowL >= res.out_lb.to(dt))[:, None]
    useU = ((-lowU) <= res.out_ub.to(dt))[:, None]
    r.Lc = torch.where(useL, lamL, res.Lc.to(dt)).to(res.Lc.dtype)
    r.L0 = torch.where(useL[:, 0], cL, res.L0.to(dt)).to(res.L0.dtype)
    r.Le = torch.where(useL[:, 0], eL, res.Le.to(dt)).to(res.Le.dtype)
    r.Uc = torch.where(useU, -lamU, res.Uc.to(dt)).to(res.Uc.dtype)
    r.U0 = torch.where(useU[:, 0], -cU, res.U0.to(dt)).to(res.U0.dtype)
    r.Ue = torch.where(useU[:, 0], eU, res.Ue.to(dt)).to(res.Ue.dtype)
    return r


@dataclass
class PhaseCrown:
    """Backward bounds of the ReLU-split search (:func:`crown_phase`), per row and sign
    (column 0: lower bound of N, column 1: lower bound of -N)."""
    low: torch.Tensor           # [R, 2] best lower bound over concretisation layers and slope policies
    split: torch.Tensor         # [R, 2] int64 hidden-neuron index to split for that bound (-1: none)
    score: torch.Tensor         # [R, 2] its score


ALPHA_POLICIES = ("adaptive", "zero", "one")


def crown_phase(ws: Sequence[torch.Tensor], bs: Sequence[torch.Tensor], lo: torch.Tensor, hi: torch.Tensor,
                res: BoundResult, phase: Optional[torch.Tensor] = None, unit: Optional[float] = None,
                policies: Sequence[str] = ALPHA_POLICIES):
    """Backward (CROWN) bounds of the logit for the ReLU-phase search, concretised at EVERY layer.

    ``res`` = forward bounds of the rows (with ``phase``, keep_layers).  For each sign and each
    lower-slope policy (adaptive = the forward pass's rule, all 0, all 1) the multipliers are
    back-substituted from the logit; at every hidden layer the bound ``sigma N >= sum lambda_j a_j +
    c`` is concretised over the post-activation ranges ``a_j in [max(lb, 0), max(ub, 0)]`` before
    the layer is relaxed, and finally over the input box.  The best value wins.

    Exact zeros: the coefficient errors are kept per coefficient (``E``, the rounding of
    ``lambda = W mu``) until the next layer, so a term whose range starts at 0 and whose
    coefficient is certainly >= 0 contributes exactly 0 with no rounding charge.  On zero-bias
    networks (the random-init bench models) a branch where every path to a positive logit is
    closed then bounds the logit by exactly 0 -- the strict ``N(x) < 0 < N(x')`` query needs that
    (csrc/relu.hip: fa_crown_phase_kernel has the same arithmetic).

    Split choice per (row, sign), from the policy with the best bound: the unstable unsplit neuron
    with the largest chord intercept ``|mu_j l_j|`` the bound pays (+ 1e-3 |lambda_j| x triangle
    gap as a tie-break); forced-active neurons have no intercept.  Returns (:class:`PhaseCrown`,
    input forms {sign: (coef [R, n0], const [R], err [R], low_at_input [R])} of the policy with
    the best input-level bound).
    """
    dt = lo.dtype
    if unit is None:
        unit = FP64_UNIT if dt == torch.float64 else FP32_UNIT
    R, n0 = lo.shape
    L = len(ws)
    dev = lo.device
    lbs, ubs = res.layer_lb, res.layer_ub
    offs = [0]
    for l in range(L - 1):
        offs.append(offs[-1] + ws[l].shape[1])
    mx_in = torch.maximum(lo.abs(), hi.abs())
    K = 4 * L + 4 + sum(2 * int(w.shape[1]) for w in ws)
    gK = gamma(K, unit)
    low = torch.full((R, 2), -float("inf"), dtype=dt, device=dev)
    split = torch.full((R, 2), -1, dtype=torch.int64, device=dev)
    score = torch.zeros(R, 2, dtype=dt, device=dev)
    forms = {}
    ar = torch.arange(R, device=dev)
    for si, sg in enumerate((1.0, -1.0)):
        best_in = None
        for pol in policies:
            lam = (sg * ws[L - 1][:, 0].to(dt))[None].expand(R, -1).clone()
            E = torch.zeros_like(lam)
            c = torch.full((R,), sg * float(bs[L - 1][0]), dtype=dt, device=dev)
            err = torch.zeros(R, dtype=dt, device=dev)
            pol_best = torch.full((R,), -float("inf"), dtype=dt, device=dev)
            sc_best = torch.full((R,), -1.0, dtype=dt, device=dev)
            sc_idx = torch.full((R,), -1, dtype=torch.int64, device=dev)
            for l in range(L - 2, -1, -1):
                W = ws[l].to(dt)
                b = bs[l].to(dt)
                n = W.shape[1]
                lb, ub = lbs[l].to(dt), ubs[l].to(dt)
                ph = phase[:, offs[l]:offs[l] + n] if phase is not None else torch.zeros_like(lb, dtype=torch.int8)
                dd = (ub <= 0) | (ph < 0)
                fact = (ph > 0) & ~dd
                act = (lb >= 0) & ~dd
                unst = ~(dd | act)
                # ---- concretise at this layer's post-activations a_j in [alo, ahi]
                alo = torch.where(dd, torch.zeros_like(lb), lb.clamp(min=0))
                ahi = torch.where(dd, torch.zeros_like(ub), ub.clamp(min=0))
                exact0 = (ahi == 0) | ((alo == 0) & (lam - E >= 0))
                prod = torch.minimum(lam * alo, lam * ahi)
                eprod = E * ahi
                term = torch.where(exact0, torch.zeros_like(prod), prod - eprod)
                tv = term.sum(1) + c
                tmag = torch.where(exact0, torch.zeros_like(prod), prod.abs() + eprod).sum(1) + c.abs()
                v = tv - err * (1 + 2 * gK) - gamma(n + 3, unit) * tmag
                pol_best = torch.maximum(pol_best, v)
                # ---- coefficients of uncertain sign (|lambda| <= E): relax lambda (the computed
                # value) and charge the difference E |a| to the constant; certain signs keep the
                # interval [lambda - E, lambda + E] through the relaxation (no charge)
                unc = ((lam - E) < 0) & ((lam + E) > 0) & ~dd
                err = err + torch.where(unc, E * ahi, torch.zeros_like(E)).sum(1)
                E = torch.where(unc | dd, torch.zeros_like(E), E)
                # ---- relax this layer's ReLUs
                if pol == "adaptive":
                    alpha = (ub > -lb).to(dt)
                elif pol == "zero":
                    alpha = torch.zeros_like(ub)
                else:
                    alpha = torch.ones_like(ub)
                chord_ok = unst & ~fact
                den = torch.where(chord_ok, ub - lb, torch.ones_like(ub))
                s_ch = torch.where(chord_ok, (ub / den) * (1 + 4 * unit), torch.ones_like(ub))
                slope = torch.where(act, torch.ones_like(ub), torch.where(dd, torch.zeros_like(ub),
                                    torch.where(lam >= 0, alpha, s_ch)))
                mu = lam * slope
                chord = chord_ok & (lam < 0)
                t = torch.where(chord, -mu * lb, torch.zeros_like(ub))
                zmax = torch.maximum(lb.abs(), ub.abs())
                # chord multipliers / intercepts are rounded (and carry E through the intercept)
                e_rel = torch.where(chord, 3 * unit * (mu.abs() * zmax + t.abs()) + E * s_ch * lb.abs(),
                                    torch.zeros_like(ub))
                Emu = E * slope * (1 + 4 * unit)            # |mu_hat - mu| from the coefficient interval
                # split score: the chord intercept this bound pays (+ tie-break on the triangle gap)
                gap = torch.where(chord_ok, -ub * lb / den, torch.zeros_like(ub))
                sc = torch.where(chord_ok, t.abs() + 1e-3 * lam.abs() * gap, torch.full_like(ub, -1.0))
                if phase is not None:
                    sc = torch.where(ph != 0, torch.full_like(sc, -1.0), sc)
                smax, sarg = sc.max(dim=1)
                better = smax > sc_best
                sc_best = torch.where(better, smax, sc_best)
                sc_idx = torch.where(better, sarg + offs[l], sc_idx)
                csum = (mu * b[None]).sum(1) + t.sum(1)
                cmag = c.abs() + (mu * b[None]).abs().sum(1) + t.abs().sum(1)
                c = c + csum
                err = err + e_rel.sum(1) + gamma(2 * n + 1, unit) * cmag + (Emu * b[None].abs()).sum(1)
                lam = mu @ W.T
                # new coefficient interval: propagated E through |W| plus the rounding of W mu
                E = (Emu @ W.abs().T) * (1 + gamma(n + 1, unit)) + gamma(n + 1, unit) * (mu.abs() @ W.abs().T)
            # ---- concretise over the input box
            err_in = (err + (E * mx_in).sum(1)) * (1 + 2 * gK)
            a_ = lam * lo
            b_ = lam * hi
            conc = torch.minimum(a_, b_).sum(1) + c
            cmg = (lam.abs() * mx_in).sum(1) + c.abs()
            low_in = conc - err_in - gamma(n0 + 1, unit) * cmg - gamma(1, unit) * conc.abs()
            pol_best = torch.maximum(pol_best, low_in)
            take = pol_best > low[:, si]
            low[:, si] = torch.where(take, pol_best, low[:, si])
            split[:, si] = torch.where(take, sc_idx, split[:, si])
            score[:, si] = torch.where(take, sc_best, score[:, si])
            if best_in is None:
                best_in = (lam, c, err_in, low_in)
            else:
                tk = low_in > best_in[3]
                best_in = (torch.where(tk[:, None], lam, best_in[0]), torch.where(tk, c, best_in[1]),
                           torch.where(tk, err_in, best_in[2]), torch.where(tk, low_in, best_in[3]))
        forms[sg] = best_in
    split = torch.where(score > 0, split, torch.full_like(split, -1))
    return PhaseCrown(low=low, split=split, score=score), forms


# ======================================================================================
# Fairness-pair certificate (branch-and-bound node test)
# ======================================================================================

@dataclass
class PairDecision:
    open_: torch.Tensor       # [Nn] bool: some valid pair not certified impossible
    score: torch.Tensor       # [Nn] best (largest) certificate value g*  (>0 means open)
    split_dim: torch.Tensor   # [Nn] int64 index into the 2n0 split space (x dims then x' dims)
    cand_x: torch.Tensor      # [Nn, n0] candidate violating x
    cand_xp: torch.Tensor     # [Nn, n0] candidate violating x'
    cand_v: torch.Tensor      # [Nn] pair index (into pairs) of the candidate
    cand_orient: torch.Tensor  # [Nn] 0: N(x)<0<N(x'), 1: N(x)>0>N(x')


def pair_certify(res_x: BoundResult, res_xp: BoundResult, xlo: torch.Tensor, xhi: torch.Tensor,
                 xplo: torch.Tensor, xphi: torch.Tensor, pairs: torch.Tensor, values: torch.Tensor,
                 pa: torch.Tensor, shared: torch.Tensor, relaxed: bool, unit: float = FP32_UNIT,
                 n_t: int = 0) -> PairDecision:
    """Decide for every node whether any fairness violation may exist inside it.

    Rows of ``res_x`` / ``res_xp`` are node-major, V rows per node (PA assignment v).  For an
    ordered pair (v, v') and orientation A (``N(x,v) < 0 < N(x',v')``) the node is clean if
    some t in [0,1] gives  max_{x,x'} t(-L_v(x) + eL) + (1-t)(U_v'(x') + eU)  <= 0 — a convex
    (minimax / LP-duality) certificate that couples x and x' through their shared features.
    t = 1 / t = 0 are the plain interval tests; the optimum t is at a breakpoint of the
    piecewise-linear objective, all of which are evaluated.  Orientation B swaps signs.  With
    no relaxed attributes orientation B of (v, v') is orientation A of (v', v) and is skipped.

    Shared features (``shared[i]``) use x_i = x'_i; PA features take the fixed row values;
    relaxed features vary independently over the x box and the (wider) x' box.
    """
    dt = xlo.dtype
    Nn, n0 = xlo.shape
    P = pairs.shape[0]
    V = values.shape[0]
    dev = xlo.device
    vals = values.to(dt)

    def fold(C, c0):
        # PA coordinates are fixed per row: move their terms into the constant
        C = C.view(Nn, V, n0).clone()
        terms = C[:, :, pa] * vals[None]
        contrib = terms.sum(-1)
        C[:, :, pa] = 0
        # rounding margin over the products' magnitudes (several PA dims can cancel in the sum)
        return C, c0.view(Nn, V) + contrib, terms.abs().sum(-1)

    Lc, L0, fL = fold(res_x.Lc, res_x.L0 - res_x.Le)      # lower form minus its error
    Uc, U0, fU = fold(res_x.Uc, res_x.U0 + res_x.Ue)
    Lcp, L0p, fLp = fold(res_xp.Lc, res_xp.L0 - res_xp.Le)
    Ucp, U0p, fUp = fold(res_xp.Uc, res_xp.U0 + res_xp.Ue)
    vi, vj = pairs[:, 0], pairs[:, 1]
    orients = [0, 1] if relaxed else [0]
    best_g = torch.full((Nn,), -math.inf, dtype=dt, device=dev)
    best = None
    sh = shared.to(dt)[None, None, :]
    for o in orients:
        if o == 0:   # t * (-L_v(x)) + (1-t) * U_v'(x')
            A_c, A_0, fA = -Lc[:, vi, :], -L0[:, vi], fL[:, vi]
            B_c, B_0, fB = Ucp[:, vj, :], U0p[:, vj], fUp[:, vj]
        else:        # t * U_v(x) + (1-t) * (-L_v'(x'))
            A_c, A_0, fA = Uc[:, vi, :], U0[:, vi], fU[:, vi]
            B_c, B_0, fB = -Lcp[:, vj, :], -L0p[:, vj], fLp[:, vj]
        # magnitudes for rounding margins
        mx = torch.maximum(xlo.abs(), xhi.abs())[:, None, :]
        mxp = torch.maximum(xplo.abs(), xphi.abs())[:, None, :]
        magA = (A_c.abs() * mx).sum(-1) + A_0.abs() + fA
        magB = (B_c.abs() * mxp).sum(-1) + B_0.abs() + fB
        # candidate t values: endpoints + breakpoints of shared coefficients
        with torch.no_grad():
            den = A_c - B_c
            tb = torch.where(den.abs() > 0, -B_c / torch.where(den.abs() > 0, den, torch.ones_like(den)),
                             torch.full_like(den, -1.0))
            tb = torch.where(sh.bool().expand_as(tb), tb, torch.full_like(tb, -1.0))
            tb = tb.clamp(min=-1.0, max=2.0)
            ts = torch.cat([torch.zeros_like(tb[..., :1]), torch.ones_like(tb[..., :1]), tb], dim=-1)
            if n_t:
                grid = torch.linspace(0, 1, n_t, dtype=dt, device=dev).expand(Nn, P, n_t)
                ts = torch.cat([ts, grid], dim=-1)
            ts = ts.clamp(0.0, 1.0)                                    # [Nn, P, T]
        T = ts.shape[-1]
        t = ts[..., :, None]                                           # [Nn,P,T,1]
        Ac = A_c[:, :, None, :]
        Bc = B_c[:, :, None, :]
        xl, xh = xlo[:, None, None, :], xhi[:, None, None, :]
        xpl, xph = xplo[:, None, None, :], xphi[:, None, None, :]
        # shared dims: combined coefficient on x
        cs = t * Ac + (1 - t) * Bc
        val_s = torch.maximum(cs * xl, cs * xh)
        # separate dims: x part and x' part
        ca = t * Ac
        cb = (1 - t) * Bc
        val_sep = torch.maximum(ca * xl, ca * xh) + torch.maximum(cb * xpl, cb * xph)
        val = torch.where(sh.bool()[:, :, None, :].expand_as(val_s), val_s, val_sep).sum(-1)
        g = val + t[..., 0] * A_0[:, :, None] + (1 - t[..., 0]) * B_0[:, :, None]
        marg = gamma(2 * n0 + 4, unit) * (t[..., 0] * magA[:, :, None] + (1 - t[..., 0]) * magB[:, :, None]) \
            + 8 * unit * (magA + magB)[:, :, None]
        g = g + marg
        gmin, targ = g.min(dim=-1)                                     # [Nn, P]
        # exact-sign shortcut from the rigorous per-row interval bounds
        olb_x, oub_x = res_x.out_lb.view(Nn, V), res_x.out_ub.view(Nn, V)
        olb_p, oub_p = res_xp.out_lb.view(Nn, V), res_xp.out_ub.view(Nn, V)
        if o == 0:
            imp = (olb_x[:, vi] >= 0) | (oub_p[:, vj] <= 0)
        else:
            imp = (oub_x[:, vi] <= 0) | (olb_p[:, vj] >= 0)
        gmin = torch.where(imp, torch.full_like(gmin, -1.0), gmin)
        gbest, pbest = gmin.max(dim=-1)                                # [Nn]
        upd = gbest > best_g
        tstar = torch.gather(ts, 2, targ[:, :, None])[..., 0]          # [Nn, P]
        tsel = tstar.gather(1, pbest[:, None])[:, 0]                   # [Nn]
        Acs = A_c.gather(1, pbest[:, None, None].expand(Nn, 1, n0))[:, 0]
        Bcs = B_c.gather(1, pbest[:, None, None].expand(Nn, 1, n0))[:, 0]
        cur = dict(g=gbest, p=pbest, t=tsel, Ac=Acs, Bc=Bcs, o=torch.full_like(pbest, o))
        if best is None:
            best = cur
        else:
            for k in best:
                if best[k].dim() == 1:
                    best[k] = torch.where(upd, cur[k], best[k])
                else:
                    best[k] = torch.where(upd[:, None], cur[k], best[k])
        best_g = torch.maximum(best_g, gbest)
    open_ = best_g > 0
    t = best["t"][:, None]
    Ac, Bc = best["Ac"], best["Bc"]
    shb = shared.bool()[None, :]
    # split score: contribution width * |coef| at t*  (x dims then x' dims for relaxed features)
    cs = t * Ac + (1 - t) * Bc
    wx = (xhi - xlo)
    wxp = (xphi - xplo)
    sx = torch.where(shb, cs.abs() * wx, (t * Ac).abs() * wx)
    sxp = torch.where(shb, torch.zeros_like(wxp), ((1 - t) * Bc).abs() * wxp)
    # tie-break toward the widest dim so that zero-coefficient dims still get split eventually
    sx = sx + 1e-9 * wx
    sxp = sxp + 1e-9 * wxp
    sx[:, pa] = -1.0                      # PA coordinates are enumerated, never split
    sxp[:, pa] = -1.0
    split_dim = torch.cat([sx, sxp], dim=1).argmax(dim=1)
    # candidate vertex maximising the objective at t*
    cx_s = torch.where(cs > 0, xhi, xlo)
    cx_a = torch.where(t * Ac > 0, xhi, xlo)
    cand_x = torch.where(shb, cx_s, cx_a)
    cxp = torch.where((1 - t) * Bc > 0, xphi, xplo)
    cand_xp = torch.where(shb, cand_x, cxp)
    return PairDecision(open_=open_, score=best_g, split_dim=split_dim, cand_x=cand_x, cand_xp=cand_xp,
                        cand_v=best["p"], cand_orient=best["o"])
