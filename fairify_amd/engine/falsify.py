"""Residual falsifier: heavy sampling + lattice local search on the BaB residue (K8, extended).

The reference finds counterexamples only through Z3 (src/AC/Verify-AC.py:158-163) and its
1 000-point simulation only nominates dead neurons (utils/prune.py:168-222).  Partitions that
stay UNKNOWN after the device branch-and-bound are often SAT with violating pairs occupying
a tiny fraction of the box (e.g. ~0.04 % of the lattice points): the first-stage simulation and
the LP-optimal vertex candidates of the BaB miss them.  For those partitions only:

1. draw ``n_samples`` fresh lattice points per partition (same counter-based hash stream as
   the simulation, different seed) and evaluate every protected-attribute assignment on the
   device (HIP forward kernel);
2. the violation margin of a point for an ordered PA pair (v, v') is
   ``f = min(-N(x, v), N(x', v'))`` — a strict violation iff ``f > 0``;
3. from the ``k_starts`` best points, coordinate ascent on the integer lattice: every ±1 move
   of a non-protected feature (and of the relaxed offset x'_r - x_r within [-tau, tau]) is
   evaluated in one batched forward, the best improving move is taken, ``iters`` rounds.
   On the HIP path all three steps -- heavy sampling, the boundary walk of
   :func:`engine.sim.boundary_walk` and the ascent -- run in ONE ``fa_falsify_kernel`` launch
   (``csrc/falsify.hip``, register-resident MFMA forward); each partition stops at its first hit.
   Relaxed queries run in the same launch: every sample carries its RA offsets (the hash stream
   below), the ascent moves them too, and both orientations of a pair count.

Hits are only *candidates*: the pipeline confirms them with the exact checker
(:mod:`fairify_amd.engine.exact`) before a partition becomes SAT.
"""
from __future__ import annotations

import os
from dataclasses import dataclass
from typing import Optional

import torch

from ..ops import reference as ref
from ..ops.backend import Backend
from ..spec import ResolvedQuery


@dataclass
class FalsifyResult:
    found: torch.Tensor       # [P] bool
    wit_x: torch.Tensor       # [P, n0] float (integral values)
    wit_xp: torch.Tensor
    how: Optional[torch.Tensor] = None   # [P] int8 (fused kernel): 1 sampling, 2 boundary walk, 3 local search


def _margins(be: Backend, X: torch.Tensor, D: torch.Tensor, pa: torch.Tensor, ra: torch.Tensor,
             vals: torch.Tensor, pairs: torch.Tensor, relaxed: bool) -> torch.Tensor:
    """X [p, K, n] points, D [p, K, nra] relaxed offsets -> margins [p, K, Q]; Q = Pp (x and x'
    share every non-protected feature, so the pair list covers both orientations) or 2 Pp."""
    p_, K, n = X.shape
    V = vals.shape[0]
    XV = X[:, :, None, :].expand(p_, K, V, n).clone()
    XV[:, :, :, pa] = vals[None, None].expand(p_, K, V, -1)
    z = be.forward(XV.reshape(-1, n)).view(p_, K, V)
    if relaxed:
        XPV = XV.clone()
        XPV[:, :, :, ra] = XV[:, :, :, ra] + D[:, :, None, :]
        zp = be.forward(XPV.reshape(-1, n)).view(p_, K, V)
    else:
        zp = z
    f = torch.minimum(-z[..., pairs[:, 0]], zp[..., pairs[:, 1]])       # N(x,v) < 0 < N(x',v')
    if relaxed:                                                          # x' may leave the box:
        f2 = torch.minimum(z[..., pairs[:, 0]], -zp[..., pairs[:, 1]])  # the other orientation
        f = torch.cat([f, f2], dim=-1)
    return f


def residual_falsify(be: Backend, q: ResolvedQuery, lo: torch.Tensor, hi: torch.Tensor, pids: torch.Tensor,
                     values: torch.Tensor, pairs: torch.Tensor, seed: int, n_samples: int = 8192,
                     k_starts: int = 16, iters: int = 24, sub: int = 1024, n_local: int = 512) -> FalsifyResult:
    """On the HIP path the heavy sampling runs in the fused simulation kernel (points never
    leave registers, plus its boundary walk); the local search then starts from the best of
    ``n_local`` materialised samples of the partitions still without a witness."""
    P, n = lo.shape
    dev = lo.device
    if be.hip and P and os.environ.get("FAIRIFY_FUSED_FALSIFY", "1") != "0":
        from ..ops import hip

        free = [d for d in range(n) if d not in set(q.pa_idx)]
        out = hip.falsify(be, q, lo, hi, pids, values, pairs, (seed ^ 0x6A09E667) & 0xFFFFFFFF, n_samples, n_local,
                          16, 12, k_starts, iters, free, dseed=(seed ^ 0x3C6EF372) & 0xFFFFFFFF)
        if out is not None:
            return FalsifyResult(out[0], out[1], out[2], how=out[3])
    if be.hip and P:
        from ..ops import hip

        sim = hip.simulate(be, q, lo, hi, pids, n_samples, (seed ^ 0x6A09E667) & 0xFFFFFFFF, values, pairs, 16, 12)
        rest = torch.nonzero(~sim.found).flatten()
        res = FalsifyResult(sim.found.clone(), sim.wit_x.clone(), sim.wit_xp.clone())
        if rest.numel():
            r2 = _local_search(be, q, lo[rest], hi[rest], pids[rest], values, pairs, seed, n_local, k_starts, iters,
                               sub)
            res.found[rest] = r2.found
            res.wit_x[rest] = torch.where(r2.found[:, None], r2.wit_x, res.wit_x[rest])
            res.wit_xp[rest] = torch.where(r2.found[:, None], r2.wit_xp, res.wit_xp[rest])
        return res
    return _local_search(be, q, lo, hi, pids, values, pairs, seed, n_samples, k_starts, iters, sub)


def _local_search(be: Backend, q: ResolvedQuery, lo: torch.Tensor, hi: torch.Tensor, pids: torch.Tensor,
                  values: torch.Tensor, pairs: torch.Tensor, seed: int, n_samples: int, k_starts: int, iters: int,
                  sub: int) -> FalsifyResult:
    P, n = lo.shape
    dev = lo.device
    pa = torch.tensor(list(q.pa_idx), device=dev, dtype=torch.long)
    relaxed = q.relaxed
    ra = torch.tensor(list(q.ra_idx) if relaxed else [], device=dev, dtype=torch.long)
    nra = int(ra.numel())
    tau = float(q.tau)
    vals = values.to(torch.float32)
    Pp = pairs.shape[0]
    found = torch.zeros(P, dtype=torch.bool, device=dev)
    wx = torch.zeros(P, n, device=dev)
    wxp = torch.zeros(P, n, device=dev)
    if P == 0 or Pp == 0:
        return FalsifyResult(found, wx, wxp)
    free = torch.ones(n, dtype=torch.bool, device=dev)
    free[pa] = False
    fdims = torch.nonzero(free).flatten()
    # move set: +-1 on every non-protected feature, +-1 on every relaxed offset
    nm = 2 * fdims.numel() + 2 * nra
    MX = torch.zeros(nm, n, device=dev)
    MD = torch.zeros(nm, nra, device=dev)
    mi = 0
    for d in fdims.tolist():
        MX[mi, d], MX[mi + 1, d] = -1.0, 1.0
        mi += 2
    for r in range(nra):
        MD[mi, r], MD[mi + 1, r] = -1.0, 1.0
        mi += 2
    for s0 in range(0, P, sub):
        sl = slice(s0, min(P, s0 + sub))
        plo, phi, ppid = lo[sl], hi[sl], pids[sl]
        p_ = plo.shape[0]
        X = ref.sample_points(plo, phi, ppid, n_samples, seed ^ 0x6A09E667)          # [p, S, n]
        if relaxed:
            h = ref.rng_u32(seed ^ 0x3C6EF372, ppid.to(torch.int64)[:, None, None],
                            torch.arange(n_samples, device=dev)[None, :, None], ra[None, None, :])
            D = (h % (2 * q.tau + 1)).to(torch.float32) - tau
        else:
            D = torch.zeros(p_, n_samples, 0, device=dev)
        f = _margins(be, X, D, pa, ra, vals, pairs, relaxed)                          # [p, S, Pp]
        fbest, pbest = f.max(dim=2)                                                   # [p, S]
        # ---- local search from the k best starts
        k = min(k_starts, n_samples)
        top = fbest.topk(k, dim=1).indices
        ar = torch.arange(p_, device=dev)[:, None]
        cx = X[ar, top]                                                               # [p, k, n]
        cd = D[ar, top]                                                               # [p, k, nra]
        cf = fbest[ar, top]
        cp = pbest[ar, top]
        if be.hip and not relaxed and nm:
            from ..ops import hip

            out = hip.ascent(be, q, plo, phi, cx, cf, cp, iters, values, pairs, fdims.tolist())
            if out is not None:
                g = torch.nonzero(out[0]).flatten()
                idx = torch.arange(s0, s0 + p_, device=dev)[g]
                found[idx] = True
                wx[idx] = out[1][g]
                wxp[idx] = out[2][g]
                continue
        for _ in range(iters if nm else 0):
            if bool((cf > 0).any(dim=1).all()):
                break
            NX = torch.minimum(torch.maximum(cx[:, :, None, :] + MX[None, None], plo[:, None, None, :]),
                               phi[:, None, None, :])
            ND = torch.clamp(cd[:, :, None, :] + MD[None, None], -tau, tau)
            nf = _margins(be, NX.view(p_, k * nm, n), ND.view(p_, k * nm, nra), pa, ra, vals, pairs,
                          relaxed).view(p_, k, nm, -1)
            nfb, npb = nf.max(dim=3)                                                  # [p, k, nm]
            mv, mj = nfb.max(dim=2)                                                   # [p, k]
            imp = mv > cf
            if not bool(imp.any()):
                break
            a2 = torch.arange(k, device=dev)[None, :]
            cx = torch.where(imp[..., None], NX[ar, a2, mj], cx)
            cd = torch.where(imp[..., None], ND[ar, a2, mj], cd)
            cp = torch.where(imp, npb[ar, a2, mj], cp)
            cf = torch.where(imp, mv, cf)
        hit = cf > 0                                                                  # [p, k]
        anyh = hit.any(dim=1)
        if bool(anyh.any()):
            j = hit.float().argmax(dim=1)
            r_ = torch.arange(p_, device=dev)
            bx = cx[r_, j]
            pp = pairs[cp[r_, j] % Pp]
            x = bx.clone()
            xp = bx.clone()
            x[:, pa] = vals[pp[:, 0]]
            xp[:, pa] = vals[pp[:, 1]]
            if relaxed:
                xp[:, ra] = bx[:, ra] + cd[r_, j]
            g = torch.nonzero(anyh).flatten()
            idx = torch.arange(s0, s0 + p_, device=dev)[g]
            found[idx] = True
            wx[idx] = x[g]
            wxp[idx] = xp[g]
    return FalsifyResult(found, wx, wxp)
