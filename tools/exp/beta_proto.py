#!/usr/bin/env python
"""CPU feasibility prototype (fp64 torch): beta-CROWN-style ReLU-phase branch-and-bound for the
coupled fairness certificate on residue partitions -- slopes alpha, split multipliers beta and the
mixing weight t optimised per node by projected gradient; nodes branch on the unstable neuron whose
chord the bound pays most.  Compare node counts with the verified LP (tools/exp/lp_tree_sizes.py).

    python tools/exp/beta_proto.py --model AC-7 --weights zoo --pids 5564,5302,12545 --budget 2000
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))

from fairify_amd.ops import reference as ref  # noqa: E402


def layer_bounds(ws, bs, lo, hi, phase):
    """Rigorous per-layer pre-activation bounds of rows [R] with fixed phases [R, NH] (fp64):
    forward symbolic with phases, clamped, back-substitution refinement, clamped again."""
    res = ref.bounds(ws, bs, lo, hi, mode="symbolic", keep_layers=True, phase=phase)
    lbs, ubs = [t.clone() for t in res.layer_lb], [t.clone() for t in res.layer_ub]
    off = 0
    for l in range(len(ws) - 1):
        n = ws[l].shape[1]
        ph = phase[:, off:off + n]
        lbs[l] = torch.where(ph > 0, lbs[l].clamp(min=0), lbs[l])
        ubs[l] = torch.where(ph < 0, ubs[l].clamp(max=0), ubs[l])
        off += n
    res.layer_lb, res.layer_ub = lbs, ubs
    rr = ref.crown_refine(ws, bs, lo, hi, res)
    lbs, ubs = rr.layer_lb, rr.layer_ub
    off = 0
    infeas = torch.zeros(lo.shape[0], dtype=torch.bool)
    for l in range(len(ws) - 1):
        n = ws[l].shape[1]
        ph = phase[:, off:off + n]
        infeas |= ((ph > 0) & (ubs[l] < 0)).any(1) | ((ph < 0) & (lbs[l] > 0)).any(1) | (lbs[l] > ubs[l]).any(1)
        lbs[l] = torch.where(ph > 0, lbs[l].clamp(min=0), lbs[l])
        ubs[l] = torch.where(ph < 0, ubs[l].clamp(max=0), ubs[l])
        off += n
    return lbs, ubs, infeas


def backsub_ab(ws, bs, lo, hi, lbs, ubs, phase, lam, alpha, beta, unit):
    """Lower bound of lam . N_pre_logit + lam*b_L (the logit scaled by lam [R]) over the box with
    free lower slopes alpha [R, NH] in [0, 1] and split multipliers beta [R, NH] >= 0 (valid on the
    region where the phases hold).  Returns (coef [R, n0], const [R], err [R])."""
    dt = lo.dtype
    L = len(ws)
    offs = [0]
    for l in range(L - 1):
        offs.append(offs[-1] + ws[l].shape[1])
    mx_in = torch.maximum(lo.abs(), hi.abs())
    lam_v = lam[:, None] * ws[L - 1].to(dt)[:, 0][None]          # multiplier of h_{L-2}
    c = lam * bs[L - 1].to(dt)[0]
    err = torch.zeros_like(c)
    for l in range(L - 2, -1, -1):
        W, b = ws[l].to(dt), bs[l].to(dt)
        n = W.shape[1]
        lb, ub = lbs[l], ubs[l]
        ph = phase[:, offs[l]:offs[l] + n]
        dd = (ub <= 0) | (ph < 0)
        act = ((lb >= 0) | (ph > 0)) & ~dd
        unst = ~(dd | act)
        den = torch.where(unst, ub - lb, torch.ones_like(ub))
        s = torch.where(unst, (ub / den) * (1 + 4 * unit), torch.zeros_like(ub))
        a = alpha[:, offs[l]:offs[l] + n]
        slope = torch.where(act, torch.ones_like(ub), torch.where(dd, torch.zeros_like(ub),
                                                                  torch.where(lam_v >= 0, a, s)))
        mu = lam_v * slope
        neg = unst & (lam_v < 0)
        t = torch.where(neg, -mu * lb, torch.zeros_like(ub))
        # split constraints: s_j z_j >= 0 on the region, so f >= f - beta_j s_j z_j
        bt = beta[:, offs[l]:offs[l] + n] * ph.to(dt)
        mu = mu - bt
        zmax = torch.maximum(lb.abs(), ub.abs())
        e_rel = torch.where(neg, 3 * unit * (mu.abs() * zmax + t.abs()), torch.zeros_like(ub)) + \
            2 * unit * bt.abs() * zmax
        csum = (mu * b[None]).sum(1) + t.sum(1)
        cmag = c.abs() + (mu * b[None]).abs().sum(1) + t.abs().sum(1)
        c = c + csum
        hm = ubs[l - 1].clamp(min=0) if l > 0 else mx_in
        lam_v = mu @ W.T
        eps = ref.gamma(n + 1, unit) * (mu.abs() @ W.abs().T)
        err = err + e_rel.sum(1) + (eps * hm).sum(1) + ref.gamma(2 * n + 1, unit) * cmag
    return lam_v, c, err


def pair_low(ws, bs, lo, hi, pa, va, vb, boundsA, boundsB, phA, phB, alA, alB, beA, beB, t, unit):
    """Lower bound over the node box of t N(x, va) - (1 - t) N(x, vb) (> 0: no x with
    N(x, va) < 0 < N(x, vb))."""
    loA, hiA = lo.clone(), hi.clone()
    loB, hiB = lo.clone(), hi.clone()
    loA[:, pa], hiA[:, pa] = va, va
    loB[:, pa], hiB[:, pa] = vb, vb
    cA, kA, eA = backsub_ab(ws, bs, loA, hiA, boundsA[0], boundsA[1], phA, t, alA, beA, unit)
    cB, kB, eB = backsub_ab(ws, bs, loB, hiB, boundsB[0], boundsB[1], phB, -(1 - t), alB, beB, unit)
    kA = kA + (cA[:, pa] * va).sum(1)
    kB = kB + (cB[:, pa] * vb).sum(1)
    cA = cA.clone(); cA[:, pa] = 0
    cB = cB.clone(); cB[:, pa] = 0
    coef = cA + cB
    conc = torch.minimum(coef * lo, coef * hi).sum(1) + kA + kB
    mag = (coef.abs() * torch.maximum(lo.abs(), hi.abs())).sum(1) + kA.abs() + kB.abs()
    n0 = lo.shape[1]
    return conc - (eA + eB) * (1 + 1e-12) - ref.gamma(2 * n0 + 4, unit) * mag, coef


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--preset", default="src/AC-sex")
    ap.add_argument("--model", default="AC-7")
    ap.add_argument("--weights", default="zoo")
    ap.add_argument("--pids", default="5564,5302,12545")
    ap.add_argument("--budget", type=int, default=2000)
    ap.add_argument("--iters", type=int, default=30)
    ap.add_argument("--no-beta", action="store_true")
    a = ap.parse_args()
    from fairify_amd import presets
    from fairify_amd.engine.bab import _pa_table
    from fairify_amd.models.zoo import get_model
    from fairify_amd.ops.backend import Backend

    torch.set_num_threads(8)
    pre = presets.get(a.preset)
    grid, q = pre.grid(), pre.resolved()
    m = get_model(a.model, weights=a.weights, seed=0)
    be = Backend(m, "cpu")
    ws = [w.double() for w in be.ws]
    bs = [b.double() for b in be.bs]
    NH = sum(int(w.shape[1]) for w in ws[:-1])
    unit = ref.FP64_UNIT
    pa = list(q.pa_idx)
    ids = np.array([int(x) for x in a.pids.split(",")])
    lo_all, hi_all = grid.decode(ids)
    vals, pairs = _pa_table(q, lo_all, hi_all)
    for k, pid in enumerate(ids):
        t0 = time.time()
        verdict, nodes_tot = "unsat", 0
        for vi, vj in pairs:
            va = torch.tensor(vals[int(vi)], dtype=torch.float64)
            vb = torch.tensor(vals[int(vj)], dtype=torch.float64)
            # frontier: boxes + phases of both copies
            lo = torch.tensor(lo_all[k], dtype=torch.float64)[None]
            hi = torch.tensor(hi_all[k], dtype=torch.float64)[None]
            phA = torch.zeros(1, NH, dtype=torch.int8)
            phB = torch.zeros(1, NH, dtype=torch.int8)
            nodes = 0
            while lo.shape[0]:
                R = lo.shape[0]
                nodes += R
                if nodes > a.budget:
                    verdict = "unknown"
                    break
                loA, hiA = lo.clone(), hi.clone(); loA[:, pa], hiA[:, pa] = va, va
                loB, hiB = lo.clone(), hi.clone(); loB[:, pa], hiB[:, pa] = vb, vb
                bA = layer_bounds(ws, bs, loA, hiA, phA)
                bB = layer_bounds(ws, bs, loB, hiB, phB)
                feas = ~(bA[2] | bB[2])
                # optimise alpha (sigmoid), beta (softplus), t (sigmoid)
                ra = torch.zeros(R, NH, dtype=torch.float64, requires_grad=True)
                rb = torch.zeros(R, NH, dtype=torch.float64, requires_grad=True)
                rA = torch.full((R, NH), -2.0, dtype=torch.float64, requires_grad=True)
                rB = torch.full((R, NH), -2.0, dtype=torch.float64, requires_grad=True)
                rt = torch.zeros(R, dtype=torch.float64, requires_grad=True)
                params = [ra, rb, rt] + ([] if a.no_beta else [rA, rB])
                opt = torch.optim.Adam(params, lr=0.2)
                best = torch.full((R,), -np.inf, dtype=torch.float64)
                for it in range(a.iters):
                    beA = torch.nn.functional.softplus(rA) if not a.no_beta else torch.zeros_like(rA)
                    beB = torch.nn.functional.softplus(rB) if not a.no_beta else torch.zeros_like(rB)
                    low, _ = pair_low(ws, bs, lo, hi, pa, va, vb, bA[:2], bB[:2], phA, phB, torch.sigmoid(ra),
                                      torch.sigmoid(rb), beA, beB, torch.sigmoid(rt), unit)
                    best = torch.maximum(best, low.detach())
                    if bool(((best > 0) | ~feas).all()):
                        break
                    opt.zero_grad()
                    (-low[feas & (best <= 0)]).sum().backward()
                    opt.step()
                closed = (best > 0) | ~feas
                keep = ~closed
                if not keep.any():
                    lo = lo[:0]
                    break
                # branch: unstable unfixed neuron with the largest chord area, either copy
                idx = torch.nonzero(keep)[:, 0]
                lo, hi, phA, phB = lo[idx], hi[idx], phA[idx], phB[idx]
                sc = []
                for (lbs, ubs, _), ph in ((bA, phA), (bB, phB)):
                    parts = []
                    for l in range(len(ws) - 1):
                        lb, ub = lbs[l][idx], ubs[l][idx]
                        u = (lb < 0) & (ub > 0)
                        parts.append(torch.where(u, -lb * ub / torch.where(u, ub - lb, torch.ones_like(ub)),
                                                 torch.zeros_like(ub)))
                    sc.append(torch.cat(parts, 1) * (ph == 0))
                S = torch.cat(sc, 1)                       # [R', 2 NH]
                mx, j = S.max(1)
                new_lo, new_hi, nA, nB = [], [], [], []
                for r in range(idx.numel()):
                    if mx[r] <= 0:
                        # no unstable neuron left: split the widest input dim
                        w = (hi[r] - lo[r]).clone(); w[pa] = -1
                        d = int(torch.argmax(w))
                        if w[d] <= 0:
                            verdict = "unknown"      # a single lattice point left open: exact check needed
                            continue
                        mid = torch.floor((lo[r, d] + hi[r, d]) / 2)
                        for lo_d, hi_d in ((lo[r, d], mid), (mid + 1, hi[r, d])):
                            l2, h2 = lo[r].clone(), hi[r].clone(); l2[d], h2[d] = lo_d, hi_d
                            new_lo.append(l2); new_hi.append(h2); nA.append(phA[r]); nB.append(phB[r])
                        continue
                    jj = int(j[r])
                    for sgn in (-1, 1):
                        a2, b2 = phA[r].clone(), phB[r].clone()
                        if jj < NH:
                            a2[jj] = sgn
                        else:
                            b2[jj - NH] = sgn
                        new_lo.append(lo[r]); new_hi.append(hi[r]); nA.append(a2); nB.append(b2)
                if not new_lo:
                    break
                lo, hi = torch.stack(new_lo), torch.stack(new_hi)
                phA, phB = torch.stack(nA), torch.stack(nB)
            nodes_tot += nodes
            if verdict != "unsat":
                break
        print(json.dumps({"pid": int(pid), "verdict": verdict, "nodes": nodes_tot, "s": round(time.time() - t0, 1)}),
              flush=True)


if __name__ == "__main__":
    main()
