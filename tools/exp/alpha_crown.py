#!/usr/bin/env python
"""CPU experiment: alpha-optimised coupled CROWN certificate (torch fp64 autograd) on the residue,
with fixed-phase ReLU splits -- does optimising the lower-relaxation slopes (and t) reach the LP
value of tools/exp/lp_residue.py?"""
from __future__ import annotations

import argparse
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
from tools.exp.crown_phase import forward_sym  # noqa: E402


def g_of(ws, bs, lo, hi, pa_idx, values, phases, orient, bnds_all, alphas, t, betas=None):
    """Coupled bound max_x t*(-N_p) + (1-t)*N_q (phase splits fixed; betas: Lagrange terms of the
    split constraints, s_j beta_j z_j added to the objective: inactive s=-1, active s=+1)."""
    n0 = lo.shape[0]
    lam_x = torch.zeros(n0, dtype=torch.float64)
    const = torch.zeros((), dtype=torch.float64)
    p, q = orient
    for c, w_ in ((p, -t), (q, 1 - t)):
        bnds = bnds_all[c]
        lam = w_ * torch.from_numpy(ws[-1][:, 0])
        cst = w_ * float(bs[-1][0])
        for l in range(len(ws) - 2, -1, -1):
            lb, ub = (torch.from_numpy(v) for v in bnds[l])
            ph = torch.from_numpy(phases[c][l])
            dead = (ub <= 0) | (ph < 0)
            act = ((lb >= 0) | (ph > 0)) & ~dead
            unst = ~(dead | act)
            s = torch.where(unst, ub / torch.where(unst, ub - lb, torch.ones_like(ub)), torch.zeros_like(ub))
            a = alphas[c][l]
            slope = torch.where(act, torch.ones_like(ub), torch.where(dead, torch.zeros_like(ub),
                                                                      torch.where(lam >= 0, s, a)))
            mu = lam * slope
            cst = cst + torch.where(unst & (lam >= 0), -mu * lb, torch.zeros_like(mu)).sum()
            if betas is not None:
                mu = mu + betas[c][l] * ph.double()     # + s_j beta_j on z_j (split neurons only)
            cst = cst + mu @ torch.from_numpy(bs[l])
            lam = torch.from_numpy(ws[l]) @ mu
        xv = torch.zeros(n0, dtype=torch.float64)
        xv[pa_idx] = torch.from_numpy(values[c])
        cst = cst + (lam * xv)[pa_idx].sum()
        lam = lam.clone()
        lam[pa_idx] = 0
        lam_x = lam_x + lam
        const = const + cst
    lo_t, hi_t = torch.from_numpy(lo), torch.from_numpy(hi)
    return torch.maximum(lam_x * lo_t, lam_x * hi_t).sum() + const


def optimise(ws, bs, lo, hi, pa_idx, values, phases, orient, iters=60, lr=0.1, use_beta=False):
    bnds_all = []
    for c in range(len(values)):
        l2, h2 = lo.copy(), hi.copy()
        l2[pa_idx] = values[c]
        h2[pa_idx] = values[c]
        bnds, _ = forward_sym(ws, bs, l2, h2, phases[c])
        # infeasible split: inactive with lb > 0 or active with ub < 0 -> empty node
        for l, (lb, ub) in enumerate(bnds[:-1]):
            if np.any((phases[c][l] < 0) & (lb > 0)) or np.any((phases[c][l] > 0) & (ub < 0)):
                return -np.inf
        bnds_all.append(bnds)
    H = [w.shape[1] for w in ws[:-1]]
    raw = [[torch.zeros(h, dtype=torch.float64, requires_grad=True) for h in H] for _ in values]
    traw = torch.zeros((), dtype=torch.float64, requires_grad=True)
    braw = [[torch.full((h,), -3.0, dtype=torch.float64, requires_grad=True) for h in H] for _ in values]
    params = [p for r in raw for p in r] + [traw] + ([p for r in braw for p in r] if use_beta else [])
    opt = torch.optim.Adam(params, lr=lr)
    best = np.inf
    for it in range(iters):
        alphas = [[torch.sigmoid(r) for r in rc] for rc in raw]
        betas = [[torch.nn.functional.softplus(r) for r in rc] for rc in braw] if use_beta else None
        g = g_of(ws, bs, lo, hi, pa_idx, values, phases, orient, bnds_all, alphas, torch.sigmoid(traw), betas)
        best = min(best, float(g))
        if best <= 0:
            break
        opt.zero_grad()
        g.backward()
        opt.step()
    return best


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--model", default="AC-8")
    ap.add_argument("--residue", default=None)
    ap.add_argument("--n", type=int, default=20)
    ap.add_argument("--iters", type=int, default=60)
    ap.add_argument("--beta", action="store_true")
    args = ap.parse_args()
    from fairify_amd import presets
    from fairify_amd.models.zoo import get_model

    pre = presets.get("src/AC-sex")
    grid, q = pre.grid(), pre.resolved()
    m = get_model(args.model, weights="random", seed=0)
    ws = [w.astype(np.float64) for w in m.weights]
    bs = [b.astype(np.float64) for b in m.biases]
    z = np.load(args.residue)
    ids = z["grid_id"][z["verdict"] == "unknown"][:args.n]
    lo, hi = grid.decode(ids)
    pa_idx = list(q.pa_idx)
    values = [np.asarray(v, float) for v in q.pa_values(lo[0], hi[0])]
    H = [w.shape[1] for w in ws[:-1]]
    zero = [[np.zeros(h, np.int64) for h in H] for _ in values]
    for k in range(len(ids)):
        l0, h0 = lo[k].astype(float), hi[k].astype(float)
        out = []
        for orient in ((0, 1), (1, 0)):
            g = optimise(ws, bs, l0, h0, pa_idx, values, zero, orient, args.iters)
            # one split: the last hidden layer's neurons of copy q, both phases
            ch = []
            qc = orient[1]
            for j in range(H[-1]):
                gs = []
                for sgn in (-1, 1):
                    ph = [[x.copy() for x in pc] for pc in zero]
                    ph[qc][-1][j] = sgn
                    gs.append(optimise(ws, bs, l0, h0, pa_idx, values, ph, orient, args.iters, use_beta=args.beta))
                ch.append(max(gs))
            out.append((g, min(ch)))
        print(ids[k], " | ".join(f"root {a:+.4f} best-split {b:+.4f}" for a, b in out), flush=True)


if __name__ == "__main__":
    main()
