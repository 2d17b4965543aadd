#!/usr/bin/env python
"""CPU experiment: ReLU-phase BaB with the alpha-optimised coupled bound at every node (fixed-phase
forms, optional beta terms); branching on |multiplier| x chord intercept (BaBSR-like)."""
from __future__ import annotations

import argparse
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
from tools.exp.crown_phase import forward_sym  # noqa: E402
from tools.exp.alpha_crown import g_of  # noqa: E402


def node_bound(ws, bs, lo, hi, pa_idx, values, phases, orient, iters, lr, use_beta):
    bnds_all = []
    for c in range(len(values)):
        l2, h2 = lo.copy(), hi.copy()
        l2[pa_idx] = values[c]
        h2[pa_idx] = values[c]
        bnds, _ = forward_sym(ws, bs, l2, h2, phases[c])
        for l, (lb, ub) in enumerate(bnds[:-1]):
            if np.any((phases[c][l] < 0) & (lb > 0)) or np.any((phases[c][l] > 0) & (ub < 0)):
                return -np.inf, None, None
        # exact-sign shortcut (rigorous row bounds): orientation needs N_p < 0 and N_q > 0
        bnds_all.append(bnds)
    p, q = orient
    if bnds_all[p][-1][0][0] >= 0 or bnds_all[q][-1][1][0] <= 0:
        return -1.0, None, None
    H = [w.shape[1] for w in ws[:-1]]
    raw = [[torch.zeros(h, dtype=torch.float64, requires_grad=True) for h in H] for _ in values]
    traw = torch.zeros((), dtype=torch.float64, requires_grad=True)
    braw = [[torch.full((h,), -2.0, dtype=torch.float64, requires_grad=True) for h in H] for _ in values]
    params = [p_ for r in raw for p_ in r] + [traw] + ([p_ for r in braw for p_ in r] if use_beta else [])
    opt = torch.optim.Adam(params, lr=lr)
    best, best_state = np.inf, None
    for it in range(iters):
        alphas = [[torch.sigmoid(r) for r in rc] for rc in raw]
        betas = [[torch.nn.functional.softplus(r) for r in rc] for rc in braw] if use_beta else None
        t = torch.sigmoid(traw)
        g = g_of(ws, bs, lo, hi, pa_idx, values, phases, orient, bnds_all, alphas, t, betas)
        if float(g) < best:
            best = float(g)
            best_state = ([[a.detach().numpy().copy() for a in ac] for ac in alphas], float(t))
        if best <= 0:
            break
        opt.zero_grad()
        g.backward()
        opt.step()
    return best, best_state, bnds_all


def scores(ws, bs, bnds_all, phases, orient, state):
    """|multiplier on a_j| x chord intercept per unstable, unsplit neuron (both copies)."""
    alphas, t = state
    best, bk = -1.0, None
    for c, w_ in ((orient[0], -t), (orient[1], 1 - t)):
        bnds = bnds_all[c]
        lam = w_ * ws[-1][:, 0]
        for l in range(len(ws) - 2, -1, -1):
            lb, ub = bnds[l]
            ph = phases[c][l]
            dead = (ub <= 0) | (ph < 0)
            act = ((lb >= 0) | (ph > 0)) & ~dead
            unst = ~(dead | act)
            s = np.where(unst, ub / np.where(unst, ub - lb, 1), 0.0)
            inter = -s * lb
            for j in np.nonzero(unst)[0]:
                sc = abs(lam[j]) * inter[j]
                if sc > best:
                    best, bk = sc, (c, l, int(j))
            slope = np.where(act, 1.0, np.where(dead, 0.0, np.where(lam >= 0, s, alphas[c][l])))
            lam = ws[l] @ (lam * slope)
    return bk


def search(ws, bs, lo, hi, pa_idx, values, orient, max_nodes, iters, lr, use_beta):
    H = [w.shape[1] for w in ws[:-1]]
    stack = [[[np.zeros(h, np.int64) for h in H] for _ in values]]
    nodes = 0
    while stack:
        ph = stack.pop()
        nodes += 1
        if nodes > max_nodes:
            return None, nodes
        g, st, bnds_all = node_bound(ws, bs, lo, hi, pa_idx, values, ph, orient, iters, lr, use_beta)
        if g <= 0:
            continue
        bk = scores(ws, bs, bnds_all, ph, orient, st)
        if bk is None:
            return False, nodes
        c, l, j = bk
        for sg in (-1, 1):
            d = [[x.copy() for x in pc] for pc in ph]
            d[c][l][j] = sg
            stack.append(d)
    return True, nodes


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--model", default="AC-8")
    ap.add_argument("--residue", default=None)
    ap.add_argument("--n", type=int, default=20)
    ap.add_argument("--skip", type=int, default=0)
    ap.add_argument("--iters", type=int, default=100)
    ap.add_argument("--lr", type=float, default=0.3)
    ap.add_argument("--max-nodes", type=int, default=64)
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
    ids = z["grid_id"][z["verdict"] == "unknown"][args.skip:args.skip + args.n]
    lo, hi = grid.decode(ids)
    pa_idx = list(q.pa_idx)
    values = [np.asarray(v, float) for v in q.pa_values(lo[0], hi[0])]
    tot, closed = [], 0
    for k in range(len(ids)):
        res = [search(ws, bs, lo[k].astype(float), hi[k].astype(float), pa_idx, values, o, args.max_nodes,
                      args.iters, args.lr, args.beta) for o in ((0, 1), (1, 0))]
        ok = all(c is True for c, _ in res)
        closed += ok
        tot.append(sum(n for _, n in res))
        print(ids[k], res, flush=True)
    print(f"closed {closed}/{len(ids)}, nodes median {np.median(tot)} max {max(tot)}")


if __name__ == "__main__":
    main()
