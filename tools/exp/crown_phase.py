#!/usr/bin/env python
"""CPU experiment: fixed-phase ReLU splits with forward-symbolic + CROWN bounds (fp64, no rounding
terms) on the residue -- the bounding the GPU kernels implement -- against the LP numbers of
tools/exp/lp_residue.py.  Coupled pair certificate: min over t of max_x t(-L_p(x)) + (1-t) U_q(x)."""
from __future__ import annotations

import argparse
import os
import sys

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))


def forward_sym(ws, bs, lo, hi, phase):
    """DeepPoly-style forward pass with fixed phases (phase[l][j] in {-1, 0, +1});
    returns per-layer (lb, ub) of pre-activations and output forms (Uc, U0, Lc, L0)."""
    n0 = len(lo)
    U = np.vstack([np.eye(n0), np.zeros((1, n0))])   # [n0+1, n] forms of the inputs
    L = U.copy()
    out = []

    def conc(E):
        C, c0 = E[:-1], E[-1]
        mn = np.minimum(C * lo[:, None], C * hi[:, None]).sum(0) + c0
        mx = np.maximum(C * lo[:, None], C * hi[:, None]).sum(0) + c0
        return mn, mx

    Ih, Il = hi.copy(), lo.copy()
    for l, (W, b) in enumerate(zip(ws, bs)):
        Wp, Wn = np.maximum(W, 0), np.minimum(W, 0)
        Un = U @ Wp + L @ Wn
        Ln = L @ Wp + U @ Wn
        Un[-1] += b
        Ln[-1] += b
        _, ubU = conc(Un)
        lbL, _ = conc(Ln)
        ihn = Ih @ Wp + Il @ Wn + b
        iln = Il @ Wp + Ih @ Wn + b
        ub = np.minimum(ubU, ihn)
        lb = np.maximum(lbL, iln)
        out.append((lb, ub))
        if l == len(ws) - 1:
            return out, (Un[:-1, 0], Un[-1, 0], Ln[:-1, 0], Ln[-1, 0])
        ph = phase[l]
        dead = (ub <= 0) | (ph < 0)
        act = (lb >= 0) & ~dead
        unst = ~(dead | act)
        # forced active (ph > 0) on the branch region {z >= 0}: upper relaxation = identity (no
        # chord), lower relaxation as an unstable neuron's, range [max(lb, 0), ub]
        chord = unst & (ph == 0)
        s = np.where(chord, ub / np.where(chord, ub - lb, 1), 1.0)
        Unew = Un * s
        Unew[-1] += np.where(chord, -s * lb, 0)
        lam = np.where(act, 1.0, np.where(unst, (ub > -lb).astype(float), 0.0))
        Lnew = Ln * lam
        Unew[:, dead] = 0
        Lnew[:, dead] = 0
        U, L = Unew, Lnew
        Ih = np.where(dead, 0, np.maximum(ub, 0))
        Il = np.where(dead, 0, np.maximum(lb, 0))


def crown(ws, bs, bnds, phase, sign, alpha=None):
    """Backward bound of sign * N: returns (coef [n0], const) with sign*N(x) <= coef.x + const."""
    Lyr = len(ws)
    lam = sign * ws[-1][:, 0].copy()
    c = sign * bs[-1][0]
    mus = []
    for l in range(Lyr - 2, -1, -1):
        lb, ub = bnds[l]
        ph = phase[l]
        dead = (ub <= 0) | (ph < 0)
        act = ((lb >= 0) | (ph > 0)) & ~dead
        unst = ~(dead | act)
        s = np.where(unst, ub / np.where(unst, ub - lb, 1), 0.0)
        a = (ub > -lb).astype(float) if alpha is None else alpha[l]
        slope = np.where(act, 1.0, np.where(dead, 0.0, np.where(lam >= 0, s, a)))
        mu = lam * slope
        c += np.where(unst & (lam >= 0), -mu * lb, 0).sum()
        mus.append((l, lam.copy()))
        c += mu @ bs[l]
        lam = ws[l] @ mu
    return lam, c, mus


def certify(ws, bs, lo, hi, pa, values, phases, orient, pa_idx):
    """g* = min_t max_x t(-N_p lower form) + (1-t)(N_q upper form) (coupled, shared x)."""
    p, q = orient
    forms = []
    for c, sg in ((p, -1.0), (q, 1.0)):
        l2, h2 = lo.copy(), hi.copy()
        l2[pa_idx] = values[c]
        h2[pa_idx] = values[c]
        bnds, fo = forward_sym(ws, bs, l2, h2, phases[c])
        lam, c0, mus = crown(ws, bs, bnds, phases[c], sg)
        # fold PA into the constant
        c0 = c0 + lam[pa_idx] @ np.asarray(values[c], float)
        lam = lam.copy()
        lam[pa_idx] = 0
        forms.append((lam, c0, bnds, mus))
    (a, a0, _, _), (bq, b0, _, _) = forms
    best = np.inf
    ts = [0.0, 1.0]
    for i in range(len(lo)):
        den = a[i] - bq[i]
        if den != 0:
            t = -bq[i] / den
            if 0 < t < 1:
                ts.append(t)
    for t in ts:
        cs = t * a + (1 - t) * bq
        g = np.maximum(cs * lo, cs * hi).sum() + t * a0 + (1 - t) * b0
        if g < best:
            best, bt = g, t
    return best, bt, forms


def relu_search(ws, bs, lo, hi, pa_idx, values, orient, max_nodes=64, branch="babsr"):
    H = [w.shape[1] for w in ws[:-1]]
    V = len(values)
    root = [[np.zeros(h, int) for h in H] for _ in range(V)]
    stack = [root]
    nodes = 0
    while stack:
        ph = stack.pop()
        nodes += 1
        if nodes > max_nodes:
            return None, nodes
        g, t, forms = certify(ws, bs, lo, hi, None, values, ph, orient, pa_idx)
        if g <= 0:
            continue
        # BaBSR-like score: |multiplier| x upper-relaxation intercept, weighted by t / 1-t
        best, bk = 0.0, None
        for ci, (c, w_) in enumerate(((orient[0], t), (orient[1], 1 - t))):
            _, _, bnds, mus = forms[ci]
            for l, lam in mus:
                lb, ub = bnds[l]
                for j in range(len(lb)):
                    if ph[c][l][j] != 0 or ub[j] <= 0 or lb[j] >= 0:
                        continue
                    inter = -ub[j] * lb[j] / (ub[j] - lb[j])
                    sc = w_ * max(lam[j], 0) * inter if branch == "babsr" else w_ * abs(lam[j]) * inter
                    if sc > best:
                        best, bk = sc, (c, l, j)
        if bk is None:
            return False, nodes
        c, l, j = bk
        for s in (-1, 1):
            d = [[x.copy() for x in pc] for pc in ph]
            d[c][l][j] = s
            stack.append(d)
    return True, nodes


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--model", default="AC-8")
    ap.add_argument("--residue", default=None)
    ap.add_argument("--n", type=int, default=30)
    ap.add_argument("--max-nodes", type=int, default=64)
    ap.add_argument("--branch", default="babsr")
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
    hist = {}
    closed = 0
    for k in range(len(ids)):
        res = []
        for orient in ((0, 1), (1, 0)):
            g0, _, _ = certify(ws, bs, lo[k].astype(float), hi[k].astype(float), None, values,
                               [[np.zeros(w.shape[1], int) for w in ws[:-1]] for _ in values], orient, pa_idx)
            c, nn = relu_search(ws, bs, lo[k].astype(float), hi[k].astype(float), pa_idx, values, orient,
                                args.max_nodes, args.branch)
            res.append((g0, c, nn))
        ok = all(c is True for _, c, _ in res)
        closed += ok
        key = tuple(n for _, _, n in res)
        hist[key] = hist.get(key, 0) + 1
        print(ids[k], " ".join(f"root {g:+.4g} closed {c} nodes {n}" for g, c, n in res), flush=True)
    print("closed", closed, "of", len(ids), "node histogram", sorted(hist.items(), key=lambda kv: -kv[1])[:10])


if __name__ == "__main__":
    main()
