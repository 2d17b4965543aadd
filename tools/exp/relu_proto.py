#!/usr/bin/env python
"""CPU prototype of the ReLU-phase BaB stage (fp64, rounding terms ignored): fixed-phase forward
symbolic bounds, backward CROWN bounds concretised at EVERY layer (hidden post-activations
included: exact zeros survive when every coefficient on a [0, u] range is non-positive), the sign
shortcut, the coupled input certificate, BaBSR-style branching.  Measures closure / node counts on
the dumped residue before the HIP implementation."""
from __future__ import annotations

import argparse
import os
import sys

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
from tools.exp.crown_phase import forward_sym  # noqa: E402


SCORE = os.environ.get("SCORE", "intercept")


def crown_multi(ws, bs, bnds, phase, lo, hi, sign):
    """Best over the alpha policies (adaptive, all 0, all 1) of crown_one."""
    best = None
    for pol in POLICIES:
        r = crown_one(ws, bs, bnds, phase, lo, hi, sign, pol)
        if best is None or r[0] > best[0]:
            best = r
    return best


POLICIES = os.environ.get("POLICIES", "adaptive,zero,one").split(",")


def crown_one(ws, bs, bnds, phase, lo, hi, sign, pol):
    """Lower bound of sign*N (best over concretisation layers), input form (lam, c), and the
    per-neuron split scores |lambda| * chord-gap of unstable neurons."""
    L = len(ws)
    lam = sign * ws[-1][:, 0].copy()
    c = sign * bs[-1][0]
    best = -np.inf
    scores = {}
    for l in range(L - 2, -1, -1):
        lb, ub = bnds[l]
        ph = phase[l]
        dead = (ph < 0) | (ub <= 0)
        act = (lb >= 0) & ~dead
        unst = ~(dead | act)
        fact = unst & (ph > 0)        # forced active: identity upper, free lower
        # concretise at the post-activations of layer l: a in [lo_a, hi_a]
        lo_a = np.where(dead, 0, np.maximum(lb, 0))
        hi_a = np.where(dead, 0, np.maximum(ub, 0))
        val = np.minimum(lam * lo_a, lam * hi_a).sum() + c
        best = max(best, val)
        s = np.where(unst, np.where(fact, 1.0, ub / np.where(unst, ub - lb, 1)), 0.0)
        alpha = (ub > -lb).astype(float) if pol == "adaptive" else (np.zeros_like(ub) if pol == "zero" else np.ones_like(ub))
        slope = np.where(act, 1.0, np.where(dead, 0.0, np.where(lam >= 0, alpha, s)))
        mu = lam * slope
        c = c + np.where(unst & ~fact & (lam < 0), -mu * lb, 0).sum() + mu @ bs[l]
        gap = np.where(unst, -ub * lb / np.where(unst, ub - lb, 1), 0)
        for j in np.nonzero(unst & ~fact)[0]:
            if SCORE == "gap":
                scores[(l, int(j))] = abs(lam[j]) * gap[j]
            else:   # the constant the chord relaxation adds (lam < 0 here: chord), tiny gap tiebreak
                scores[(l, int(j))] = (abs(mu[j] * lb[j]) if lam[j] < 0 else 0.0) + 1e-3 * abs(lam[j]) * gap[j]
        lam = ws[l] @ mu
    val = np.minimum(lam * lo, lam * hi).sum() + c
    best = max(best, val)
    return best, lam, c, scores


def node(ws, bs, lo, hi, pa, values, phases, orients):
    """Returns (open orientations, split choice)."""
    V = len(values)
    rows = []
    for v in range(V):
        l2, h2 = lo.copy(), hi.copy()
        l2[pa] = values[v]
        h2[pa] = values[v]
        bnds, _ = forward_sym(ws, bs, l2, h2, phases[v])
        infeas = any(np.any((phases[v][l] < 0) & (lb > 0)) or np.any((phases[v][l] > 0) & (ub < 0))
                     for l, (lb, ub) in enumerate(bnds[:-1]))
        if infeas:
            return [], None
        lwb, lamL, cL, scL = crown_multi(ws, bs, bnds, phases[v], l2, h2, 1.0)
        upb, lamU, cU, scU = crown_multi(ws, bs, bnds, phases[v], l2, h2, -1.0)
        olb = max(lwb, bnds[-1][0][0])
        oub = min(-upb, bnds[-1][1][0])
        lamL = lamL.copy(); lamU = lamU.copy()
        cL += lamL[pa] @ values[v]; cU += lamU[pa] @ values[v]
        lamL[pa] = 0; lamU[pa] = 0
        rows.append(dict(olb=olb, oub=oub, L=(lamL, cL), U=(-lamU, -cU), scL=scL, scU=scU))
    still = []
    best_sc, choice = np.inf, None
    for (p, q) in orients:
        if rows[p]["olb"] >= 0 or rows[q]["oub"] <= 0:
            continue
        # coupled certificate: min_t max_x t(-L_p(x)) + (1-t) U_q(x)
        a_, a0 = -rows[p]["L"][0], -rows[p]["L"][1]
        b_, b0 = rows[q]["U"]
        ts = [0.0, 1.0] + [float(-b_[i] / (a_[i] - b_[i])) for i in range(len(lo)) if a_[i] != b_[i]]
        g = min(np.maximum((t * a_ + (1 - t) * b_) * lo, (t * a_ + (1 - t) * b_) * hi).sum() + t * a0 + (1 - t) * b0
                for t in ts if 0 <= t <= 1)
        if g <= 0:
            continue
        still.append((p, q))
        # the pass closest to closing (lower bound of N_p -> 0, or upper bound of N_q -> 0), then
        # its neuron with the largest chord intercept
        cands = [(-rows[p]["olb"], p, rows[p]["scL"]), (rows[q]["oub"], q, rows[q]["scU"])]
        cands.sort(key=lambda t: t[0])
        for gap, v, sc_ in cands:
            if sc_ and max(sc_.values()) > 0:
                (l, j), sc = max(sc_.items(), key=lambda kv: kv[1])
                if choice is None or gap < best_sc:
                    best_sc, choice = gap, (v, l, j)
                break
    return still, choice


def search(ws, bs, lo, hi, pa, values, max_nodes):
    """One independent ReLU-split tree per orientation (splits made for one orientation do not
    multiply the other's tree)."""
    V = len(values)
    tot = 0
    for o in [(p, q) for p in range(V) for q in range(V) if p != q]:
        c, n = search_one(ws, bs, lo, hi, pa, values, max_nodes, [o])
        tot += n
        if c is not True:
            return c, tot
    return True, tot


def search_one(ws, bs, lo, hi, pa, values, max_nodes, orients):
    H = [w.shape[1] for w in ws[:-1]]
    V = len(values)
    stack = [([[np.zeros(h, np.int64) for h in H] for _ in range(V)], orients)]
    nodes = 0
    while stack:
        ph, ors = stack.pop()
        nodes += 1
        if nodes > max_nodes:
            return None, nodes
        still, ch = node(ws, bs, lo, hi, pa, values, ph, ors)
        if not still:
            continue
        if ch is None:
            return False, nodes
        v, l, j = ch
        if os.environ.get("VERB") == "1":
            print("  split", ch, "depth", sum(int((x != 0).sum()) for pc in ph for x in pc), "open", still)
        for sg in (-1, 1):
            d = [[x.copy() for x in pc] for pc in ph]
            d[v][l][j] = sg
            stack.append((d, still))
    return True, nodes


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--model", default="AC-8")
    ap.add_argument("--n", type=int, default=40)
    ap.add_argument("--max-nodes", type=int, default=256)
    args = ap.parse_args()
    from fairify_amd import presets
    from fairify_amd.models.zoo import get_model

    pre = presets.get("src/AC-sex")
    grid, q = pre.grid(), pre.resolved()
    m = get_model(args.model, weights="random", seed=0)
    ws = [w.astype(np.float64) for w in m.weights]
    bs = [b.astype(np.float64) for b in m.biases]
    z = np.load(f"gpurun_out/residue/{args.model}.npz")
    ids = z["grid_id"][z["verdict"] == "unknown"][:args.n]
    lo, hi = grid.decode(ids)
    pa = list(q.pa_idx)
    values = [np.asarray(v, float) for v in q.pa_values(lo[0], hi[0])]
    res = []
    for k in range(len(ids)):
        c, n = search(ws, bs, lo[k].astype(float), hi[k].astype(float), pa, values, args.max_nodes)
        res.append((c, n))
    cl = [n for c, n in res if c is True]
    print(f"{args.model}: closed {len(cl)}/{len(ids)}  nodes median {np.median(cl) if cl else 0} "
          f"p90 {np.percentile(cl, 90) if cl else 0} max {max(cl) if cl else 0}; "
          f"open-leaf {sum(1 for c, _ in res if c is False)} budget {sum(1 for c, _ in res if c is None)}")


if __name__ == "__main__":
    main()
