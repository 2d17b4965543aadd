#!/usr/bin/env python
"""CPU experiment (not part of the product): how hard is the sound-UNKNOWN residue for an
LP-based relational bound?  For each residue partition: the coupled triangle-relaxation LP of the
two network copies (shared non-PA inputs, one per PA value) at the root, then a ReLU-phase-split
BaB on top of it (scipy HiGHS, fp64, NOT rigorous -- a measurement of search-tree sizes only).

    python tools/exp/lp_residue.py --model AC-8 --residue gpurun_out/residue/AC-8.npz --n 50
"""
from __future__ import annotations

import argparse
import os
import sys
import time

import numpy as np
from scipy.optimize import linprog

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))


def ibp(ws, bs, lo, hi):
    """Pre-activation interval bounds per layer (fp64, no rounding care)."""
    out = []
    l, h = lo.astype(np.float64), hi.astype(np.float64)
    for k, (W, b) in enumerate(zip(ws, bs)):
        Wp, Wn = np.maximum(W, 0), np.minimum(W, 0)
        zl = l @ Wp + h @ Wn + b
        zh = h @ Wp + l @ Wn + b
        out.append((zl, zh))
        l, h = np.maximum(zl, 0), np.maximum(zh, 0)
    return out


def lp_a_index(lp, c, l, j):
    idx = lp.n0
    for cc in range(lp.V):
        for ll, h in enumerate(lp.H):
            if (cc, ll) == (c, l):
                return idx + j
            idx += h
    raise KeyError


class PairLP:
    """Triangle LP of V copies of the net on a shared box; PA dims fixed per copy."""

    def __init__(self, ws, bs, lo, hi, pa, values):
        self.ws = [np.asarray(w, np.float64) for w in ws]
        self.bs = [np.asarray(b, np.float64) for b in bs]
        self.lo, self.hi, self.pa, self.values = lo.astype(np.float64), hi.astype(np.float64), pa, values
        self.n0 = len(lo)
        self.V = len(values)
        self.H = [w.shape[1] for w in self.ws[:-1]]
        self.bounds = []
        for v in values:
            l, h = self.lo.copy(), self.hi.copy()
            l[pa], h[pa] = v, v
            self.bounds.append(ibp(self.ws, self.bs, l, h))

    def solve(self, orient, phases, bnds=None):
        """max s s.t. s <= -N_a, s <= N_b (orient (a, b)); phases: dict (copy, layer, j) -> +1/-1."""
        bnds = bnds or self.bounds
        n0 = self.n0
        # variable layout: x[n0], per copy per hidden layer: a[h], then s
        idx = n0
        aoff = {}
        for c in range(self.V):
            for l, h in enumerate(self.H):
                aoff[(c, l)] = idx
                idx += h
        sidx = idx
        nv = idx + 1
        A, bvec, Aeq, beq = [], [], [], []
        vb = [(self.lo[i], self.hi[i]) for i in range(n0)]
        vb += [(None, None)] * (nv - n0)
        for i in self.pa:
            vb[i] = (0, 0)   # PA dims enter through constants

        def zrow(c, l):
            """z of layer l, copy c as (coef matrix [h, nv], const [h])."""
            W, b = self.ws[l], self.bs[l]
            h = W.shape[1]
            M = np.zeros((h, nv))
            k = b.copy()
            if l == 0:
                M[:, :n0] = W.T
                for i, p in enumerate(self.pa):
                    M[:, p] = 0
                    k = k + W[p] * self.values[c][i]
            else:
                o = aoff[(c, l - 1)]
                M[:, o:o + W.shape[0]] = W.T
            return M, k

        for c in range(self.V):
            for l, h in enumerate(self.H):
                M, k = zrow(c, l)
                zl, zh = bnds[c][l]
                o = aoff[(c, l)]
                for j in range(h):
                    ph = phases.get((c, l, j), 0)
                    lj, uj = zl[j], zh[j]
                    if ph < 0 or uj <= 0:
                        vb[o + j] = (0, 0)
                        if ph < 0 and not NOCON:      # z <= 0
                            A.append(M[j]); bvec.append(-k[j])
                        continue
                    if ph > 0 or lj >= 0:
                        r = -M[j].copy(); r[o + j] += 1   # a - z = 0
                        Aeq.append(r); beq.append(k[j])
                        if ph > 0 and not NOCON:      # z >= 0  ->  -z <= 0
                            A.append(-M[j]); bvec.append(k[j])
                        continue
                    vb[o + j] = (0, None)
                    r = M[j].copy(); r[o + j] -= 1        # z - a <= 0
                    A.append(r); bvec.append(-k[j])
                    s = uj / (uj - lj)                    # a <= s (z - l)
                    r = -s * M[j].copy(); r[o + j] += 1
                    A.append(r); bvec.append(s * (k[j] - lj))
        # outputs
        a_, b_ = orient
        for c, sg in ((a_, -1.0), (b_, 1.0)):
            Wl, bl = self.ws[-1], self.bs[-1]
            o = aoff[(c, len(self.H) - 1)]
            r = np.zeros(nv)
            r[o:o + Wl.shape[0]] = -sg * Wl[:, 0]
            r[sidx] = 1.0                          # s - sg*N <= 0
            A.append(r); bvec.append(sg * bl[0])
        cost = np.zeros(nv); cost[sidx] = -1.0
        vb[sidx] = (None, 1e6)
        res = linprog(cost, A_ub=np.array(A) if A else None, b_ub=np.array(bvec) if A else None,
                      A_eq=np.array(Aeq) if Aeq else None, b_eq=np.array(beq) if Aeq else None, bounds=vb,
                      method="highs")
        if res.status == 2:
            return -np.inf, None
        if res.status != 0:
            return np.inf, None
        return -res.fun, res.x


BRANCH = "area"
NOCON = False
VERB = os.environ.get("VERB") == "1"


def relu_bab(lp: PairLP, orient, max_nodes=2000):
    """DFS ReLU-phase BaB on the coupled LP; returns (closed?, nodes)."""
    stack = [dict()]
    nodes = 0
    while stack:
        ph = stack.pop()
        nodes += 1
        if nodes > max_nodes:
            return None, nodes
        val, x = lp.solve(orient, ph)
        if val <= 1e-9:
            continue
        if x is None:
            return None, nodes
        # pick the unstable unfixed neuron with the largest triangle violation at the LP point
        best, bk = -1.0, None
        n0 = lp.n0
        for c in range(lp.V):
            xx = x[:n0].copy()
            for i, p in enumerate(lp.pa):
                xx[p] = lp.values[c][i]
            act = xx
            for l, h in enumerate(lp.H):
                z = act @ lp.ws[l] + lp.bs[l]
                zl, zh = lp.bounds[c][l]
                for j in range(h):
                    if (c, l, j) in ph or zh[j] <= 0 or zl[j] >= 0:
                        continue
                    sc = -zl[j] * zh[j] / (zh[j] - zl[j])
                    if BRANCH == "viol":      # triangle violation at the LP point
                        aj = x[lp_a_index(lp, c, l, j)]
                        sc = aj - max(z[j], 0.0)
                    elif BRANCH == "late":    # last hidden layer first
                        sc = sc + 1e6 * l
                    elif BRANCH == "late_copy":  # only the copy whose output must be positive
                        sc = sc + 1e6 * l + (1e9 if c == orient[1] else 0)
                    if sc > best:
                        best, bk = sc, (c, l, j)
                act = np.maximum(z, 0)
        if bk is None:
            if VERB: print("   open leaf", ph, val)
            return False, nodes        # LP exact with all phases fixed: real-valued violation
        if VERB: print("   split", bk, "at", ph, "val", round(val, 5))
        for s in (-1, 1):
            d = dict(ph); d[bk] = s
            stack.append(d)
    return True, nodes


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--model", default="AC-8")
    ap.add_argument("--residue", default=None)
    ap.add_argument("--n", type=int, default=30)
    ap.add_argument("--max-nodes", type=int, default=2000)
    ap.add_argument("--branch", default="area")
    ap.add_argument("--nocon", action="store_true")
    args = ap.parse_args()
    global BRANCH
    BRANCH = args.branch
    global NOCON
    NOCON = args.nocon
    from fairify_amd import presets
    from fairify_amd.models.zoo import get_model
    from fairify_amd.partition import processing_order

    pre = presets.get("src/AC-sex")
    grid, q = pre.grid(), pre.resolved()
    m = get_model(args.model, weights="random", seed=0)
    if args.residue:
        z = np.load(args.residue)
        ids = z["grid_id"][z["verdict"] == "unknown"][:args.n]
    else:
        ids = processing_order(grid, 0)[:args.n]
    lo, hi = grid.decode(ids)
    pa = list(q.pa_idx)
    values = q.pa_values(lo[0], hi[0])
    stats = []
    for k in range(len(ids)):
        lp = PairLP(m.weights, m.biases, lo[k], hi[k], pa, values)
        t0 = time.time()
        res = []
        for orient in ((0, 1), (1, 0)):
            root, _ = lp.solve(orient, {})
            closed, nodes = relu_bab(lp, orient, args.max_nodes)
            res.append((root, closed, nodes))
        dt = time.time() - t0
        stats.append(res)
        print(f"{ids[k]}: " + "  ".join(f"root {r:+.4g} closed {c} nodes {n}" for r, c, n in res) + f"  {dt:.1f}s",
              flush=True)
    roots_closed = sum(all(r <= 1e-9 for r, _, _ in s) for s in stats)
    bab_closed = sum(all(c is True for _, c, _ in s) for s in stats)
    real_sat = sum(any(c is False for _, c, _ in s) for s in stats)
    print(f"root LP closes {roots_closed}/{len(stats)}; ReLU BaB closes {bab_closed}; real-valued violation {real_sat}")


if __name__ == "__main__":
    main()
