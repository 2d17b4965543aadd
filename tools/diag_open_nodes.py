#!/usr/bin/env python
"""Where does the BaB budget go on the hard residue?  (CPU diagnostic, torch reference ops)

Runs a plain breadth-first BaB (same bounding + certificate + split rule as the device BaB) on
a few partitions and, for the partitions still open at the budget, reports the open frontier:
how many nodes are fully stable (every hidden neuron of every PA row has a fixed phase, so both
logits are affine on the node) and how many lattice points they hold.

    python tools/diag_open_nodes.py --model AC-8 --partitions 256 --budget 2048
"""
from __future__ import annotations

import argparse
import os
import sys
import time

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def crown(be, res, lo, hi):
    """Backward (CROWN/DeepPoly-style) output forms from the forward pass's per-neuron bounds
    (fp64 prototype: no rounding terms)."""
    from fairify_amd.ops.reference import BoundResult
    ws = [w.double() for w in be.ws]
    bs = [b.double() for b in be.bs]
    L = len(ws)
    lbs = [t.double() for t in res.layer_lb]
    ubs = [t.double() for t in res.layer_ub]
    R = lo.shape[0]
    out = {}
    for sign in (1.0, -1.0):             # +1: lower bound of y, -1: lower bound of -y (upper of y)
        lam = sign * ws[-1][:, 0].expand(R, -1).clone()       # [R, n_{L-1}]
        c = sign * bs[-1][0].expand(R).clone()
        for k in range(L - 2, -1, -1):
            l, u = lbs[k], ubs[k]
            dead = u <= 0
            act = l >= 0
            unst = ~(dead | act)
            s = torch.where(unst, u / torch.where(unst, u - l, torch.ones_like(u)), torch.zeros_like(u))
            alpha = (u > -l).double()
            slope = torch.where(act, torch.ones_like(u), torch.where(dead, torch.zeros_like(u),
                                torch.where(lam >= 0, alpha, s)))
            c = c + torch.where(unst & (lam < 0), -lam * s * l, torch.zeros_like(u)).sum(1)
            mu = lam * slope
            c = c + mu @ bs[k]
            lam = mu @ ws[k].T
        out[sign] = (lam, c)
    (lc, l0), (uc, u0) = out[1.0], out[-1.0]
    r = BoundResult(out_lb=res.out_lb, out_ub=res.out_ub)
    r.Lc, r.L0, r.Le = lc.float(), l0.float(), torch.zeros_like(l0).float()
    r.Uc, r.U0, r.Ue = (-uc).float(), (-u0).float(), torch.zeros_like(u0).float()
    return r


def _score(be, lo, hi, V, q, values, pairs, pa, shared):
    N = lo.shape[0]
    rlo = lo[:, None, :].expand(N, V, q.n).clone()
    rhi = hi[:, None, :].expand(N, V, q.n).clone()
    rlo[:, :, pa] = values.float()[None]
    rhi[:, :, pa] = values.float()[None]
    res = be.bounds(rlo.reshape(-1, q.n), rhi.reshape(-1, q.n), mode="symbolic")
    dec = be.pair_certify(res, res, lo, hi, lo, hi, pairs, values, pa, shared, False)
    return dec.score.clamp(min=0)


def strong_dims(be, lo, hi, V, q, values, pairs, pa, shared):
    N, n = lo.shape
    best = torch.full((N,), float("inf"))
    bd = torch.zeros(N, dtype=torch.long)
    for i in range(n):
        if i in pa.tolist():
            continue
        w = hi[:, i] - lo[:, i]
        mid = torch.floor((lo[:, i] + hi[:, i]) / 2)
        h1 = hi.clone(); h1[:, i] = mid
        l2 = lo.clone(); l2[:, i] = mid + 1
        s = _score(be, lo, h1, V, q, values, pairs, pa, shared) + _score(be, l2, hi, V, q, values, pairs, pa, shared)
        s = torch.where(w > 0, s, torch.full_like(s, float("inf")))
        upd = s < best
        best = torch.where(upd, s, best)
        bd = torch.where(upd, torch.full_like(bd, i), bd)
    return bd


def smear_dims(be, lo, hi, values, pa):
    """sum over unstable first-layer neurons of |W0[i, j]| * width_i (both PA rows)."""
    W = be.ws[0]
    N, n = lo.shape
    sc = torch.zeros(N, n)
    for v in range(values.shape[0]):
        a, b = lo.clone(), hi.clone()
        a[:, pa] = values[v].float(); b[:, pa] = values[v].float()
        z_lo = torch.clamp(a, min=0) @ W.clamp(min=0) + b @ W.clamp(max=0)
        z_lo = a @ W.clamp(min=0) + b @ W.clamp(max=0) + be.bs[0]
        z_hi = b @ W.clamp(min=0) + a @ W.clamp(max=0) + be.bs[0]
        unst = ((z_lo < 0) & (z_hi > 0)).float()
        sc += (W.abs()[None] * unst[:, None, :]).sum(-1) * (b - a)
    sc[:, pa] = -1
    return sc.argmax(dim=1)


def full_crown(be, lo, hi):
    """CROWN with backward-computed intermediate bounds (fp64 prototype, no rounding terms):
    every hidden layer's pre-activation bounds come from back-substitution to the input box
    through the relaxations of the layers below, then the output forms likewise."""
    from fairify_amd.ops.reference import BoundResult
    ws = [w.double() for w in be.ws]
    bs = [b.double() for b in be.bs]
    lo = lo.double(); hi = hi.double()
    R = lo.shape[0]
    L = len(ws)
    lbs, ubs = [], []

    def backsub(lam, c, upto):
        # lam [R, n_upto]: coefficients on pre-activations z_upto ... wait: on h_{upto-1}
        for k in range(upto - 1, -1, -1):
            l, u = lbs[k], ubs[k]
            dead = u <= 0
            act = l >= 0
            unst = ~(dead | act)
            s = torch.where(unst, u / torch.where(unst, u - l, torch.ones_like(u)), torch.zeros_like(u))
            alpha = (u > -l).double()
            slope = torch.where(act, torch.ones_like(u), torch.where(dead, torch.zeros_like(u),
                                torch.where(lam >= 0, alpha, s)))
            c = c + torch.where(unst & (lam < 0), -lam * s * l, torch.zeros_like(u)).sum(1)
            mu = lam * slope
            c = c + mu @ bs[k]
            lam = mu @ ws[k].T
        return lam, c

    def concretize_lower(lam, c):
        return (torch.where(lam >= 0, lam * lo, lam * hi)).sum(1) + c

    for k in range(L):
        n_out = ws[k].shape[1]
        # bounds of z_k = W_k^T h_{k-1} + b_k for all neurons j: lower via lam = e_j^T W_k^T
        Wt = ws[k].T                                   # [n_out, n_in]
        lam = Wt[None].expand(R, n_out, -1).reshape(R * n_out, -1)
        c = bs[k][None].expand(R, n_out).reshape(-1)
        # backsub over layers below k (batch rows x neurons)
        def rep(t):
            return t.repeat_interleave(n_out, dim=0)
        saved = (lbs, ubs)
        lbs_r = [rep(t) for t in lbs]; ubs_r = [rep(t) for t in ubs]
        lo_r, hi_r = rep(lo), rep(hi)
        res = []
        for sign in (1.0, -1.0):
            lam_s, c_s = sign * lam, sign * c
            for kk in range(k - 1, -1, -1):
                l, u = lbs_r[kk], ubs_r[kk]
                dead = u <= 0; act = l >= 0; unst = ~(dead | act)
                s = torch.where(unst, u / torch.where(unst, u - l, torch.ones_like(u)), torch.zeros_like(u))
                alpha = (u > -l).double()
                slope = torch.where(act, torch.ones_like(u), torch.where(dead, torch.zeros_like(u),
                                    torch.where(lam_s >= 0, alpha, s)))
                c_s = c_s + torch.where(unst & (lam_s < 0), -lam_s * s * l, torch.zeros_like(u)).sum(1)
                mu = lam_s * slope
                c_s = c_s + mu @ bs[kk]
                lam_s = mu @ ws[kk].T
            res.append(((torch.where(lam_s >= 0, lam_s * lo_r, lam_s * hi_r)).sum(1) + c_s, lam_s, c_s))
        low = res[0][0].view(R, n_out)
        up = (-res[1][0]).view(R, n_out)
        if k < L - 1:
            lbs.append(low); ubs.append(up)
        else:
            r = BoundResult(out_lb=low[:, 0].float(), out_ub=up[:, 0].float())
            r.Lc, r.L0, r.Le = res[0][1].float(), res[0][2].float(), torch.zeros(R)
            r.Uc, r.U0, r.Ue = (-res[1][1]).float(), (-res[1][2]).float(), torch.zeros(R)
            return r


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--preset", default="src/AC-sex")
    ap.add_argument("--model", default="AC-8")
    ap.add_argument("--partitions", type=int, default=256)
    ap.add_argument("--budget", type=int, default=2048)
    ap.add_argument("--weights", default="random")
    ap.add_argument("--bound", default="fwd", choices=["fwd", "crown", "both", "zero", "one", "fwd+zero", "fwd+zero+one",
                                                       "fullcrown", "fwd+fullcrown"])
    ap.add_argument("--split", default="cert", choices=["cert", "strong", "smear"])
    ap.add_argument("--residue", default=None, help="npz of tools/dump_residue.py: its UNKNOWN ids instead of the order")
    ap.add_argument("--summary-only", action="store_true")
    args = ap.parse_args()
    from fairify_amd import presets
    from fairify_amd.engine.bab import _pa_table
    from fairify_amd.models.zoo import get_model
    from fairify_amd.ops.backend import Backend
    from fairify_amd.partition import processing_order

    torch.set_num_threads(8)
    pre = presets.get(args.preset)
    grid = pre.grid()
    q = pre.resolved()
    order = processing_order(grid, seed=0)[:args.partitions]
    if args.residue:
        z = np.load(args.residue)
        order = z["grid_id"][z["verdict"] == "unknown"][:args.partitions]
    m = get_model(args.model, weights=args.weights, seed=0)
    be = Backend(m, device="cpu")
    lo_np, hi_np = grid.decode(order)
    values_np, pairs_np = _pa_table(q, lo_np, hi_np)
    values = torch.from_numpy(values_np)
    pairs = torch.from_numpy(pairs_np)
    pa = torch.tensor(list(q.pa_idx))
    V = values.shape[0]
    shared = torch.ones(q.n, dtype=torch.bool)
    P = len(order)
    xlo = torch.from_numpy(lo_np).float()
    xhi = torch.from_numpy(hi_np).float()
    part = torch.arange(P)
    nodes = torch.zeros(P, dtype=torch.long)
    t0 = time.time()
    while xlo.shape[0]:
        alive = nodes[part] < args.budget
        if not bool(alive.any()):
            break
        over_lo, over_hi, over_part = xlo[~alive], xhi[~alive], part[~alive]
        xlo, xhi, part = xlo[alive], xhi[alive], part[alive]
        nodes.index_add_(0, part, torch.ones_like(part))
        N = xlo.shape[0]
        rlo = xlo[:, None, :].expand(N, V, q.n).clone()
        rhi = xhi[:, None, :].expand(N, V, q.n).clone()
        rlo[:, :, pa] = values.float()[None]
        rhi[:, :, pa] = values.float()[None]
        res = be.bounds(rlo.reshape(-1, q.n), rhi.reshape(-1, q.n), mode="symbolic", keep_layers=True)
        if args.bound == "fwd":
            dec = be.pair_certify(res, res, xlo, xhi, xlo, xhi, pairs, values, pa, shared, False)
        elif args.bound in ("zero", "one", "fwd+zero", "fwd+zero+one"):
            from fairify_amd.ops import reference as ref
            slopes = {"zero": ["zero"], "one": ["one"], "fwd+zero": ["adaptive", "zero"],
                      "fwd+zero+one": ["adaptive", "zero", "one"]}[args.bound]
            dec = None
            for sl in slopes:
                rz = ref.bounds(be.ws, be.bs, rlo.reshape(-1, q.n), rhi.reshape(-1, q.n), mode="symbolic",
                                unit=be.unit, lower_slope=sl)
                dz = be.pair_certify(rz, rz, xlo, xhi, xlo, xhi, pairs, values, pa, shared, False)
                if dec is None:
                    dec = dz
                else:
                    dec.open_ = dec.open_ & dz.open_
        elif args.bound in ("fullcrown", "fwd+fullcrown"):
            rf = full_crown(be, rlo.reshape(-1, q.n), rhi.reshape(-1, q.n))
            dec = be.pair_certify(rf, rf, xlo, xhi, xlo, xhi, pairs, values, pa, shared, False)
            if args.bound == "fwd+fullcrown":
                d2 = be.pair_certify(res, res, xlo, xhi, xlo, xhi, pairs, values, pa, shared, False)
                dec.open_ = dec.open_ & d2.open_
        else:
            rc = crown(be, res, rlo.reshape(-1, q.n), rhi.reshape(-1, q.n))
            dec = be.pair_certify(rc, rc, xlo, xhi, xlo, xhi, pairs, values, pa, shared, False)
            if args.bound == "both":
                d2 = be.pair_certify(res, res, xlo, xhi, xlo, xhi, pairs, values, pa, shared, False)
                dec.open_ = dec.open_ & d2.open_
        width = (xhi - xlo).amax(dim=1)
        leaf = dec.open_ & (width == 0)
        sp = dec.open_ & ~leaf
        idx = torch.nonzero(sp).flatten()
        d = dec.split_dim[idx]
        if args.split == "strong" and len(idx):
            d = strong_dims(be, xlo[idx], xhi[idx], V, q, values, pairs, pa, shared)
        elif args.split == "smear" and len(idx):
            d = smear_dims(be, xlo[idx], xhi[idx], values, pa)
        a, b = xlo[idx], xhi[idx]
        ar = torch.arange(len(idx))
        mid = torch.floor((a[ar, d] + b[ar, d]) / 2)
        h1 = b.clone()
        h1[ar, d] = mid
        l2 = a.clone()
        l2[ar, d] = mid + 1
        xlo = torch.cat([over_lo, a, l2])
        xhi = torch.cat([over_hi, h1, b])
        part = torch.cat([over_part, part[idx], part[idx]])
    print(f"BaB {time.time() - t0:.1f}s", flush=True)
    open_parts = torch.unique(part)
    print(f"partitions open at budget {args.budget}: {open_parts.numel()} / {P}")
    closed = np.setdiff1d(np.arange(P), open_parts.numpy())
    print("nodes of closed partitions:", sorted(nodes[closed].tolist()), "total nodes", int(nodes.sum()))
    if args.summary_only:
        return
    # classify the open partitions by sampled logit range (row v = each PA value)
    ws = [w.double() for w in be.ws]; bs_ = [b.double() for b in be.bs]
    def net(x):
        h = x
        for i, (w, b) in enumerate(zip(ws, bs_)):
            h = h @ w + b
            if i < len(ws) - 1:
                h = h.clamp(min=0)
        return h[..., 0]
    cats = {}
    for p in open_parts.tolist():
        l = torch.from_numpy(lo_np[p]).double(); h = torch.from_numpy(hi_np[p]).double()
        X = torch.floor(l + torch.rand(20000, q.n, dtype=torch.float64) * (h - l + 1))
        key = []
        for v in range(V):
            Xv = X.clone(); Xv[:, pa] = values[v].double()
            z = net(Xv)
            key.append("cross" if (z.min() < 0 < z.max()) else ("pos" if z.min() > 0 else
                       ("neg" if z.max() < 0 else ("zero" if (z == 0).all() else ("nonpos0" if z.max() == 0 else "nonneg0")))))
        k = "/".join(key)
        cats[k] = cats.get(k, 0) + 1
    print("open partitions by sampled sign pattern (row per PA value):", cats)
    if not xlo.shape[0]:
        return
    N = xlo.shape[0]
    rlo = xlo[:, None, :].expand(N, V, q.n).clone()
    rhi = xhi[:, None, :].expand(N, V, q.n).clone()
    rlo[:, :, pa] = values.float()[None]
    rhi[:, :, pa] = values.float()[None]
    res = be.bounds(rlo.reshape(-1, q.n), rhi.reshape(-1, q.n), mode="symbolic")
    stable = (res.dead | res.active).view(N, V, -1).all(dim=2).all(dim=1)
    n_unst = (~(res.dead | res.active)).view(N, V, -1).sum(dim=(1, 2))
    pts = (xhi - xlo + 1).double().prod(dim=1)
    print(f"open frontier nodes: {N}; fully stable {int(stable.sum())} ({100.0 * stable.float().mean():.1f}%)")
    print("unstable neurons per node (both rows): hist", torch.bincount(n_unst.clamp(max=20)).tolist())
    print(f"lattice points per node: median {pts.median().item():.3g}, p90 {pts.quantile(0.9).item():.3g}, "
          f"max {pts.max().item():.3g}")
    fr = []
    for p in open_parts.tolist():
        s = part == p
        fr.append(float(stable[s].float().mean()))
    fr = np.array(fr)
    print(f"per open partition: all-stable frontier {int((fr == 1).sum())}, >=90% stable {int((fr >= .9).sum())}, "
          f"median stable fraction {np.median(fr):.2f}")


if __name__ == "__main__":
    main()
