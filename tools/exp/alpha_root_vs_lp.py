#!/usr/bin/env python
"""CPU check: alpha-optimised coupled CROWN bound at a trained AC-7 partition root vs the verified
LP root value (tools/exp/beta_proto.py functions): converges to the LP with enough iterations."""
import sys, numpy as np, torch
import os; _R = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))); sys.path.insert(0, _R); sys.path.insert(0, os.path.join(_R, "tools", "exp"))
from beta_proto import layer_bounds, pair_low
from fairify_amd import presets
from fairify_amd.engine.bab import _pa_table
from fairify_amd.models.zoo import get_model
from fairify_amd.ops.backend import Backend
from fairify_amd.ops import reference as ref
from fairify_amd.smt import lpbab, milp
pre = presets.get("src/AC-sex"); grid, q = pre.grid(), pre.resolved()
m = get_model("AC-7", weights="zoo", seed=0); be = Backend(m, "cpu")
ws = [w.double() for w in be.ws]; bs = [b.double() for b in be.bs]
NH = sum(int(w.shape[1]) for w in ws[:-1]); pa = list(q.pa_idx)
ids = np.array([12596]); lo_all, hi_all = grid.decode(ids)
vals, pairs = _pa_table(q, lo_all, hi_all)
lbs, ubs = milp.layer_bounds_rows(be, lo_all, hi_all, q, vals, widen_ra=False)
for vi, vj in pairs:
    rb = {v: ([lb[0, v] for lb in lbs], [ub[0, v] for ub in ubs]) for v in range(vals.shape[0])}
    lp = lpbab._LP(m.weights, m.biases, lo_all[0], hi_all[0], pa, vals[int(vi)], vals[int(vj)], rb[int(vi)], rb[int(vj)])
    t_lp, cert, v, basis = lp.solve(lp.lb, lp.ub)
    va = torch.tensor(vals[int(vi)], dtype=torch.float64); vb = torch.tensor(vals[int(vj)], dtype=torch.float64)
    lo = torch.tensor(lo_all[0], dtype=torch.float64)[None]; hi = torch.tensor(hi_all[0], dtype=torch.float64)[None]
    ph = torch.zeros(1, NH, dtype=torch.int8)
    loA, hiA = lo.clone(), hi.clone(); loA[:, pa], hiA[:, pa] = va, va
    loB, hiB = lo.clone(), hi.clone(); loB[:, pa], hiB[:, pa] = vb, vb
    bA = layer_bounds(ws, bs, loA, hiA, ph); bB = layer_bounds(ws, bs, loB, hiB, ph)
    # compare interval widths with the LP's bounds
    wl = sum(float((bA[1][l] - bA[0][l]).sum()) for l in range(len(ws)-1))
    wlp = sum(float((rb[int(vi)][1][l] - rb[int(vi)][0][l]).sum()) for l in range(len(ws)-1))
    ra = torch.zeros(1, NH, dtype=torch.float64, requires_grad=True); rb_ = torch.zeros(1, NH, dtype=torch.float64, requires_grad=True)
    rt = torch.zeros(1, dtype=torch.float64, requires_grad=True)
    opt = torch.optim.Adam([ra, rb_, rt], lr=0.05); best = -1e9
    z = torch.zeros(1, NH, dtype=torch.float64)
    for it in range(3000):
        low, _ = pair_low(ws, bs, lo, hi, pa, va, vb, bA[:2], bB[:2], ph, ph, torch.sigmoid(ra), torch.sigmoid(rb_), z, z, torch.sigmoid(rt), ref.FP64_UNIT)
        best = max(best, float(low)); opt.zero_grad(); (-low.sum()).backward(); opt.step()
    print("pair", vi, vj, "LP t*", t_lp, "cert", cert, "| ours -low(best)", -best, "widths ours", round(wl,2), "lp", round(wlp,2))
