#!/usr/bin/env python
"""One residue partition, tree by tree: the verified LP-BaB's node count per (ordered pair, orientation)
(smt/lpbab.py:lp_bab_pair) next to the beta BaB's on the same tree (BetaConfig.trees), CPU.

    python tools/exp/beta_trees.py --gid 11368 --budget 4096 --set it256:iters=256
"""
from __future__ import annotations

import argparse
import os
import sys
import time
from dataclasses import replace

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--preset", default="relaxed/BM")
    ap.add_argument("--model", default="BM-8")
    ap.add_argument("--gid", type=int, required=True)
    ap.add_argument("--budget", type=int, default=4096, help="nodes per tree")
    ap.add_argument("--set", action="append", default=[], help="beta setting 'name:key=value,...'")
    args = ap.parse_args()
    import torch

    from fairify_amd import presets
    from fairify_amd.engine import exact
    from fairify_amd.engine.bab import SAT, UNSAT, _pa_table
    from fairify_amd.engine.beta_bab import BetaBaBSolver, BetaConfig
    from fairify_amd.models.zoo import get_model
    from fairify_amd.ops.backend import Backend
    from fairify_amd.smt import lpbab, milp

    torch.set_num_threads(max(1, (os.cpu_count() or 2) - 1))
    pre = presets.get(args.preset)
    grid, q = pre.grid(), pre.resolved()
    lo, hi = grid.decode(np.array([args.gid]))
    m = get_model(args.model, weights="zoo", seed=0)
    be = Backend(m, device="cpu")
    values, pairs = _pa_table(q, lo, hi)
    Pp = pairs.shape[0]
    O = 2 if q.relaxed else 1
    lbs, ubs = milp.layer_bounds_rows(be, lo, hi, q, values, widen_ra=False)
    lbp, ubp = milp.layer_bounds_rows(be, lo, hi, q, values, widen_ra=True) if q.relaxed else (lbs, ubs)
    rb = {v: ([lb[0, v] for lb in lbs], [ub[0, v] for ub in ubs]) for v in range(values.shape[0])}
    rbp = {v: ([lb[0, v] for lb in lbp], [ub[0, v] for ub in ubp]) for v in range(values.shape[0])}

    def confirm(xs, xps):
        ok = exact.check_pair_constraints(xs[None], xps[None], lo, hi, q.pa_idx, q.ra_idx, q.tau)
        return bool(ok[0] and exact.is_violation(m, xs[None], xps[None])[0])

    # node_budget of the beta config = per-tree budget (one tree per call: x Pp / 2 x O undone)
    nb = max(1, int(args.budget / (max(1.0, Pp / 2.0) * O)))
    base = BetaConfig(node_budget=nb, native=False)
    sets = {"default": base}
    for spec in args.set:
        name, _, kv = spec.partition(":")
        kw = {}
        for item in filter(None, kv.split(",")):
            k, v = item.split("=")
            cur = getattr(base, k)
            kw[k] = type(cur)(v) if not isinstance(cur, bool) else v in ("1", "true", "True")
        sets[name] = replace(base, **kw)
    name = {SAT: "sat", UNSAT: "unsat"}
    for j in range(Pp):
        vi, vj = int(pairs[j, 0]), int(pairs[j, 1])
        for o in ((1, -1) if q.relaxed else (1,)):
            t0 = time.time()
            st, _, n = lpbab.lp_bab_pair(m.weights, m.biases, lo[0].astype(np.float64), hi[0].astype(np.float64),
                                         q.pa_idx, values[vi], values[vj], rb[vi], rbp[vj], args.budget,
                                         time.time() + 600, confirm, ra_idx=q.ra_idx if q.relaxed else (),
                                         tau=float(q.tau) if q.relaxed else 0.0, orient=o)
            row = [f"pair {j} ({vi},{vj}) orient {o:+d}: LP {st:7s} {n:5d} ({time.time() - t0:4.1f}s)"]
            for sname, cfg in sets.items():
                t0 = time.time()
                s = BetaBaBSolver(be, q, replace(cfg, trees=((j, o),), sign_prune=False))
                r = s.solve(lo, hi, m)
                row.append(f"{sname} {name.get(int(r.status[0]), 'unk'):5s} {int(r.nodes[0]):5d} "
                           f"({time.time() - t0:4.1f}s)")
            print(" | ".join(row), flush=True)


if __name__ == "__main__":
    main()
