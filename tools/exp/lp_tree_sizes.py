#!/usr/bin/env python
"""CPU experiment: LP branch-and-bound tree sizes on a trained model's partitions (smt/lpbab.py,
the verified-LP stage) -- does the coupled LP close a partition at its root (then optimised
CROWN slopes, whose optimum is that LP, would close it on the GPU) or only after ReLU-phase
branching (split constraints: beta terms)?

    python tools/exp/lp_tree_sizes.py --model AC-7 --weights zoo --n 40 --skip 0
"""
from __future__ import annotations

import argparse
import collections
import json
import os
import sys
import time

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--preset", default="src/AC-sex")
    ap.add_argument("--model", default="AC-7")
    ap.add_argument("--weights", default="zoo")
    ap.add_argument("--n", type=int, default=40)
    ap.add_argument("--skip", type=int, default=0)
    ap.add_argument("--budget", type=int, default=4000)
    a = ap.parse_args()
    import torch

    from fairify_amd import presets
    from fairify_amd.engine import exact
    from fairify_amd.models.zoo import get_model
    from fairify_amd.ops.backend import Backend
    from fairify_amd.partition import processing_order
    from fairify_amd.smt import lpbab, milp

    torch.set_num_threads(4)
    pre = presets.get(a.preset)
    grid, q = pre.grid(), pre.resolved()
    m = get_model(a.model, weights=a.weights, seed=0)
    be = Backend(m, "cpu")
    ids = processing_order(grid, 0)[a.skip:a.skip + a.n]
    lo, hi = grid.decode(ids)
    from fairify_amd.engine.bab import _pa_table

    vals, pairs = _pa_table(q, lo, hi)
    lbs, ubs = milp.layer_bounds_rows(be, lo, hi, q, vals, widen_ra=False)
    hist = collections.Counter()
    for k in range(len(lo)):
        rb = {v: ([lb[k, v] for lb in lbs], [ub[k, v] for ub in ubs]) for v in range(vals.shape[0])}

        def confirm(xs, xps):
            ok = exact.check_pair_constraints(xs[None], xps[None], lo[k][None], hi[k][None], q.pa_idx, (), 0)
            return bool(ok[0] and exact.is_violation(m, xs[None], xps[None])[0])

        t = time.time()
        per = []
        verdict = "unsat"
        for vi, vj in pairs:
            st, wit, nodes = lpbab.lp_bab_pair(m.weights, m.biases, lo[k], hi[k], q.pa_idx, vals[int(vi)],
                                              vals[int(vj)], rb[int(vi)], rb[int(vj)], a.budget, time.time() + 120,
                                              confirm)
            per.append((st, nodes))
            if st == "sat":
                verdict = "sat"
                break
            if st != "unsat":
                verdict = "unknown"
                break
        tot = sum(n for _, n in per)
        key = "sat" if verdict == "sat" else (verdict if verdict != "unsat" else
                                             ("root" if all(n <= 1 for _, n in per) else
                                              ("<=16" if tot <= 16 else ("<=256" if tot <= 256 else ">256"))))
        hist[key] += 1
        print(json.dumps({"pid": int(ids[k]), "verdict": verdict, "pairs": per, "s": round(time.time() - t, 2)}),
              flush=True)
    print(json.dumps({"summary": dict(hist)}), flush=True)


if __name__ == "__main__":
    main()
