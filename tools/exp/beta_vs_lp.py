#!/usr/bin/env python
"""Per-partition tree sizes of the verified LP-BaB (smt/lpbab.py) and the beta BaB (engine/beta_bab.py)
on the same residue partitions (CPU; the LP is the reference the GPU beta stage is measured against).

    python tools/exp/beta_vs_lp.py --npz tools/exp/data/relaxedBM_BM-8_unknown.npz --n 10 --budget 2048

Prints one line per partition: LP verdict / nodes, beta verdict / nodes per setting.
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
    ap.add_argument("--npz", required=True)
    ap.add_argument("--n", type=int, default=10)
    ap.add_argument("--skip", type=int, default=0)
    ap.add_argument("--budget", type=int, default=2048)
    ap.add_argument("--lp-budget", type=int, default=4096)
    ap.add_argument("--set", action="append", default=[], help="beta setting 'name:key=value,...'")
    args = ap.parse_args()
    import torch

    from fairify_amd import presets
    from fairify_amd.engine.bab import SAT, UNSAT, _pa_table
    from fairify_amd.engine.beta_bab import BetaBaBSolver, BetaConfig
    from fairify_amd.models.zoo import get_model
    from fairify_amd.ops.backend import Backend
    from fairify_amd.smt import lpbab

    torch.set_num_threads(max(1, (os.cpu_count() or 2) - 1))
    pre = presets.get(args.preset)
    grid, q = pre.grid(), pre.resolved()
    d = np.load(args.npz)
    ids = d["grid_id"][d["verdict"] == "unknown"][args.skip:args.skip + args.n]
    lo, hi = grid.decode(ids)
    m = get_model(args.model, weights="zoo", seed=0)
    be = Backend(m, device="cpu")
    base = BetaConfig(node_budget=args.budget // 2, native=False)
    sets = {"pgap8": base}
    for spec in args.set:
        name, _, kv = spec.partition(":")
        kw = {}
        for item in filter(None, kv.split(",")):
            k, v = item.split("=")
            cur = getattr(base, k)
            kw[k] = type(cur)(v) if not isinstance(cur, bool) else v in ("1", "true", "True")
        sets[name] = replace(base, **kw)
    name = {SAT: "sat", UNSAT: "unsat"}
    for i, gid in enumerate(ids):
        l1, h1 = lo[i:i + 1], hi[i:i + 1]
        values_np, pairs_np = _pa_table(q, l1, h1)
        t0 = time.time()
        fut = lpbab.submit(be, m, q, l1, h1, values_np, pairs_np, args.lp_budget, 600.0, workers=1)
        v, _, lp_nodes = fut[0].result()
        t_lp = time.time() - t0
        row = [f"{gid:8d} LP {v:7s} {lp_nodes:5d} ({t_lp:5.1f}s)"]
        for sname, cfg in sets.items():
            t0 = time.time()
            s = BetaBaBSolver(be, q, cfg)
            r = s.solve(l1, h1, m)
            row.append(f"{sname} {name.get(int(r.status[0]), 'unk'):5s} {int(r.nodes[0]):5d} ({time.time() - t0:5.1f}s)")
        print(" | ".join(row), flush=True)


if __name__ == "__main__":
    main()
