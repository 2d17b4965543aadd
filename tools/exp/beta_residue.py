#!/usr/bin/env python
"""beta stage settings on a dumped residue (tools/dump_residue.py): decided counts and time.

    python tools/exp/beta_residue.py --preset relaxed/BM --model BM-8 --npz gpurun_out/res/BM-8.npz --n 400

Each setting runs the stage alone (no probe) on the same UNKNOWN partitions; prints one line per
setting: decided SAT / UNSAT, the stage's stats, wall seconds.
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
    ap.add_argument("--weights", default="zoo")
    ap.add_argument("--npz", required=True)
    ap.add_argument("--n", type=int, default=400)
    ap.add_argument("--set", action="append", default=[],
                    help="extra setting 'name:key=value,key=value' over BetaConfig(node_budget=64) "
                         "(e.g. pg_b1024:branch=pgap,node_budget=1024,lookahead=0); given: only these run")
    args = ap.parse_args()
    import torch

    from fairify_amd import presets
    from fairify_amd.engine.beta_bab import SAT, UNSAT, BetaBaBSolver, BetaConfig
    from fairify_amd.models.zoo import get_model
    from fairify_amd.ops.backend import Backend

    pre = presets.get(args.preset)
    grid, q = pre.grid(), pre.resolved()
    d = np.load(args.npz)
    ids = d["grid_id"][d["verdict"] == "unknown"][:args.n]
    lo, hi = grid.decode(ids)
    m = get_model(args.model, weights=args.weights, seed=0)
    be = Backend(m, device="cuda" if torch.cuda.device_count() else "cpu")
    base = BetaConfig(node_budget=64)
    only = os.environ.get("BETA_RES_ONLY")
    settings = {
        "default(64)": base,
        "iters512_root2000": replace(base, iters=512, root_iters=2000),
        "lpgap_b1024": replace(base, branch="lpgap", node_budget=1024),
        "lpgap_b4096": replace(base, branch="lpgap", node_budget=4096),
        "it256_b1024": replace(base, iters=256, root_iters=1000, node_budget=1024),
        "it256_b4096": replace(base, iters=256, root_iters=1000, node_budget=4096),
        "b4096": replace(base, node_budget=4096),
        "la0_b256": replace(base, lookahead=0, node_budget=256),
        "la0_b1024": replace(base, lookahead=0, node_budget=1024),
        "la2_b1024": replace(base, lookahead=2, node_budget=1024),
        "la0_input2_b1024": replace(base, lookahead=0, node_budget=1024, input_every=2),
        "iters1024_root4000_lr_half": replace(base, iters=1024, root_iters=4000, lr_a=0.05, lr_b=0.25, lr_t=0.05,
                                              decay=0.995),
        "budget256": replace(base, node_budget=256),
        "budget1024": replace(base, node_budget=1024),
        "iters128": replace(base, iters=128, root_iters=400),
        "lookahead16": replace(base, lookahead=16),
        "no_tighten": replace(base, tighten=False),
        "lr_x2": replace(base, lr_a=0.2, lr_b=1.0, lr_t=0.2),
        "lr_t_x10": replace(base, lr_t=1.0),
        "lr_t_x10_b256": replace(base, lr_t=1.0, node_budget=256),
        "lr_t_x30_it128_b256": replace(base, lr_t=3.0, iters=128, root_iters=400, node_budget=256),
        "input_every1_b256": replace(base, node_budget=256, input_every=1),
        "input_every2_b256": replace(base, node_budget=256, input_every=2),
        "input_every3_b256": replace(base, node_budget=256, input_every=3),
    }
    if args.set:
        settings = {}
        for spec in args.set:
            name, _, kv = spec.partition(":")
            kw = {}
            for item in filter(None, kv.split(",")):
                k, v = item.split("=")
                cur = getattr(base, k)
                kw[k] = type(cur)(v) if not isinstance(cur, bool) else v in ("1", "true", "True")
            settings[name] = replace(base, **kw)
    print(f"{args.model}: {len(ids)} residue partitions", flush=True)
    for name, cfg in settings.items():
        if only and name not in only.split(","):
            continue
        t0 = time.time()
        s = BetaBaBSolver(be, q, cfg)
        r = s.solve(lo, hi, m)
        if be.hip:
            torch.cuda.synchronize()
        print(f"{name:14s} sat {(r.status == SAT).sum():5d} unsat {(r.status == UNSAT).sum():5d} "
              f"{time.time() - t0:7.2f}s {s.stats}", flush=True)


if __name__ == "__main__":
    main()
