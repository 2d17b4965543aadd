#!/usr/bin/env python
"""ReLU-phase BaB with / without phase-aware refined hidden-layer bounds on the input-split residue
of a (trained) model: how many residue partitions each closes, nodes and wall time.

    python tools/exp/relu_refine_ac7.py --model AC-7 --weights zoo --n 2000 --budgets 2048,16384
"""
from __future__ import annotations

import argparse
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
    ap.add_argument("--n", type=int, default=2000)
    ap.add_argument("--bab-budget", type=int, default=8192)
    ap.add_argument("--budgets", default="2048,16384")
    ap.add_argument("--modes", default="off,auto")
    a = ap.parse_args()
    import torch

    from fairify_amd import presets
    from fairify_amd.engine.bab import SAT, UNSAT, BaBConfig, BaBSolver
    from fairify_amd.engine.relu_bab import ReluBaBSolver, ReluConfig
    from fairify_amd.models.zoo import get_model
    from fairify_amd.ops.backend import Backend
    from fairify_amd.partition import processing_order

    pre = presets.get(a.preset)
    grid, q = pre.grid(), pre.resolved()
    m = get_model(a.model, weights=a.weights, seed=0)
    be = Backend(m, torch.device("cuda"))
    ids = processing_order(grid, 0)[:a.n]
    lo, hi = grid.decode(ids)
    t = time.time()
    r = BaBSolver(be, q, BaBConfig(node_budget=a.bab_budget)).solve(lo, hi, m)
    unk = np.nonzero(~np.isin(r.status, (SAT, UNSAT)))[0]
    print(json.dumps({"stage": "input-split", "n": a.n, "sat": int((r.status == SAT).sum()),
                      "unsat": int((r.status == UNSAT).sum()), "unknown": int(unk.size),
                      "nodes": int(r.nodes.sum()), "s": round(time.time() - t, 2)}), flush=True)
    for b in (int(x) for x in a.budgets.split(",")):
        for mode in a.modes.split(","):
            t = time.time()
            rr = ReluBaBSolver(be, q, ReluConfig(node_budget=b, refine=mode)).solve(lo[unk], hi[unk], m)
            print(json.dumps({"stage": "relu", "budget": b, "refine": mode, "residue": int(unk.size),
                              "sat": int((rr.status == SAT).sum()), "unsat": int((rr.status == UNSAT).sum()),
                              "nodes": int(np.asarray(rr.nodes).sum()), "s": round(time.time() - t, 2)}), flush=True)


if __name__ == "__main__":
    main()
