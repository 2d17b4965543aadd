#!/usr/bin/env python
"""CPU experiment: how many input-split BaB nodes does the bench residue need?  Runs the torch
BaB (same bounds / certificate / split rule as the device BaB) with growing budgets on residue
partitions dumped by tools/dump_residue.py and reports decided counts per budget.

    python tools/exp/residue_depth.py --model AC-7 --residue gpurun_out/r4a/residue/AC-7.npz --n 20
"""
from __future__ import annotations

import argparse
import os
import sys
import time

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--model", default="AC-7")
    ap.add_argument("--residue", required=True)
    ap.add_argument("--n", type=int, default=20)
    ap.add_argument("--budgets", default="4096,16384,65536")
    args = ap.parse_args()
    import torch

    from fairify_amd import presets
    from fairify_amd.engine.bab import BaBConfig, BaBSolver, SAT, UNSAT
    from fairify_amd.models.zoo import get_model
    from fairify_amd.ops.backend import Backend

    torch.set_num_threads(8)
    pre = presets.get("src/AC-sex")
    grid, q = pre.grid(), pre.resolved()
    m = get_model(args.model, weights="random", seed=0)
    be = Backend(m, device="cpu")
    z = np.load(args.residue)
    ids = z["grid_id"][z["verdict"] == "unknown"][:args.n]
    lo, hi = grid.decode(ids)
    for b in (int(v) for v in args.budgets.split(",")):
        t0 = time.time()
        res = BaBSolver(be, q, BaBConfig(node_budget=b, batch_nodes=65536)).solve(lo, hi, m)
        st = res.status
        print(f"budget {b}: sat {(st == SAT).sum()} unsat {(st == UNSAT).sum()} of {len(ids)}; "
              f"nodes median {int(np.median(res.nodes))} max {int(res.nodes.max())} ({time.time() - t0:.1f}s)",
              flush=True)
        dec = np.isin(st, (SAT, UNSAT))
        print("   decided nodes:", sorted(res.nodes[dec].tolist()))


if __name__ == "__main__":
    main()
