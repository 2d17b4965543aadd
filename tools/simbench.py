#!/usr/bin/env python
"""Micro-benchmark of the simulation kernel (fa_sim_kernel, K3+K8): ``simulate`` on --partitions
partitions of every AC model, one stream, median of --reps timed launches after a warm launch.
Prints one JSON line per model plus a checksum of the activation counts / flip keys, so two
builds can be compared for both speed and bitwise-identical results.

    python tools/simbench.py --partitions 8192 --reps 5
"""
from __future__ import annotations

import argparse
import hashlib
import json
import os
import sys
import time

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--preset", default="src/AC-sex")
    ap.add_argument("--models", default=None)
    ap.add_argument("--partitions", type=int, default=8192)
    ap.add_argument("--reps", type=int, default=5)
    args = ap.parse_args()
    import torch

    from fairify_amd import presets
    from fairify_amd.engine.bab import _pa_table
    from fairify_amd.engine.sim import simulate
    from fairify_amd.models.zoo import get_model
    from fairify_amd.ops import hip as H
    from fairify_amd.ops.backend import Backend
    from fairify_amd.partition import processing_order

    dev = torch.device("cuda")
    pre = presets.get(args.preset)
    grid, q = pre.grid(), pre.resolved()
    ids = processing_order(grid, 0)[:args.partitions]
    lo_np, hi_np = grid.decode(ids)
    values_np, pairs_np = _pa_table(q, lo_np, hi_np)
    values = torch.from_numpy(values_np).to(dev)
    pairs = torch.from_numpy(pairs_np).to(dev)
    pids = torch.from_numpy(ids).to(dev)
    names = args.models.split(",") if args.models else list(pre.models)
    for name in names:
        m = get_model(name, weights="random", seed=0)
        be = Backend(m, device=dev)
        assert be.hip
        lo, hi = H.decode(grid, pids)
        res = simulate(be, q, lo, hi, pids, pre.sim_size, 0, values, pairs, 0, 0)
        torch.cuda.synchronize()
        ts = []
        for _ in range(args.reps):
            t0 = time.perf_counter()
            res = simulate(be, q, lo, hi, pids, pre.sim_size, 0, values, pairs, 0, 0)
            torch.cuda.synchronize()
            ts.append(time.perf_counter() - t0)
        h = hashlib.sha1(res.counts.cpu().numpy().tobytes() + res.found.cpu().numpy().tobytes()).hexdigest()[:12]
        print(json.dumps({"model": name, "ms": round(1e3 * float(np.median(ts)), 3), "found": int(res.found.sum()),
                          "hash": h}), flush=True)


if __name__ == "__main__":
    main()
