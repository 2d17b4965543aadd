#!/usr/bin/env python
"""Does the open frontier a partition leaves at the first-pass budget predict whether the
escalated pass decides it?  Per model: BaB at --budget on --partitions partitions, then the
UNKNOWN ones at --escalate; resolution rate and escalation node cost per open_left bucket.

    python tools/diag_escalate.py --models AC-4,AC-8 --partitions 4096
"""
from __future__ import annotations

import argparse
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
    ap.add_argument("--partitions", type=int, default=4096)
    ap.add_argument("--budget", type=int, default=2048)
    ap.add_argument("--escalate", type=int, default=8192)
    ap.add_argument("--json-out", default=None)
    args = ap.parse_args()
    import torch

    from fairify_amd import presets
    from fairify_amd.engine.bab import BaBConfig, BaBSolver
    from fairify_amd.models.zoo import get_model
    from fairify_amd.ops.backend import Backend
    from fairify_amd.partition import processing_order

    dev = torch.device("cuda")
    pre = presets.get(args.preset)
    grid = pre.grid()
    q = pre.resolved()
    ids = processing_order(grid, seed=0)[:args.partitions]
    lo, hi = grid.decode(ids)
    edges = [0, 16, 64, 128, 256, 512, 1024, 1 << 30]
    out = []
    for name in (args.models.split(",") if args.models else list(pre.models)):
        m = get_model(name, weights="random", seed=0)
        be = Backend(m, device=dev)
        r1 = BaBSolver(be, q, BaBConfig(node_budget=args.budget)).solve(lo, hi, m)
        unk = np.nonzero(r1.status == 0)[0]
        if unk.size == 0:
            continue
        ol = r1.open_left[unk]
        t0 = time.time()
        r2 = BaBSolver(be, q, BaBConfig(node_budget=args.escalate)).solve(lo[unk], hi[unk], m)
        torch.cuda.synchronize()
        dt = time.time() - t0
        res = r2.status != 0
        rows = []
        for a, b in zip(edges[:-1], edges[1:]):
            s = (ol >= a) & (ol < b)
            if s.any():
                rows.append(dict(bucket=f"[{a},{b})", n=int(s.sum()), resolved=int(res[s].sum()),
                                 nodes=int(r2.nodes[s].sum())))
        row = dict(model=name, unknown=int(unk.size), resolved=int(res.sum()), escalate_s=round(dt, 3),
                   nodes=int(r2.nodes.sum()), buckets=rows)
        out.append(row)
        print(json.dumps(row), flush=True)
    if args.json_out:
        json.dump(out, open(args.json_out, "w"), indent=1)


if __name__ == "__main__":
    main()
