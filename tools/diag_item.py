#!/usr/bin/env python
"""Critical-path diagnostic of one bench work item (bench.py's configuration, one stream).

Runs the (model, shard) item the way bench.py does, alone on the GPU, and prints the per-stage
timer breakdown (synchronised), the BaB level / launch / node statistics and the verdict split:
which stage of the longest item of a 1/8 shard is worth shortening.

    python tools/diag_item.py --models AC-12,AC-4 --shard 0/8
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
    ap.add_argument("--models", default="AC-12")
    ap.add_argument("--shard", default="0/8")
    ap.add_argument("--repeat", type=int, default=2)
    ap.add_argument("--escalate-budget", type=int, default=32768)
    ap.add_argument("--escalate-max-open", type=int, default=384)
    ap.add_argument("--no-heuristic", action="store_true")
    ap.add_argument("--escalate-probation", default="2048:768,4096:768,8192:768,16384:1024")
    args = ap.parse_args()
    import torch

    from fairify_amd import presets
    from fairify_amd.engine import bab as B
    from fairify_amd.engine.pipeline import VerifyConfig, verify_chunk
    from fairify_amd.models.zoo import get_model
    from fairify_amd.ops.backend import Backend
    from fairify_amd.partition import processing_order
    from fairify_amd.utils.timer import StageTimer

    dev = torch.device("cuda")
    pre = presets.get(args.preset)
    grid, q = pre.grid(), pre.resolved()
    order = processing_order(grid, seed=0)
    r, n = (int(v) for v in args.shard.split("/"))
    ids = order[r::n][:4096]
    cfg = VerifyConfig(sim_size=pre.sim_size, chunk=4096, soft_timeout=pre.soft_timeout,
                       hard_timeout=pre.hard_timeout, node_budget=512, heuristic_p=pre.heuristic_p,
                       heuristic_node_budget=512, escalate_budget=args.escalate_budget,
                       escalate_max_open=args.escalate_max_open, heuristic=not args.no_heuristic, smt_backend="none",
                       escalate_probation=tuple(tuple(int(v) for v in st.split(":"))
                                                for st in args.escalate_probation.split(",") if st))
    for name in args.models.split(","):
        m = get_model(name, weights="random", seed=0)
        be = Backend(m, device=dev)
        verify_chunk(be, m, q, grid, ids, cfg)
        torch.cuda.synchronize()
        for rep in range(args.repeat):
            for k in B.STATS:
                B.STATS[k] = 0
            tm = StageTimer(dev, sync=True)
            t0 = time.time()
            recs = verify_chunk(be, m, q, grid, ids, cfg, timer=tm)
            torch.cuda.synchronize()
            wall = time.time() - t0
            c = recs.cols
            row = dict(model=name, rep=rep, n=len(recs), wall_ms=round(1e3 * wall, 1),
                       stages_ms={k: round(1e3 * t, 1) for k, t in tm.t.items()},
                       bab=dict(B.STATS), nodes_sum=int(c["nodes"].sum()),
                       nodes_p50=float(np.median(c["nodes"])), nodes_max=int(c["nodes"].max()),
                       verdicts={v: int((c["verdict"] == v).sum()) for v in ("sat", "unsat", "unknown")},
                       heuristic=int((c["stage"] == "heuristic").sum()),
                       nodes_unknown=int(c["nodes"][c["verdict"] == "unknown"].sum()),
                       escalate=args.escalate_budget)
            print(json.dumps(row), flush=True)


if __name__ == "__main__":
    main()
