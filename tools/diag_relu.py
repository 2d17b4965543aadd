#!/usr/bin/env python
"""Per-model cost / yield of the ReLU-phase stage (engine/relu_bab.py) on the bench schedule.

For each model: verify the first --limit partitions of the seeded order with the bench's sound
schedule (heuristic off), relu stage off vs on (budgets from --budgets), and print decided counts
and wall time per stage (synchronised).  The input of the per-model relu policy.

    python tools/diag_relu.py --models AC-7,AC-8,AC-12 --limit 4000 --budgets 0,256,2048
"""
from __future__ import annotations

import argparse
import os
import sys
import time

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--preset", default="src/AC-sex")
    ap.add_argument("--models", default="AC-1,AC-2,AC-3,AC-4,AC-5,AC-6,AC-7,AC-8,AC-9,AC-10,AC-11,AC-12")
    ap.add_argument("--limit", type=int, default=4000)
    ap.add_argument("--budgets", default="0,2048")
    ap.add_argument("--escalate-budget", type=int, default=32768)
    ap.add_argument("--escalate-probation", default="2048:768,4096:768,8192:768,16384:1024")
    ap.add_argument("--weights", default="random", help="random | zoo (the reference's trained nets)")
    ap.add_argument("--offset", type=int, default=0, help="first position of the seeded order")
    args = ap.parse_args()
    import torch

    from fairify_amd import presets
    from fairify_amd.engine.pipeline import VerifyConfig, verify_chunk
    from fairify_amd.models.zoo import get_model
    from fairify_amd.ops.backend import Backend
    from fairify_amd.partition import processing_order
    from fairify_amd.utils.timer import StageTimer

    dev = torch.device("cuda" if torch.cuda.device_count() else "cpu")
    pre = presets.get(args.preset)
    grid, q = pre.grid(), pre.resolved()
    ids = processing_order(grid, seed=0)[args.offset:args.offset + args.limit]
    for name in args.models.split(","):
        m = get_model(name, weights=args.weights, seed=0)
        be = Backend(m, device=dev)
        for rb in (int(b) for b in args.budgets.split(",")):
            cfg = VerifyConfig(sim_size=pre.sim_size, chunk=4096, soft_timeout=pre.soft_timeout,
                               hard_timeout=pre.hard_timeout, node_budget=512, heuristic=False,
                               escalate_budget=args.escalate_budget, escalate_max_open=384, smt_backend="none",
                               relu_budget=rb, relu_max_width=1 << 20,
                               escalate_probation=tuple(tuple(int(v) for v in st.split(":"))
                                                        for st in args.escalate_probation.split(",") if st))
            verify_chunk(be, m, q, grid, ids[:256], cfg)            # warm caches / runtimes
            tm = StageTimer(dev, sync=True)
            t0 = time.time()
            recs = verify_chunk(be, m, q, grid, ids, cfg, timer=tm)
            if dev.type == "cuda":
                torch.cuda.synchronize()
            wall = time.time() - t0
            v, st = recs.cols["verdict"], recs.cols["stage"]
            relu_dec = int(((v != "unknown") & (st == "relu")).sum())
            stimes = {k: round(s, 3) for k, s in tm.t.items() if k in ("bab", "relu", "falsify", "sim")}
            print(f"{name} relu_budget {rb}: wall {wall:.3f}s decided {(v != 'unknown').sum()} "
                  f"unknown {(v == 'unknown').sum()} relu-decided {relu_dec} stages {stimes}", flush=True)


if __name__ == "__main__":
    main()
