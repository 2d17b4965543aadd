#!/usr/bin/env python
"""Dump the sound-UNKNOWN residue of the bench configuration (heuristic retry off) per model.

Runs bench.py's default sound schedule (node budget 512, inline escalation to 32 768 behind the
frontier gates, residual falsifier) on the first --limit partitions of the seeded order and
writes OUT/<model>.npz with the grid ids, verdicts, stages, nodes and open-frontier sizes, the
input of the CPU experiments on the residue (tools/exp_*.py).

    python tools/dump_residue.py --models AC-8,AC-12,AC-7 --limit 4000 --out gpurun_out/residue
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
    ap.add_argument("--out", default="gpurun_out/residue")
    ap.add_argument("--weights", default="random", help="random | zoo (trained weights)")
    ap.add_argument("--big", action="store_true",
                    help="the big-grid schedule of tools/baseline_configs.py (escalation to 8 192 nodes)")
    ap.add_argument("--cfg", default="", help="VerifyConfig overrides 'key=value,...'")
    args = ap.parse_args()
    import torch

    from fairify_amd import presets
    from fairify_amd.engine.pipeline import VerifyConfig, verify_chunk
    from fairify_amd.models.zoo import get_model
    from fairify_amd.ops.backend import Backend
    from fairify_amd.partition import processing_order

    dev = torch.device("cuda" if torch.cuda.device_count() else "cpu")
    pre = presets.get(args.preset)
    grid, q = pre.grid(), pre.resolved()
    ids = processing_order(grid, seed=0)[:args.limit]
    cfg = VerifyConfig(sim_size=pre.sim_size, chunk=4096, soft_timeout=pre.soft_timeout, hard_timeout=pre.hard_timeout,
                       node_budget=512, heuristic=False, heuristic_p=pre.heuristic_p,
                       escalate_budget=8192 if args.big else 32768, escalate_max_open=384, smt_backend="none",
                       escalate_probation=((2048, 768), (4096, 768)) if args.big else
                       ((2048, 768), (4096, 768), (8192, 768), (16384, 1024)),
                       relu_budget=1024, relu_max_width=16, relu_escalate_cap=2048)
    if args.cfg:      # VerifyConfig overrides 'key=value,...'
        from dataclasses import replace as _rp

        kv = {}
        for item in filter(None, args.cfg.split(",")):
            k, v = item.split("=")
            kv[k] = type(getattr(cfg, k))(v)
        cfg = _rp(cfg, **kv)
    os.makedirs(args.out, exist_ok=True)
    for name in args.models.split(","):
        m = get_model(name, weights=args.weights, seed=0)
        be = Backend(m, device=dev)
        t0 = time.time()
        recs = verify_chunk(be, m, q, grid, ids, cfg)
        if dev.type == "cuda":
            torch.cuda.synchronize()
        c = recs.cols
        v = c["verdict"]
        np.savez_compressed(os.path.join(args.out, f"{name}.npz"), grid_id=c["grid_id"], verdict=v.astype(str),
                            stage=c["stage"].astype(str), nodes=c["nodes"],
                            stage_nodes=c.get("stage_nodes", np.zeros((len(v), 0), np.int64)))
        print(f"{name}: {len(ids)} partitions in {time.time() - t0:.2f}s: sat {(v == 'sat').sum()} "
              f"unsat {(v == 'unsat').sum()} unknown {(v == 'unknown').sum()}", flush=True)


if __name__ == "__main__":
    main()
