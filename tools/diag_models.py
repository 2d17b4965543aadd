#!/usr/bin/env python
"""Per-model diagnostic of the verification pipeline (one model at a time, one stream).

Prints, per model: wall time, SAT/UNSAT/UNK, which stage decided, BaB node statistics and the
per-stage timer breakdown.  Used to decide where kernel / algorithm work pays off.

    python tools/diag_models.py --preset src/AC-sex --models AC-4,AC-11 [--node-budget 2048]
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
    ap.add_argument("--node-budget", type=int, default=2048)
    ap.add_argument("--chunk", type=int, default=4096)
    ap.add_argument("--max-partitions", type=int, default=None)
    ap.add_argument("--no-heuristic", action="store_true")
    ap.add_argument("--weights", default="random")
    ap.add_argument("--json-out", default=None)
    ap.add_argument("--bench-config", action="store_true",
                    help="bench.py's defaults (inline escalation to 32768 with probation, relu stage, "
                         "chunk 8192) instead of the fixed-budget config above")
    ap.add_argument("--residual-samples", type=int, default=8192)
    ap.add_argument("--residual-iters", type=int, default=24)
    ap.add_argument("--residual-starts", type=int, default=16)
    ap.add_argument("--deep-budget", type=int, default=0,
                    help="re-run the sound BaB with this node budget on the partitions left UNKNOWN "
                         "before the heuristic stage, and report how they resolve")
    args = ap.parse_args()
    import torch

    from fairify_amd import presets
    from fairify_amd.engine.pipeline import VerifyConfig, verify_chunk
    from fairify_amd.models.zoo import get_model
    from fairify_amd.ops.backend import Backend
    from fairify_amd.partition import processing_order
    from fairify_amd.utils.timer import StageTimer

    dev = torch.device("cuda" if torch.cuda.is_available() else "cpu")
    pre = presets.get(args.preset)
    grid = pre.grid()
    q = pre.resolved()
    order = processing_order(grid, seed=0)
    if args.max_partitions:
        order = order[:args.max_partitions]
    names = args.models.split(",") if args.models else list(pre.models)
    cfg = VerifyConfig(sim_size=pre.sim_size, chunk=args.chunk, node_budget=args.node_budget,
                       heuristic=not args.no_heuristic, heuristic_p=pre.heuristic_p,
                       heuristic_node_budget=args.node_budget, residual_samples=args.residual_samples,
                       residual_iters=args.residual_iters, residual_starts=args.residual_starts)
    if args.bench_config:
        cfg = VerifyConfig(sim_size=pre.sim_size, chunk=8192, node_budget=512, heuristic=not args.no_heuristic,
                           heuristic_p=pre.heuristic_p, heuristic_node_budget=512, escalate_budget=32768,
                           escalate_max_open=384, batch_nodes=65536, smt_backend="none", relu_budget=1024,
                           relu_max_width=16, relu_escalate_cap=2048,
                           escalate_probation=((2048, 768), (4096, 768), (8192, 768), (16384, 1024)))
    out = []
    for name in names:
        m = get_model(name, weights=args.weights, seed=0)
        be = Backend(m, device=dev)
        # warm (allocations, runtime construction)
        verify_chunk(be, m, q, grid, order[:256], cfg)
        if dev.type == "cuda":
            torch.cuda.synchronize()
        tm = StageTimer(dev, sync=True)
        t0 = time.time()
        recs = []
        for s in range(0, len(order), cfg.chunk):
            recs += verify_chunk(be, m, q, grid, order[s:s + cfg.chunk], cfg, timer=tm)
        if dev.type == "cuda":
            torch.cuda.synchronize()
        wall = time.time() - t0
        v = np.array([r["verdict"] for r in recs])
        st = np.array([r["stage"] for r in recs])
        nodes = np.array([r["nodes"] for r in recs])
        row = dict(model=name, widths=m.hidden, wall=round(wall, 3), n=len(recs),
                   sat=int((v == "sat").sum()), unsat=int((v == "unsat").sum()), unk=int((v == "unknown").sum()),
                   by_stage={k: int((st == k).sum()) for k in set(st.tolist())},
                   nodes_sum=int(nodes.sum()), nodes_p50=float(np.median(nodes)), nodes_p99=float(np.percentile(nodes, 99)),
                   nodes_max=int(nodes.max()), stages={k: round(t, 3) for k, t in tm.t.items()},
                   # where the node expansions go: by final verdict / stage, and past the first budget
                   nodes_by={f"{vv}/{ss}": int(nodes[(v == vv) & (st == ss)].sum())
                             for vv, ss in sorted(set(zip(v.tolist(), st.tolist())))},
                   nodes_over_first=int(np.maximum(nodes - cfg.node_budget, 0).sum()))
        if args.deep_budget:
            from fairify_amd.engine.bab import SAT, UNSAT, BaBConfig, BaBSolver

            unk = np.nonzero((v == "unknown") | (st == "heuristic"))[0]
            if unk.size:
                ids = order[unk]
                lo_np, hi_np = grid.decode(ids)
                t1 = time.time()
                res = BaBSolver(be, q, BaBConfig(node_budget=args.deep_budget)).solve(lo_np, hi_np, m)
                if dev.type == "cuda":
                    torch.cuda.synchronize()
                row["deep"] = dict(budget=args.deep_budget, n=int(unk.size), wall=round(time.time() - t1, 3),
                                   sat=int((res.status == SAT).sum()), unsat=int((res.status == UNSAT).sum()),
                                   unk=int(((res.status != SAT) & (res.status != UNSAT)).sum()),
                                   nodes_p50=float(np.median(res.nodes)),
                                   nodes_p90=float(np.percentile(res.nodes, 90)))
        out.append(row)
        print(json.dumps(row), flush=True)
    if args.json_out:
        with open(args.json_out, "w") as f:
            json.dump(out, f, indent=1)


if __name__ == "__main__":
    main()
