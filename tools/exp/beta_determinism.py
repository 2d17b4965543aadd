#!/usr/bin/env python
"""Run the fixed beta pass (engine/pipeline.py:_beta_round) repeatedly on one residue set and compare
verdicts and node counts run to run, under toggles (native loop / torch loop, forced weight placement,
no tightening), to find where run-to-run differences come from.

    python tools/exp/beta_determinism.py --preset relaxed/BM --model BM-4 --limit 40000
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
    ap.add_argument("--preset", default="relaxed/BM")
    ap.add_argument("--model", default="BM-4")
    ap.add_argument("--limit", type=int, default=40000)
    ap.add_argument("--settings", default="nat,nat,nat,wm0,wm0,torch,torch")
    ap.add_argument("--threads", type=int, default=0,
                    help="> 0: also run the residue split in this many parts, serially and then concurrently "
                         "from host threads with a stream each (the runner's workers), and compare")
    args = ap.parse_args()
    import torch
    from dataclasses import replace

    from fairify_amd import presets
    from fairify_amd.engine.bab import UNKNOWN
    from fairify_amd.engine.pipeline import VerifyConfig, _beta_round, verify_chunk
    from fairify_amd.models.zoo import get_model
    from fairify_amd.ops.backend import Backend
    from fairify_amd.partition import processing_order

    dev = torch.device("cuda")
    pre = presets.get(args.preset)
    grid, q = pre.grid(), pre.resolved()
    ids = processing_order(grid, seed=0)[:args.limit]
    cfg = VerifyConfig(sim_size=pre.sim_size, chunk=8192, soft_timeout=pre.soft_timeout, hard_timeout=pre.hard_timeout,
                       node_budget=512, heuristic=False, heuristic_p=pre.heuristic_p, escalate_budget=8192,
                       escalate_max_open=384, smt_backend="none", escalate_probation=((2048, 768), (4096, 768)),
                       relu_budget=1024, relu_escalate_cap=2048)
    m = get_model(args.model, weights="zoo", seed=0)
    be = Backend(m, device=dev)
    t0 = time.time()
    recs = verify_chunk(be, m, q, grid, ids, replace(cfg, beta_budget=0))
    v = recs.cols["verdict"]
    unk = np.asarray(recs.cols["grid_id"])[v == "unknown"]
    lo_np, hi_np = grid.decode(unk)
    P = unk.size
    print(f"{args.model}: {ids.size} partitions, residue {P} ({time.time() - t0:.1f}s)", flush=True)
    ref = None
    for name in args.settings.split(","):
        env = {"nat": {}, "wm0": {"FAIRIFY_BETA_WM": "0"}, "wm2": {"FAIRIFY_BETA_WM": "2"},
               "torch": {"FAIRIFY_TORCH_BETA": "1"}}[name.split("_")[0]]
        old = {k: os.environ.get(k) for k in env}
        os.environ.update(env)
        status = np.full(P, UNKNOWN, dtype=np.int8)
        stage = np.empty(P, dtype=object)
        cx = np.zeros((P, lo_np.shape[1]), np.int64)
        cxp = np.zeros_like(cx)
        nodes = np.zeros(P, np.int64)
        t1 = time.time()
        _beta_round(be, q, m, np.arange(P), lo_np, hi_np, cfg.beta_budget, 1e9, cfg.batch_nodes, status, stage, cx, cxp,
                    nodes, probe_levels=cfg.beta_probe_levels, cfg=cfg)
        torch.cuda.synchronize()
        for k, x in old.items():
            if x is None:
                os.environ.pop(k, None)
            else:
                os.environ[k] = x
        dec = int((status != UNKNOWN).sum())
        line = f"{name:8s} decided {dec:5d} (sat {int((status == 1).sum())}) nodes {int(nodes.sum()):8d} {time.time() - t1:5.2f}s"
        if ref is None:
            ref = (status.copy(), nodes.copy())
        else:
            line += f"  vs first: status differs on {int((status != ref[0]).sum())}, nodes on {int((nodes != ref[1]).sum())}"
        print(line, flush=True)
    if args.threads > 0:
        from concurrent.futures import ThreadPoolExecutor

        parts = np.array_split(np.arange(P), args.threads)
        streams = [torch.cuda.Stream(dev) for _ in parts]

        def run(k):
            idx = parts[k]
            with torch.cuda.stream(streams[k]):
                st = np.full(idx.size, UNKNOWN, dtype=np.int8)
                nd = np.zeros(idx.size, np.int64)
                cx = np.zeros((idx.size, lo_np.shape[1]), np.int64)
                _beta_round(be, q, m, np.arange(idx.size), lo_np[idx], hi_np[idx], cfg.beta_budget, 1e9,
                            cfg.batch_nodes, st, np.empty(idx.size, dtype=object), cx, cx.copy(), nd,
                            probe_levels=cfg.beta_probe_levels, cfg=cfg)
                torch.cuda.current_stream().synchronize()
            return st, nd

        serial = [run(k) for k in range(len(parts))]
        for rep in range(3):
            with ThreadPoolExecutor(len(parts)) as ex:
                conc = list(ex.map(run, range(len(parts))))
            diff = [(int((a[0] != b[0]).sum()), int((a[1] != b[1]).sum())) for a, b in zip(serial, conc)]
            dec = [int((c[0] != UNKNOWN).sum()) for c in conc]
            print(f"concurrent rep {rep}: decided per part {dec} (serial {[int((s_[0] != UNKNOWN).sum()) for s_ in serial]}),"
                  f" (status, nodes) differing vs serial {diff}", flush=True)


if __name__ == "__main__":
    main()
