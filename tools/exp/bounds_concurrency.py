#!/usr/bin/env python
"""be.bounds (symbolic + refine + backward logit pass: the beta stage's root bounds) from several host
threads with a stream each, against the same calls run serially: any difference is a cross-stream
hazard.  Also counts crossed (lb > ub) hidden bounds, which sound bounds of a box never have.

    python tools/exp/bounds_concurrency.py --model BM-4 --rows 2000 --threads 4 --reps 5
"""
from __future__ import annotations

import argparse
import os
import sys
from concurrent.futures import ThreadPoolExecutor

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--model", default="BM-4")
    ap.add_argument("--preset", default="relaxed/BM")
    ap.add_argument("--rows", type=int, default=2000)
    ap.add_argument("--threads", type=int, default=4)
    ap.add_argument("--reps", type=int, default=5)
    args = ap.parse_args()
    import torch

    from fairify_amd import presets
    from fairify_amd.models.zoo import get_model
    from fairify_amd.ops.backend import Backend
    from fairify_amd.partition import processing_order

    dev = torch.device("cuda")
    pre = presets.get(args.preset)
    grid = pre.grid()
    m = get_model(args.model, weights="zoo", seed=0)
    be = Backend(m, device=dev)
    ids = processing_order(grid, seed=0)[: args.rows * args.threads]
    lo_np, hi_np = grid.decode(ids)
    NH = be.n_hidden
    parts = [(torch.from_numpy(lo_np[k::args.threads].astype(np.float32)),
              torch.from_numpy(hi_np[k::args.threads].astype(np.float32))) for k in range(args.threads)]
    streams = [torch.cuda.Stream(dev) for _ in parts]

    def run(k):
        with torch.cuda.stream(streams[k]):
            lo, hi = parts[k][0].to(dev), parts[k][1].to(dev)
            res = be.bounds(lo, hi, mode="symbolic", keep_layers=True, crown=True, refine=True)
            lb = torch.cat([t.float() for t in res.layer_lb], 1)[:, :NH]
            ub = torch.cat([t.float() for t in res.layer_ub], 1)[:, :NH]
            out = (lb.cpu(), ub.cpu(), res.out_lb.cpu(), res.out_ub.cpu())
        return out

    serial = [run(k) for k in range(args.threads)]
    crossed = sum(int((s[0] > s[1]).any(1).sum()) for s in serial)
    print(f"{args.model}: {args.threads} x {parts[0][0].shape[0]} rows; serial crossed rows {crossed}", flush=True)
    for rep in range(args.reps):
        with ThreadPoolExecutor(args.threads) as ex:
            conc = list(ex.map(run, range(args.threads)))
        diff = [sum(int((a != b).any(1).sum()) if a.dim() > 1 else int((a != b).sum()) for a, b in zip(s, c))
                for s, c in zip(serial, conc)]
        cr = [int((c[0] > c[1]).any(1).sum()) for c in conc]
        print(f"rep {rep}: rows differing vs serial per thread {diff}, crossed {cr}", flush=True)


if __name__ == "__main__":
    main()
