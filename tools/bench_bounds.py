#!/usr/bin/env python
"""Micro-benchmark of the fused bound-propagation kernel (K2/K4) per zoo architecture.

Times ``Backend.bounds`` on R random boxes of the preset's domain and reports rows/s and the
achieved GEMM rate.  FLOPs counted are those of the layer GEMMs as formulated
(out_U = [U|L].[W+;W-]): 2 * (2*rb rows per box) * (2*n_in) * n_out per layer, rb = n0+4 for the
symbolic mode and 2 for IBP.

    python tools/bench_bounds.py --models AC-1,AC-4,AC-11 --rows 65536 --mode symbolic
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def gemm_flops(dims, rows, symbolic):
    n0 = dims[0]
    rb = n0 + 4 if symbolic else 2
    f = 0
    for l in range(len(dims) - 1):
        f += 2 * (2 * rb) * (2 * dims[l]) * dims[l + 1]
    return f * rows


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--preset", default="src/AC-sex")
    ap.add_argument("--models", default=None)
    ap.add_argument("--rows", type=int, default=65536)
    ap.add_argument("--mode", default="symbolic")
    ap.add_argument("--iters", type=int, default=20)
    ap.add_argument("--json-out", default=None)
    ap.add_argument("--no-fold", action="store_true", help="do not fix/fold the protected attribute")
    args = ap.parse_args()
    import torch

    from fairify_amd import presets
    from fairify_amd.models.zoo import get_model
    from fairify_amd.ops.backend import Backend

    dev = torch.device("cuda")
    pre = presets.get(args.preset)
    dom = pre.domain()
    lo_d = dom.lo().astype(np.float32)
    hi_d = dom.hi().astype(np.float32)
    rng = np.random.default_rng(0)
    a = rng.uniform(lo_d, hi_d, size=(args.rows, len(lo_d)))
    b = rng.uniform(lo_d, hi_d, size=(args.rows, len(lo_d)))
    lo_n = np.floor(np.minimum(a, b)).astype(np.float32)
    hi_n = np.ceil(np.maximum(a, b)).astype(np.float32)
    fold = () if args.no_fold else tuple(pre.resolved().pa_idx)
    for d in fold:      # BaB node rows: the protected attribute is fixed per row
        hi_n[:, d] = lo_n[:, d]
    lo = torch.from_numpy(lo_n).to(dev)
    hi = torch.from_numpy(hi_n).to(dev)
    out = []
    for name in (args.models.split(",") if args.models else list(pre.models)):
        m = get_model(name, weights="random", seed=0)
        be = Backend(m, device=dev)
        def run():
            if args.mode == "points":
                be.point_bounds(lo)
            else:
                be.bounds(lo, hi, mode=args.mode, fold=fold)

        for _ in range(3):
            run()
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for _ in range(args.iters):
            run()
        torch.cuda.synchronize()
        dt = (time.perf_counter() - t0) / args.iters
        dims = [m.n_in] + m.widths
        fl = gemm_flops(dims, args.rows, args.mode == "symbolic") if args.mode != "points" else \
            sum(2 * 2 * dims[l] * dims[l + 1] for l in range(len(dims) - 1)) * args.rows
        row = dict(model=name, dims=dims, rows=args.rows, mode=args.mode, ms=round(dt * 1e3, 4),
                   mrows_per_s=round(args.rows / dt / 1e6, 3), gemm_tflops=round(fl / dt / 1e12, 2))
        out.append(row)
        print(json.dumps(row), flush=True)
    if args.json_out:
        with open(args.json_out, "w") as f:
            json.dump(out, f, indent=1)


if __name__ == "__main__":
    main()
