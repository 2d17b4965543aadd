#!/usr/bin/env python
"""Micro-benchmark of the backward (CROWN) bound kernel in isolation, one process per variant:

    python tools/bench_crown.py --models AC-1,AC-4,AC-7 --rows 131072            # MFMA variant
    FAIRIFY_CROWN_MFMA=0 python tools/bench_crown.py ...                        # scalar variant

Forward symbolic bounds (forms + per-layer bounds) are computed once per model on R random
boxes of the preset's domain (PA dims set, as in the BaB node rows); the crown launch is then
timed alone (it refines the forms in place, so repeated launches redo the same work).
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
    ap.add_argument("--models", default="AC-1,AC-4,AC-7,AC-11")
    ap.add_argument("--rows", type=int, default=131072)
    ap.add_argument("--iters", type=int, default=20)
    args = ap.parse_args()
    import torch

    from fairify_amd import presets
    from fairify_amd.models.zoo import get_model
    from fairify_amd.ops import hip
    from fairify_amd.ops.backend import Backend

    dev = torch.device("cuda")
    pre = presets.get(args.preset)
    dom = pre.domain()
    g = np.random.default_rng(0)
    lo0, hi0 = dom.lo(), dom.hi()
    R = args.rows
    lo = g.integers(lo0, hi0 + 1, size=(R, dom.n))
    hi = np.minimum(lo + g.integers(0, 10, size=(R, dom.n)), hi0)
    lo_t = torch.from_numpy(lo).float().to(dev)
    hi_t = torch.from_numpy(hi).float().to(dev)
    variant = "scalar" if os.environ.get("FAIRIFY_CROWN_MFMA") == "0" else "mfma"
    for name in args.models.split(","):
        m = get_model(name, weights="random", seed=0)
        be = Backend(m, device=dev)
        res = be.bounds(lo_t, hi_t, mode="symbolic", keep_layers=True)
        hip.crown(be, lo_t, hi_t, res)
        torch.cuda.synchronize()
        t0 = time.time()
        for _ in range(args.iters):
            hip.crown(be, lo_t, hi_t, res)
        torch.cuda.synchronize()
        dt = (time.time() - t0) / args.iters
        print(json.dumps({"variant": variant, "model": name, "rows": R, "ms": round(1000 * dt, 3),
                          "rows_per_s": round(R / dt, 1)}), flush=True)


if __name__ == "__main__":
    main()
