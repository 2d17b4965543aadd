#!/usr/bin/env python
"""Micro-benchmark of the BaB node certificate (fa_pair_eval + fa_pair_pick) on the device.

Builds N random BaB nodes inside partitions of the preset grid, computes their symbolic row
bounds once, then times ``Backend.pair_certify`` alone.

    python tools/certbench.py --models AC-4,AC-8 --nodes 32768
"""
from __future__ import annotations

import argparse
import json
import os
import sys

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--preset", default="src/AC-sex")
    ap.add_argument("--models", default="AC-4,AC-8")
    ap.add_argument("--nodes", type=int, default=32768)
    ap.add_argument("--iters", type=int, default=50)
    args = ap.parse_args()
    import torch

    from fairify_amd import presets
    from fairify_amd.engine.bab import _pa_table
    from fairify_amd.models.zoo import get_model
    from fairify_amd.ops.backend import Backend
    from fairify_amd.partition import processing_order

    dev = torch.device("cuda")
    pre = presets.get(args.preset)
    grid = pre.grid()
    q = pre.resolved()
    ids = processing_order(grid, seed=0)[:args.nodes]
    lo, hi = grid.decode(ids)
    rng = np.random.default_rng(0)
    # random sub-boxes (what the BaB frontier looks like a few levels down)
    a = lo + np.floor(rng.random(lo.shape) * (hi - lo + 1) * 0.5).astype(lo.dtype)
    b = np.minimum(hi, a + np.floor(rng.random(lo.shape) * (hi - lo + 1) * 0.6).astype(lo.dtype))
    values_np, pairs_np = _pa_table(q, lo, hi)
    values = torch.from_numpy(values_np).to(dev)
    pairs = torch.from_numpy(pairs_np).to(dev)
    pa = torch.tensor(list(q.pa_idx), device=dev)
    shared = torch.ones(q.n, dtype=torch.bool, device=dev)
    xlo = torch.from_numpy(a).to(dev, torch.float32)
    xhi = torch.from_numpy(b).to(dev, torch.float32)
    N, V = xlo.shape[0], values.shape[0]
    rlo = xlo[:, None, :].expand(N, V, q.n).clone()
    rhi = xhi[:, None, :].expand(N, V, q.n).clone()
    rlo[:, :, pa] = values.float()[None]
    rhi[:, :, pa] = values.float()[None]
    out = []
    for name in args.models.split(","):
        m = get_model(name, weights="random", seed=0)
        be = Backend(m, device=dev)
        res = be.bounds(rlo.reshape(-1, q.n), rhi.reshape(-1, q.n), mode="symbolic", fold=tuple(q.pa_idx))
        dec = be.pair_certify(res, res, xlo, xhi, xlo, xhi, pairs, values, pa, shared, False)
        torch.cuda.synchronize()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        for _ in range(args.iters):
            dec = be.pair_certify(res, res, xlo, xhi, xlo, xhi, pairs, values, pa, shared, False)
        e1.record()
        torch.cuda.synchronize()
        us = 1000.0 * e0.elapsed_time(e1) / args.iters
        row = dict(model=name, nodes=N, us_per_call=round(us, 1), open=int(dec.open_.sum()),
                   score_sum=float(dec.score.double().sum()))
        out.append(row)
        print(json.dumps(row), flush=True)


if __name__ == "__main__":
    main()
