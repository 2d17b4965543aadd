"""Per-model decided counts of the bench configuration on a fixed slice of the AC grid.

The GPU tests check every bound kernel for SOUNDNESS (bounds enclose the exact values); a
change can keep them green and still loosen the bounds enough to lose verdicts (the reverted
centre/radius GEMM of round 2: 95.09 % -> 88.80 % on the bench, profiles/r2/s4/README.md).
``tests/test_tightness_gpu.py`` therefore compares today's decided counts against the pins this
script writes (``tests/data/tightness_ac_sex.json``).

    python tools/pin_tightness.py [--n 1024] [--out tests/data/tightness_ac_sex.json]
"""
from __future__ import annotations

import argparse
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
if ROOT not in sys.path:
    sys.path.insert(0, ROOT)

PIN_PATH = os.path.join(ROOT, "tests", "data", "tightness_ac_sex.json")


def decided_counts(n: int, device: str = "cuda:0", models=None) -> dict:
    """{model: {"attempted", "sat", "unsat_sound", "unknown"}} for the first ``n`` partitions of
    the bench order (seed 0, random-init weights), with bench.py's default configuration minus
    the heuristic retry (its UNSAT is unsound by design and not a bound-tightness signal)."""
    import numpy as np
    import torch

    from fairify_amd import presets
    from fairify_amd.engine.pipeline import VerifyConfig, verify_chunk
    from fairify_amd.models.zoo import get_model
    from fairify_amd.ops.backend import Backend
    from fairify_amd.partition import processing_order

    pre = presets.get("src/AC-sex")
    grid, q = pre.grid(), pre.resolved()
    ids = processing_order(grid, seed=0)[:n]
    cfg = VerifyConfig(sim_size=pre.sim_size, seed=0, chunk=4096, soft_timeout=pre.soft_timeout,
                       hard_timeout=pre.hard_timeout, node_budget=512, heuristic=False,
                       escalate_budget=8192, escalate_max_open=384, batch_nodes=65536, smt_backend="none")
    dev = torch.device(device)
    out = {}
    for name in models or pre.models:
        m = get_model(name, weights="random", seed=0)
        be = Backend(m, device=dev)
        if dev.type == "cuda" and not be.hip:
            raise RuntimeError("HIP extension inactive on a GPU run")
        recs = verify_chunk(be, m, q, grid, np.asarray(ids), cfg)
        if dev.type == "cuda":
            torch.cuda.synchronize(dev)
        v = recs.cols["verdict"]
        out[name] = {"attempted": int(len(v)), "sat": int((v == "sat").sum()),
                     "unsat_sound": int((v == "unsat").sum()), "unknown": int((v == "unknown").sum())}
    return out


def main() -> None:
    ap = argparse.ArgumentParser()
    ap.add_argument("--n", type=int, default=1024)
    ap.add_argument("--out", default=PIN_PATH)
    args = ap.parse_args()
    res = decided_counts(args.n)
    doc = {"preset": "src/AC-sex", "weights": "random", "seed": 0, "n": args.n, "heuristic": False,
           "models": res}
    os.makedirs(os.path.dirname(args.out), exist_ok=True)
    with open(args.out, "w") as f:
        json.dump(doc, f, indent=1, sort_keys=True)
    print("PINS " + json.dumps(doc, sort_keys=True), flush=True)   # one line: gpu.sh keeps stdout


if __name__ == "__main__":
    main()
