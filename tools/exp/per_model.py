#!/usr/bin/env python
"""Per-model bench A/B: one bench.py child per (model, env setting), JSON lines to stdout.

    python tools/exp/per_model.py --models AC-7,AC-11 --env REFINE=off --env REFINE=auto \
        -- --steps 2 --warmup 1 --budget-pass 0

Each child is a fresh process (no GPU state shared), under its own time limit.
"""
from __future__ import annotations

import argparse
import json
import os
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--models", default=",".join(f"AC-{i}" for i in range(1, 13)))
    ap.add_argument("--env", action="append", default=[],
                    help="VAR=VAL (repeatable; FAIRIFY_ prefix implied; '' = no override)")
    ap.add_argument("--timeout", type=int, default=240)
    ap.add_argument("rest", nargs=argparse.REMAINDER)
    a = ap.parse_args()
    rest = [x for x in a.rest if x != "--"]
    envs = a.env or [""]
    for m in a.models.split(","):
        for ev in envs:
            env = dict(os.environ)
            if ev:
                k, v = ev.split("=", 1)
                env[k if k.startswith("FAIRIFY") else "FAIRIFY_" + k] = v   # gpu.sh turns "_" into " "
            cmd = [sys.executable, "-u", os.path.join(ROOT, "bench.py"), "--models", m] + rest
            p = subprocess.run(cmd, env=env, capture_output=True, text=True, timeout=a.timeout)
            if p.returncode != 0:
                print(json.dumps({"model": m, "env": ev, "rc": p.returncode, "err": p.stderr[-2000:]}), flush=True)
                raise SystemExit(p.returncode)
            line = [ln for ln in p.stdout.splitlines() if ln.startswith("{")][-1]
            r = json.loads(line)
            print(json.dumps({"model": m, "env": ev, "ms_per_step": r["ms_per_step"], "unknown": r["unknown"],
                              "sat": r["sat"], "unsat_sound": r["unsat_sound"], "steps": r["steps"],
                              "pct_sound": r["pct_verified_sound"], "stages": p.stderr[-3000:] if "--profile" in rest
                              else None}), flush=True)


if __name__ == "__main__":
    main()
