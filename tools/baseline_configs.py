#!/usr/bin/env python
"""One-HEAD re-measurement of every BASELINE.json config, sound verdicts only.

    python tools/baseline_configs.py --group tablev  --out gpurun_out/r4/base --head <sha>
    python tools/baseline_configs.py --group stress  --out ...
    python tools/baseline_configs.py --group relaxed --out ...
    python tools/baseline_configs.py --group targeted --out ...
    python tools/baseline_configs.py --report gpurun_out/r4/base > profiles/r4/baseline_configs.md

Groups (BASELINE.json ``configs``; reference constants per SURVEY §2.5):

* ``tablev``   -- Table V of the paper with the reference's TRAINED weights: src/AC-sex, src/AC-race,
                  src/BM-age, src/GC-sex, src/GC-age, every model, anytime mode (the reference spends up
                  to its hard timeout per model, src/AC/Verify-AC.py:318-320; here ``--anytime-budget``
                  seconds per model);
* ``stress``   -- stress/AC, stress/BM, stress/GC full grids (3.29 M / 1.0 M / 18 009 partitions);
* ``relaxed``  -- relaxed/AC, relaxed/BM, relaxed/GC (|x_r - x'_r| <= tau, x' unclipped);
* ``targeted`` -- targeted/* and targeted2/* (domain overrides).

Every preset runs every model of the preset (trained weights where the zoo has them, else the
preset's random-init shape), with the heuristic retry OFF: every UNSAT is a proof and every SAT an
exactly confirmed pair.  Each run writes ``<out>/<preset>/summary.json`` (per-model Table-V rows
with ``Cov_sound%``, ``UNSAT_heuristic``, wall time) and the HEAD sha; the
report turns all of them into one markdown table.
"""
from __future__ import annotations

import argparse
import glob
import json
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

GROUPS = {
    "tablev": ["src/AC-sex", "src/AC-race", "src/BM-age", "src/GC-sex", "src/GC-age"],
    "stress": ["stress/AC", "stress/BM", "stress/GC"],
    "relaxed": ["relaxed/AC", "relaxed/BM", "relaxed/GC"],
    "targeted": ["targeted/AC", "targeted/BM", "targeted/GC", "targeted2/AC", "targeted2/BM", "targeted2/GC"],
}


def run_group(args) -> None:
    import torch

    from fairify_amd import presets
    from fairify_amd.engine.pipeline import VerifyConfig
    from fairify_amd.engine.runner import run_preset
    from fairify_amd.models.zoo import has_weights
    from fairify_amd.parallel import dist as D

    info = D.init("cuda" if torch.cuda.device_count() else "cpu")
    names = GROUPS[args.group] if args.group in GROUPS else args.group.split(",")
    # heartbeat: a stress model (3.29 M partitions) runs for minutes without a per-model line, and a
    # silent GPU command is taken to be hung
    import threading

    cur = {"what": "start", "t": time.time()}

    def beat():
        while True:
            time.sleep(60)
            print(f"[hb] {cur['what']} {time.time() - cur['t']:.0f}s", flush=True)

    threading.Thread(target=beat, daemon=True).start()
    for name in names:
        pre = presets.get(name)
        models = list(pre.models) if not args.models else args.models.split(",")
        # one directory per (preset, model subset, part): calls of one group never overwrite each other
        sub = ("@" + args.models.replace(",", "+")) if args.models else ""
        part = f"@{args.start}" if (args.start or args.max_partitions) else ""
        out = os.path.join(args.out, name.replace("/", "_") + sub + part)
        os.makedirs(out, exist_ok=True)
        # per-partition CSVs (MBs per model) go to scratch: gpurun copies back <= 64 MiB of gpurun_out
        scratch = os.path.join(args.scratch, name.replace("/", "_"))
        anytime = args.anytime_budget if (args.group == "tablev" or args.anytime_budget > 0 and args.all_anytime) else 0
        # the large grids (stress / relaxed / targeted: 0.2-3.3 M partitions per model) run the GPU
        # stages only (--smt none) with a shorter escalation; Table V adds the host LP (anytime)
        big = args.group != "tablev" and not args.all_anytime
        cfg = VerifyConfig(sim_size=pre.sim_size, soft_timeout=pre.soft_timeout, hard_timeout=pre.hard_timeout,
                           heuristic=False, heuristic_p=pre.heuristic_p, node_budget=512,
                           escalate_budget=8192 if big else 32768, escalate_max_open=384,
                           escalate_probation=((2048, 768), (4096, 768)) if big else
                           ((2048, 768), (4096, 768), (8192, 768), (16384, 1024)),
                           relu_budget=1024, relu_escalate_cap=2048, smt_backend=args.smt or ("none" if big else "auto"),
                           chunk=8192)
        if args.cfg:      # A/B overrides of VerifyConfig fields: --cfg key=value,key=value
            from dataclasses import replace as _rp

            kv = {}
            for item in filter(None, args.cfg.split(",")):
                k, v = item.split("=")
                kv[k] = type(getattr(cfg, k))(v)
            cfg = _rp(cfg, **kv)
        t0 = time.time()
        weights = {m: ("zoo" if has_weights(m) else "random") for m in models}
        rows = []
        for m in models:
            cur["what"], cur["t"] = f"{name} {m}", time.time()
            r = run_preset(pre, models=[m], weights=weights[m], out_dir=os.path.join(scratch, m), cfg=cfg, info=info,
                           seed=0, accuracy=False, verbose=False, concurrency=4,
                           anytime_budget=anytime or None, max_partitions=args.max_partitions,
                           start_partition=args.start)
            for row in r:
                row["weights"] = weights[m]
                rows.append(row)
                print(f"[{name}] {m} ({weights[m]}): {row['SAT']} sat / {row['UNSAT']} unsat / {row['UNK']} unk "
                      f"of {row['#P']}, Cov_sound {row.get('Cov_sound%')} %, {row.get('wall_s')} s",
                      flush=True)
            # after every model: a run cut by its time limit keeps the finished models
            with open(os.path.join(out, "summary.json"), "w") as f:
                json.dump({"preset": name, "models": rows, "head": args.head, "wall_s": round(time.time() - t0, 2),
                           "start": args.start, "max_partitions": args.max_partitions,
                           "anytime_budget_s": anytime, "heuristic": False, "smt": cfg.smt_backend,
                           "escalate_budget": cfg.escalate_budget}, f, indent=2)
        print(f"[{name}] done in {time.time() - t0:.1f}s", flush=True)
    D.destroy(info)


def report(root: str) -> None:
    rows = []
    heads = set()
    parts = {}
    for path in sorted(glob.glob(os.path.join(root, "*", "summary.json"))):
        s = json.load(open(path))
        heads.add(s.get("head"))
        for r in s["models"]:
            if s.get("start") or s.get("max_partitions"):
                # one part of a model's grid (--start / --max-partitions): counts and walls add up
                key = (s["preset"], r["model"])
                if key not in parts:
                    parts[key] = (s["preset"], s.get("anytime_budget_s", 0), dict(r), [s.get("start", 0)])
                    continue
                m = parts[key][2]
                for k in ("SAT", "UNSAT", "UNK", "UNSAT_heuristic", "UNSAT_sound", "#P"):
                    if k in r:
                        m[k] = m.get(k, 0) + r[k]
                m["wall_s"] = round(float(m.get("wall_s", 0)) + float(r.get("wall_s", 0)), 3)
                parts[key][3].append(s.get("start", 0))
                continue
            rows.append((s["preset"], s.get("anytime_budget_s", 0), r))
    for pre_, any_s, m, starts in parts.values():
        sat_h = 0
        m["Cov_sound%"] = round(100.0 * (m["SAT"] + m.get("UNSAT_sound", m["UNSAT"]) - sat_h) / max(1, m["Grid"]), 2)
        m["partitions_per_s"] = round(m.get("#P", m["SAT"] + m["UNSAT"] + m["UNK"]) / max(1e-9, m["wall_s"]), 3)
        m["parts"] = len(starts)
        rows.append((pre_, any_s, m))
    print(f"# BASELINE configs at one HEAD ({', '.join(sorted(h or '?' for h in heads))}), sound verdicts only\n")
    print("`tools/baseline_configs.py` on 1x MI355X; heuristic retry off (every UNSAT a proof, every SAT an exactly "
          "confirmed pair).  Cov_sound% = (SAT + sound UNSAT) / grid.\n")
    print("| preset | model | weights | grid | SAT | UNSAT | UNK | Cov_sound % | UNSAT_heuristic | anytime s | wall s | "
          "partitions/s |")
    print("|---|---|---|---|---|---|---|---|---|---|---|---|")
    tot = {}
    for preset, any_s, r in rows:
        mname = r['model'] + (f" ({r['parts']} parts)" if r.get("parts", 1) > 1 else "")
        print(f"| {preset} | {mname} | {r.get('weights', '?')} | {r['Grid']} | {r['SAT']} | {r['UNSAT']} | "
              f"{r['UNK']} | {r.get('Cov_sound%')} | {r.get('UNSAT_heuristic', 0)} | {any_s or '-'} | "
              f"{r.get('wall_s', '?')} | {r.get('partitions_per_s', '?')} |")
        t = tot.setdefault(preset, [0, 0, 0, 0.0])
        t[0] += r["Grid"]
        t[1] += r["SAT"] + r.get("UNSAT_sound", r["UNSAT"])
        t[2] += r.get("UNSAT_heuristic", 0)
        t[3] += float(r.get("wall_s", 0) or 0)
    print("\n| preset | grid (all models) | sound decided | Cov_sound % | UNSAT_heuristic | wall s |")
    print("|---|---|---|---|---|---|")
    for preset, (g, d, h, w) in tot.items():
        print(f"| {preset} | {g} | {d} | {100.0 * d / max(1, g):.3f} | {h} | {w:.1f} |")


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--group", default=None)
    ap.add_argument("--models", default=None)
    ap.add_argument("--out", default=os.environ.get("FAIRIFY_BASE_OUT", "gpurun_out/base"))
    ap.add_argument("--head", default=os.environ.get("FAIRIFY_HEAD", ""))
    ap.add_argument("--anytime-budget", type=float, default=120.0, help="tablev: seconds per model")
    ap.add_argument("--all-anytime", action="store_true", help="anytime mode for the other groups too")
    ap.add_argument("--max-partitions", type=int, default=None, help="CPU rehearsal: first N of each grid")
    ap.add_argument("--report", default=None)
    ap.add_argument("--cfg", default="", help="VerifyConfig overrides 'key=value,...' (A/B runs)")
    ap.add_argument("--start", type=int, default=0,
                    help="first position of the seeded order (with --max-partitions: one part of a model's grid; "
                         "the report adds the parts of a (preset, model) up)")
    ap.add_argument("--smt", default=None, help="host back-end (default: auto for tablev, none for the big grids)")
    ap.add_argument("--scratch", default=os.path.join(os.environ.get("TMPDIR", "/tmp"), "fairify_base"),
                    help="per-partition CSVs (not copied back)")
    args = ap.parse_args()
    if args.report:
        report(args.report)
    else:
        run_group(args)


if __name__ == "__main__":
    main()
