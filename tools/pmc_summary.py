#!/usr/bin/env python
"""Summarise rocprofv3 ``--pmc`` counter CSVs per kernel (sums over dispatches).

    python tools/pmc_summary.py gpurun_out/pmc2/p1/run_counter_collection.csv [...] > table.md
"""
from __future__ import annotations

import collections
import csv
import re
import sys


def short(name: str) -> str:
    name = name.replace("(anonymous namespace)::", "")
    name = re.sub(r"\(.*", "", name)
    return name.replace("void ", "")[:48]


def main(paths):
    tot = collections.defaultdict(lambda: collections.defaultdict(float))
    disp = collections.defaultdict(set)
    for p in paths:
        with open(p, newline="") as fh:
            for row in csv.DictReader(fh):
                k = short(row.get("Kernel_Name", "?"))
                tot[k][row["Counter_Name"]] += float(row["Counter_Value"])
                disp[k].add((p, row.get("Dispatch_Id", row.get("Correlation_Id", ""))))
    counters = sorted({c for v in tot.values() for c in v})
    keep = sorted(tot, key=lambda k: -max(tot[k].get("SQ_WAVE_CYCLES", 0), tot[k].get("SQ_BUSY_CYCLES", 0),
                                          tot[k].get("FETCH_SIZE", 0)))[:14]
    print("| kernel | dispatches | " + " | ".join(counters) + " |")
    print("|---|---|" + "---|" * len(counters))
    for k in keep:
        print(f"| {k} | {len(disp[k])} | " + " | ".join(f"{tot[k].get(c, 0):.4g}" for c in counters) + " |")
    print()
    print("Derived (per kernel): MFMA share of issued vector instructions, LDS bank-conflict cycles per")
    print("LDS instruction, VALU+MFMA instructions per wave.")
    print()
    print("| kernel | MFMA / (VALU+MFMA) | LDS conflict cyc / LDS inst | (VALU+MFMA) / wave |")
    print("|---|---|---|---|")
    for k in keep:
        t = tot[k]
        v, m, lds = t.get("SQ_INSTS_VALU", 0), t.get("SQ_INSTS_MFMA", 0), t.get("SQ_INSTS_LDS", 0)
        w = t.get("SQ_WAVES", 0)
        conf = t.get("SQ_LDS_BANK_CONFLICT", float("nan"))
        print(f"| {k} | {m / max(v + m, 1):.3f} | {conf / max(lds, 1):.3f} | {(v + m) / max(w, 1):.1f} |")


if __name__ == "__main__":
    main(sys.argv[1:])
