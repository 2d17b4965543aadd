#!/usr/bin/env python
"""Aggregate every ``summary.json`` under a results root into one Table-V style markdown table
(the paper's aggregation was done offline)."""
import glob
import json
import os
import sys


def main(root: str) -> None:
    rows = []
    for path in sorted(glob.glob(os.path.join(root, "**", "summary.json"), recursive=True)):
        s = json.load(open(path))
        for r in s.get("models", []):
            rows.append((s.get("preset", os.path.dirname(path)), r))
    cols = ["model", "PA", "Ver", "#P", "Grid", "Cov%", "SAT", "UNSAT", "UNK", "#H", "#HS", "C(S)", "C(H)",
            "SV", "HV", "Total", "partitions_per_s"]
    print("| preset | " + " | ".join(cols) + " |")
    print("|---" * (len(cols) + 1) + "|")
    for preset, r in rows:
        print(f"| {preset} | " + " | ".join(str(r.get(c, "")) for c in cols) + " |")


if __name__ == "__main__":
    main(sys.argv[1] if len(sys.argv) > 1 else "results")
