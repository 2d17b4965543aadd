#!/usr/bin/env python
"""Summarise a rocprofv3 ``--stats`` kernel_stats.csv as markdown (for profiles/).

    python tools/prof_summary.py gpurun_out/X/prof3/run_kernel_stats.csv --title "..." [--top 25] > profiles/Y.md

Groups dispatches by origin (our HIP kernels ``fa_*``, PyTorch ``at::native``, HIP runtime blits,
other library kernels) and lists the top kernels by total duration.
"""
from __future__ import annotations

import argparse
import csv
import re


def origin(name: str) -> str:
    if re.search(r"\bfa_\w+", name):
        return "fairify HIP kernels (fa_*)"
    if "at::native" in name or "at::" in name:
        return "PyTorch elementwise/reduce (at::native)"
    if "__amd_rocclr" in name:
        return "HIP runtime copy/fill blits"
    return "other library kernels (rocprim, ...)"


def short(name: str, width: int = 72) -> str:
    name = name.replace("|", "\\|")
    return name if len(name) <= width else name[:width - 3] + "..."


def main() -> None:
    ap = argparse.ArgumentParser()
    ap.add_argument("csv")
    ap.add_argument("--title", default="rocprofv3 kernel stats")
    ap.add_argument("--top", type=int, default=25)
    ap.add_argument("--note", default="")
    a = ap.parse_args()
    rows = []
    with open(a.csv) as f:
        for r in csv.DictReader(f):
            rows.append((r["Name"], int(r["Calls"]), int(r["TotalDurationNs"]), float(r["AverageNs"])))
    tot_calls = sum(r[1] for r in rows)
    tot_ns = sum(r[2] for r in rows)
    print(f"# {a.title}\n")
    if a.note:
        print(a.note + "\n")
    print(f"Dispatches: **{tot_calls}**; sum of kernel durations {tot_ns / 1e9:.3f} s.\n")
    groups = {}
    for name, calls, ns, _ in rows:
        g = groups.setdefault(origin(name), [0, 0])
        g[0] += calls
        g[1] += ns
    print("| origin | dispatches | share of dispatches | kernel s | share of kernel time |")
    print("|---|---:|---:|---:|---:|")
    for g, (c, ns) in sorted(groups.items(), key=lambda kv: -kv[1][1]):
        print(f"| {g} | {c} | {100.0 * c / max(1, tot_calls):.1f} % | {ns / 1e9:.3f} | {100.0 * ns / max(1, tot_ns):.1f} % |")
    print(f"\n| kernel | calls | total ms | avg us | share |")
    print("|---|---:|---:|---:|---:|")
    for name, calls, ns, avg in sorted(rows, key=lambda r: -r[2])[:a.top]:
        print(f"| `{short(name)}` | {calls} | {ns / 1e6:.1f} | {avg / 1e3:.1f} | {100.0 * ns / max(1, tot_ns):.2f} % |")


if __name__ == "__main__":
    main()
