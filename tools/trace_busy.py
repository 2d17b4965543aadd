#!/usr/bin/env python
"""GPU busy fraction from a rocprofv3 kernel trace CSV: union of kernel intervals vs the
span from first start to last end, plus per-kernel totals.  Usage: trace_busy.py trace.csv"""
import csv
import sys
from collections import defaultdict

rows = list(csv.DictReader(open(sys.argv[1])))
iv = sorted((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), r["Kernel_Name"]) for r in rows)
busy, cur_s, cur_e = 0, None, None
for s, e, _ in iv:
    if cur_e is None or s > cur_e:
        if cur_e is not None:
            busy += cur_e - cur_s
        cur_s, cur_e = s, e
    else:
        cur_e = max(cur_e, e)
busy += cur_e - cur_s
span = iv[-1][1] - iv[0][0]
tot = defaultdict(int)
for s, e, k in iv:
    tot[k.split("(")[0][:48]] += e - s
print(f"span {span/1e9:.3f}s  busy(union) {busy/1e9:.3f}s  ({100*busy/span:.1f}%)  kernels {len(iv)}")
for k, v in sorted(tot.items(), key=lambda kv: -kv[1])[:12]:
    print(f"  {k:50s} {v/1e9:8.3f}s")
