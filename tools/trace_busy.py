#!/usr/bin/env python
"""GPU busy fraction from a rocprofv3 kernel trace CSV: union of kernel intervals vs the
span, plus per-kernel totals.

    trace_busy.py trace.csv            span = first kernel start .. last kernel end
    trace_busy.py trace.csv --window   span = between the first and the last
                                       fa_trace_marker_kernel (bench.py launches one right
                                       before and one right after the timed steps), so
                                       start-up, warmup and the untimed budget pass are
                                       excluded
"""
import csv
import sys
from collections import defaultdict

MARK = "fa_trace_marker_kernel"
rows = list(csv.DictReader(open(sys.argv[1])))
iv = sorted((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), r["Kernel_Name"].replace("(anonymous namespace)::", ""))
            for r in rows)
window = "--window" in sys.argv[2:]
marks = [(s, e) for s, e, k in iv if k.startswith(MARK)]
if window:
    if len(marks) < 2:
        sys.exit("--window: fewer than two fa_trace_marker_kernel launches in the trace")
    w0, w1 = marks[0][1], marks[-1][0]
    iv = [(max(s, w0), min(e, w1), k) for s, e, k in iv if e > w0 and s < w1 and not k.startswith(MARK)]
    span = w1 - w0
else:
    span = iv[-1][1] - iv[0][0]
busy, cur_s, cur_e = 0, None, None
for s, e, _ in iv:
    if cur_e is None or s > cur_e:
        if cur_e is not None:
            busy += cur_e - cur_s
        cur_s, cur_e = s, e
    else:
        cur_e = max(cur_e, e)
if cur_e is not None:
    busy += cur_e - cur_s
tot = defaultdict(int)
cnt = defaultdict(int)
durs = defaultdict(list)
for s, e, k in iv:
    tot[k.split("(")[0][:48]] += e - s
    cnt[k.split("(")[0][:48]] += 1
    durs[k.split("(")[0][:48]].append(e - s)
what = "timed window" if window else "span"
print(f"{what} {span/1e9:.3f}s  busy(union) {busy/1e9:.3f}s  ({100*busy/max(1, span):.1f}%)  kernels {len(iv)}  "
      f"sum of kernel time {sum(tot.values())/1e9:.3f}s")
print(f"  {'kernel':50s} {'total':>9s}  {'launches':>7s}  {'p50 us':>8s}  {'p90 us':>8s}")
for k, v in sorted(tot.items(), key=lambda kv: -kv[1])[:14]:
    d = sorted(durs[k])
    p50, p90 = d[len(d) // 2] / 1e3, d[min(len(d) - 1, (9 * len(d)) // 10)] / 1e3
    print(f"  {k:50s} {v/1e9:8.3f}s  {cnt[k]:7d}  {p50:8.1f}  {p90:8.1f}")
