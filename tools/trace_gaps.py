#!/usr/bin/env python
"""Idle gaps of the GPU inside the timed window of a rocprofv3 trace and what the host threads
were doing during them.

    trace_gaps.py KERNEL_TRACE.csv [HIP_API_TRACE.csv] [--min-ms 3]

For every gap (no kernel running anywhere) longer than --min-ms between the two
fa_trace_marker_kernel launches bench.py brackets the timed steps with: its position, the last
kernel before and the first after it, and -- with the HIP API trace -- every API call that
overlaps the gap by more than 10 % of it (name, thread, duration).  A call that spans the gap on
one thread while the others are idle is the stall.
"""
import csv
import sys
from collections import defaultdict

args = [a for a in sys.argv[1:] if not a.startswith("--")]
min_ms = float(sys.argv[sys.argv.index("--min-ms") + 1]) if "--min-ms" in sys.argv else 3.0
if "--min-ms" in sys.argv:
    args.remove(sys.argv[sys.argv.index("--min-ms") + 1])
rows = list(csv.DictReader(open(args[0])))
iv = sorted((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), r["Kernel_Name"]) for r in rows)
marks = [(s, e) for s, e, k in iv if k.startswith("fa_trace_marker_kernel")]
w0, w1 = (marks[0][1], marks[-1][0]) if len(marks) >= 2 else (iv[0][0], iv[-1][1])
api = []
if len(args) > 1:
    for r in csv.DictReader(open(args[1])):
        api.append((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), r.get("Function", r.get("Operation", "?")),
                    r.get("Thread_Id", "?")))
gaps = []
end = None
for s, e, k in iv:
    if e <= w0 or s >= w1 or k.startswith("fa_trace_marker_kernel"):
        continue
    if end is not None and s - end > min_ms * 1e6:
        gaps.append((end, s))
    end = e if end is None else max(end, e)
print(f"window {(w1 - w0) / 1e6:.1f} ms, {len(gaps)} gaps > {min_ms} ms, total "
      f"{sum(b - a for a, b in gaps) / 1e6:.1f} ms")
for a, b in gaps:
    print(f"gap {(b - a) / 1e6:.1f} ms at +{(a - w0) / 1e6:.1f} ms")
    tot = defaultdict(float)
    for s, e, f, t in api:
        ov = min(e, b) - max(s, a)
        if ov > 0.1 * (b - a):
            print(f"    {f:40s} tid {t:>8s} {(e - s) / 1e6:9.2f} ms  (overlap {ov / 1e6:.2f})")

# launch -> start delay per kernel (queueing behind other streams' work on the shared hardware
# queues + dispatch), from the Correlation_Id shared by the API call and the dispatch
if len(args) > 1:
    import numpy as np

    launch = {}
    for r in csv.DictReader(open(args[1])):
        if "Launch" in r.get("Function", ""):
            launch[r["Correlation_Id"]] = (int(r["End_Timestamp"]), r["Thread_Id"])
    d = []
    for r in rows:
        c = r["Correlation_Id"]
        s = int(r["Start_Timestamp"])
        if c in launch and w0 < s < w1:
            d.append(s - launch[c][0])
    if d:
        d = np.array(d) / 1e3
        print(f"launch->start delay (us) over {len(d)} kernels in the window: p10/50/90/99 "
              f"{np.percentile(d, [10, 50, 90, 99]).round(1).tolist()}  sum {d.sum() / 1e3:.1f} ms")
    # host-side time per thread inside the window by API function (where the threads wait)
    per = defaultdict(float)
    for s, e, f, t in api:
        if e > w0 and s < w1:
            per[f] += (min(e, w1) - max(s, w0)) / 1e6
    print("API time in the window, summed over threads (ms):")
    for f, v in sorted(per.items(), key=lambda x: -x[1])[:15]:
        print(f"    {f:40s} {v:9.1f}")
