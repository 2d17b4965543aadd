#!/bin/bash
set -eo pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out/diag512
timeout -k 10 300 python tools/diag_escalate.py --budget 512 --escalate 16384 --json-out gpurun_out/diag512/b512_e16384.json > gpurun_out/diag512/b512.log 2>&1
python - <<'PY'
import json
d = json.load(open("gpurun_out/diag512/b512_e16384.json"))
agg = {}
for r in d:
    for b in r["buckets"]:
        a = agg.setdefault(b["bucket"], [0, 0, 0])
        a[0] += b["n"]; a[1] += b["resolved"]; a[2] += b["nodes"]
    print(r["model"], "unknown@512", r["unknown"], "resolved@16384", r["resolved"], "nodes", r["nodes"])
for k, (n, res, nodes) in agg.items():
    print(k, n, res, nodes)
PY
