#!/bin/bash
# Table V (src/AC-sex, trained weights) with escalation schedules through the CLI runner.
set -eo pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out/tvs
for spec in "4096|0|0" "512|16384|256" "1024|32768|512"; do
  IFS='|' read nb eb eo <<< "$spec"; tag=$(echo "$spec" | tr "|" "_")
  timeout -k 10 400 python -u -m fairify_amd.cli verify --preset src/AC-sex --out /tmp/tvs_$tag --no-accuracy \
    --node-budget $nb --escalate-budget $eb --escalate-max-open $eo > gpurun_out/tvs/$tag.log 2>&1
  cp /tmp/tvs_$tag/summary.json gpurun_out/tvs/$tag.summary.json
  python - "$tag" <<'PY'
import json, sys
d = json.load(open(f"gpurun_out/tvs/{sys.argv[1]}.summary.json"))
n = sum(r["#P"] for r in d["models"]); dec = sum(r["SAT"] + r["UNSAT"] for r in d["models"]); w = sum(r["wall_s"] for r in d["models"])
print(sys.argv[1], "decided %.2f%%" % (100 * dec / n), "wall %.1fs" % w, {r["model"]: r["Cov%"] for r in d["models"]})
PY
done
