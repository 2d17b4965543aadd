#!/bin/bash
# round 6, call M: the headline step's residue -- default step + its budget pass (which stages decide
# the residue), and the beta fixed pass inside the timed step at budgets 64 / 128
set -o pipefail
OUT=gpurun_out/r6m; mkdir -p $OUT
timeout -k 10 400 python -u bench.py --steps 3 --warmup 1 > $OUT/def.json 2> $OUT/def.err || { tail -20 $OUT/def.err; exit 1; }
python - $OUT/def.json <<'PY'
import json, sys
d = json.load(open(sys.argv[1]))
print("default", d["ms_per_step"], d["pct_verified_sound"], d["unknown"], "budget", d.get("pct_verified_at_budget_sound"))
print(json.dumps(d.get("budget_pass", {}).get("unsat_by_stage")), json.dumps(d.get("budget_pass", {}).get("sat_by_stage")))
print({k: v["unknown"] for k, v in d["per_model"].items()})
PY
for b in 64 128; do
  timeout -k 10 400 python -u bench.py --steps 3 --warmup 1 --budget-pass 0 --beta-budget $b > $OUT/b$b.json 2> $OUT/b$b.err || { tail -20 $OUT/b$b.err; exit 1; }
  python -c "import json;d=json.load(open('$OUT/b$b.json'));print('beta $b', d['ms_per_step'], d['pct_verified_sound'], d['unknown'], d['unsat_by_stage']['beta'], d['sat_by_stage']['beta'], {k: v['unknown'] for k, v in d['per_model'].items()})"
done
