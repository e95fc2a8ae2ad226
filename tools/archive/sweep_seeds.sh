#!/bin/bash
# euro30 (or --preset ...) over seeds 1-8 for each argument line of $1;
# one summary line per configuration.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
: > gpurun_out/sweep_seeds.jsonl
while IFS= read -r cfg; do
  [ -z "$cfg" ] && continue
  : > gpurun_out/ss_one.jsonl
  for s in ${SEEDS:-1 2 3 4 5 6 7 8}; do
    timeout -k 10 200 python bench.py --steps 5 --warmup 2 --seed $s $cfg > gpurun_out/ss_one.log 2>&1 || { tail -n 20 gpurun_out/ss_one.log; exit 1; }
    tail -n 1 gpurun_out/ss_one.log >> gpurun_out/ss_one.jsonl
  done
  python3 - "$cfg" <<'PY'
import json, sys, numpy as np
rows = [json.loads(l) for l in open("gpurun_out/ss_one.jsonl")]
p = [r["quality"]["terminal_pnl_std"] for r in rows]; ms = [r["ms_per_step"] for r in rows]
rec = {"cfg": sys.argv[1], "ms": float(np.mean(ms)), "pnl": p, "mean": float(np.mean(p)), "worst": float(max(p)),
       "resid": [r["quality"]["terminal_residual_std"] for r in rows]}
open("gpurun_out/sweep_seeds.jsonl", "a").write(json.dumps(rec) + "\n")
print(sys.argv[1], "ms", round(rec["ms"], 2), "pnl", np.round(p, 4).tolist(), "mean", round(rec["mean"], 4), "worst", round(rec["worst"], 4))
PY
done < "$1"
