#!/bin/bash
# euro30 first-date multi-start over seeds 1-8 (two budgets)
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
for cfg in "--lm-starts 4 --lm-explore-passes 45 --lm-passes-first 25" "--lm-starts 4 --lm-explore-passes 35 --lm-passes-first 20"; do
  tag=$(echo "$cfg" | tr -d ' -' | cut -c1-40)
  : > gpurun_out/ms_$tag.jsonl
  for s in 1 2 3 4 5 6 7 8; do
    timeout -k 10 200 python bench.py --steps 5 --warmup 2 --seed $s $cfg > gpurun_out/ms_one.log 2>&1 || { tail -n 20 gpurun_out/ms_one.log; exit 1; }
    tail -n 1 gpurun_out/ms_one.log >> gpurun_out/ms_$tag.jsonl
  done
  python3 - "gpurun_out/ms_$tag.jsonl" "$cfg" <<'PY'
import json, sys, numpy as np
rows = [json.loads(l) for l in open(sys.argv[1])]
p = [r["quality"]["terminal_pnl_std"] for r in rows]; ms = [r["ms_per_step"] for r in rows]
print(sys.argv[2], "ms", round(np.mean(ms), 2), "pnl", np.round(p, 4).tolist(), "mean", round(np.mean(p), 4), "worst", round(max(p), 4))
PY
done
