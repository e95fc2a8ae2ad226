#!/bin/bash
# basket5 quality levers: Gram subsample size, later-date passes, multi-start
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
: > gpurun_out/bk.jsonl
for a in "--lm-gram-paths 16384" "--lm-gram-paths 8192" "--lm-passes-rest 3" "--lm-starts 4 --lm-explore-passes 45 --lm-passes-first 40"; do
  timeout -k 10 300 python bench.py --preset basket5 --steps 1 --warmup 1 --seed 1 $a > gpurun_out/one.log 2>&1 || { tail -20 gpurun_out/one.log; exit 1; }
  tail -n 1 gpurun_out/one.log >> gpurun_out/bk.jsonl
  echo "done $a"
done
python3 - <<'PY'
import json
for l in open("gpurun_out/bk.jsonl"):
    r = json.loads(l); q = r["quality"]; c = r["config"]
    print(c.get("lm_gram_paths"), c.get("lm_passes_rest"), c.get("lm_multistart"), round(r["ms_per_step"], 1), round(q["terminal_pnl_std"], 4),
          "ratio", round(q["terminal_pnl_std"] / q["hedge_anchor"]["pnl_std"], 4), "resid", round(q["terminal_residual_std"], 4))
PY
