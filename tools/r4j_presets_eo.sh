#!/bin/bash
# presets with the single-start exploration warm-up on the first date
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
: > gpurun_out/peo.jsonl
run() { timeout -k 10 300 python bench.py "$@" > gpurun_out/one.log 2>&1 || { tail -20 gpurun_out/one.log; exit 1; }; tail -n 1 gpurun_out/one.log >> gpurun_out/peo.jsonl; }
for s in 1 2 3; do run --preset heston30 --steps 3 --warmup 1 --seed $s --lm-explore-one 1 --lm-explore-passes 45 --lm-passes-first 35; done
for s in 1 2 3; do run --preset euro252 --steps 2 --warmup 1 --seed $s --lm-explore-one 1 --lm-explore-passes 60 --lm-passes-first 60; done
for s in 1 2; do run --preset basket5 --steps 2 --warmup 1 --seed $s --lm-explore-one 1 --lm-explore-passes 40 --lm-passes-first 40; done
python3 - <<'PY'
import json
for l in open("gpurun_out/peo.jsonl"):
    r = json.loads(l); q = r["quality"]
    print(r["config"]["preset"], r["config"].get("seed"), round(r["ms_per_step"], 2), round(q["terminal_pnl_std"], 4),
          "ratio", round(q["terminal_pnl_std"] / q["hedge_anchor"]["pnl_std"], 4), "resid", round(q["terminal_residual_std"], 4), "V0", round(q["V0"], 4))
PY
