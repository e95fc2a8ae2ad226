#!/bin/bash
# Multi-start first date on euro252 / heston30 over seeds, and the quality
# test's 2^18-path ratios (tests/test_gpu_quality.py) for its bounds.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
: > gpurun_out/msp.jsonl; : > gpurun_out/q18.jsonl
for s in 1 2 3; do
  timeout -k 10 300 python bench.py --preset euro252 --steps 2 --warmup 1 --seed $s --lm-starts 4 --lm-explore-passes 45 --lm-passes-first 60 > gpurun_out/one.log 2>&1 || { tail -20 gpurun_out/one.log; exit 1; }
  tail -n 1 gpurun_out/one.log >> gpurun_out/msp.jsonl
  timeout -k 10 300 python bench.py --preset heston30 --steps 3 --warmup 1 --seed $s --lm-starts 4 --lm-explore-passes 45 --lm-passes-first 30 > gpurun_out/one.log 2>&1 || { tail -20 gpurun_out/one.log; exit 1; }
  tail -n 1 gpurun_out/one.log >> gpurun_out/msp.jsonl
done
for p in euro30 heston30 euro252 basket5; do
  timeout -k 10 300 python bench.py --preset $p --paths-log2 18 --steps 1 --warmup 1 > gpurun_out/one.log 2>&1 || { tail -20 gpurun_out/one.log; exit 1; }
  tail -n 1 gpurun_out/one.log >> gpurun_out/q18.jsonl
done
python3 - <<'PY'
import json
for f in ("gpurun_out/msp.jsonl", "gpurun_out/q18.jsonl"):
    for l in open(f):
        r = json.loads(l); q = r["quality"]; a = q["hedge_anchor"]["pnl_std"]
        print(f[11:], r["config"]["preset"], r["config"].get("seed"), round(r["ms_per_step"], 2), round(q["terminal_pnl_std"], 4),
              "ratio", round(q["terminal_pnl_std"] / a, 4), "resid", round(q["terminal_residual_std"], 4), "V0", round(q["V0"], 4))
PY
