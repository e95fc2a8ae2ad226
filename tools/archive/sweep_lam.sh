#!/bin/bash
# LM damping constants x pass budget on a preset (quality vs time), one JSON line per run.
# CFGS: "passes_first passes_rest lam0 lam_up lam_down;..."
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
IFS=';' read -ra LIST <<< "${CFGS}"
for cfg in "${LIST[@]}"; do
  set -- $cfg
  timeout -k 10 200 python bench.py --preset ${PRESET:-euro30} --lm-passes-first $1 --lm-passes-rest $2 \
    --lm-lam0 $3 --lm-lam-up $4 --lm-lam-down $5 --steps 2 --warmup 1 > gpurun_out/sweep_one.log 2>&1 || exit 1
  grep '^{' gpurun_out/sweep_one.log >> gpurun_out/sweep_lam.jsonl
done
