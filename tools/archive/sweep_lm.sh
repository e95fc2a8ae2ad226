#!/bin/bash
# LM pass-budget sweep of a preset (quality vs time), one JSON line per config.
# usage: PRESET=euro30 CFGS="40 2;60 3" bash tools/archive/sweep_lm.sh
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
IFS=';' read -ra LIST <<< "${CFGS:-30 2;40 2;50 2;50 3;60 2;60 3;80 3;80 2}"
for cfg in "${LIST[@]}"; do
  set -- $cfg
  timeout -k 10 200 python bench.py --preset ${PRESET:-euro30} --optimizer lm --lm-passes-first $1 --lm-passes-rest $2 \
    --steps 2 --warmup 1 > gpurun_out/sweep_one.log 2>&1 || exit 1
  grep '^{' gpurun_out/sweep_one.log >> gpurun_out/sweep_lm.jsonl
done
