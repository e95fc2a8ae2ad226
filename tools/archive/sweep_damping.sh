#!/bin/bash
# LM damping update (simple vs Nielsen) x pass budget on a preset, one JSON line per run.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
IFS=';' read -ra LIST <<< "${CFGS:-40 2;60 2;80 2}"
for damp in ${DAMPINGS:-simple nielsen}; do
  for cfg in "${LIST[@]}"; do
    set -- $cfg
    timeout -k 10 200 python bench.py --preset ${PRESET:-euro30} --lm-damping $damp --lm-passes-first $1 \
      --lm-passes-rest $2 --steps 2 --warmup 1 > gpurun_out/sweep_one.log 2>&1 || exit 1
    grep '^{' gpurun_out/sweep_one.log >> gpurun_out/sweep_damping.jsonl
  done
done
