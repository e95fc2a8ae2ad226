#!/bin/bash
# LM on every GPU BASELINE preset, one JSON line per run (quality vs time).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
out=gpurun_out/sweep_lm_only.jsonl
for p in ${PRESETS:-euro30 heston30 euro252}; do
  timeout -k 10 200 python bench.py --preset $p --optimizer lm --steps 3 --warmup 1 $EXTRA > gpurun_out/sweep_one.log 2>&1 || exit 1
  grep '^{' gpurun_out/sweep_one.log >> $out
done
