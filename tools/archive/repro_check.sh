#!/bin/bash
# Run-to-run reproducibility: the same preset in separate processes, one JSON
# line each (V0 / P&L std must be bitwise identical for a deterministic path).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
out=gpurun_out/repro.jsonl
for p in ${PRESETS:-euro252 euro30_adam}; do
  for k in 1 2 3; do
    timeout -k 10 200 python bench.py --preset $p --steps 1 --warmup 1 > gpurun_out/repro_one.log 2>&1 || exit 1
    grep '^{' gpurun_out/repro_one.log >> $out
  done
done
