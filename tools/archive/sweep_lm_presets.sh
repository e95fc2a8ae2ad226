#!/bin/bash
# LM vs Adam on every BASELINE preset (quality vs time), one JSON line per run.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
out=gpurun_out/sweep_presets_lm.jsonl
for p in euro30 heston30 euro252; do
  for opt in adam lm; do
    timeout -k 10 200 python bench.py --preset $p --optimizer $opt --steps 3 --warmup 1 > gpurun_out/sweep_one.log 2>&1 || exit 1
    grep '^{' gpurun_out/sweep_one.log >> $out
  done
done
timeout -k 10 300 python bench.py --preset basket5 --optimizer lm --steps 1 --warmup 1 > gpurun_out/sweep_one.log 2>&1 || exit 1
grep '^{' gpurun_out/sweep_one.log >> $out
