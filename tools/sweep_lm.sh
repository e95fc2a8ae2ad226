#!/bin/bash
# LM pass-budget sweep of the euro30 preset (quality vs time), one JSON line per config.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
for cfg in "40 2" "60 2" "60 3" "80 3" "80 4" "120 4" "80 6"; do
  set -- $cfg
  timeout -k 10 120 python bench.py --optimizer lm --lm-passes-first $1 --lm-passes-rest $2 --steps 2 --warmup 1 \
    | grep '^{' >> gpurun_out/sweep_lm.jsonl || exit 1
done
