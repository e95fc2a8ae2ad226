#!/bin/bash
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
for v in spread; do
  BENCH_ARGS="--init $v ${EXTRA}" LIBS=main tools/archive/seed_sweep.sh || exit 1
  mv gpurun_out/seeds_main.jsonl gpurun_out/seeds_init_$v.jsonl
done
SEEDS=1234 BENCH_ARGS="--init spread ${EXTRA}" LIBS=main tools/archive/seed_sweep.sh && mv gpurun_out/seeds_main.jsonl gpurun_out/seeds_init_spread_1234.jsonl
SEEDS=1234 BENCH_ARGS="${EXTRA}" LIBS=main tools/archive/seed_sweep.sh && mv gpurun_out/seeds_main.jsonl gpurun_out/seeds_init_ref_1234.jsonl
