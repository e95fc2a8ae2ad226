#!/bin/bash
# GPU: round-3 evidence collection (MTS parity variants, LM pass stamps,
# 8-seed flagship sweep); every step under its own time limit, stop at the
# first failure.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
timeout -k 10 600 python tools/mts_variants.py --seeds 8 > gpurun_out/mts_variants8.jsonl 2> gpurun_out/mts_variants.err || exit $?
timeout -k 10 120 python tools/stamp_lm.py 20 > gpurun_out/stamp20.json || exit $?
timeout -k 10 120 python tools/stamp_lm.py 16 > gpurun_out/stamp16.json || exit $?
bash tools/sweep_bench.sh tools/sweeps/seeds_r3_abc.txt seeds_r3_abce
