#!/bin/bash
# round-5: quality of every preset at 2^18 paths (the GPU quality test's size), 3 seeds
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
A="--paths-log2 18 --steps 1 --warmup 1"
tools/r5/step.sh \
 "q1:::timeout -k 10 300 python tools/r5/seeds.py gpurun_out/r5/q18_euro30.jsonl 1-3 $A --preset euro30" \
 "q2:::timeout -k 10 300 python tools/r5/seeds.py gpurun_out/r5/q18_heston30.jsonl 1-3 $A --preset heston30" \
 "q3:::timeout -k 10 300 python tools/r5/seeds.py gpurun_out/r5/q18_euro252.jsonl 1-3 $A --preset euro252" \
 "q4:::timeout -k 10 300 python tools/r5/seeds.py gpurun_out/r5/q18_basket5.jsonl 1-3 $A --preset basket5"
