#!/bin/bash
# round-5 seed sweep 2: multi-start width / exploration prefix (8 seeds each)
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
L=16.384000778198242
B="--steps 5 --warmup 2 --preset euro30_ms --lm-lam0-first $L"
tools/r5/step.sh \
 "s_k8_e35:::timeout -k 10 300 python tools/r5/seeds.py gpurun_out/r5/sw_k8_e35.jsonl 1-8 $B --lm-starts 8 --lm-explore-passes 35" \
 "s_k6_e35:::timeout -k 10 300 python tools/r5/seeds.py gpurun_out/r5/sw_k6_e35.jsonl 1-8 $B --lm-starts 6 --lm-explore-passes 35" \
 "s_k4_e45_x17:::timeout -k 10 300 python tools/r5/seeds.py gpurun_out/r5/sw_k4_e45_x17.jsonl 1-8 $B --lm-explore-log2 17" \
 "s_k8_e25:::timeout -k 10 300 python tools/r5/seeds.py gpurun_out/r5/sw_k8_e25.jsonl 1-8 $B --lm-starts 8 --lm-explore-passes 25" \
 "s_k16_e25:::timeout -k 10 300 python tools/r5/seeds.py gpurun_out/r5/sw_k16_e25.jsonl 1-8 $B --lm-starts 16 --lm-explore-passes 25"
