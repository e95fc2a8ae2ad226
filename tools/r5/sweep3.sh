#!/bin/bash
# round-5 seed sweep 3: around 16 starts x 25 exploration passes (8 seeds each)
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
L=16.384000778198242
B="--steps 5 --warmup 2 --preset euro30_ms --lm-lam0-first $L"
tools/r5/step.sh \
 "s_k16_e20:::timeout -k 10 300 python tools/r5/seeds.py gpurun_out/r5/sw_k16_e20.jsonl 1-8 $B --lm-starts 16 --lm-explore-passes 20" \
 "s_k16_e25_p20:::timeout -k 10 300 python tools/r5/seeds.py gpurun_out/r5/sw_k16_e25_p20.jsonl 1-8 $B --lm-starts 16 --lm-explore-passes 25 --lm-passes-first 20" \
 "s_k12_e25:::timeout -k 10 300 python tools/r5/seeds.py gpurun_out/r5/sw_k12_e25.jsonl 1-8 $B --lm-starts 12 --lm-explore-passes 25" \
 "s_k16_e20_x15:::timeout -k 10 300 python tools/r5/seeds.py gpurun_out/r5/sw_k16_e20_x15.jsonl 1-8 $B --lm-starts 16 --lm-explore-passes 20 --lm-explore-log2 15" \
 "s_k32_e20_x15:::timeout -k 10 300 python tools/r5/seeds.py gpurun_out/r5/sw_k32_e20_x15.jsonl 1-8 $B --lm-starts 32 --lm-explore-passes 20 --lm-explore-log2 15" \
 "s_k16_e25_s916:::timeout -k 10 300 python tools/r5/seeds.py gpurun_out/r5/sw_k16_e25_s916.jsonl 9-16 $B --lm-starts 16 --lm-explore-passes 25"
