#!/bin/bash
# round-5 seed sweep 4: candidate defaults on seeds 1-8 and 9-16
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
L=16.384000778198242
B="--steps 5 --warmup 2 --preset euro30_ms --lm-lam0-first $L"
tools/r5/step.sh \
 "a:::timeout -k 10 300 python tools/r5/seeds.py gpurun_out/r5/sw_k16_e20_x15_s916.jsonl 9-16 $B --lm-starts 16 --lm-explore-passes 20 --lm-explore-log2 15" \
 "b:::timeout -k 10 300 python tools/r5/seeds.py gpurun_out/r5/sw_k16_e20_x15_p20.jsonl 1-8 $B --lm-starts 16 --lm-explore-passes 20 --lm-explore-log2 15 --lm-passes-first 20" \
 "c:::timeout -k 10 300 python tools/r5/seeds.py gpurun_out/r5/sw_k16_e20_x15_p20_s916.jsonl 9-16 $B --lm-starts 16 --lm-explore-passes 20 --lm-explore-log2 15 --lm-passes-first 20" \
 "d:::timeout -k 10 300 python tools/r5/seeds.py gpurun_out/r5/sw_k24_e20_x15.jsonl 1-8 $B --lm-starts 24 --lm-explore-passes 20 --lm-explore-log2 15" \
 "e:::timeout -k 10 300 python tools/r5/seeds.py gpurun_out/r5/sw_k16_e25_p20_s916.jsonl 9-16 $B --lm-starts 16 --lm-explore-passes 25 --lm-passes-first 20" \
 "f:::timeout -k 10 300 python tools/r5/seeds.py gpurun_out/r5/sw_default_s916.jsonl 9-16 --steps 5 --warmup 2" \
 "g:::timeout -k 10 300 python tools/r5/seeds.py gpurun_out/r5/sw_k16_e20_x15_r3.jsonl 1-8 $B --lm-starts 16 --lm-explore-passes 20 --lm-explore-log2 15 --lm-passes-rest 3"
