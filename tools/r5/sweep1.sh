#!/bin/bash
# round-5 seed sweep 1: default vs multi-start variants (8 seeds each)
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
L=16.384000778198242
tools/r5/step.sh \
 "s_default:::timeout -k 10 300 python tools/r5/seeds.py gpurun_out/r5/sw_default.jsonl 1-8 --steps 5 --warmup 2" \
 "s_ms:::timeout -k 10 300 python tools/r5/seeds.py gpurun_out/r5/sw_ms.jsonl 1-8 --steps 5 --warmup 2 --preset euro30_ms" \
 "s_ms_l0:::timeout -k 10 300 python tools/r5/seeds.py gpurun_out/r5/sw_ms_l0.jsonl 1-8 --steps 5 --warmup 2 --preset euro30_ms --lm-lam0-first $L" \
 "s_ms_l0_e35:::timeout -k 10 300 python tools/r5/seeds.py gpurun_out/r5/sw_ms_l0_e35.jsonl 1-8 --steps 5 --warmup 2 --preset euro30_ms --lm-lam0-first $L --lm-explore-passes 35" \
 "s_ms_l0_p20:::timeout -k 10 300 python tools/r5/seeds.py gpurun_out/r5/sw_ms_l0_p20.jsonl 1-8 --steps 5 --warmup 2 --preset euro30_ms --lm-lam0-first $L --lm-passes-first 20"
