#!/bin/bash
# round-5 preset sweep 2: euro252 first-date budgets, heston30 variants
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
L=16.384000778198242
tools/r5/step.sh \
 "e1:::timeout -k 10 300 python tools/r5/seeds.py gpurun_out/r5/sp_e252_k4e45x16p80.jsonl 1-3 --steps 3 --warmup 1 --preset euro252 --lm-starts 4 --lm-explore-passes 45 --lm-explore-log2 16 --lm-passes-first 80" \
 "e2:::timeout -k 10 300 python tools/r5/seeds.py gpurun_out/r5/sp_e252_k8e40x16p80.jsonl 1-3 --steps 3 --warmup 1 --preset euro252 --lm-starts 8 --lm-explore-passes 40 --lm-explore-log2 16 --lm-passes-first 80" \
 "e3:::timeout -k 10 300 python tools/r5/seeds.py gpurun_out/r5/sp_e252_p160.jsonl 1-3 --steps 3 --warmup 1 --preset euro252 --lm-passes-first 160" \
 "e4:::timeout -k 10 300 python tools/r5/seeds.py gpurun_out/r5/sp_e252_k16e30x16p80.jsonl 1-3 --steps 3 --warmup 1 --preset euro252 --lm-starts 16 --lm-explore-passes 30 --lm-explore-log2 16 --lm-passes-first 80 --lm-lam0-first $L" \
 "e5:::timeout -k 10 300 python tools/r5/seeds.py gpurun_out/r5/sp_e252_init_spread.jsonl 1-3 --steps 3 --warmup 1 --preset euro252 --init spread" \
 "h2:::timeout -k 10 300 python tools/r5/seeds.py gpurun_out/r5/sp_heston_ms_e25_p35.jsonl 1-3 --steps 5 --warmup 2 --preset heston30 --lm-starts 16 --lm-explore-passes 25 --lm-explore-log2 15 --lm-explore-one 0 --lm-lam0-first $L --lm-passes-first 35"
