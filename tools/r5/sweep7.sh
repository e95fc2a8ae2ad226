#!/bin/bash
# round-5 preset sweep 3: euro252 later-date budget
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
M="--preset euro252 --lm-starts 8 --lm-explore-passes 40 --lm-explore-log2 16 --lm-passes-first 80"
tools/r5/step.sh \
 "e1:::timeout -k 10 300 python tools/r5/seeds.py gpurun_out/r5/sp_e252_k8_r3.jsonl 1-3 --steps 3 --warmup 1 $M --lm-passes-rest 3" \
 "e2:::timeout -k 10 300 python tools/r5/seeds.py gpurun_out/r5/sp_e252_k8_r4s.jsonl 1-3 --steps 3 --warmup 1 $M --lm-passes-rest 4 --lm-stop-tol 0.01 --lm-stop-min 2" \
 "e3:::timeout -k 10 300 python tools/r5/seeds.py gpurun_out/r5/sp_e252_k8_r3_c2.jsonl 1-3 --steps 3 --warmup 1 $M --lm-passes-rest 3 --lm-lam-carry 2"
