#!/bin/bash
# round-5 preset sweep: heston30 / euro252 / basket5, current vs 16-start first date
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
L=16.384000778198242
M="--lm-starts 16 --lm-explore-passes 20 --lm-explore-log2 15 --lm-explore-one 0 --lm-lam0-first $L"
tools/r5/step.sh \
 "h0:::timeout -k 10 300 python tools/r5/seeds.py gpurun_out/r5/sp_heston_base.jsonl 1-3 --steps 5 --warmup 2 --preset heston30" \
 "h1:::timeout -k 10 300 python tools/r5/seeds.py gpurun_out/r5/sp_heston_ms.jsonl 1-3 --steps 5 --warmup 2 --preset heston30 $M --lm-passes-first 25" \
 "e0:::timeout -k 10 300 python tools/r5/seeds.py gpurun_out/r5/sp_e252_base.jsonl 1-3 --steps 3 --warmup 1 --preset euro252" \
 "e1:::timeout -k 10 300 python tools/r5/seeds.py gpurun_out/r5/sp_e252_ms.jsonl 1-3 --steps 3 --warmup 1 --preset euro252 $M --lm-passes-first 40" \
 "b0:::timeout -k 10 400 python tools/r5/seeds.py gpurun_out/r5/sp_b5_base.jsonl 1-2 --steps 2 --warmup 1 --preset basket5" \
 "b1:::timeout -k 10 400 python tools/r5/seeds.py gpurun_out/r5/sp_b5_ms.jsonl 1-2 --steps 2 --warmup 1 --preset basket5 $M --lm-passes-first 40"
