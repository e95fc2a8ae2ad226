#!/bin/bash
# lm_gram_skip timing sweep of the euro30 bench (RPH_LM_GRAM_SKIP), one box
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
mkdir -p gpurun_out/r5
for gs in "$@"; do
  RPH_LM_GRAM_SKIP=$gs timeout -k 10 200 python bench.py --steps 20 --warmup 3 > gpurun_out/r5/gs$gs.log 2>&1 || exit 1
  python3 -c "
import json; r=json.loads([l for l in open('gpurun_out/r5/gs$gs.log') if l.startswith('{')][-1]); print('gram_skip', $gs, round(r['ms_per_step'],3), r['quality']['terminal_pnl_std'])"
done
