#!/bin/bash
# basket5 (2^23 paths, 252 dates) seeds 1-8: longer first date / multi-start
# with the output-step trust region (round 6 sweep; profiles/r6/basket5/).
# usage: bash tools/archive/basket5_first_tr.sh OUTDIR "VARIANT" ...
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
export TMPDIR=/tmp
O=$1; shift
mkdir -p $O
i=0
for v in "$@"; do
  i=$((i+1))
  timeout -k 10 400 python tools/seeds.py $O/v$i.jsonl ${SEEDS:-1-8} --steps 2 --warmup 1 --preset basket5 $v > $O/v$i.log 2>&1 || { echo "v$i failed"; tail -3 $O/v$i.log; exit 1; }
  echo "v$i: $v"
done
python tools/seed_summary.py $O/v*.jsonl
