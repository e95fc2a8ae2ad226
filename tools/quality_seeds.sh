#!/bin/bash
# 16-seed quality sweeps of the LM presets (tools/seeds.py, one process per
# preset) + their summary; usage: bash tools/quality_seeds.sh OUTDIR [presets]
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=${1:-gpurun_out/seeds}; shift
mkdir -p $OUT
export TMPDIR=/tmp
for pre in ${@:-euro30 euro252 heston30}; do
  S=1-16; [ $pre = basket5 ] && S=${BASKET_SEEDS:-1-8}
  rm -f $OUT/$pre.jsonl
  timeout -k 10 400 python tools/seeds.py $OUT/$pre.jsonl $S --steps 2 --warmup 1 --preset $pre > $OUT/$pre.log 2>&1 || { echo "$pre failed"; tail -3 $OUT/$pre.log; exit 1; }
done
python tools/seed_summary.py $OUT/*.jsonl | tee $OUT/SUMMARY.txt
