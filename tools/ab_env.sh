#!/bin/bash
# Same-box A/B of bench.py variants: each argument is "ENV=.. ENV2=..|bench args"
# (either side may be empty); prints ms per step, the P&L std and V0 per variant.
# usage: bash tools/ab_env.sh OUTDIR "RPH_X=0|" "|--lm-leaf-paths 1024" ...
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=$1; shift
mkdir -p $OUT
export TMPDIR=/tmp
i=0
for a in "$@"; do
  e=${a%%|*}; f=${a#*|}; i=$((i + 1))
  env $e timeout -k 10 150 python bench.py --steps ${STEPS:-20} --warmup 3 $f > $OUT/v$i.json 2> $OUT/v$i.err || { echo "variant $i failed"; tail -3 $OUT/v$i.err; exit 1; }
  python -c "import json,sys; d=json.loads(open('$OUT/v$i.json').read().strip().splitlines()[-1]); q=d['quality']; print('$e | $f |', round(d['ms_per_step'],4), q['terminal_pnl_std'], q['V0'])"
done
