#!/bin/bash
# rocprofv3 kernel trace of bench.py (default: the euro30 flagship) and the
# per-kernel / per-phase summaries of ONE graph replay.
# usage: bash tools/prof_bench.sh OUTDIR [bench.py args...]
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=${1:-gpurun_out/prof}; shift
mkdir -p $OUT
export TMPDIR=/tmp
rm -rf $OUT/prof
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $OUT/prof -o run -- python3 bench.py --steps 6 --warmup 1 "$@" > $OUT/prof.log 2>&1 || { echo prof failed; tail -5 $OUT/prof.log; exit 1; }
db=$(find $OUT/prof -name "*results.db" | head -1)
python3 tools/kstats.py "$db" > $OUT/kernel_stats.txt
python3 tools/phases.py "$db" > $OUT/phases.txt
head -12 $OUT/kernel_stats.txt
head -3 $OUT/phases.txt
