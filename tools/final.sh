#!/bin/bash
# Round-end rehearsal on one GPU: smoke, the GPU suite, the euro30 bench and a
# rocprofv3 kernel-stats run of it; outputs under gpurun_out/final/.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=${1:-gpurun_out/final}
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 120 python -u -c "import __graft_entry__ as g; g.smoke()" > $OUT/smoke.log 2>&1 || { echo smoke failed; tail -5 $OUT/smoke.log; exit 1; }
timeout -k 10 900 python -u -m pytest tests -m gpu -q --timeout 200 --timeout-method thread -p no:cacheprovider > $OUT/pytest_gpu.log 2>&1
tail -2 $OUT/pytest_gpu.log
timeout -k 10 200 python bench.py --steps 20 --warmup 3 > $OUT/bench.log 2>&1 || { echo bench failed; exit 1; }
tail -c 400 $OUT/bench.log
rm -rf $OUT/prof
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $OUT/prof -o run -- python3 bench.py --steps 6 --warmup 1 > $OUT/prof.log 2>&1 || { echo prof failed; exit 1; }
db=$(find $OUT/prof -name "*results.db" | head -1)
python3 tools/kstats.py "$db" > $OUT/kernel_stats.txt
python3 tools/phases.py "$db" > $OUT/phases.txt
head -8 $OUT/kernel_stats.txt
