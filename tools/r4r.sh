#!/bin/bash
# Round-4 final GPU step: the whole GPU suite, euro30 seeds 1-8, the other
# presets, and a kernel-stats profile of the default bench.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out/r4r
export TMPDIR=/tmp
true
printf '%s\n' "--steps 5 --warmup 2" > /tmp/r4o_lines.txt
bash tools/sweep_seeds.sh /tmp/r4o_lines.txt || exit $?
cp gpurun_out/sweep_seeds.jsonl gpurun_out/r4r/seeds_euro30.jsonl
for p in heston30 euro252 basket5; do
  timeout -k 10 300 python bench.py --preset $p --steps 5 --warmup 2 > gpurun_out/r4r/bench_$p.log 2>&1 || exit 1
  tail -1 gpurun_out/r4r/bench_$p.log | cut -c1-200
done
cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $GRAFT_REPO_ROOT/gpurun_out/r4r/prof -o run --output-format csv -- python3 $GRAFT_REPO_ROOT/bench.py --steps 10 --warmup 3 > $GRAFT_REPO_ROOT/gpurun_out/r4r/prof.log 2>&1 || exit 1
