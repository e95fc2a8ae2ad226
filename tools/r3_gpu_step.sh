#!/bin/bash
# GPU: LM / DP / multi-start tests, then an 8-seed sweep file ($1 -> gpurun_out/$2.jsonl) and a
# rocprofv3 kernel-stats run of the default bench; stop at the first failure.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_gpu_dp.py tests/test_gpu_lm.py tests/test_gpu_lm_multistart.py -x -q \
    --timeout 300 --timeout-method thread -p no:cacheprovider > gpurun_out/pt.log 2>&1
rc=$?; tail -5 gpurun_out/pt.log; [ $rc -ne 0 ] && exit $rc
bash tools/sweep_bench.sh "$1" "$2" || exit $?
export TMPDIR=/tmp
timeout -k 10 200 rocprofv3 --kernel-trace --stats -d gpurun_out/prof -o run --output-format csv -- \
    python3 bench.py --steps 2 --warmup 1 > gpurun_out/prof.log 2>&1
