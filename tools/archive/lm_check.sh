#!/bin/bash
# LM kernel iteration loop on the GPU box: LM tests, rocprof of the default
# bench, solve-kernel stamps (NINS: network input counts to stamp).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
rm -rf gpurun_out/prof
timeout -k 10 300 python -u -m pytest tests/test_gpu_lm.py -q -p no:cacheprovider --timeout=200 --timeout-method thread > gpurun_out/pytest.log 2>&1 || exit 1
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof -o run --output-format csv -- python3 bench.py --steps 2 --warmup 1 > gpurun_out/prof.log 2>&1 || exit 1
: > gpurun_out/stamp.log
for nin in ${NINS:-1}; do
  timeout -k 10 200 python tools/stamp_lm.py 20 $nin >> gpurun_out/stamp.log 2>&1 || exit 1
done
