#!/bin/bash
# GPU: direct k_lm_solve tests (+ $EXTRA_TESTS) with the current library, the
# per-shape solve timing with an A/B library ($AB_LIB), the flagship bench
# with the current library, and (PROF=1) its rocprofv3 kernel statistics.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
T="python -u -m pytest --timeout 120 --timeout-method thread -p no:cacheprovider"
timeout -k 10 600 $T tests/test_gpu_lm_solve.py ${EXTRA_TESTS} -v > gpurun_out/solve_tests.log 2>&1
rc=$?; echo "tests rc=$rc"; [ $rc -gt 1 ] && exit $rc
if [ -n "$STAMPS" ]; then
  timeout -k 10 200 python -u tools/archive/solve_stamps.py > gpurun_out/solve_stamps.jsonl 2> gpurun_out/solve_stamps.err
  echo "stamps rc=$?"
fi
if [ -n "$AB_LIB" ]; then
  RPH_NATIVE_LIB=$AB_LIB timeout -k 10 200 $T tests/test_gpu_lm_solve.py -k time_per_shape -s > gpurun_out/solve_time_ab.log 2>&1
  echo "ab timing rc=$?"
fi
timeout -k 10 300 python bench.py --steps 10 --warmup 2 ${BENCH_ARGS} > gpurun_out/bench.log 2>&1
rc=$?; echo "bench rc=$rc"; [ $rc -ne 0 ] && exit $rc
if [ -n "$PROF" ]; then
  timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof -o run --output-format csv -- python3 bench.py --steps 2 --warmup 1 ${BENCH_ARGS} > gpurun_out/prof.log 2>&1
  echo "prof rc=$?"
fi
