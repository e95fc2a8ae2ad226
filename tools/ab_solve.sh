#!/bin/bash
# GPU: direct k_lm_solve tests with the current library, then the per-shape
# solve timing with the current library and an A/B library ($AB_LIB), then the
# flagship bench with the current library.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
T="python -u -m pytest --timeout 120 --timeout-method thread -p no:cacheprovider"
timeout -k 10 500 $T tests/test_gpu_lm_solve.py -x -v ${EXTRA_TESTS} > gpurun_out/solve_tests.log 2>&1
rc=$?; echo "tests rc=$rc"; [ $rc -gt 1 ] && exit $rc
if [ -n "$AB_LIB" ]; then
  RPH_NATIVE_LIB=$AB_LIB timeout -k 10 200 $T tests/test_gpu_lm_solve.py -k time_per_shape -s > gpurun_out/solve_time_ab.log 2>&1
  echo "ab timing rc=$?"
fi
timeout -k 10 300 python bench.py --steps 10 --warmup 2 ${BENCH_ARGS} > gpurun_out/bench.log 2>&1
echo "bench rc=$?"
