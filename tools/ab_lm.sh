#!/bin/bash
# A/B of two native builds on the LM path: A = librphedge_debug.so slot (the
# previous build, copied there by hand), B = the current librphedge.so.
cd "${GRAFT_REPO_ROOT}"
export TMPDIR=/tmp
O=gpurun_out/ab
mkdir -p $O
T="timeout -k 10"
RPH_NATIVE_LIB=debug $T 200 python -u -m pytest tests/test_gpu_lm.py -q -p no:cacheprovider --timeout 120 --timeout-method thread -k fit_matches > $O/tests_A.log 2>&1; echo "A tests rc=$?"
$T 300 python -u -m pytest tests/test_gpu_lm.py -q -p no:cacheprovider --timeout 120 --timeout-method thread > $O/tests_B.log 2>&1; rc=$?; echo "B tests rc=$rc"
[ $rc -gt 1 ] && exit $rc
for pre in euro30 heston30; do
  RPH_NATIVE_LIB=debug $T 200 python bench.py --preset $pre --steps 10 --warmup 2 > $O/bench_${pre}_A.log 2>&1 || exit 1
  $T 200 python bench.py --preset $pre --steps 10 --warmup 2 > $O/bench_${pre}_B.log 2>&1 || exit 1
done
echo ALLDONE
