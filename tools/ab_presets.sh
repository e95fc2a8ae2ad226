#!/bin/bash
# A/B of two native builds over bench presets: A = rphedge/_lib/ab/librphedge_A.so
# (an older tree's csrc/ built with the same flags; RPH_NATIVE_LIB=<path>.so
# loads exactly that file, never building it), B = rphedge/_lib/librphedge.so.
# PRESETS (default "euro30 euro30_adam basket5"); TESTS=1 also runs pytest -m gpu on B.
cd "${GRAFT_REPO_ROOT}"
export TMPDIR=/tmp
O=gpurun_out/ab
mkdir -p $O
T="timeout -k 10"
if [ "${TESTS:-0}" = 1 ]; then
  $T 500 python -u -m pytest tests -m gpu -q -p no:cacheprovider --timeout 120 --timeout-method thread > $O/tests_B.log 2>&1
  rc=$?; echo "B tests rc=$rc"; tail -3 $O/tests_B.log
  [ $rc -gt 1 ] && exit $rc
fi
for pre in ${PRESETS:-euro30 euro30_adam basket5}; do
  for v in A B; do
    if [ $v = A ]; then export RPH_NATIVE_LIB=$PWD/rphedge/_lib/ab/librphedge_A.so; else unset RPH_NATIVE_LIB; fi
    $T 300 python bench.py --preset $pre --steps ${STEPS:-5} --warmup 2 > $O/bench_${pre}_$v.log 2>&1 || exit 1
    echo "$pre $v $(grep -o '"native[^,]*' $O/bench_${pre}_$v.log | head -1) $(grep -o '"ms_per_step": [0-9.]*\|"V0": [0-9.]*\|"terminal_pnl_std": [0-9.]*' $O/bench_${pre}_$v.log | tr '\n' ' ')"
  done
done
echo ALLDONE
