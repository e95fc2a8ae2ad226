#!/bin/bash
# GPU A/B of native-library variants: for each name in $LIBS ("main" = the
# in-tree library, else rphedge/_lib/ab/librphedge_<name>.so) run the LM
# tests ($TESTS), the pass/solve stamps (tools/stamp_lm.py) and the flagship
# bench; logs under gpurun_out/ab_<name>.*
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
T="python -u -m pytest --timeout 120 --timeout-method thread -p no:cacheprovider -q"
for v in ${LIBS:-main}; do
  if [ "$v" = main ]; then unset RPH_NATIVE_LIB; else export RPH_NATIVE_LIB=rphedge/_lib/ab/librphedge_$v.so; fi
  if [ -n "$TESTS" ]; then
    timeout -k 10 300 $T $TESTS > gpurun_out/ab_$v.tests.log 2>&1; echo "$v tests rc=$?"
  fi
  timeout -k 10 120 python tools/stamp_lm.py 20 1 > gpurun_out/ab_$v.stamp.json 2> gpurun_out/ab_$v.stamp.err
  rc=$?; echo "$v stamp rc=$rc"; [ $rc -gt 1 ] && exit $rc
  timeout -k 10 300 python bench.py --steps 10 --warmup 2 ${BENCH_ARGS} > gpurun_out/ab_$v.bench.log 2>&1
  rc=$?; echo "$v bench rc=$rc"; [ $rc -ne 0 ] && exit $rc
done
exit 0
