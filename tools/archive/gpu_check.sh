#!/bin/bash
# GPU validation round: smoke -> pytest -m gpu -> bench -> rocprofv3 kernel stats.
# Stops at the first fault/abort/timeout (rc 124/134/137/139 or >128); a plain
# test failure (rc 1) still lets the bench run.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out
mkdir -p $OUT
export TMPDIR=/tmp
STEPS=${STEPS:-smoke,tests,bench,prof}
fatal() { local rc=$1; [ "$rc" -eq 124 ] || [ "$rc" -eq 134 ] || [ "$rc" -eq 137 ] || [ "$rc" -eq 139 ] || [ "$rc" -gt 128 ]; }
run() {
  local name=$1; shift
  echo "=== $name: $*" | tee -a $OUT/steps.log
  local t0=$(date +%s)
  "$@" > $OUT/$name.log 2>&1
  local rc=$?
  echo "=== $name rc=$rc ($(( $(date +%s) - t0 ))s)" | tee -a $OUT/steps.log
  tail -n 25 $OUT/$name.log
  if fatal $rc; then echo "FATAL in $name (rc=$rc): stopping"; exit $rc; fi
  return 0
}
[[ $STEPS == *smoke* ]] && run smoke timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()"
[[ $STEPS == *tests* ]] && run pytest_gpu timeout -k 10 600 python -m pytest tests -m gpu -q -p no:cacheprovider --timeout=240 ${PYTEST_ARGS}
[[ $STEPS == *bench* ]] && run bench timeout -k 10 420 python bench.py --steps ${BENCH_STEPS:-5} --warmup 2 ${BENCH_ARGS}
if [[ $STEPS == *prof* ]]; then
  run rocprof timeout -k 10 420 rocprofv3 --kernel-trace --stats -d $OUT/prof -o run --output-format csv -- python3 bench.py --steps 2 --warmup 1 ${BENCH_ARGS}
fi
echo ALLDONE
