#!/bin/bash
# Round-5 GPU step runner: each argument is "name:::command"; every step runs
# under its own timeout, output to gpurun_out/r5/<name>.log; the run stops at
# the first fault / abort / timeout (rc 124/134/137/139 or >128).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
OUT=gpurun_out/r5
mkdir -p $OUT
export TMPDIR=/tmp
fatal() { local rc=$1; [ "$rc" -eq 124 ] || [ "$rc" -eq 134 ] || [ "$rc" -eq 137 ] || [ "$rc" -eq 139 ] || [ "$rc" -gt 128 ]; }
for spec in "$@"; do
  name=${spec%%:::*}; cmd=${spec#*:::}
  echo "=== $name: $cmd"
  t0=$(date +%s)
  bash -c "$cmd" > $OUT/$name.log 2>&1
  rc=$?
  echo "=== $name rc=$rc ($(( $(date +%s) - t0 ))s)"
  tail -n 6 $OUT/$name.log | cut -c1-600
  if fatal $rc; then echo "FATAL in $name (rc=$rc): stopping"; exit $rc; fi
done
echo ALLDONE
