#!/bin/bash
# GPU: run bench.py once per argument line of $1 (one JSON line each, into
# gpurun_out/$2.jsonl); every run under its own time limit, stop at the first
# failure.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
out=gpurun_out/${2:-sweep}.jsonl
: > "$out"
while IFS= read -r line; do
  [ -z "$line" ] && continue
  echo "== $line"
  timeout -k 10 ${SWEEP_TIMEOUT:-240} python bench.py $line > gpurun_out/sweep_one.log 2>&1
  rc=$?
  if [ $rc -ne 0 ]; then echo "rc=$rc for: $line"; tail -n 20 gpurun_out/sweep_one.log; exit $rc; fi
  tail -n 1 gpurun_out/sweep_one.log >> "$out"
done < "$1"
