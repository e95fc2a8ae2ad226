#!/bin/bash
# Run bench.py for every GPU BASELINE preset (1 GPU), one JSON line each into
# gpurun_out/presets.jsonl; stops at the first fault/timeout.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
for p in ${PRESETS:-euro30 heston30 euro252 basket5}; do
  echo "=== preset $p"
  timeout -k 10 ${PRESET_TIMEOUT:-300} python bench.py --preset $p --steps ${STEPS:-3} --warmup 1 \
      --json-out gpurun_out/preset_$p.json > gpurun_out/preset_$p.log 2>&1
  rc=$?
  tail -n 3 gpurun_out/preset_$p.log
  [ $rc -ne 0 ] && { echo "preset $p rc=$rc: stopping"; exit $rc; }
  cat gpurun_out/preset_$p.json >> gpurun_out/presets.jsonl
done
echo ALLDONE
