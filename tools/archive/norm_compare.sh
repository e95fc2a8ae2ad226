#!/bin/bash
# Quality of the fused input standardisation: each GPU preset with
# --feature-norm date / global / none (1 GPU), JSON lines into gpurun_out/norm.jsonl.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
for p in ${PRESETS:-euro30 heston30 euro30_mfma}; do
  for fn in ${NORMS:-date none}; do
    echo "=== preset $p norm $fn"
    timeout -k 10 ${PRESET_TIMEOUT:-240} python bench.py --preset $p --steps ${STEPS:-2} --warmup 1 \
        --feature-norm $fn $EXTRA --json-out gpurun_out/n_${p}_$fn.json > gpurun_out/n_${p}_$fn.log 2>&1
    rc=$?
    [ $rc -ne 0 ] && { tail -n 5 gpurun_out/n_${p}_$fn.log; echo "rc=$rc: stopping"; exit $rc; }
    cat gpurun_out/n_${p}_$fn.json >> gpurun_out/norm.jsonl
  done
done
echo ALLDONE
