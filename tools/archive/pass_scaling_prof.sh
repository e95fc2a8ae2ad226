#!/bin/bash
cd "${GRAFT_REPO_ROOT}"
export TMPDIR=/tmp
for n in 20 19 18; do
  timeout -k 10 120 rocprofv3 --kernel-trace --stats -d gpurun_out/pp$n -o run --output-format csv -- python3 tools/stamp_lm.py $n 1 > gpurun_out/pp$n.log 2>&1 || exit 1
done
