#!/bin/bash
# The whole GPU test suite (as the round-end driver runs it), one process,
# per-test time limits; the summary line and failures to stdout.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp HSA_ENABLE_IPC_MODE_LEGACY=0
timeout -k 10 1150 python -u -m pytest tests -m gpu -q --timeout 300 --timeout-method thread -p no:cacheprovider \
    -rf ${PYTEST_EXTRA} > gpurun_out/pt_full.log 2>&1
rc=$?
grep -E "^(FAILED|ERROR)|passed|failed" gpurun_out/pt_full.log | tail -n 30
exit $rc
