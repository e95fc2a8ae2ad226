#!/bin/bash
# Run the notebook-equivalent example scripts and the CLI end to end on one GPU,
# one log per step under gpurun_out/examples/; stops at the first fault or timeout.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/examples
export PYTHONPATH="$PWD${PYTHONPATH:+:$PYTHONPATH}"  # the example scripts import rphedge from the repo root
mkdir -p $OUT
step() {
  local name=$1 secs=$2; shift 2
  echo "=== $name: $*"
  local t0=$(date +%s)
  timeout -k 10 "$secs" "$@" > $OUT/$name.log 2>&1
  local rc=$?
  echo "=== $name rc=$rc ($(( $(date +%s) - t0 ))s)"
  tail -n 12 $OUT/$name.log
  # a plain error (rc 1) lets the next script run; a fault/abort/timeout ends the call
  if [ $rc -eq 124 ] || [ $rc -gt 128 ]; then echo "stopping after $name"; exit $rc; fi
  [ $rc -ne 0 ] && FAILED="$FAILED $name"
  return 0
}
step info 120 python -m rphedge info
step cli_run_euro30 300 python -m rphedge run --config examples/euro_call_30.json --out /tmp/rph_euro30_model && ls -la /tmp/rph_euro30_model >> $OUT/cli_run_euro30.log
step cli_run_heston30 300 python -m rphedge run --config examples/heston_call_30.json
step cli_run_basket5 300 python -m rphedge run --config examples/basket5_call.json
step european 300 python examples/european_options.py
step single_time_step 300 python examples/single_time_step.py
step multi_time_step 600 python examples/multi_time_step.py --sweep --sv
step stochastic_volatility 300 python examples/stochastic_volatility.py
[ -n "$FAILED" ] && { echo "FAILED:$FAILED"; exit 1; }
echo ALLDONE
