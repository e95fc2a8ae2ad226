#!/bin/bash
# Round-4 step d: LM GPU tests, every preset, the grouped-panel A/B and the
# instruction-cache counters.  Test failures do not stop the benches.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_gpu_lm_multistart.py tests/test_gpu_lm.py tests/test_gpu_dp.py \
    tests/test_gpu_gram_side.py -q --timeout 240 --timeout-method thread -p no:cacheprovider > gpurun_out/pt_r4d.log 2>&1
rc=$?; tail -n 12 gpurun_out/pt_r4d.log; [ $rc -gt 1 ] && exit $rc
printf '%s\n' "--steps 20 --warmup 5" "--preset heston30 --steps 10 --warmup 3" "--preset euro252 --steps 5 --warmup 2" \
    "--preset basket5 --steps 3 --warmup 1" > /tmp/r4d_lines.txt
bash tools/sweep_bench.sh /tmp/r4d_lines.txt bench_r4d || exit $?
python - <<'PY'
import json
for l in open("gpurun_out/bench_r4d.jsonl"):
    r = json.loads(l); q = r["quality"]
    print(r["config"]["preset"], round(r["ms_per_step"], 3), q["terminal_pnl_std"], q["terminal_residual_std"], q["V0"])
PY
bash tools/ab_lib.sh grouped || exit $?
bash tools/pmc_icache.sh
