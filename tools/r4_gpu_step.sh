#!/bin/bash
# Round-4 GPU step: the new / changed GPU tests first (world-invariant Gram
# subsample, DP exchange, LM, output-layer Gram on the matrix cores), then the
# default bench and its round-3 equivalent (lam0 1e-3, 80 first-date passes),
# stop at the first failure.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
timeout -k 10 700 python -u -m pytest tests/test_gpu_gram_side.py tests/test_gpu_lm_multistart.py tests/test_gpu_lm.py \
    tests/test_gpu_dp.py -x -q --timeout 300 --timeout-method thread -p no:cacheprovider > gpurun_out/pt_r4.log 2>&1
rc=$?; tail -8 gpurun_out/pt_r4.log; [ $rc -ne 0 ] && exit $rc
printf '%s\n' "--steps 20 --warmup 5" "--steps 20 --warmup 5 --lm-lam0-first 0 --lm-passes-first 80" > /tmp/r4_lines.txt
bash tools/sweep_bench.sh /tmp/r4_lines.txt bench_r4a || exit $?
printf '%s\n' "--steps 20 --warmup 5" > /tmp/r4_mg.txt
RPH_LM_MFMA_GRAD=1 bash tools/sweep_bench.sh /tmp/r4_mg.txt bench_r4a_mg || exit $?
cat gpurun_out/bench_r4a_mg.jsonl >> gpurun_out/bench_r4a.jsonl
python - <<'PY'
import json
for l in open("gpurun_out/bench_r4a.jsonl"):
    r = json.loads(l); q = r["quality"]
    print(round(r["ms_per_step"], 3), q["terminal_pnl_std"], q["terminal_residual_std"], q["V0"], r["lm"]["first_date"]["best_loss"])
PY
