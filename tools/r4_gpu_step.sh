#!/bin/bash
# Round-4 GPU step: the new / changed GPU tests first (world-invariant Gram
# subsample, DP exchange, LM, output-layer Gram on the matrix cores), then the
# default bench, its round-3 equivalent (lam0 1e-3, 80 first-date passes) and
# the MFMA-gradient A/B body, the other presets, and a kernel-stats profile.
# Test FAILURES do not stop the step (the benches are independent of them);
# a crash, abort or time limit does.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest ${R4_TESTS:-tests/test_gpu_gram_side.py tests/test_gpu_lm_multistart.py \
    tests/test_gpu_lm.py tests/test_gpu_dp.py} -q --timeout 240 --timeout-method thread -p no:cacheprovider \
    > gpurun_out/pt_r4.log 2>&1
rc=$?; tail -n 12 gpurun_out/pt_r4.log
[ $rc -gt 1 ] && { echo "pytest rc=$rc: stopping"; exit $rc; }
printf '%s\n' "--steps 20 --warmup 5" "--steps 20 --warmup 5 --lm-lam0-first 0 --lm-passes-first 80" > /tmp/r4_lines.txt
bash tools/sweep_bench.sh /tmp/r4_lines.txt bench_r4a || exit $?
printf '%s\n' "--steps 20 --warmup 5" > /tmp/r4_mg.txt
RPH_LM_MFMA_GRAD=1 bash tools/sweep_bench.sh /tmp/r4_mg.txt bench_r4a_mg || exit $?
cat gpurun_out/bench_r4a_mg.jsonl >> gpurun_out/bench_r4a.jsonl
printf '%s\n' "--preset heston30 --steps 10 --warmup 3" "--preset euro252 --steps 5 --warmup 2" \
    "--preset basket5 --steps 3 --warmup 1" > /tmp/r4_presets.txt
bash tools/sweep_bench.sh /tmp/r4_presets.txt bench_r4a_presets || exit $?
python - <<'PY'
import json
for f in ("gpurun_out/bench_r4a.jsonl", "gpurun_out/bench_r4a_presets.jsonl"):
    for l in open(f):
        r = json.loads(l); q = r.get("quality", {}); lm = (r.get("lm") or {}).get("first_date") or {}
        print(r["config"]["model"], round(r["ms_per_step"], 3), q.get("terminal_pnl_std"), q.get("terminal_residual_std"),
              q.get("V0"), lm.get("best_loss"))
PY
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_r4a -o r4a -- python3 bench.py --steps 10 --warmup 3 \
    > gpurun_out/prof_r4a.log 2>&1 || { echo "rocprof rc=$?"; tail -n 20 gpurun_out/prof_r4a.log; exit 1; }
find gpurun_out/prof_r4a -name '*kernel_stats.csv'
