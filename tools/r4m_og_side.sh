cd "${GRAFT_REPO_ROOT:-.}"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests/test_gpu_lm_multistart.py tests/test_gpu_lm.py tests/test_gpu_gram_side.py -q --timeout 240 --timeout-method thread -p no:cacheprovider > gpurun_out/pt_side.log 2>&1
rc=$?; tail -n 4 gpurun_out/pt_side.log; [ $rc -gt 1 ] && exit $rc
for v in 1 0; do
  RPH_LM_OG_SIDE=$v timeout -k 10 200 python bench.py --steps 20 --warmup 5 > gpurun_out/bs.log 2>&1 || { tail -20 gpurun_out/bs.log; exit 1; }
  echo "og_side=$v $(tail -n 1 gpurun_out/bs.log | python3 -c 'import json,sys; r=json.loads(sys.stdin.read()); print(r["ms_per_step"], r["quality"]["terminal_pnl_std"], r["quality"]["V0"])')"
done
timeout -k 10 300 rocprofv3 --kernel-trace -d gpurun_out/trace_side -o tr -- python3 bench.py --steps 5 --warmup 2 > gpurun_out/trace_side.log 2>&1 && python3 tools/trace_gaps.py gpurun_out/trace_side/tr_results.db | head -9
