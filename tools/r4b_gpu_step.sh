cd "${GRAFT_REPO_ROOT:-.}"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 python -u tools/og_diag.py 13 20 > gpurun_out/og_diag.log 2>&1 || { cat gpurun_out/og_diag.log; exit 1; }
cat gpurun_out/og_diag.log
timeout -k 10 400 python -u -m pytest tests/test_gpu_lm_multistart.py tests/test_gpu_lm.py -q --timeout 240 --timeout-method thread -p no:cacheprovider > gpurun_out/pt_r4b.log 2>&1
rc=$?; tail -n 6 gpurun_out/pt_r4b.log; [ $rc -gt 1 ] && exit $rc
timeout -k 10 200 python bench.py --steps 20 --warmup 5 > gpurun_out/b4b.log 2>&1 || { tail -5 gpurun_out/b4b.log; exit 1; }
python -c "
import json; r=json.loads(open('gpurun_out/b4b.log').read().strip().splitlines()[-1]); q=r['quality']
print('euro30', r['ms_per_step'], q['terminal_pnl_std'], q['V0'])"
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_r4b -o r4b -- python3 bench.py --steps 10 --warmup 3 > gpurun_out/prof_r4b.log 2>&1 || { echo rocprof failed; exit 1; }
