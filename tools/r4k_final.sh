#!/bin/bash
# eval-grid sweep + the default euro30's kernel statistics (replay kernels)
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
for w in 512 1024 2048; do
  RPH_EVAL_WGS=$w timeout -k 10 200 python bench.py --steps 20 --warmup 5 > gpurun_out/ew.log 2>&1 || { tail -20 gpurun_out/ew.log; exit 1; }
  echo "eval_wgs $w $(tail -n 1 gpurun_out/ew.log | python3 -c 'import json,sys; r=json.loads(sys.stdin.read()); print(r["ms_per_step"], r["quality"]["terminal_pnl_std"])')"
done
timeout -k 10 300 rocprofv3 --kernel-trace -d gpurun_out/trace_fin -o tr -- python3 bench.py --steps 10 --warmup 3 > gpurun_out/trace_fin.log 2>&1 || { tail -20 gpurun_out/trace_fin.log; exit 1; }
python3 tools/trace_gaps.py gpurun_out/trace_fin/tr_results.db | head -8
python3 tools/rocpd_stats.py gpurun_out/trace_fin/tr_results.db gpurun_out/rocprof_r4_final_kernel_stats.csv > /dev/null
