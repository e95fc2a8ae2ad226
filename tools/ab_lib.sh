#!/bin/bash
# A/B of two native-library builds (default vs rphedge/_lib/ab/librphedge_$1.so):
# LM solve/pass stamps (tools/stamp_lm.py) and the euro30 bench, each build.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
for lib in default "$1"; do
  if [ "$lib" = default ]; then unset RPH_NATIVE_LIB; else export RPH_NATIVE_LIB=$PWD/rphedge/_lib/ab/librphedge_$lib.so; fi
  timeout -k 10 120 python tools/stamp_lm.py 20 1 > gpurun_out/ab_stamp_$lib.json || exit 1
  timeout -k 10 200 python bench.py --steps 20 --warmup 5 > gpurun_out/ab_bench_$lib.log 2>&1 || { tail -5 gpurun_out/ab_bench_$lib.log; exit 1; }
done
unset RPH_NATIVE_LIB
python - "$1" <<'PY'
import json, sys
for lib in ("default", sys.argv[1]):
    r = json.load(open(f"gpurun_out/ab_stamp_{lib}.json"))
    b = json.loads(open(f"gpurun_out/ab_bench_{lib}.log").read().strip().splitlines()[-1])
    print(lib, "us/pass", round(r["us_per_pass"], 2), "solve", r.get("tile_solver_us"), "| bench ms", round(b["ms_per_step"], 3),
          "pnl", b["quality"]["terminal_pnl_std"])
PY
