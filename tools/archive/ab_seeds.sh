#!/bin/bash
# A/B of a library build on euro30 quality and time: stamps (default vs
# variant) and seeds 1-8 with the variant library.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
V=$1
export RPH_NATIVE_LIB=$PWD/rphedge/_lib/ab/librphedge_$V.so
timeout -k 10 120 python tools/stamp_lm.py 20 1 > gpurun_out/ab_stamp_$V.json || exit 1
: > gpurun_out/ab_seeds_$V.jsonl
for s in 1 2 3 4 5 6 7 8; do
  timeout -k 10 200 python bench.py --steps 5 --warmup 2 --seed $s > gpurun_out/ab_one.log 2>&1 || { tail -n 20 gpurun_out/ab_one.log; exit 1; }
  tail -n 1 gpurun_out/ab_one.log >> gpurun_out/ab_seeds_$V.jsonl
done
python3 - "$V" <<'PY'
import json, sys, numpy as np
v = sys.argv[1]
r = json.load(open(f"gpurun_out/ab_stamp_{v}.json"))
rows = [json.loads(l) for l in open(f"gpurun_out/ab_seeds_{v}.jsonl")]
p = [x["quality"]["terminal_pnl_std"] for x in rows]; ms = [x["ms_per_step"] for x in rows]
print(v, "us/pass", round(r["us_per_pass"], 2), "solve", r.get("tile_solver_us", {}).get("factor_total"),
      "| ms", round(np.mean(ms), 2), "pnl", np.round(p, 4).tolist(), "mean", round(np.mean(p), 4), "worst", round(max(p), 4))
PY
