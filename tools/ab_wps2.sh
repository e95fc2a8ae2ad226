#!/bin/bash
# A/B: LM pass kernel at two workgroups per CU (RPH_LM_PAIR_WPS=2 build in
# rphedge/_lib/ab/) vs the default build: pass-phase stamps + euro30 bench.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
AB=rphedge/_lib/ab/librphedge_${1:-wps2}.so
RPH_NATIVE_LIB=$PWD/$AB timeout -k 10 120 python tools/stamp_lm.py 20 1 > gpurun_out/stamp_ab_plain.json || exit 1
RPH_NATIVE_LIB=$PWD/$AB timeout -k 10 120 python tools/stamp_lm.py 20 1 og > gpurun_out/stamp_ab_og.json || exit 1
RPH_NATIVE_LIB=$PWD/$AB timeout -k 10 200 python bench.py --steps 20 --warmup 5 > gpurun_out/bench_ab.log 2>&1 || { tail -5 gpurun_out/bench_ab.log; exit 1; }
python - <<'PY'
import json
for f in ("gpurun_out/stamp_ab_plain.json", "gpurun_out/stamp_ab_og.json"):
    r = json.load(open(f)); p = r["pass_wg_us_min_med_max"]
    print(f, "us/pass", round(r["us_per_pass"], 2), "paths other", p["paths_other_wgs"], "end", p["end_other_wgs"], p["end_gram_wgs"])
r = json.loads(open("gpurun_out/bench_ab.log").read().strip().splitlines()[-1])
print("bench", r["ms_per_step"], r["quality"]["terminal_pnl_std"], r["quality"]["V0"])
PY
