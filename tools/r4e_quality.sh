#!/bin/bash
# Round-4 quality step: euro30 over 8 weight-init seeds, the presets over 3
# seeds, basket5 at 2^25 paths; every run under its own limit.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
run() {  # out-file, args...
  local out=$1; shift
  timeout -k 10 300 python bench.py "$@" > gpurun_out/q_one.log 2>&1 || { echo "rc=$? for $*"; tail -n 20 gpurun_out/q_one.log; exit 1; }
  tail -n 1 gpurun_out/q_one.log >> gpurun_out/$out
}
: > gpurun_out/q_euro30.jsonl; : > gpurun_out/q_presets.jsonl
for s in 1 2 3 4 5 6 7 8; do run q_euro30.jsonl --steps 5 --warmup 2 --seed $s; echo "euro30 seed $s"; done
for p in heston30 euro252; do for s in 1 2 3; do run q_presets.jsonl --preset $p --steps 3 --warmup 1 --seed $s; echo "$p seed $s"; done; done
for s in 1 2; do run q_presets.jsonl --preset basket5 --steps 2 --warmup 1 --seed $s; echo "basket5 seed $s"; done
run q_presets.jsonl --preset basket5 --steps 1 --warmup 1 --paths-log2 25
python3 - <<'PY'
import json, numpy as np
for f in ("gpurun_out/q_euro30.jsonl", "gpurun_out/q_presets.jsonl"):
    rows = [json.loads(l) for l in open(f)]
    for r in rows:
        q = r["quality"]
        print(r["config"]["preset"], r["config"].get("seed"), r["config"]["paths_per_gpu"], round(r["ms_per_step"], 2),
              round(q["terminal_pnl_std"], 4), round(q["terminal_residual_std"], 4), round(q["V0"], 4))
PY
