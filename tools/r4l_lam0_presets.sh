cd "${GRAFT_REPO_ROOT:-.}"
mkdir -p gpurun_out
: > gpurun_out/l0.jsonl
for s in 1 2 3; do
  timeout -k 10 300 python bench.py --preset heston30 --steps 3 --warmup 1 --seed $s --lm-lam0-first 16.384000778198242 --lm-explore-passes 38 > gpurun_out/one.log 2>&1 || { tail -20 gpurun_out/one.log; exit 1; }
  tail -n 1 gpurun_out/one.log >> gpurun_out/l0.jsonl
done
for s in 1 2; do
  timeout -k 10 300 python bench.py --preset basket5 --steps 2 --warmup 1 --seed $s --lm-lam0-first 16.384000778198242 --lm-explore-passes 33 > gpurun_out/one.log 2>&1 || { tail -20 gpurun_out/one.log; exit 1; }
  tail -n 1 gpurun_out/one.log >> gpurun_out/l0.jsonl
done
python3 - <<'PY'
import json
for l in open("gpurun_out/l0.jsonl"):
    r = json.loads(l); q = r["quality"]
    print(r["config"]["preset"], r["config"].get("seed"), round(r["ms_per_step"], 2), round(q["terminal_pnl_std"], 4), round(q["V0"], 4))
PY
