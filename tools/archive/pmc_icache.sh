#!/bin/bash
# Instruction-cache counters of the LM kernels (k_lm_solve's fully unrolled
# panels: is the solve instruction-fetch bound?).  One short PMC pass.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out/pmc_icache
export TMPDIR=/tmp
timeout -s KILL 90 rocprofv3 --output-format csv --pmc SQC_ICACHE_MISSES SQC_ICACHE_HITS SQ_WAIT_ANY SQ_IFETCH SQ_WAVES SQ_BUSY_CYCLES \
    -d gpurun_out/pmc_icache -o ic -- python3 tools/stamp_lm.py 16 1 > gpurun_out/pmc_icache/run.log 2>&1 \
    || { echo "rc=$?"; tail -n 20 gpurun_out/pmc_icache/run.log; exit 1; }
python3 - <<'PY'
import csv, collections
agg = collections.defaultdict(lambda: collections.defaultdict(float)); n = collections.defaultdict(set)
for r in csv.DictReader(open("gpurun_out/pmc_icache/ic_counter_collection.csv")):
    k = r["Kernel_Name"].split("(")[0].replace("void rph::", "")[:60]
    agg[k][r["Counter_Name"]] += float(r["Counter_Value"]); n[k].add(r["Dispatch_Id"])
for k, c in agg.items():
    m = len(n[k])
    print(f"{k:60s} n={m}", {a: round(b / m) for a, b in sorted(c.items())})
PY
