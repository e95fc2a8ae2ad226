#!/bin/bash
# Where the LM pass kernel's waves spend their cycles (one PMC pass of 8 SQ
# counters over tools/stamp_lm.py 2^20, 1-input net).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out/pmc_stall
export TMPDIR=/tmp
timeout -s KILL 90 rocprofv3 --output-format csv --pmc SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY \
    SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_VMEM SQ_ACTIVE_INST_LDS SQ_INSTS_VMEM_RD \
    -d gpurun_out/pmc_stall -o st -- python3 tools/stamp_lm.py 20 1 > gpurun_out/pmc_stall/run.log 2>&1 \
    || { echo "rc=$?"; tail -n 20 gpurun_out/pmc_stall/run.log; exit 1; }
python3 - <<'PY'
import csv, collections
agg = collections.defaultdict(lambda: collections.defaultdict(float)); n = collections.defaultdict(set)
for r in csv.DictReader(open("gpurun_out/pmc_stall/st_counter_collection.csv")):
    k = r["Kernel_Name"].split("(")[0].replace("void rph::", "")[:60]
    if "k_lm" not in k: continue
    agg[k][r["Counter_Name"]] += float(r["Counter_Value"]); n[k].add(r["Dispatch_Id"])
for k, c in agg.items():
    m = len(n[k])
    print(f"{k:60s} n={m}", {a: round(b / m) for a, b in sorted(c.items())})
PY
