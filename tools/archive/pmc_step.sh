#!/bin/bash
# PMC passes over the flagship bench (one counter group per run; each run
# bounded).  Output: gpurun_out/pmc_<n>/...counter_collection.csv
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out
i=0
while read -r grp; do
  [ -z "$grp" ] && continue
  i=$((i+1))
  echo "=== pmc pass $i: $grp"
  timeout -s KILL 120 rocprofv3 --pmc $grp --kernel-include-regex 'k_hedge_step_lag|k_hedge_eval|k_sim_scan' \
      -d gpurun_out/pmc_$i -o run --output-format csv -- python3 bench.py --steps 1 --warmup 0 ${BENCH_ARGS} \
      > gpurun_out/pmc_$i.log 2>&1
  rc=$?
  tail -n 2 gpurun_out/pmc_$i.log
  [ $rc -ne 0 ] && { echo "pmc pass $i rc=$rc: stopping"; exit $rc; }
done <<'GROUPS'
SQ_WAVES SQ_INSTS_VALU SQ_ACTIVE_INST_VALU SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_INSTS_SALU SQ_INSTS_LDS SQ_WAIT_INST_ANY
SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_ACTIVE_INST_LDS SQ_INST_CYCLES_VMEM_RD SQ_WAIT_ANY SQ_ACTIVE_INST_ANY GRBM_GUI_ACTIVE GRBM_COUNT
TCC_HIT_sum TCC_MISS_sum TCC_EA0_RDREQ_sum TCC_EA0_WRREQ_sum
GROUPS
echo ALLDONE
