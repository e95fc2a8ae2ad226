#!/bin/bash
# PMC passes over the LM kernels of the flagship bench (matrix-core use of
# k_lm_pass / k_lm_solve); one counter group per run, each run bounded.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out
i=0
while read -r grp; do
  [ -z "$grp" ] && continue
  i=$((i+1))
  echo "=== pmc pass $i: $grp"
  timeout -s KILL 120 rocprofv3 --pmc $grp --kernel-include-regex 'k_lm_' \
      -d gpurun_out/pmc_lm_$i -o run --output-format csv -- python3 bench.py --steps 1 --warmup 0 ${BENCH_ARGS} \
      > gpurun_out/pmc_lm_$i.log 2>&1
  rc=$?
  tail -n 2 gpurun_out/pmc_lm_$i.log
  [ $rc -ne 0 ] && { echo "pmc pass $i rc=$rc: stopping"; exit $rc; }
done <<'GROUPS'
SQ_WAVES SQ_INSTS_VALU SQ_INSTS_VALU_MFMA_F32 SQ_INSTS_VALU_MFMA_F64 SQ_VALU_MFMA_BUSY_CYCLES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_INSTS_LDS
GROUPS
echo ALLDONE
