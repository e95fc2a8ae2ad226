#!/bin/bash
# Round-4 diagnostics: pass-phase stamps of the plain and the output-Gram LM
# pass, and PMC counters of the MFMA-gradient A/B pass body (VALU vs MFMA).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out/pmc_r4
export TMPDIR=/tmp
timeout -k 10 120 python tools/stamp_lm.py 20 1 > gpurun_out/stamp_r4_plain.json 2> gpurun_out/stamp_r4.err || exit 1
timeout -k 10 120 python tools/stamp_lm.py 20 1 og > gpurun_out/stamp_r4_og.json 2>> gpurun_out/stamp_r4.err || exit 1
for mg in 0 1; do
  RPH_LM_MFMA_GRAD=$mg timeout -s KILL 120 rocprofv3 --output-format csv \
      --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_MFMA SQ_VALU_MFMA_BUSY_CYCLES SQ_ACTIVE_INST_VALU SQ_INSTS_LDS SQ_WAIT_INST_LDS SQ_BUSY_CYCLES \
      -d gpurun_out/pmc_r4/mg$mg -o pmc -- python3 bench.py --steps 1 --warmup 0 > gpurun_out/pmc_r4/mg$mg.log 2>&1 \
      || { echo "pmc mg=$mg rc=$?"; tail -n 15 gpurun_out/pmc_r4/mg$mg.log; exit 1; }
done
echo ok
