#!/bin/bash
# GPU: the flagship bench over weight-init seeds for library variants
# ($LIBS; "main" = in-tree) -> gpurun_out/seeds_<lib>.jsonl
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
for v in ${LIBS:-main}; do
  if [ "$v" = main ]; then unset RPH_NATIVE_LIB; else export RPH_NATIVE_LIB=rphedge/_lib/ab/librphedge_$v.so; fi
  : > gpurun_out/seeds_$v.jsonl
  for s in ${SEEDS:-1 2 3 4 5 6 7 8}; do
    timeout -k 10 200 python bench.py --steps 3 --warmup 1 --seed $s ${BENCH_ARGS} > gpurun_out/seed_one.log 2>&1 || { tail -n 20 gpurun_out/seed_one.log; exit 1; }
    tail -n 1 gpurun_out/seed_one.log >> gpurun_out/seeds_$v.jsonl
  done
  echo "$v done"
done
