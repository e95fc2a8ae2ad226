cd "${GRAFT_REPO_ROOT}"
for lr in 0 0.03 0.3; do
  BENCH_ARGS="--lm-lam0-rest $lr" LIBS=main tools/archive/seed_sweep.sh || exit 1
  mv gpurun_out/seeds_main.jsonl gpurun_out/seeds_lamrest_$lr.jsonl
done
