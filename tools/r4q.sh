cd "${GRAFT_REPO_ROOT}"
mkdir -p gpurun_out/r4q
export TMPDIR=/tmp
timeout -k 10 120 python tools/stamp_lm.py 20 1 > gpurun_out/r4q/stamp.json || exit 1
for i in 1 2 3; do timeout -k 10 200 python bench.py --steps 20 --warmup 5 > gpurun_out/r4q/bench_$i.log 2>&1 || exit 1; done
bash tools/gpu_full_tests.sh
