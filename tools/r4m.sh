cd "${GRAFT_REPO_ROOT}"
mkdir -p gpurun_out/r4m
export TMPDIR=/tmp
for i in 1 2 3; do timeout -k 10 200 python bench.py --steps 20 --warmup 5 > gpurun_out/r4m/bench_$i.log 2>&1 || exit 1; done
timeout -k 10 120 python tools/stamp_lm.py 20 1 > gpurun_out/r4m/stamp.json || exit 1
cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $GRAFT_REPO_ROOT/gpurun_out/r4m/prof -o run --output-format csv -- python3 $GRAFT_REPO_ROOT/bench.py --steps 10 --warmup 3 > $GRAFT_REPO_ROOT/gpurun_out/r4m/prof.log 2>&1 || exit 1
cd $GRAFT_REPO_ROOT && timeout -k 10 600 python -u -m pytest tests -m gpu -q -x --timeout 300 --timeout-method thread -p no:cacheprovider -k "lm or reduce or distributed or parity" > gpurun_out/r4m/pt.log 2>&1; rc=$?; tail -3 gpurun_out/r4m/pt.log; exit $rc
