cd "${GRAFT_REPO_ROOT}"
mkdir -p gpurun_out/r4n
export TMPDIR=/tmp
timeout -k 10 120 python tools/stamp_lm.py 20 1 > gpurun_out/r4n/stamp.json || exit 1
for i in 1 2 3; do timeout -k 10 200 python bench.py --steps 20 --warmup 5 > gpurun_out/r4n/bench_$i.log 2>&1 || exit 1; done
timeout -k 10 600 python -u -m pytest tests -m gpu -q -x --timeout 300 --timeout-method thread -p no:cacheprovider -k "lm or chol or solve or basket or distributed" > gpurun_out/r4n/pt.log 2>&1; rc=$?; tail -3 gpurun_out/r4n/pt.log; exit $rc
