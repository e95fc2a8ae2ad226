cd "${GRAFT_REPO_ROOT}"
mkdir -p gpurun_out/r4s
export TMPDIR=/tmp
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > gpurun_out/r4s/smoke.log 2>&1 || { tail -20 gpurun_out/r4s/smoke.log; exit 1; }
tail -1 gpurun_out/r4s/smoke.log
timeout -k 10 300 python bench.py > gpurun_out/r4s/bench_default.log 2>&1 || exit 1
tail -1 gpurun_out/r4s/bench_default.log | cut -c1-400
