#!/bin/bash
# Same-box A/B of native-library builds: the in-tree library ("default") and
# rphedge/_lib/ab/librphedge_<name>.so for every name given.  Per build: the
# euro30 bench (20 timed steps) and a rocprofv3 kernel-stats run (its own
# process; kernel means from tools/kstats.py).  Output under gpurun_out/ab/.
# usage: bash tools/archive/r5/ab_prof.sh NAME [NAME ...] [-- extra bench args]
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
names=(default)
extra=()
while [ $# -gt 0 ]; do
  if [ "$1" = "--" ]; then shift; extra=("$@"); break; fi
  names+=("$1"); shift
done
OUT=gpurun_out/ab
mkdir -p $OUT
export TMPDIR=/tmp
for lib in "${names[@]}"; do
  if [ "$lib" = default ]; then unset RPH_NATIVE_LIB; else export RPH_NATIVE_LIB=$PWD/rphedge/_lib/ab/librphedge_$lib.so; fi
  timeout -k 10 200 python bench.py --steps 20 --warmup 3 "${extra[@]}" > $OUT/bench_$lib.log 2>&1 || { echo "bench $lib failed"; tail -5 $OUT/bench_$lib.log; exit 1; }
  rm -rf $OUT/prof_$lib
  timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $OUT/prof_$lib -o run -- python3 bench.py --steps 6 --warmup 1 "${extra[@]}" > $OUT/prof_$lib.log 2>&1 || { echo "prof $lib failed"; tail -5 $OUT/prof_$lib.log; exit 1; }
done
unset RPH_NATIVE_LIB
for lib in "${names[@]}"; do
  python3 - "$lib" "$OUT" <<'PY'
import json, sys
lib, out = sys.argv[1], sys.argv[2]
b = json.loads([l for l in open(f"{out}/bench_{lib}.log") if l.startswith("{")][-1])
print(lib, "ms", round(b["ms_per_step"], 3), "pnl", repr(b["quality"]["terminal_pnl_std"]), "V0", b["quality"]["V0"])
PY
  db=$(find $OUT/prof_$lib -name "*results.db" | head -1)
  [ -n "$db" ] && python3 tools/kstats.py "$db" rph | head -6
done
