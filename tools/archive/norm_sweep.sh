#!/bin/bash
# Seed sweeps of bench.py variants in one GPU call (round 6: horizon-aware input
# standardisation A/B).  usage: bash tools/norm_sweep.sh OUTDIR SEEDS VARIANT...
#   VARIANT = preset~flag=value~flag=value (bench.py flags without the dashes),
#   e.g. euro252~feature-norm=horizon~feature-norm-floor=0.1
set -o pipefail
out=$1; seeds=$2; shift 2
mkdir -p "$out"
for v in "$@"; do
  IFS='~' read -ra parts <<< "$v"
  args=(--preset "${parts[0]}")
  for kv in "${parts[@]:1}"; do args+=("--${kv%%=*}" "${kv#*=}"); done
  name=$(echo "$v" | tr '~=' '_-')
  sd=$seeds
  [[ "$v" == basket5* ]] && sd=${BASKET_SEEDS:-$seeds}
  timeout -k 10 ${VTIMEOUT:-400} python -u tools/seeds.py "$out/$name.jsonl" "$sd" --steps 2 --warmup 1 "${args[@]}" \
    > "$out/$name.log" 2>&1 || { echo "FAILED $name"; exit 1; }
  echo "done $name"
done
