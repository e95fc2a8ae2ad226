cd "${GRAFT_REPO_ROOT}"
for v in main wps1; do
  if [ $v = main ]; then unset RPH_NATIVE_LIB; else export RPH_NATIVE_LIB=rphedge/_lib/ab/librphedge_$v.so; fi
  for k in 0 2 3; do
    RPH_LM_GRAM_SKIP=$k timeout -k 10 120 python tools/stamp_lm.py 20 1 > gpurun_out/gs_${v}_$k.json 2>/dev/null || exit 1
    RPH_LM_GRAM_SKIP=$k timeout -k 10 200 python bench.py --steps 10 --warmup 2 > gpurun_out/gs_${v}_$k.bench 2>&1 || exit 1
    echo "$v $k done"
  done
done
