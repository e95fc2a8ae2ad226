#!/bin/bash
# DP rehearsal of the bench on ONE GPU (2 and 4 ranks share the card; RCCL
# or the mailbox transport between processes), + the multi-start preset.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp HSA_ENABLE_IPC_MODE_LEGACY=0
for n in 2 4; do
  timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node $n --master-addr 127.0.0.1 --master-port $((29500 + n)) \
      bench.py --gpus $n --steps 5 --warmup 2 > gpurun_out/dp$n.log 2>&1 || { echo "dp$n rc=$?"; tail -n 30 gpurun_out/dp$n.log; exit 1; }
  grep '^{' gpurun_out/dp$n.log | tail -n 1 | python3 -c "
import json,sys; r=json.loads(sys.stdin.read()); print('dp', r['n_gpus'], r['ms_per_step'], r['quality']['terminal_pnl_std'], r['quality']['V0'], r.get('lm_exchange'), r['config'].get('lm_dp_transport'))"
done
timeout -k 10 300 python bench.py --preset euro30_ms --steps 10 --warmup 3 > gpurun_out/ms_preset.log 2>&1 && tail -n 1 gpurun_out/ms_preset.log | cut -c1-200
