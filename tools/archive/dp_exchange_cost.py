"""Cost of the in-kernel DP exchange of the lagged schedule, measured on ONE
GPU: W processes share the card (IPC mailboxes in local HBM instead of peer
HBM over xGMI), each runs a lag-mode fit with a small grid (all ranks' grids
co-resident), and the per-step time is compared with one process.  This
isolates the protocol (push, sentinel wait, tagged reads, fixed-order sum);
xGMI link latency comes on top on a real multi-GPU node.

usage: python tools/archive/dp_exchange_cost.py [W] [batch_log2_per_rank]"""
import json
import os
import socket
import sys
import tempfile

import torch
import torch.multiprocessing as mp

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def _fit_time(world, rank, n, bl2, mb, epochs=200):
    from rphedge.engine import DateData, FitConfig, HipBackend, TrainConfig
    from rphedge.models.hedge_mlp import NetSpec, init_weights

    dev = torch.device("cuda", 0)
    spec = NetSpec(nin=1, hidden=8, nout=2, head=0)
    g = torch.Generator().manual_seed(rank)
    x = (torch.rand(n, generator=g) * 0.6 + 0.7).to(dev)
    tc = TrainConfig(batch_size=(1 << bl2) * world, chunk_log2=6, step_mode="lag")
    be = HipBackend(spec, n, tc, device=dev, world=world, rank=rank, mailbox=mb)
    data = DateData(feats=[x], prices_next=[x * 1.01], bond_next=1.0, target=torch.relu(x - 1.0), prices_now=[x])
    fc = FitConfig(epochs=epochs, patience=10 ** 6, early_stopping=False)
    w0 = init_weights(spec, [0.5, 0.0])
    times = []
    for _ in range(3):
        w, o, f = be.new_weights(w0), be.new_opt(), be.new_fit()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        be.fit(w, o, f, data, fc, seed=1)
        e1.record()
        torch.cuda.synchronize()
        times.append(e0.elapsed_time(e1) * 1e3 / (epochs * be.steps_per_epoch))
    return min(times), be.num_wgs, be.step_mode()


def _worker(rank, world, port, n, bl2, out):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    import torch.distributed as dist
    from torch.distributed import distributed_c10d as c10d

    from rphedge.ops.native import IpcMailbox

    torch.cuda.set_device(0)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    mb = IpcMailbox(rank, world, 128, c10d._get_default_store(), torch.device("cuda", 0), tag="dpcost")
    dist.barrier()
    t, wgs, mode = _fit_time(world, rank, n, bl2, mb)
    mb.check()
    if rank == 0:
        with open(out, "w") as f:
            json.dump({"us_per_step": t, "num_wgs": wgs, "mode": mode}, f)
    dist.barrier()
    mb.close()
    dist.destroy_process_group()


if __name__ == "__main__":
    W = int(sys.argv[1]) if len(sys.argv) > 1 else 2
    bl2 = int(sys.argv[2]) if len(sys.argv) > 2 else 14
    n = 1 << (bl2 + 2)
    t1, wgs1, m1 = _fit_time(1, 0, n, bl2, None)
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    with tempfile.TemporaryDirectory() as td:
        out = os.path.join(td, "r.json")
        ctx = mp.get_context("spawn")
        ps = [ctx.Process(target=_worker, args=(r, W, port, n, bl2, out)) for r in range(W)]
        for p in ps:
            p.start()
        for p in ps:
            p.join(300)
        rw = json.load(open(out))
    print(json.dumps({"world": W, "batch_per_rank_log2": bl2, "num_wgs": wgs1, "single_us_per_step": t1,
                      "dp_us_per_step": rw["us_per_step"], "dp_mode": rw["mode"],
                      "exchange_cost_us": rw["us_per_step"] - t1}), flush=True)
