#!/usr/bin/env python
"""Flagship benchmark: MC paths/sec training a 30-step hedge MLP + terminal P&L std.

BASELINE.json metric: "MC paths/sec training 30-step hedge-MLP + terminal P&L
std-dev, 1/2/4/8 MI355X"; config "European call, 30-step GBM, 1M Sobol paths,
bf16 hedge-MLP on 1 MI355X".

One benchmark STEP = one complete replicating-portfolio training run, captured
as ONE hipGraph and replayed:
  Sobol/ndtri + log-GBM path kernel (2^20 paths per GPU, 30 dates) -> call payoff
  -> backward induction over the 30 dates (per date: E epochs of minibatch
  Keras-Adam on the hedge MLP 1-8-8-2, fused train-step kernels, RCCL gradient
  all-reduce per step when N>1) -> value/holdings/residual epilogue per date
  (terminal one-step P&L statistics included).
Nothing is skipped inside the timed region; weights and Adam state are reset
from the same initialisation at the start of every replay.

value = training path-samples per second over the whole job
      = (global paths x sum over dates of epochs) / seconds per run,
i.e. the same unit as the reference's Keras throughput (BASELINE.md:
"Keras training step, batch 512 ... ≈85 k samples/s"), so
vs_baseline = value / 85,333.  Scaling is weak (2^20 paths per GPU).
Compute dtype is fp32 (>= the bf16 the config names).
"""
from __future__ import annotations

import argparse
import json
import math
import os
import sys
import time

import torch

BASELINE_SAMPLES_PER_S = 512 / 0.006   # median 6 ms per 512-sample Keras step
METRIC = "MC paths/sec training 30-step hedge-MLP + terminal P&L std-dev, 1/2/4/8 MI355X"


def parse(argv=None):
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=5)
    ap.add_argument("--warmup", type=int, default=2)
    ap.add_argument("--paths-log2", type=int, default=20, help="paths PER GPU (weak scaling)")
    ap.add_argument("--dates", type=int, default=30)
    ap.add_argument("--epochs-first", type=int, default=512)
    ap.add_argument("--epochs-rest", type=int, default=12)
    ap.add_argument("--batch-log2", type=int, default=18, help="per-GPU minibatch (global = N x this)")
    ap.add_argument("--lr", type=float, default=2e-2)
    ap.add_argument("--lr-rest", type=float, default=4e-3)
    ap.add_argument("--lr-decay", type=float, default=0.02, help="per-date geometric LR decay factor (last/first epoch)")
    ap.add_argument("--hidden", type=int, default=8, help="hidden width (8 = reference net; 32 = MFMA kernel)")
    ap.add_argument("--mfma-precision", default="bf16", choices=["bf16", "fp32"])
    ap.add_argument("--no-graph", action="store_true")
    ap.add_argument("--cpu", action="store_true", help="torch reference backend (plumbing only)")
    ap.add_argument("--json-out", default=None)
    return ap.parse_args(argv)


def build_run(a, world: int):
    from rphedge.config import RunConfig, TrainingParams, ParityFlags
    from rphedge.api import HedgeRun

    tr = TrainingParams(batch_size=(1 << a.batch_log2) * world, epochs_first=a.epochs_first,
                        epochs_rest=a.epochs_rest, patience_first=10 ** 6, patience_rest=10 ** 6,
                        lr=a.lr, lr_schedule_first=False, early_stopping=False, q99=False, shuffle=True,
                        chunk_log2=6, seed=1234, hidden=a.hidden, mfma_precision=a.mfma_precision)
    cfg = RunConfig(Y=100.0, K=100.0, T=1.0, mu=0.08, r=0.08, sigma=0.15, rebalancing=1.0 / a.dates,
                    dt=1.0 / a.dates, n_paths=a.paths_log2 + int(math.log2(world)), payoff="call",
                    option_type="CALL", model="gbm_log", mortality=False, N=1, P=1.0, keep_paths=False,
                    verbose=False, train=tr, parity=ParityFlags(), backend="torch" if a.cpu else None)
    return cfg


def main(argv=None):
    a = parse(argv)
    world = int(os.environ.get("WORLD_SIZE", "1"))
    if world != a.gpus:
        if a.gpus > 1 and world == 1:
            print(f"bench.py: --gpus {a.gpus} needs torch.distributed.run with {a.gpus} processes", file=sys.stderr)
            return 2
    from rphedge.parallel import dist as D
    from rphedge.api import HedgeRun

    di = D.init() if world > 1 else None
    if di is not None and not a.cpu:
        D.select_transport(di)  # in-kernel xGMI exchange if a probe fit is clean, else RCCL
    cfg = build_run(a, world)
    if a.cpu and di is None:
        di = D.DistInfo(device=torch.device("cpu"))
    run = HedgeRun(cfg, dist_info=di)
    rank = run.di.rank
    gpu = run.device.type == "cuda"
    # lr schedule: first date a.lr, later dates a.lr_rest (constant per date; see FitConfig)
    run.build()
    def sched(lr0, n):
        if n <= 1 or a.lr_decay == 1.0:
            return tuple([lr0] * n)
        return tuple(lr0 * a.lr_decay ** (e / (n - 1)) for e in range(n))

    sched_first = sched(a.lr, a.epochs_first)
    sched_rest = sched(a.lr_rest, a.epochs_rest)
    ind = run.induction
    orig = ind._fcfg

    def fcfg(first, loss):
        f = orig(first, loss)
        f.lr_schedule = sched_first if first else sched_rest
        return f

    ind._fcfg = fcfg
    use_graph = gpu and not a.no_graph and (world == 1 or os.environ.get("RPH_GRAPH_DP", "1") == "1")
    if use_graph:
        try:
            run.capture(include_simulation=True)
        except Exception as e:  # e.g. a collective that refuses stream capture: run eagerly
            if rank == 0:
                print(f"bench.py: graph capture failed ({e}); timing eager launches", file=sys.stderr)
            torch.cuda.synchronize(run.device)
            use_graph = False

    def one():
        if use_graph:
            run.replay()
        else:
            if gpu:
                run._enqueue_sim_into_existing()
            run.enqueue()

    def sync():
        if gpu:
            torch.cuda.synchronize(run.device)
        if world > 1:
            D.barrier()
            if gpu:
                torch.cuda.synchronize(run.device)

    for _ in range(a.warmup):
        one()
    sync()
    t0 = time.perf_counter()
    for _ in range(a.steps):
        one()
    sync()
    dt = time.perf_counter() - t0
    if world > 1:
        dt = D.all_reduce_scalar(dt, op="max", device=run.device)
    res = run.collect()
    ms = 1000.0 * dt / max(a.steps, 1)
    n_total = run.n_total
    n_dates = run.paths.n_coarse - 1
    epochs = a.epochs_first + (n_dates - 1) * a.epochs_rest
    samples = float(n_total) * epochs
    value = samples / (ms / 1000.0)
    out = {
        "metric": METRIC,
        "value": value,
        "unit": "path-samples/s (global paths x epochs x dates per second, full training run)",
        "n_gpus": world,
        "steps": a.steps,
        "warmup": a.warmup,
        "ms_per_step": ms,
        "higher_is_better": True,
        "scaling": "weak",
        "vs_baseline": value / BASELINE_SAMPLES_PER_S,
        "dtype": "fp32" if (a.hidden == 8 or a.mfma_precision == "fp32") else "bf16",
        "data": "synthetic (Sobol-QMC GBM paths generated on device; random-init N(0,0.1) weights)",
        "config": {"model": f"hedge-MLP 1-{a.hidden}-{a.hidden}-2 (LeakyReLU 0.3), European call S0=K=100 r=0.08 sigma=0.15 T=1",
                   "global_batch": cfg.train.batch_size, "seq_len": n_dates,
                   "parallelism": f"dp{world}", "paths_global": n_total, "paths_per_gpu": run.n_local,
                   "epochs_first": a.epochs_first, "epochs_rest": a.epochs_rest,
                   "steps_per_epoch": run.backend.steps_per_epoch, "graph": use_graph,
                   "backend": run.backend_kind,
                   "step_schedule": run.backend.step_mode() if hasattr(run.backend, "step_mode") else "torch",
                   "dp_transport": (run.di.dp_mode if world > 1 else None)},
        "quality": {"terminal_pnl_std": res.terminal_pnl["std"], "terminal_pnl_mean": res.terminal_pnl["mean"],
                    "V0": res.v0, "bs_price": res.summary.get("bs_price"), "phi0": res.phi,
                    "bs_delta": res.summary.get("bs_delta"),
                    "reference_terminal_pnl_std_52step": 1.7504, "reference_V0": 11.352},
        "paths_per_sec_full_run": n_total / (ms / 1000.0),
    }
    if rank == 0:
        line = json.dumps(out)
        print(line, flush=True)
        if a.json_out:
            with open(a.json_out, "w") as f:
                f.write(line + "\n")
    D.shutdown()
    return 0


if __name__ == "__main__":
    sys.exit(main())
