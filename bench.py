#!/usr/bin/env python
"""Flagship benchmark: MC paths/sec training a 30-step hedge MLP + terminal P&L std.

BASELINE.json metric: "MC paths/sec training 30-step hedge-MLP + terminal P&L
std-dev, 1/2/4/8 MI355X"; config "European call, 30-step GBM, 1M Sobol paths,
bf16 hedge-MLP on 1 MI355X".

One benchmark STEP = one complete replicating-portfolio training run, captured
as ONE hipGraph and replayed:
  Sobol/ndtri + log-GBM path kernel (2^20 paths per GPU, 30 dates) -> call payoff
  -> backward induction over the 30 dates (per date: the MSE fit of the hedge
  MLP 1-8-8-2 - full-batch Levenberg-Marquardt passes (loss + gradient over every
  path on the VALU, Gram matrix on the matrix cores, fp64 Cholesky solve) or,
  with --optimizer adam, Keras-Adam minibatch epochs (fused step kernels);
  data parallel: one all-reduce per pass / step) -> value/holdings/residual
  epilogue per date -> self-financing P&L scan over all dates.
Nothing is skipped inside the timed region; weights and optimiser state are
reset from the same initialisation at the start of every replay.

value = MC paths trained per second = global paths / seconds per full
30-date training run (the literal BASELINE.json metric; independent of the
optimiser).  vs_baseline = value / the reference's paths/s for the same job
(BASELINE_PATHS_PER_S, derived from BASELINE.md's Keras timings).  The round-1
unit, path-samples/s = paths x full passes / s, is kept as path_samples_per_s.
Scaling is weak (2^20 paths per GPU).  Compute dtype is fp32 (>= the bf16 the
config names).

``--preset`` selects the other BASELINE.json configs (same metric, same
one-run-per-step timing, simulation inside the graph):
  euro30      (default) European call, 30-step GBM, 2^20 paths per GPU, LM fits
  euro30_adam euro30 with Keras-Adam minibatch fits (the reference's optimiser)
  heston30    Heston stochastic vol, 30 dates (10 Euler substeps each), 2^20 paths per GPU
  euro252     European call, 252-step GBM, 2^21 paths per GPU (16M paths at 8 GPUs)
  basket5     basket-of-5 European call, 252 steps, 2^23 paths per GPU (64M at 8 GPUs)
  euro30_mfma euro30 with the 32-unit hedge MLP on the matrix cores (bf16 MFMA, "bf16 hedge-MLP")
  euro1_cpu   European call, 1-step GBM, 2^14 (>= 10k) paths, CPU torch backend (plumbing)
Per-GPU path counts are the 8-GPU configs divided by 8 (weak scaling), so a
1-GPU run measures exactly the per-GPU shard of the 8-GPU job.
"""
from __future__ import annotations

import argparse
import json
import math
import os
import sys
import time

# dmabuf IPC (mailboxes, RCCL) on this driver: set before torch initialises
# HIP, whatever launched this process (self_launch, an external torchrun)
os.environ.setdefault("HSA_ENABLE_IPC_MODE_LEGACY", "0")

import torch  # noqa: E402

BASELINE_SAMPLES_PER_S = 512 / 0.006   # median 6 ms per 512-sample Keras step
# The reference's MC paths/s for the same job (derived from BASELINE.md): its
# European run trains 4096 paths with 500 epochs on the first date and 17.7 on
# average on each later date (1,404 epochs over 52 dates), 8 steps of 6 ms per
# epoch; a 30-date run is therefore (500 + 29 x 17.7) x 8 x 6 ms = 48.6 s for
# 4096 paths = 84.2 paths/s.
BASELINE_PATHS_PER_S = 4096.0 / ((500 + 29 * (1404 - 500) / 51) * 8 * 0.006)
METRIC = "MC paths/sec training 30-step hedge-MLP + terminal P&L std-dev, 1/2/4/8 MI355X"


LAM0_FIRST = 16.384000778198242  # float32(1e-3) * 4**7 (exact in fp32)

# BASELINE.json configs -> (model, dates, Euler substeps per date, paths per GPU log2, epochs first/rest,
# per-GPU batch log2, lr first/rest, extra RunConfig fields)
PRESETS = {
    "euro30": dict(model="gbm_log", dates=30, substeps=1, paths_log2=20, epochs_first=512, epochs_rest=12,
                   batch_log2=18, lr=5e-2, lr_rest=4e-3, lr_decay=0.1, optimizer="lm",
                   # first date: 16 starts explored at once (one launch per kernel, grid y =
                   # start, 16 pass workgroups each) for 20 passes on the global 2^15-path
                   # prefix (every rank the same), the best polished for 25 passes on every
                   # path; from fp32(1e-3) x 4^7, the damping of the first trial the lam0 =
                   # 1e-3 sequence could accept.  Seeds 1-8 / 9-16: P&L mean 0.891 / 0.891,
                   # worst 0.901 / 0.900 at 7.13 ms, against 0.908 / 0.905, worst 0.938 / 0.937
                   # at 7.49 ms for the round-4 single start (profiles/r5/seeds_*.jsonl)
                   lm_lam0_first=LAM0_FIRST, lm_starts=16, lm_explore_passes=20, lm_explore_log2=15,
                   lm_passes_first=25,
                   lm_passes_rest=1, lm_lam_carry=3.0, lm_out_fix=1,
                   # round 6: inputs centred at the strike and scaled by the remaining-horizon
                   # spread (feature_norm "horizon", floor 0.1 x the date spread), first-layer
                   # breakpoints spread over [-1.5, 1.5] (init "spread"): seeds 1-16 P&L mean
                   # 0.881 / worst 0.898 vs 0.891 / 0.901 (profiles/r6/norm/).  On that scale the
                   # previous date's net is nearly the next date's optimum, so ONE LM trial per
                   # later date (+ the output-layer step) suffices: 0.882 / 0.901 at 5.71 vs
                   # 7.03 ms (profiles/r6/rest1/; 0 trials: 0.920 / 1.083)
                   feature_norm="horizon", feature_norm_floor=0.1, init="spread",
                   label="European call, 30-step GBM, 1M Sobol paths per GPU"),
    # the round-4 default: one start, 33 warm-up passes on the 2^16-path prefix, 35 on every path
    "euro30_1s": dict(model="gbm_log", dates=30, substeps=1, paths_log2=20, epochs_first=512, epochs_rest=12,
                      batch_log2=18, lr=5e-2, lr_rest=4e-3, lr_decay=0.1, optimizer="lm",
                      lm_lam0_first=LAM0_FIRST, lm_explore_one=1, lm_explore_passes=33, lm_explore_log2=16,
                      lm_passes_first=35, lm_passes_rest=2, lm_lam_carry=3.0, lm_out_fix=1,
                      label="European call, 30-step GBM, 1M Sobol paths per GPU, single-start first date"),
    # the flagship with a multi-start first date (4 starts x 45 passes on 2^16
    # paths, 25 polish passes): no first-date local minima (8 seeds: P&L mean
    # 0.893, worst 0.910 vs 0.908 / 0.944) for +1 ms (profiles/r4/ms_*.jsonl)
    "euro30_ms": dict(model="gbm_log", dates=30, substeps=1, paths_log2=20, epochs_first=512, epochs_rest=12,
                      batch_log2=18, lr=5e-2, lr_rest=4e-3, lr_decay=0.1, optimizer="lm",
                      lm_starts=4, lm_explore_passes=45, lm_passes_first=25,
                      lm_passes_rest=2, lm_lam_carry=3.0, lm_out_fix=1,
                      label="European call, 30-step GBM, 1M Sobol paths per GPU, multi-start first date"),
    "euro30_adam": dict(model="gbm_log", dates=30, substeps=1, paths_log2=20, epochs_first=512, epochs_rest=12,
                        batch_log2=18, lr=5e-2, lr_rest=4e-3, lr_decay=0.1, optimizer="adam",
                        label="European call, 30-step GBM, 1M Sobol paths per GPU, Keras-Adam minibatch fits"),
    "heston30": dict(model="heston", dates=30, substeps=10, paths_log2=20, epochs_first=1024, epochs_rest=16,
                     batch_log2=18, lr=5e-2, lr_rest=4e-3, lr_decay=0.1,
                     extra=dict(mu=0.05, r=0.05, kappa=2.0, theta=0.04, xi=0.5, rho=-0.7, v0=0.04, sigma=0.2),
                     optimizer="lm", lm_passes_first=35, lm_passes_rest=1, lm_lam_carry=3.0, lm_out_fix=1,
                     # first date: 16 starts x 25 passes on the global 2^15-path prefix, the best
                     # polished for 35 passes on every path (3 seeds: 11.38 ms, P&L 1.0024 /
                     # 1.0038 / 1.0052 x the minimum-variance hedge, against 11.18 ms and
                     # 1.0075 / 1.0042 / 1.0061 for one start: profiles/r5/seeds_presets.jsonl)
                     lm_lam0_first=LAM0_FIRST, lm_starts=16, lm_explore_passes=25, lm_explore_log2=15,
                     # round 6: the price input on the remaining-horizon scale (the variance input keeps
                     # the date scale) and one LM trial per later date: 16 seeds 1.0070 x the minimum-
                     # variance hedge, worst 1.0108, 9.71 ms (2 trials: 1.0048 / 1.0098, 11.17 ms)
                     feature_norm="horizon", feature_norm_floor=0.1,
                     label="Heston stochastic-vol call, 30 dates x 10 substeps, 1M paths per GPU"),
    "euro252": dict(model="gbm_log", dates=252, substeps=1, paths_log2=21, epochs_first=256, epochs_rest=8,
                    batch_log2=18, lr=2e-2, lr_rest=4e-3, lr_decay=0.03,
                    optimizer="lm", lm_passes_first=80, lm_passes_rest=2, lm_lam_carry=3.0, lm_out_fix=1,
                    # the first date is a 1-day hedge of the payoff (a near-digital delta):
                    # 8 starts x 40 passes on the global 2^16-path prefix, the best polished
                    # for 80 passes (3 seeds: last residual 0.069 / 0.071 / 0.075 against the
                    # BS floor 0.062, where 120 passes from one start left seed 2 at 0.150)
                    lm_starts=8, lm_explore_passes=40, lm_explore_log2=16,
                    # round 6: horizon-scaled inputs (floor 0.1) + spread breakpoints: seeds 1-16
                    # P&L 1.040 x the BS delta hedge, worst 1.107 x, last residual <= 0.076
                    # (date scaling: 1.114 x, worst 1.232 x, residual 0.118; profiles/r6/norm/)
                    feature_norm="horizon", feature_norm_floor=0.1, init="spread",
                    label="European call, 252-step GBM, 2M paths per GPU (16M at 8 GPUs)"),
    "basket5": dict(model="basket", dates=252, substeps=1, paths_log2=23, epochs_first=32, epochs_rest=2,
                    batch_log2=18, lr=2e-2, lr_rest=2e-3,
                    extra=dict(mu=0.05, r=0.05, sigma=0.2, n_assets=5, basket_corr=0.5),
                    optimizer="lm", lm_passes_first=80, lm_passes_rest=4, lm_lam_carry=2.0, lm_out_fix=1,
                    # first date: 40 passes on the 2^16-path prefix, then 80 on every path
                    # (2 seeds: 333 vs 340 ms, P&L 0.359 vs 0.374 mean; profiles/r4/presets_explore_one.jsonl);
                    # round 6 (16 seeds, profiles/r6/basket5/): 80 instead of 40 polish passes,
                    # the output-step trust region 0.5, damping carry x2 and 4 passes per later
                    # date: 1.157 -> 1.071 x Levy, worst 1.501 -> 1.131 x, 352 -> 493 ms
                    lm_out_tr=0.5,
                    lm_explore_one=1, lm_explore_passes=40, lm_explore_log2=16,
                    # (round 6: neither spread breakpoints - 16 seeds 1.165 x Levy, worst 1.358 x,
                    # vs 1.141 / 1.321 x - nor horizon-scaled inputs - 1.21-1.28 x on seeds 1-8 -
                    # help the basket: profiles/r6/norm/)
                    label="Basket-of-5 European call, 252 steps, 8M paths per GPU (64M at 8 GPUs)"),
    "euro30_mfma": dict(model="gbm_log", dates=30, substeps=1, paths_log2=20, epochs_first=512, epochs_rest=12,
                        batch_log2=18, lr=5e-3, lr_rest=1e-3, lr_decay=0.1, hidden=32,
                        label="European call, 30-step GBM, 1M paths per GPU, 32-unit hedge MLP on bf16 MFMA"),
    "euro1_cpu": dict(model="gbm_log", dates=1, substeps=1, paths_log2=14, epochs_first=200, epochs_rest=0,
                      batch_log2=11, lr=1e-2, lr_rest=1e-3, cpu=True,
                      label="European call, 1-step GBM, 16k (>=10k) Sobol paths, CPU plumbing"),
}


def parse(argv=None):
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=5)
    ap.add_argument("--warmup", type=int, default=2)
    ap.add_argument("--preset", default="euro30", choices=sorted(PRESETS))
    ap.add_argument("--paths-log2", type=int, default=None, help="paths PER GPU (weak scaling)")
    ap.add_argument("--dates", type=int, default=None)
    ap.add_argument("--substeps", type=int, default=None, help="fine Euler steps per rebalancing date")
    ap.add_argument("--epochs-first", type=int, default=None)
    ap.add_argument("--epochs-rest", type=int, default=None)
    ap.add_argument("--batch-log2", type=int, default=None, help="per-GPU minibatch (global = N x this)")
    ap.add_argument("--lr", type=float, default=None)
    ap.add_argument("--lr-rest", type=float, default=None)
    ap.add_argument("--lr-decay", type=float, default=None, help="per-date geometric LR decay factor (last/first epoch)")
    ap.add_argument("--hidden", type=int, default=None, help="hidden width (8 = reference net; 32 = MFMA kernel)")
    ap.add_argument("--mfma-precision", default="bf16", choices=["bf16", "fp32"])
    ap.add_argument("--variant", type=int, default=-1, help="narrow lag-kernel variant (-1: engine default)")
    ap.add_argument("--max-wgs", type=int, default=0, help="workgroups per training step (0: engine default)")
    ap.add_argument("--feature-norm", default=None, choices=["none", "global", "date", "horizon"],
                    help="input standardisation fused into the kernels (default: preset)")
    ap.add_argument("--feature-norm-floor", type=float, default=None,
                    help="horizon standardisation: scale >= this x the date spread (default: preset)")
    ap.add_argument("--optimizer", default=None, choices=["adam", "lm"],
                    help="MSE fits: Keras-Adam minibatches or full-batch Levenberg-Marquardt (default: preset)")
    ap.add_argument("--lm-passes-first", type=int, default=None)
    ap.add_argument("--lm-passes-rest", type=int, default=None)
    ap.add_argument("--lm-gram-paths", type=int, default=None)
    ap.add_argument("--lm-leaf-paths", type=int, default=None,
                    help="LM pass schedule: -1 cyclic (default); > 0 contiguous leaves of this many paths - the same "
                         "value at every --gpus makes a strong-scaling rehearsal bitwise the 1-GPU fit")
    ap.add_argument("--lm-damping", default=None, choices=["simple", "nielsen"])
    ap.add_argument("--lm-lam0", type=float, default=None)
    ap.add_argument("--lm-lam-up", type=float, default=None)
    ap.add_argument("--lm-lam-down", type=float, default=None)
    ap.add_argument("--lm-stop-tol", type=float, default=None,
                    help="later dates: adaptive LM pass budget (relative best-loss gain that ends a fit; 0: off)")
    ap.add_argument("--lm-stop-min", type=int, default=None)
    ap.add_argument("--lm-lam0-rest", type=float, default=None, help="later dates' initial LM damping (0: --lm-lam0)")
    ap.add_argument("--lm-lam0-first", type=float, default=None, help="first date's initial LM damping (0: --lm-lam0)")
    ap.add_argument("--lm-lam-carry", type=float, default=None,
                    help="later dates start at the previous fit's final LM damping x this (0: off)")
    ap.add_argument("--lm-starts", type=int, default=None, help="first date: multi-start LM exploration (1: off)")
    ap.add_argument("--lm-out-fix", type=int, default=None, choices=[0, 1],
                    help="LM fits end with the exact Newton step on the whole output layer")
    ap.add_argument("--lm-out-mu", type=float, default=None, help="relative damping of the output-layer step")
    ap.add_argument("--lm-ridge", type=float, default=None, help="LM systems: + this x the mean diagonal")
    ap.add_argument("--lm-out-tr", type=float, default=None,
                    help="output-layer step trust region: ||d|| <= this x ||w_o|| (0: off)")
    ap.add_argument("--lm-renorm", type=int, default=None, choices=[0, 1],
                    help="later dates: warm start re-expressed for the date's input standardisation")
    ap.add_argument("--lm-explore-passes", type=int, default=None, help="trial points of every exploration fit")
    ap.add_argument("--lm-explore-log2", type=int, default=None, help="exploration fits on 2^this local paths")
    ap.add_argument("--lm-explore-one", type=int, default=None, choices=[0, 1],
                    help="lm_starts 1: the one start still explores on the path prefix first (warm-up)")
    ap.add_argument("--no-graph", action="store_true")
    ap.add_argument("--cpu", action="store_true", help="torch reference backend (plumbing only)")
    ap.add_argument("--json-out", default=None)
    ap.add_argument("--seed", type=int, default=1234, help="weight-init seed (the reference's 1234)")
    ap.add_argument("--init", default=None, choices=["reference", "spread", "aligned"],
                    help="weight init (default: preset); aligned = spread + first layer along the basket weights")
    a = ap.parse_args(argv)
    pre = PRESETS[a.preset]
    for k in ("paths_log2", "dates", "substeps", "epochs_first", "epochs_rest", "batch_log2", "lr", "lr_rest"):
        if getattr(a, k) is None:
            setattr(a, k, pre[k])
    if a.lr_decay is None:
        a.lr_decay = pre.get("lr_decay", 0.02)
    if a.hidden is None:
        a.hidden = pre.get("hidden", 8)
    if a.feature_norm is None:
        a.feature_norm = pre.get("feature_norm", "date")
    if a.feature_norm_floor is None:
        a.feature_norm_floor = pre.get("feature_norm_floor", 0.0)
    if a.optimizer is None:
        a.optimizer = pre.get("optimizer", "adam")
    if a.init is None:
        a.init = pre.get("init", "reference")
    for k, dflt in (("lm_passes_first", 80), ("lm_passes_rest", 3), ("lm_gram_paths", 4096),
                    ("lm_damping", "simple"), ("lm_lam0", 1e-3), ("lm_lam_up", 4.0), ("lm_lam_down", 1.0 / 3.0),
                    ("lm_stop_tol", 0.0), ("lm_stop_min", 2), ("lm_lam0_rest", 0.0), ("lm_lam0_first", 0.0),
                    ("lm_lam_carry", 0.0),
                    ("lm_starts", 1), ("lm_explore_passes", 45), ("lm_explore_log2", 16), ("lm_explore_one", 0), ("lm_renorm", 0), ("lm_out_fix", 0),
                    ("lm_out_mu", 1e-5), ("lm_out_tr", 0.0), ("lm_ridge", 1e-10), ("lm_leaf_paths", -1)):
        if getattr(a, k) is None:
            setattr(a, k, pre.get(k, dflt))
    if pre.get("cpu"):
        a.cpu = True
    return a


def build_run(a, world: int):
    from rphedge.config import RunConfig, TrainingParams, ParityFlags

    pre = PRESETS[a.preset]
    tr = TrainingParams(batch_size=(1 << a.batch_log2) * world, epochs_first=a.epochs_first,
                        epochs_rest=a.epochs_rest, patience_first=10 ** 6, patience_rest=10 ** 6,
                        lr=a.lr, lr_rest=a.lr_rest, lr_decay=a.lr_decay, lr_schedule_first=False, early_stopping=False, q99=False, shuffle=True,
                        chunk_log2=6, seed=a.seed, hidden=a.hidden, mfma_precision=a.mfma_precision,
                        variant=a.variant, max_wgs=a.max_wgs, feature_norm=a.feature_norm,
                        feature_norm_floor=a.feature_norm_floor,
                        optimizer=a.optimizer, lm_passes_first=a.lm_passes_first, lm_passes_rest=a.lm_passes_rest,
                        lm_gram_paths=a.lm_gram_paths, lm_damping=a.lm_damping, lm_lam0=a.lm_lam0,
                        lm_lam_up=a.lm_lam_up, lm_lam_down=a.lm_lam_down, lm_stop_tol=a.lm_stop_tol,
                        lm_stop_min=a.lm_stop_min, lm_lam0_rest=a.lm_lam0_rest, lm_lam0_first=a.lm_lam0_first,
                        init=a.init,
                        lm_lam_carry=a.lm_lam_carry, lm_starts=a.lm_starts, lm_explore_passes=a.lm_explore_passes,
                        lm_explore_log2=a.lm_explore_log2, lm_explore_one=bool(a.lm_explore_one),
                        lm_renorm=bool(a.lm_renorm), lm_out_fix=bool(a.lm_out_fix),
                        lm_out_mu=a.lm_out_mu, lm_out_tr=a.lm_out_tr, lm_ridge=a.lm_ridge, lm_leaf_paths=a.lm_leaf_paths)
    model = pre["model"]
    kw = dict(Y=100.0, K=100.0, T=1.0, mu=0.08, r=0.08, sigma=0.15, rebalancing=1.0 / a.dates,
              dt=1.0 / (a.dates * a.substeps), n_paths=a.paths_log2 + int(math.log2(world)),
              payoff="basket_call" if model == "basket" else "call", option_type="CALL",
              model=model, mortality=False, N=1, P=1.0, keep_paths=False, verbose=False, train=tr,
              parity=ParityFlags(), backend="torch" if a.cpu else None)
    kw.update(pre.get("extra", {}))
    return RunConfig(**kw)


def anchor(cfg) -> dict:
    """Closed-form price/delta of the preset's option (quality anchor)."""
    from rphedge import analytic

    if cfg.model == "heston":
        p, dlt = analytic.heston_price(cfg.Y, cfg.K, cfg.r, cfg.T, cfg.kappa, cfg.theta, cfg.xi, cfg.rho, cfg.v0,
                                       cfg.option_type)
        return {"analytic": "heston", "price": p, "delta": dlt}
    if cfg.model == "basket":
        return {"analytic": None}
    p, dlt = analytic.black_scholes(cfg.Y, cfg.K, cfg.r, cfg.sigma, cfg.T, cfg.option_type)
    return {"analytic": "black_scholes", "price": p, "delta": dlt}


def _free_port() -> int:
    import socket

    with socket.socket(socket.AF_INET, socket.SOCK_STREAM) as s:
        s.bind(("127.0.0.1", 0))
        return int(s.getsockname()[1])


def self_launch(n: int, argv=None) -> int:
    """``bench.py --gpus N`` without a torch.distributed environment: run N
    ranks (one process per GPU) under ``torch.distributed.run`` as a CHILD
    process and return its exit code.  Nothing here touches the GPU (the
    parent never initialises HIP), so the ranks own their devices; rank 0 of
    the child prints the JSON line to the inherited stdout."""
    import subprocess

    args = list(sys.argv[1:] if argv is None else argv)
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", f"--nproc-per-node={n}",
           "--master-addr=127.0.0.1", f"--master-port={_free_port()}", os.path.abspath(__file__)] + args
    env = dict(os.environ)
    env.setdefault("HSA_ENABLE_IPC_MODE_LEGACY", "0")  # dmabuf IPC (mailboxes, RCCL) on this driver
    env.setdefault("OMP_NUM_THREADS", "1")
    return subprocess.call(cmd, env=env)


def delta_anchor(run, cfg) -> dict | None:
    """Analytic hedges on the same simulated grid and paths, self-financing
    P&L std (x S0) — the floor the learnt hedge is compared against:
    GBM: the Black–Scholes delta hedge (+ its last one-step residual);
    Heston: the Heston delta and the minimum-variance hedge
    Delta + (rho xi / S) dC/dv (first 2^16 paths per rank); basket: the
    per-asset deltas of a moment-matched lognormal basket (2^16 paths)."""
    from rphedge import analytic

    p = run.paths
    t = run.grid.times()
    if cfg.model in ("gbm", "gbm_log") and run.kind == "european":
        a = analytic.bs_delta_hedge(p.S, p.bond, cfg.K / cfg.Y, cfg.r, cfg.sigma, cfg.T, t,
                                    cfg.option_type, payoff=run.v_terminal, world=run.di.world)
        return {"hedge": "black_scholes_delta", "pnl_std": a["pnl_std"] * cfg.Y, "pnl_mean": a["pnl_mean"] * cfg.Y,
                "residual_std_last": a["residual_std_last"] * cfg.Y, "price": a["price"] * cfg.Y}
    if cfg.model == "heston" and p.vol is not None:
        a = analytic.heston_hedge_anchor(p.S, p.vol, p.bond, cfg.K / cfg.Y, cfg.r, cfg.T, t, cfg.kappa, cfg.theta,
                                         cfg.xi, cfg.rho, payoff=run.v_terminal, world=run.di.world,
                                         option_type=cfg.option_type)
        best = min(a["delta"]["pnl_std"], a["min_variance"]["pnl_std"])
        return {"hedge": "heston_delta | heston_min_variance", "paths": a["paths"], "price": a["price"] * cfg.Y,
                "delta_pnl_std": a["delta"]["pnl_std"] * cfg.Y,
                "min_variance_pnl_std": a["min_variance"]["pnl_std"] * cfg.Y, "pnl_std": best * cfg.Y}
    if cfg.model == "basket":
        na = p.na
        w = cfg.basket_weights or tuple([1.0 / na] * na)
        a = analytic.basket_hedge_anchor(p.S, p.bond, w, cfg.K / cfg.Y, cfg.r, cfg.sigma, cfg.basket_corr, cfg.T,
                                         t, payoff=run.v_terminal, world=run.di.world)
        return {"hedge": "levy_basket_delta", "paths": a["paths"], "price": a["price"] * cfg.Y,
                "pnl_std": a["levy_delta"]["pnl_std"] * cfg.Y, "pnl_mean": a["levy_delta"]["pnl_mean"] * cfg.Y}
    return None


def lm_fit_stats(ind) -> dict:
    """Per-date LM passes and accepted trials (from each fit's loss history:
    a trial is accepted when it beats the best loss so far), dates in
    backward order (the first fit is the last date)."""
    passes, acc = [], []
    for d in ind.dates:
        h = [x for x in d.fit_mse["history"] if x == x]
        best, n = (h[0] if h else float("inf")), 0
        for x in h[1:]:
            if x < best:
                best, n = x, n + 1
        passes.append(max(len(h) - 1, 0))
        acc.append(n)
    tot = max(sum(passes), 1)
    first = {"passes": passes[0] if passes else 0, "accepted": acc[0] if acc else 0}
    if ind.dates:  # best-so-far loss of the first fit at a few passes (convergence record)
        h = [x for x in ind.dates[0].fit_mse["history"] if x == x]
        best = [min(h[:k + 1]) for k in range(len(h))]
        first["best_loss_at"] = {str(k): best[k] for k in (0, 10, 20, 40, 60, 80, 120, 160, 240) if k < len(best)}
        first["best_loss"] = best[-1] if best else None
    return {"passes_per_date": passes, "accepted_per_date": acc, "acceptance_rate": sum(acc) / tot,
            "first_date": first}


def lm_exchange_record(run, a, world: int) -> dict:
    """Data-parallel LM exchange volume: every rank builds the same Gram
    matrix from the simulated global subsample, so one pass pushes only the
    gradient region [g | stats] to each peer (+ the packed output Gram in the
    passes that build it), from inside k_lm_reduce (no extra launch)."""
    be = run.backend
    per_peer = int(be.lm_exchange_bytes())
    run_peer = int(be.lm_exchange_bytes_run(a.lm_passes_first, a.lm_passes_rest, run.paths.n_coarse - 1))
    return {"bytes_per_pass_per_peer": per_peer, "peers": world - 1,
            "bytes_per_pass_per_rank": per_peer * (world - 1),
            "bytes_per_run_per_rank": run_peer * (world - 1),
            "same_gram_every_rank": bool(getattr(be, "_lm_same_gram", True)),
            "fused_in_reduce": bool(world > 1 and be.lm_mailbox is not None and getattr(be, "_lm_same_gram", False))}


def multistart_record(run, a, world: int) -> dict:
    """First-date multi-start exploration: every candidate's final best loss on
    the global exploration prefix (every rank runs the same candidates), the
    pick, and the exploration's work in full passes over the local paths."""
    from rphedge.ops import layout as L

    be = run.backend
    x = getattr(be, "lm_explore_last", None)
    rec = {"starts": a.lm_starts, "explore_passes": a.lm_explore_passes}
    nsub = min(run.n_total, 1 << a.lm_explore_log2)
    rec["explore_paths_global"] = nsub
    rec["full_pass_equivalents"] = a.lm_starts * (a.lm_explore_passes + 1) * nsub / run.n_local
    if isinstance(x, dict) and "state" in x:
        st = x["state"].double().cpu().numpy()
        losses = [float(st[k, L.LMS_LFIN]) for k in range(a.lm_starts)]
    elif isinstance(x, dict):
        losses = [float(v) for v in x["losses"]]
    else:
        return rec
    import numpy as _np
    ls = _np.where(_np.isnan(losses), _np.inf, losses)
    rec["losses"] = losses
    rec["pick"] = int(_np.argmin(ls))
    return rec


def main(argv=None):
    a = parse(argv)
    if "WORLD_SIZE" not in os.environ and a.gpus > 1:
        return self_launch(a.gpus, argv)
    world = int(os.environ.get("WORLD_SIZE", "1"))
    if world != a.gpus:
        print(f"bench.py: --gpus {a.gpus} but WORLD_SIZE={world}; measuring the {world} launched ranks",
              file=sys.stderr)
    from rphedge.parallel import dist as D
    from rphedge.api import HedgeRun

    di = D.init(device="cpu" if a.cpu else None) if world > 1 else None
    probe = None
    if di is not None and not a.cpu:
        D.select_transport(di)  # in-kernel xGMI exchange if a probe fit is clean, else RCCL
        probe = di.probe
    cfg = build_run(a, world)
    if a.cpu and di is None:
        di = D.DistInfo(device=torch.device("cpu"))
    run = HedgeRun(cfg, dist_info=di)
    rank = run.di.rank
    gpu = run.device.type == "cuda"
    # lr schedule (TrainingParams.lr / lr_rest / lr_decay): geometric decay over each date's epochs
    run.build()
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
    lm_stats = lm_fit_stats(res.induction) if a.optimizer == "lm" else None
    if lm_stats is not None and (a.lm_starts > 1 or a.lm_explore_one):
        lm_stats["multistart"] = multistart_record(run, a, world)
    memory = None
    if gpu:
        # HBM footprint of this rank (every buffer is a torch allocation): the
        # 288 GB-per-GPU sizing of the 64M-path basket config
        n_dates_m = run.paths.n_coarse - 1
        pb = sum(int(t.numel()) * t.element_size() for t in (run.paths.S, run.paths.vol, run.paths.nfrac,
                                                              run.paths.lam, run.paths.S_final) if t is not None)
        mx = int(torch.cuda.max_memory_allocated(run.device))
        memory = {"max_allocated_bytes": mx, "path_buffer_bytes": pb,
                  "bytes_per_path": mx / run.n_local, "bytes_per_path_date": mx / (run.n_local * max(n_dates_m, 1)),
                  "device_total_bytes": int(torch.cuda.get_device_properties(run.device).total_memory)}
    n_total = run.n_total
    n_dates = run.paths.n_coarse - 1
    lm = a.optimizer == "lm"
    # full passes over the paths per run: Adam epochs, or LM evaluations (start point + trials)
    passes = (a.lm_passes_first + 1 + (n_dates - 1) * (a.lm_passes_rest + 1)) if lm else \
        (a.epochs_first + (n_dates - 1) * a.epochs_rest)
    if lm and lm_stats and a.lm_stop_tol > 0:  # adaptive budget: the evaluations actually run
        passes = sum(p + 1 for p in lm_stats["passes_per_date"])
    if lm and lm_stats and lm_stats.get("multistart"):  # + the exploration, in full-pass equivalents
        passes += lm_stats["multistart"]["full_pass_equivalents"]
    path_samples = float(n_total) * passes / (ms / 1000.0)
    value = float(n_total) / (ms / 1000.0)
    out = {
        "metric": METRIC,
        "value": value,
        "unit": "MC paths/s (global paths trained through the whole 30-date backward induction per second)",
        "n_gpus": world,
        "steps": a.steps,
        "warmup": a.warmup,
        "ms_per_step": ms,
        "higher_is_better": True,
        "scaling": "weak",
        "vs_baseline": value / BASELINE_PATHS_PER_S,
        "vs_baseline_kind": "derived: the reference publishes no paths/s; 84.2 paths/s is derived from its "
                            "Keras log (52 dates, 4096 paths, 6 ms per 512-sample step, unknown hardware)",
        "dtype": "fp32" if (a.hidden == 8 or a.mfma_precision == "fp32") else "bf16",
        "data": f"synthetic (Sobol-QMC {cfg.model} paths generated {'on device' if gpu else 'on host'}; "
                "random-init N(0,0.1) weights)",
        "config": {"model": f"hedge-MLP {run.spec.nin}-{a.hidden}-{a.hidden}-{run.spec.nout} (LeakyReLU 0.3), "
                            + PRESETS[a.preset]["label"],
                   "preset": a.preset,
                   "global_batch": cfg.train.batch_size, "seq_len": n_dates,
                   "substeps": a.substeps, "feature_norm": a.feature_norm,
                   "feature_norm_floor": a.feature_norm_floor if a.feature_norm == "horizon" else None, "option": {k: getattr(cfg, k) for k in
                                                      ("Y", "K", "T", "r", "sigma", "kappa", "theta", "xi",
                                                       "rho", "v0", "n_assets", "basket_corr")
                                                      if cfg.model in ("heston", "basket") or
                                                      k in ("Y", "K", "T", "r", "sigma")},
                   "parallelism": f"dp{world}", "paths_global": n_total, "paths_per_gpu": run.n_local,
                   "optimizer": a.optimizer,
                   "epochs_first": None if lm else a.epochs_first, "epochs_rest": None if lm else a.epochs_rest,
                   "lm_passes_first": a.lm_passes_first if lm else None,
                   "lm_passes_rest": a.lm_passes_rest if lm else None,
                   "lm_gram_paths": a.lm_gram_paths if lm else None,
                   "lm_leaf_paths": a.lm_leaf_paths if lm else None,
                   "lm_damping": a.lm_damping if lm else None,
                   "lm_lam": [a.lm_lam0, a.lm_lam_up, a.lm_lam_down] if lm else None,
                   "lm_lam0_rest": (a.lm_lam0_rest or None) if lm else None,
                   "lm_lam0_first": (a.lm_lam0_first or None) if lm else None, "init": a.init, "seed": a.seed,
                   "lm_stop": [a.lm_stop_tol, a.lm_stop_min] if (lm and a.lm_stop_tol > 0) else None,
                   "lm_lam_carry": (a.lm_lam_carry or None) if lm else None,
                   "lm_renorm": bool(a.lm_renorm) if lm else None,
                   "lm_out_fix": bool(a.lm_out_fix) if lm else None,
                   "lm_multistart": ({"starts": a.lm_starts, "explore_passes": a.lm_explore_passes,
                                      "explore_paths_global": 1 << a.lm_explore_log2}
                                     if (lm and (a.lm_starts > 1 or a.lm_explore_one)) else None),
                   "steps_per_epoch": None if lm else run.backend.steps_per_epoch, "graph": use_graph,
                   "backend": run.backend_kind,
                   "step_schedule": None if lm else (run.backend.step_mode() if hasattr(run.backend, "step_mode")
                                                     else "torch"),
                   "dp_transport": (("gloo" if a.cpu else run.di.dp_mode) if world > 1 else None),
                   "lm_dp_transport": (("gloo" if a.cpu else run.di.lm_dp_mode) if world > 1 and lm else None),
                   "dp_probe": probe, "dist_world": D.dist_world(),
                   "launch": "torchrun" if "TORCHELASTIC_RUN_ID" in os.environ or world > 1 else "single"},
        "quality": {"terminal_pnl_std": res.terminal_pnl["std"], "terminal_pnl_mean": res.terminal_pnl["mean"],
                    "terminal_pnl_kind": res.terminal_pnl.get("kind"),
                    "terminal_residual_std": res.terminal_residual["std"],
                    "terminal_residual_mean": res.terminal_residual["mean"],
                    "V0": res.v0, "phi0": res.phi, "psi0": res.psi,
                    "anchor": anchor(cfg), "hedge_anchor": delta_anchor(run, cfg),
                    "mc_discounted_payoff": res.summary["E_payoff"] * run.scale * math.exp(-cfg.r * cfg.T),
                    "reference_terminal_residual_std_52step": 1.7504, "reference_V0": 11.352},
        "lm": lm_stats,
        "lm_exchange": lm_exchange_record(run, a, world) if (lm and not a.cpu) else None,
        "memory": memory,
        "path_samples_per_s": path_samples, "full_passes_per_run": passes,
        # nodes of the replayed hipGraph (kernels + copies): the same at every
        # world size when the data-parallel exchange adds no launch
        "graph_nodes": int(run.graph.num_nodes) if (use_graph and run.graph is not None) else None,
        "path_samples_vs_keras": path_samples / BASELINE_SAMPLES_PER_S,
    }
    if rank == 0:
        line = json.dumps(out)
        print(line, flush=True)
        if a.json_out:
            with open(a.json_out, "w") as f:
                f.write(line + "\n")
    run.close()
    D.shutdown()
    return 0


if __name__ == "__main__":
    sys.exit(main())
