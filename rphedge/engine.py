"""Training / evaluation engine: device-resident state + two backends.

* :class:`HipBackend` — the MI355X path.  Every optimizer step runs the same
  fused body (forward + loss + backward + in-wave reduce-scatter + workgroup
  sum: ``NarrowBody`` VALU for the 8-unit nets, ``WideBody`` MFMA for the
  32-unit nets) under one of three schedules (:attr:`TrainConfig.step_mode`,
  resolved by :meth:`HipBackend.step_mode`):

  - ``lag`` — one ``k_hedge_step_lag`` launch per step; every workgroup
    applies the Keras-Adam / LR / EarlyStopping update of the PREVIOUS step
    redundantly in its prologue from float-atomic accumulators, so the kernel
    boundary is the only global synchronisation (large grids; data parallel
    with the in-kernel xGMI exchange);
  - ``persistent`` — one ``k_hedge_fit`` launch per Keras fit with an
    in-kernel barrier (small grids, e.g. the reference's batch 512);
  - ``ticket`` — ``k_hedge_train_step`` with a last-arriver update
    (deterministic slab reduction, ranks sharing a GPU, RCCL all-reduce of the
    gradient packet on the compute stream between step and update kernels).

  Whole fits are launched from the native runtime (``rph_train_*_fit``), the
  ``k_hedge_eval`` epilogue produces values / holdings / residuals / stats, and
  nothing synchronises with the host, so a whole backward-induction run is
  captured into ONE hipGraph (:mod:`rphedge.driver`).  Input standardisation
  (:attr:`DateData.fmu` / ``fisd``) is fused into the feature loads.
* :class:`TorchBackend` — CPU (or any torch device) reference with identical
  semantics: same chunk permutation (Philox), same Adam formula, same early
  stopping; multi-process via ``torch.distributed`` (gloo).  It is the oracle
  for GPU numerics tests and the "CPU plumbing" configuration of BASELINE.

State blocks are flat float32 tensors (layout in :mod:`rphedge.ops.layout`).
Reference semantics: ``Replicating_Portfolio.py:128-221`` (C17-C24).
"""
from __future__ import annotations

import math
import os
from dataclasses import dataclass, field

import numpy as np
import torch

from .models.hedge_mlp import NetSpec, torch_forward
from .ops import layout as L


# ---------------------------------------------------------------------------
# configuration
# ---------------------------------------------------------------------------
def keras_lr_schedule(epochs: int) -> list:
    """``scheduler`` of RP:128-136 evaluated per epoch (NaN = keep current lr)."""
    out = []
    for e in range(epochs):
        if e < 100:
            out.append(1e-2)
        elif e < 200:
            out.append(1e-3)
        elif e < 400:
            out.append(5e-4)
        else:
            out.append(float("nan"))
    return out


def geometric_lr_schedule(lr0: float, epochs: int, decay: float = 1.0) -> tuple:
    """Per-epoch learning rates ``lr0 * decay**(e / (epochs-1))``: decays from
    ``lr0`` to ``lr0 * decay`` over one date's fit (``decay = 1``: constant).
    Throughput-mode counterpart of the reference's step schedule for the large
    global batches; ``TrainingParams.lr_rest`` / ``lr_decay``."""
    n = max(int(epochs), 1)
    if n == 1 or decay == 1.0:
        return tuple([float(lr0)] * n)
    return tuple(float(lr0) * decay ** (e / (n - 1)) for e in range(n))


@dataclass
class FitConfig:
    epochs: int = 100
    patience: int = 7
    loss: int = L.LOSS_MSE
    quantile: float = 0.99
    lr_schedule: tuple | None = None      # per-epoch learning rates (NaN keeps current)
    restore_best: bool = True
    restore_at_end: bool = False          # Keras-3 behaviour; Keras-2 restores only on early stop
    early_stopping: bool = True
    # "adam" (the reference's Keras-Adam minibatch fit) or "lm": full-batch
    # Levenberg-Marquardt passes (MSE fits of the 8-unit nets; ``epochs`` = the
    # number of trial points after the start point; csrc/hedge_lm.hip)
    optimizer: str = "adam"
    # LM adaptive pass budget: from pass lm_stop_min on, an accepted pass that
    # lowers the best loss by less than lm_stop_tol (relative) ends the fit
    # (rejections never do; 0: off;
    # ``epochs`` stays the cap)
    lm_stop_tol: float = 0.0
    lm_stop_min: int = 2
    lm_lam0: float | None = None          # initial LM damping of this fit (None: TrainConfig.lm_lam0)
    # > 0: the fit starts at the previous LM fit's final damping x lm_lam_carry
    # (later dates: a warm start's curvature scale is the last fit's)
    lm_lam_carry: float = 0.0
    # multi-start exploration (first date; on when lm_starts >= 1 AND
    # lm_explore_passes > 0 - one start is a warm-up on the path prefix, which
    # also needs lm_w0s): lm_starts fits from the start
    # points lm_w0s[k] ([starts, P]; row 0 = the run's initial weights),
    # lm_explore_passes trial points each on the first lm_explore_paths global
    # paths (lm_explore_data; every rank runs all of them on the same data),
    # then the candidate with the lowest final loss is the start point of the
    # ``epochs`` polish passes on every path (at its damping)
    # (mu, isd) of the inputs the start weights were fitted on (the previous
    # date): the first layer is re-expressed for this fit's standardisation, so
    # a warm start is the previous hedge as a function of the raw state
    lm_renorm: tuple | None = None
    lm_starts: int = 1
    lm_explore_passes: int = 0
    lm_explore_paths: int = 0
    lm_w0s: object = None
    # the exploration's data: the first lm_explore_paths GLOBAL paths of the
    # date (DateData, simulated on every rank; None: this rank's shard prefix,
    # the global prefix on one rank) - every rank runs the same starts on the
    # same paths, so the pick is the same at every world size with no exchange
    lm_explore_data: object = None
    # pinball LM fits (loss = LOSS_PINBALL): IRLS Gram weights
    # 1 / (2 max(|r|, delta)), delta = max(lm_q_delta, lm_q_kappa x the mean |r|
    # of the path's 64-path Gram tile) (target units; lm_q_delta 0: 1e-6)
    lm_q_delta: float = 0.0
    lm_q_kappa: float = 3.0

    def key(self):
        return (self.epochs, self.patience if self.early_stopping else 1 << 30, self.restore_best,
                self.restore_at_end, tuple(self.lr_schedule) if self.lr_schedule is not None else None)


@dataclass
class TrainConfig:
    batch_size: int = 512          # GLOBAL minibatch (reference: 512)
    shuffle: bool = True           # Keras fit(shuffle=True)
    chunk_log2: int = 0            # shuffle granularity: 0 = per path (Keras), 6 = 64-path chunks
    seed: int = 1234
    lr: float = 1e-3               # Adam(learning_rate=1e-3)
    beta1: float = 0.9
    beta2: float = 0.999
    eps: float = 1e-7              # Keras epsilon
    max_wgs: int = 0               # workgroups per training step; 0 = auto: 256 (one per CU), 512 for
                                   # the 1-input 32-unit bf16 net (2 resident waves/SIMD:
                                   # the MFMA tile chain is latency-bound, profiles/r1/sweep_r1n_wide_wgs.jsonl)
    paths_per_thread: int = 1      # target work per thread per step
    deterministic: bool = False    # fixed-order slab reduction instead of float atomics
    split_update: bool = False     # force the standalone update kernel (the world_size>1 path)
    mfma_fp32: bool = False        # 32-unit nets: exact fp32 MFMA instead of bf16 operands
    # Levenberg-Marquardt fits (FitConfig.optimizer == "lm"): Gram matrix from a
    # subsample of lm_gram_paths paths (global; 64-path tiles on the matrix
    # cores), Marquardt damping lam0, x lam_up on a rejected trial, x lam_down
    # on an accepted one, clamped to [lam_min, lam_max]; ridge x mean diagonal
    lm_gram_paths: int = 4096
    lm_lam0: float = 1e-3
    lm_lam_up: float = 4.0
    lm_lam_down: float = 1.0 / 3.0
    lm_lam_min: float = 1e-9
    lm_lam_max: float = 1e10
    lm_ridge: float = 1e-10
    # damping diagonal floor (relative to the mean of diag 2G): a parameter with
    # no curvature on the Gram subsample is still damped, so lam -> inf shortens
    # its step (tests/test_lm_cpu.py: a teacher fit that stalls at lam_max
    # without it).  0 = plain Marquardt scaling (the presets: 1e-6 moved the
    # euro30 8-seed P&L 0.890 -> 0.897 in tools/lm_lab.py, 1e-9 changed nothing)
    lm_diag_floor: float = 0.0
    # damping update: "simple" (x lam_down on accept, x lam_up on reject) or
    # "nielsen" (gain ratio rho of actual / predicted reduction: accept
    # x max(1/3, 1 - (2 rho - 1)^3), reject x nu with nu doubling)
    lm_damping: str = "simple"
    # after the last pass: exact Newton step on the bond holding's output bias
    # (free heads), so the fitted values' mean over all paths equals the
    # target's and no mean error drifts down the backward induction
    lm_bias_fix: bool = True
    # pass kernel load balance (cyclic schedule only, lm_leaf_paths < 0): the
    # Gram workgroups' waves take this many 128-path blocks fewer than an even
    # split (their Gram tile follows)
    lm_gram_skip: int = 3
    # pass kernel schedule: every wave sums one contiguous "leaf" of paths
    # (LmDesc.leaf_blocks): 0 = auto (the shard over 4 x the pass workgroups),
    # > 0 = this many paths per leaf (a multiple of 128: the same leaves at
    # every world size over the same global paths - the strong-scaling
    # rehearsal reproduces the one-rank fit bit for bit), < 0 = the cyclic
    # block schedule with lm_gram_skip (default: 0.7 ms faster on the euro30
    # flagship, whose Gram workgroups then take fewer path blocks)
    lm_leaf_paths: int = -1
    # the Gram tiles in Gram-only workgroups after the path grid (LmDesc.gram_base),
    # co-resident with the path workgroups, instead of in the first path
    # workgroups; None = auto: on with contiguous leaves (no gram_skip balance
    # there: euro30 6.04 -> 5.86 ms), off on the cyclic schedule (5.69 vs 5.75)
    lm_gram_overlap: bool | None = None
    # after the last pass: exact Newton step on the whole output layer (the
    # value is linear in it; 2 G_oo d = -g_o), subsuming the bias step
    lm_out_fix: bool = False
    # its relative Marquardt damping (near-collinear hidden units: the output
    # Gram's condition number reaches 1e9+; below ~1e-5 of its scale the
    # fp32-accumulated matrix is rounding noise, tools/og_precision.py)
    lm_out_mu: float = 1e-5
    lm_out_tr: float = 0.0  # output step trust region: ||d|| <= this x max(||w_o||, 1e-3 sqrt(n_o)) (0: off)
    # run the data-parallel LM sequence (pass + reduce -> all-reduce of the
    # reduced block -> solve, one launch each) even on one rank: the test hook
    # that exercises the RCCL / mailbox exchange path at world size 1
    lm_split: bool = False
    expose_packet: bool = False    # lagged fits: the finalize kernel writes the last step's summed (and
                                   # data-parallel exchanged) gradient packet to HipBackend.grad (tests)
    # optimizer-step schedule on the GPU:
    #   "lag"        one kernel per step, the Adam update of step k applied by every
    #                workgroup in the prologue of kernel k+1 (no in-kernel sync)
    #   "ticket"     one kernel per step, last-arriving workgroup reduces + updates
    #                (deterministic slab / split update / fused xGMI DP)
    #   "persistent" one resident kernel per fit with an in-kernel grid barrier
    #   "auto"       1 rank: persistent up to PERSISTENT_MAX_WGS workgroups, lag above;
    #                data parallel: lag (fused xGMI) where valid, else ticket
    step_mode: str = "auto"
    # narrow lag kernel: 0 = weights hoisted into registers (1 wave/SIMD);
    # 1 = 2 waves/SIMD with LDS weight re-reads; 2/3 = 0/1 with the path-data
    # prefetch 2 iterations deeper; 4 = LDS weight re-reads at 1 wave/SIMD;
    # -1 = auto (4 for nets whose gradient packet is 256 wide - no scratch
    # spills - else 0)
    variant: int = -1


@dataclass
class DateData:
    """Inputs of one backward-induction fit (RP:200-201)."""

    feats: list                    # state_t features, each [n_local]
    prices_next: list              # traded assets at t+1 (bond excluded), each [n_local]
    bond_next: float               # B_{t+1} (normalised)
    target: torch.Tensor           # V_{t+1} [n_local]
    prices_now: list = field(default_factory=list)   # assets at t (for V_t)
    bond_now: float = 1.0
    # input standardisation x' = (x - fmu) * fisd, fused into the kernels'
    # feature loads (empty: identity = the reference's raw inputs)
    fmu: tuple = ()
    fisd: tuple = ()
    # LM fits: the global Gram subsample (gram_subsample) simulated on this
    # rank, slot order: state_t features and traded assets at t+1, each [ns]
    # (None: the Gram reads the shard; data parallel it is then summed over ranks)
    gram_feats: list | None = None
    gram_prices_next: list | None = None
    # pinball LM fits: V_{t+1} on the same subsample paths ([ns]), so the IRLS
    # Gram weights need no shard data and the fit is world-invariant (None:
    # pinball fits read the subsample from the shard)
    gram_target: torch.Tensor | None = None


@dataclass
class PnlData:
    """Inputs of the self-financing P&L scan (k_hedge_pnl / TorchBackend.pnl)."""

    n_dates: int
    features: object               # t -> list of [n_local] state-feature tensors at date t (raw)
    prices: object                 # t -> list of [n_local] traded-asset tensors at date t (bond excluded)
    bond: torch.Tensor             # [n_dates + 1] float64 bank account B_t (device)
    fmu: torch.Tensor              # [n_dates, MAXIN] float32 per-date standardisation (device)
    fisd: torch.Tensor             # [n_dates, MAXIN]
    w0: torch.Tensor               # [n_local] initial wealth (the fitted V_0)
    payoff: torch.Tensor           # [n_local] terminal liability


PNL_PPT = 4  # paths per thread of k_hedge_pnl (csrc/hedge_mlp.hip PNL_PPT)
GRAM_BLOCKS = 8  # global blocks of the LM Gram subsample (the largest single-node world size)


def _lm_bias_index(spec, t) -> int:
    """LmDesc.bias_index: the bond holding's output bias (the last parameter of
    a free-head net), -1 for the complement head or with lm_bias_fix off."""
    return spec.nparams - 1 if (t.lm_bias_fix and spec.head == L.HEAD_FREE) else -1


def lm_out_nu(spec) -> int:
    """Output-layer parameters of a net (csrc/hedge_narrow.h NarrowPairBody::NU):
    free head H x NO + NO, complement head H + 1."""
    return spec.hidden * spec.nout + spec.nout if spec.head == L.HEAD_FREE else spec.hidden + 1


def lm_out_gram(spec) -> bool:
    """The LM pass can build the full-batch output-layer Gram matrix on the
    matrix cores (NarrowPairBody OG: at most LM_OG_MAX output parameters)."""
    return spec.hidden == 8 and lm_out_nu(spec) <= L.LM_OG_MAX


def lm_og_wgs(spec) -> int:
    """Output-Gram workgroups of k_lm_reduce (64 packed entries each)."""
    nu = lm_out_nu(spec)
    npk = nu * (nu + 1) // 2
    epw = 16 if npk <= 512 else 64  # (csrc/hedge_lm.hip lm_og_epw)
    return (npk + epw - 1) // epw if nu <= L.LM_OG_MAX else 0


def _lm_out_n(spec, t) -> int:
    """LmDesc.out_n: output-layer parameters of the final exact Newton step
    with the full-batch output Gram (TrainConfig.lm_out_fix), 0 = the bias
    step alone."""
    return lm_out_nu(spec) if (t.lm_out_fix and lm_out_gram(spec)) else 0


def gram_subsample(n_total: int, lm_gram_paths: int) -> tuple[int, int, int]:
    """(ns, blk, stride) of the LM Gram subsample of a ``n_total``-path run: the
    first ``blk`` paths of each of ns / blk aligned global blocks of ``stride``
    paths (GRAM_BLOCKS blocks where the sizes allow: aligned prefixes of a
    Sobol sequence are nets; a strided subset is not).  The same global paths
    at every world size: every rank simulates them (index-addressable Sobol /
    Philox) and builds the identical Gram matrix, so the data-parallel exchange
    carries only the gradient region [g | stats | out-means]."""
    n_total = int(n_total)
    ns = max(L.LM_TILE, min(int(lm_gram_paths), n_total) // L.LM_TILE * L.LM_TILE)
    nb = GRAM_BLOCKS
    while nb > 1 and (ns % (L.LM_TILE * nb) or n_total % nb):
        nb //= 2
    return ns, ns // nb, n_total // nb


def lm_pass_wgs(n_local: int, wps: int = 1) -> int:
    """Workgroups of the LM pass kernel (HipBackend._lm_buffers; the torch
    oracle derives its Gram subsample from the same number): ``wps`` per CU
    (256 CUs; 2 for the nets whose plain pass body fits twice on a CU,
    native.lm_pass_wps), at most one per 256 local paths."""
    return int(max(1, min(256 * max(1, min(int(wps), L.LM_PASS_WGS_MAX // 256)), n_local // 256)))


def lm_pass_schedule(n_local: int, leaf_paths: int = 0, wps: int = 1) -> tuple[int, int]:
    """(pass workgroups, leaf blocks) of an LM pass over ``n_local`` paths
    (TrainConfig.lm_leaf_paths): auto (0) = lm_pass_wgs workgroups, the shard
    split into 4 x that many contiguous leaves; > 0 = leaves of that many
    paths (the workgroups to cover them, at most 256 x wps); < 0 = the cyclic
    schedule (leaf 0)."""
    nw = lm_pass_wgs(n_local, wps)
    nmax = lm_pass_wgs(1 << 40, wps)
    nblk = (int(n_local) + 127) // 128
    if leaf_paths < 0:
        return nw, 0
    if leaf_paths > 0:
        if leaf_paths % 128:
            raise ValueError(f"lm_leaf_paths must be a multiple of 128, got {leaf_paths}")
        # the world-invariance contract (a rank's rows form a complete subtree of
        # the one-rank contiguous-halves tree): whole leaves per shard and a
        # power-of-two number of pass workgroups per rank
        if int(n_local) % leaf_paths:
            raise ValueError(f"lm_leaf_paths {leaf_paths} does not divide the {n_local}-path shard")
        lb = leaf_paths // 128
        nw = int(min(nmax, max(1, -(-nblk // (4 * lb)))))
        if 4 * nw * lb < nblk:
            raise ValueError(f"{leaf_paths}-path leaves need more than {nmax} pass workgroups for {n_local} paths")
        if nw & (nw - 1):
            raise ValueError(f"lm_leaf_paths {leaf_paths} gives {nw} pass workgroups for {n_local} paths; world "
                             "invariance needs a power of two (choose a power-of-two shard and leaf size)")
        return nw, lb
    return nw, int(-(-nblk // (4 * nw)))


def lm_tpack_len(P: int, nblk: int) -> int:
    """Doubles of the solve's tile-store image of the Gram that k_lm_reduce
    writes after the 32 x 32 blocks (csrc/hedge_lm.hip LmTPack: nets with up
    to 48 tiles whose blocks and image fit the Gram region), else 0.  A Gram
    all-reduce over the ranks carries it with the blocks."""
    nt = (P + 1 + 15) // 16
    ntile = nt * (nt + 1) // 2
    nx = (P + 15) // 16 - 1 if ntile <= 48 else 0
    ln = ntile * 256
    return ln if nx > 0 and nblk * 1024 + ln <= L.LM_GBLK_MAX else 0


def lm_tpack_image(blocks, P: int, nblk: int):
    """The tile-store image k_lm_reduce writes at red[nblk * 1024:] (strictly
    lower Gram entries x2 at their csrc/lm_chol.h tile-store offsets) from the
    32 x 32 blocks red[:nblk * 1024], for code that builds a reduced block on
    the host (tests); None when the net has no image (lm_tpack_len 0)."""
    import numpy as np
    ln = lm_tpack_len(P, nblk)
    if ln == 0:
        return None
    nbg, nt = (P + 31) // 32, (P + 1 + 15) // 16
    e = np.arange(nblk * 1024)
    b, f = e >> 10, e & 1023
    starts = np.cumsum([0] + [nbg - m for m in range(nbg)])
    mb = np.searchsorted(starts, b, side="right") - 1
    nb = mb + (b - starts[mb])
    q, h = f >> 6, (f >> 5) & 1
    lo = 32 * mb + (q & 3) + 4 * h + 8 * (q >> 2)
    hi = 32 * nb + (f & 31)
    ok = (lo < hi) & (hi < P)
    ib, jb, r, c = hi >> 4, lo >> 4, hi & 15, lo & 15
    t = jb * nt - jb * (jb - 1) // 2 + (ib - jb)
    off = t * 256 + r * 16 + (c ^ ((r >> 1) << 1))
    img = np.zeros(ln)
    img[off[ok]] = 2.0 * np.asarray(blocks, dtype=np.float64)[:nblk * 1024][ok]
    return img


def lm_gram_geometry(n_local: int, ns_local: int, world: int) -> tuple[int, int]:
    """(gram_blk, gram_blk_stride) of the LM Gram subsample (LmDesc): the
    global path range is cut into GRAM_BLOCKS aligned blocks and the first
    paths of each block are used, so the subsample is the same set of global
    paths at world size 1, 2, 4, 8 (aligned prefixes of a Sobol sequence are
    nets; a strided subset is not: every 2^k-th point shares k digits)."""
    bpr = max(1, GRAM_BLOCKS // max(int(world), 1))   # blocks per rank
    while bpr > 1 and (ns_local % bpr or n_local % bpr):
        bpr //= 2
    return max(1, ns_local // bpr), max(1, n_local // bpr)
MAXIN = 8


def _set_norm(d, data: DateData):
    for i, (m, s) in enumerate(zip(data.fmu, data.fisd)):
        d.fmu[i], d.fisd[i] = float(m), float(s)


def _normalise(X: torch.Tensor, data: DateData) -> torch.Tensor:
    if not data.fmu:
        return X
    mu = torch.tensor(data.fmu, dtype=X.dtype, device=X.device)
    isd = torch.tensor(data.fisd, dtype=X.dtype, device=X.device)
    return (X - mu) * isd


def fit_seed(seed: int, date: int, net: int) -> int:
    return (int(seed) * 1000003 + int(date) * 7919 + int(net) * 104729) & 0xFFFFFFFF


# ---------------------------------------------------------------------------
# state helpers (shared by both backends)
# ---------------------------------------------------------------------------
def make_weights(spec: NetSpec, w0: np.ndarray, device) -> torch.Tensor:
    t = torch.zeros(L.NETW_FLOATS, dtype=torch.float32)
    t[: spec.nparams] = torch.from_numpy(np.asarray(w0, np.float32))
    t[L.PMAX: L.PMAX + spec.nparams] = t[: spec.nparams]
    t[L.W_CUR] = 0.0
    return t.to(device)


def make_opt(tcfg: TrainConfig, device) -> torch.Tensor:
    t = torch.zeros(L.OPT_FLOATS, dtype=torch.float32)
    t[L.O_LR] = tcfg.lr
    t[L.O_B1] = tcfg.beta1
    t[L.O_B2] = tcfg.beta2
    t[L.O_EPS] = tcfg.eps
    return t.to(device)


def fit_template(fcfg: FitConfig, device) -> torch.Tensor:
    t = torch.zeros(L.FIT_FLOATS, dtype=torch.float32)
    t[L.F_BEST] = float("inf")
    t[L.F_PATIENCE] = float(fcfg.patience if fcfg.early_stopping else 1e30)
    t[L.F_MAXEP] = float(fcfg.epochs)
    t[L.F_RESTORE] = 1.0 if (fcfg.restore_best and fcfg.early_stopping) else 0.0
    t[L.F_RESTORE_END] = 1.0 if fcfg.restore_at_end else 0.0
    t[L.F_HIST:] = float("nan")
    return t.to(device)


def current_weights(spec: NetSpec, wts: torch.Tensor) -> np.ndarray:
    w = wts.detach().cpu().numpy()
    cur = int(w[L.W_CUR])
    return w[cur * L.PMAX: cur * L.PMAX + spec.nparams].copy()


def set_weights(spec: NetSpec, wts: torch.Tensor, w: np.ndarray):
    t = torch.from_numpy(np.asarray(w, np.float32)).to(wts.device)
    wts[: spec.nparams] = t
    wts[L.PMAX: L.PMAX + spec.nparams] = t
    wts[L.W_CUR] = 0.0


def fit_summary(fit: torch.Tensor) -> dict:
    f = fit.detach().cpu().numpy()
    ep = int(f[L.F_EPOCH])
    return {"epochs": ep, "stopped": bool(f[L.F_STOPPED]), "best_loss": float(f[L.F_BEST]),
            "last_loss": float(f[L.F_LAST_LOSS]), "mae": float(f[L.F_LAST_MAE]),
            "mape": float(f[L.F_LAST_MAPE]), "history": f[L.F_HIST:L.F_HIST + min(ep, L.MAXHIST)].tolist()}


class _Cache:
    def __init__(self):
        self.d = {}

    def get(self, key, make):
        v = self.d.get(key)
        if v is None:
            v = make()
            self.d[key] = v
        return v


def _steps(n_local: int, tcfg: TrainConfig, world: int) -> tuple[int, int]:
    if tcfg.batch_size % world:
        raise ValueError(f"global batch {tcfg.batch_size} not divisible by world size {world}")
    bl = min(tcfg.batch_size // world, n_local)
    steps = max(1, math.ceil(n_local / bl))
    if n_local % bl:
        raise ValueError(f"local paths {n_local} must be a multiple of the local batch {bl}")
    return bl, steps


# ---------------------------------------------------------------------------
# HIP backend
# ---------------------------------------------------------------------------
PERSISTENT_MAX_WGS = 64  # "auto" picks the persistent per-fit kernel up to this grid (1 rank)


class HipBackend:
    name = "hip"

    def __init__(self, spec: NetSpec, n_local: int, tcfg: TrainConfig, device=None, comm=None,
                 world: int = 1, rank: int = 0, stream=None, mailbox=None, lm_mailbox=None, lm_comm=None):
        from .ops import native

        self.mailbox = mailbox  # native.IpcMailbox: fused xGMI all-reduce inside the step kernel
        self.lm_mailbox = lm_mailbox  # native.IpcMailbox (LM_DP_PITCH pitch): LM block exchange
        self._lm_nccl = lm_comm       # RCCL communicator of the LM block when its xGMI probe failed
        self.native = native
        native.load(required=True)
        self.spec, self.n_local, self.tcfg = spec, int(n_local), tcfg
        self.device = torch.device(device) if device is not None else torch.device("cuda", torch.cuda.current_device())
        self.comm, self.world, self.rank = comm, world, rank
        self.stream = stream
        self.P, self.R = native.net_nparams(spec.nin, spec.hidden, spec.nout, spec.head)
        assert self.P == spec.nparams
        self.batch_local, self.steps_per_epoch = _steps(self.n_local, tcfg, world)
        # narrow-body variant (csrc/hedge_mlp.hip launcher): 5 = W2 hoisted in
        # VGPRs + the rest from LDS, 2 waves/SIMD at 512 WGs (1-2 input nets:
        # 9.83 -> 9.64 / 10.05 -> 9.69 us per 2^18 step; the 3-input net is
        # slower that way), 4 = all weights from LDS (256-wide packets),
        # 0 = all weights hoisted (profiles/r1/stamp_r1u_hybrid.jsonl)
        # 512 workgroups only on one rank (with the in-kernel xGMI exchange every
        # workgroup polls the mailbox, so data-parallel runs keep 256) and only
        # where the hybrid body fits 2 waves/SIMD (<= 3 inputs, 128-wide packet);
        # the 256-wide-packet nets (basket 5-8-6) run it at 1 wave/SIMD, still
        # faster than all-LDS weights (16.6 -> 14.8 us, profiles/r1/stamp_r1v_masks.jsonl)
        hyb512 = spec.hidden == 8 and spec.nin <= 3 and self.R <= 128 and world == 1
        auto_v = 5 if (hyb512 or (spec.hidden == 8 and self.R > 128)) else 0
        self.variant = int(tcfg.variant) if int(tcfg.variant) >= 0 else auto_v
        work = max(1, self.batch_local // (256 * max(1, tcfg.paths_per_thread)))
        mw = int(tcfg.max_wgs)
        if mw <= 0:
            # 512 workgroups = 2 per CU only where two fit (the 1-input bf16
            # net); the wider-input nets run 1 per CU, so a 512 grid starts in
            # two waves (+15 us start spread, profiles/r1/stamp_r1s_wide_wgs.jsonl)
            mw = 512 if (spec.hidden == 32 and not tcfg.mfma_fp32 and spec.nin == 1) else 256
            if (self.variant == 5 and hyb512 and tcfg.step_mode in ("auto", "lag") and not tcfg.deterministic
                    and not tcfg.split_update):
                mw = 512  # lagged steps: 2 workgroups (2 waves/SIMD) per CU
        self.num_wgs = int(max(1, min(mw, work)))
        dev = self.device
        self.slab = torch.zeros(self.num_wgs, self.R, dtype=torch.float32, device=dev)
        self.counter = torch.zeros(4, dtype=torch.int32, device=dev)
        self.grad = torch.zeros(self.R, dtype=torch.float32, device=dev)
        self.acc = torch.zeros(8, self.R, dtype=torch.float32, device=dev)
        # persistent per-fit kernel: 3 rotating accumulator buffers + [arrivals, error] counters
        self.acc_fit = torch.zeros(3, L.LAG_SLOTS, self.R, dtype=torch.float32, device=dev)
        self.fit_ctl = torch.zeros(4, dtype=torch.int32, device=dev)
        self.lag = torch.zeros(2, L.LAG_FLOATS, dtype=torch.float32, device=dev)
        self._acc_clean = False  # acc_fit known zero (set by a lagged fit's finalize)
        self.stamps = None  # set to an int64 [num_wgs, 8] tensor for phase diagnostics
        # eval epilogue (k_hedge_eval): weights read from LDS, up to 4 resident
        # waves per SIMD, each thread walks its paths with a 4-deep load ring;
        # 2048 workgroups (2 paths per thread at 2^20): euro30 8.42 -> 8.28 ms
        # against 512 (profiles/r4/eval_wgs_sweep.txt)
        ewg = int(os.environ.get("RPH_EVAL_WGS", "2048"))
        self.eval_wgs = int(max(1, min(ewg, (self.n_local + 255) // 256)))
        self._cache = _Cache()
        self.lm_last_fused = False  # the last LM fit summed its gradient region inside k_lm_reduce
        self._lm_same_gram = True  # the last LM fit built the world-invariant Gram (exchange: gradient region only)

    # -- state ---------------------------------------------------------------
    def new_weights(self, w0):
        return make_weights(self.spec, w0, self.device)

    def new_opt(self):
        return make_opt(self.tcfg, self.device)

    def new_fit(self):
        return torch.zeros(L.FIT_FLOATS, dtype=torch.float32, device=self.device)

    def new_stats(self):
        return torch.zeros(self.eval_wgs, L.EVAL_NSTAT, dtype=torch.float64, device=self.device)

    def _template(self, fcfg: FitConfig):
        return self._cache.get(("fit", fcfg.key()), lambda: fit_template(fcfg, self.device))

    def _lr(self, fcfg: FitConfig):
        if fcfg.lr_schedule is None:
            return None
        return self._cache.get(("lr", tuple(fcfg.lr_schedule)),
                               lambda: torch.tensor(list(fcfg.lr_schedule), dtype=torch.float32, device=self.device))

    # -- ops -----------------------------------------------------------------
    def _train_desc(self, wts, opt, fit, data: DateData, fcfg: FitConfig, seed: int, lr_t):
        n = self.native
        d = n.TrainDesc()
        for i, f in enumerate(data.feats):
            d.feat[i] = f.data_ptr()
        for i, p in enumerate(data.prices_next):
            d.price[i] = p.data_ptr()
        d.target = data.target.data_ptr()
        d.wts, d.opt, d.fit = wts.data_ptr(), opt.data_ptr(), fit.data_ptr()
        d.lr_sched = lr_t.data_ptr() if lr_t is not None else None
        d.slab, d.counter, d.grad_out = self.slab.data_ptr(), self.counter.data_ptr(), self.grad.data_ptr()
        d.bond = float(data.bond_next)
        d.alpha = float(self.spec.alpha)
        d.quantile = float(fcfg.quantile)
        d.inv_batch = 1.0 / float(self.batch_local * self.world)
        d.loss = int(fcfg.loss)
        d.n_local = self.n_local
        d.batch = self.batch_local
        d.steps_per_epoch = self.steps_per_epoch
        d.chunk_log2 = int(self.tcfg.chunk_log2)
        d.shuffle = 1 if self.tcfg.shuffle else 0
        d.seed = int(seed) & 0xFFFFFFFF
        fused_dp = self.mailbox is not None and self.world > 1
        d.fused_update = 1 if ((self.world == 1 or fused_dp) and not self.tcfg.split_update) else 0
        if self.world > 1 and self.comm is None and not fused_dp:
            raise RuntimeError("HipBackend with world_size > 1 needs an RCCL communicator or an IPC mailbox")
        if fused_dp:
            self.mailbox.fill(d)
        else:
            d.dp_world, d.dp_rank = 1, 0
        d.acc = self.acc.data_ptr()
        d.deterministic = 1 if self.tcfg.deterministic else 0
        d.mfma_fp32 = 1 if self.tcfg.mfma_fp32 else 0
        d.variant = self.variant
        d.stamps = self.stamps.data_ptr() if self.stamps is not None else None
        d.num_wgs = self.num_wgs
        d.nin, d.h, d.nout, d.head = self.spec.nin, self.spec.hidden, self.spec.nout, self.spec.head
        _set_norm(d, data)
        return d

    def fit(self, wts, opt, fit, data: DateData, fcfg: FitConfig, seed: int, poll_every: int = 0):
        """Enqueue a full Keras ``fit`` (epochs x steps).  With ``poll_every``>0 the
        host checks the device early-stop flag every that many epochs and stops
        enqueueing; otherwise everything is asynchronous (graph-capturable) and
        surplus steps after an early stop are device-side no-ops."""
        assert len(data.feats) == self.spec.nin and len(data.prices_next) == self.spec.nhold - 1
        if fcfg.optimizer == "lm":
            return self._lm_fit(wts, opt, fit, data, fcfg)
        lr_t = self._lr(fcfg)
        d = self._train_desc(wts, opt, fit, data, fcfg, seed, lr_t)
        n, S = self.native, self.steps_per_epoch
        mode = self.step_mode(poll_every)
        if mode == "lag" and not self.tcfg.expose_packet:
            d.grad_out = None  # (the finalize kernel writes the packet only when asked)
        if mode == "lag" and fcfg.epochs > 0:
            # kernel 0 reads the fit-state template and publishes it as `fit`;
            # the previous lag fit's finalize left the accumulators zeroed
            d.fit_init = self._template(fcfg).data_ptr()
            if not self._acc_clean:
                n.memset_async(self.acc_fit, 0, self.stream)
        else:
            fit.copy_(self._template(fcfg), non_blocking=True)
        self._acc_clean = False
        if mode == "persistent":
            n.memset_async(self.acc_fit, 0, self.stream)
            n.memset_async(self.fit_ctl, 0, self.stream)
            d.acc, d.counter = self.acc_fit.data_ptr(), self.fit_ctl.data_ptr()
            n.train_fit(d, fcfg.epochs, self.stream)
            return
        if mode == "lag":
            d.acc, d.lag = self.acc_fit.data_ptr(), self.lag.data_ptr()
            if not poll_every:  # whole fit launched from the native runtime
                n.train_lag_fit(d, fcfg.epochs, self.stream)
                self._acc_clean = fcfg.epochs > 0
                return
            k = 0
            for e in range(fcfg.epochs):
                for s in range(S):
                    n.train_lag_step(d, k, e, self.stream)
                    k += 1
                if poll_every and (e + 1) % poll_every == 0 and e + 1 < fcfg.epochs:
                    if float(fit[L.F_STOPPED].item()) != 0.0:
                        break
            n.train_lag_finalize(d, k, self.stream)
            self._acc_clean = True  # (finalize zeroes the three accumulators)
            return
        per_step_host = (self.world > 1 and d.fused_update == 0) or self.tcfg.split_update
        if not poll_every and not per_step_host:
            n.train_ticket_fit(d, fcfg.epochs, self.stream)
            return
        for e in range(fcfg.epochs):
            for s in range(S):
                n.train_step(d, s, e, self.stream)
                if (self.world > 1 and d.fused_update == 0) or self.tcfg.split_update:
                    if self.comm is not None:
                        self.comm.allreduce_(self.grad, self.stream)
                    n.train_update(d, s, e, self.stream)
            if poll_every and (e + 1) % poll_every == 0 and e + 1 < fcfg.epochs:
                if float(fit[L.F_STOPPED].item()) != 0.0:
                    break

    # -- Levenberg-Marquardt ----------------------------------------------------
    def lm_supported(self) -> bool:
        return self.native.lm_shape(self.spec.nin, self.spec.hidden, self.spec.nout, self.spec.head) is not None

    def _lm_buffers(self, loss: int = L.LOSS_MSE):
        """LM state, reduced block, slabs and descriptor of this backend's fits
        of one loss (MSE and pinball fits keep separate states: each carries
        its own damping across dates)."""
        pin = int(loss) == L.LOSS_PINBALL

        def make():
            shp = self.native.lm_shape(self.spec.nin, self.spec.hidden, self.spec.nout, self.spec.head)
            if shp is None:
                raise ValueError(f"no Levenberg-Marquardt solver for net {self.spec} (8-unit nets up to 174 parameters)")
            P, R, nblk = shp
            t = self.tcfg
            wps = self.native.lm_pass_wps(self.spec.nin, self.spec.hidden, self.spec.nout, self.spec.head)
            wps = int(os.environ.get("RPH_LM_WPS", wps))  # (env: A/B)
            nw, leaf = lm_pass_schedule(self.n_local, int(os.environ.get("RPH_LM_LEAF", t.lm_leaf_paths)), wps)
            W = max(self.world, 1)
            # the global Gram subsample (every rank: gw = ns / 64 Gram workgroups,
            # past the path grid where it is larger)
            ns, gblk, gstride = gram_subsample(self.n_local * W, t.lm_gram_paths)
            gw = ns // L.LM_TILE
            # fallback without simulated subsample data, data parallel: this
            # rank's part of the subsample from its shard, the Gram summed over ranks
            ns_local = max(L.LM_TILE, min(int(t.lm_gram_paths) // W, self.n_local))
            gw_local = int(max(1, min(ns_local // L.LM_TILE, nw)))
            dev = self.device
            lm = self.native.LmDesc()
            bufs = dict(state=torch.zeros(L.LMS_FLOATS, dtype=torch.float64, device=dev),
                        red=torch.zeros(L.LM_RED, dtype=torch.float64, device=dev),
                        slab_b=torch.zeros(nw, R, dtype=torch.float32, device=dev),
                        slab_o=torch.zeros(nw if _lm_out_n(self.spec, t) else 1, 3 * 1024, dtype=torch.float32,
                                           device=dev),
                        slab_g=torch.zeros(max(gw, gw_local), nblk * 1024, dtype=torch.float32, device=dev))
            lm.state, lm.slab_b, lm.slab_g = (bufs[k].data_ptr() for k in ("state", "slab_b", "slab_g"))
            lm.slab_o = bufs["slab_o"].data_ptr()
            lm.num_wgs, lm.red_wgs = nw, nblk * 1024 // 64 + R // 4 + lm_og_wgs(self.spec)
            lm.inv_n = 1.0 / float(self.n_local * W)
            # (Gram geometry: per fit, _lm_gram_mode)
            bufs["gram"] = dict(side=(gw, gblk, gstride, 1.0 / float(ns)),
                                local=(gw_local,) + lm_gram_geometry(self.n_local, gw_local * L.LM_TILE, W) +
                                (1.0 / float(gw_local * L.LM_TILE * W),))
            # default (no subsample data): one rank reads the global subsample from its shard
            lm.gram_side = 0
            lm.gram_wgs, lm.gram_blk, lm.gram_blk_stride, lm.inv_ns = bufs["gram"]["side" if W == 1 else "local"]
            lm.lam0, lm.lam_up, lm.lam_down = t.lm_lam0, t.lm_lam_up, t.lm_lam_down
            lm.lam_min, lm.lam_max, lm.ridge = t.lm_lam_min, t.lm_lam_max, t.lm_ridge
            lm.diag_floor = float(t.lm_diag_floor)
            # (pinball fits: no output-layer / bias Newton step - the loss is not quadratic)
            lm.bias_index = -1 if pin else _lm_bias_index(self.spec, t)
            lm.out_n, lm.out_mu = (0 if pin else _lm_out_n(self.spec, t)), float(t.lm_out_mu)
            lm.out_tr = float(t.lm_out_tr)
            lm.out_gram = 1 if lm.out_n > 0 else 0
            lm.damping = 1 if str(t.lm_damping).lower() == "nielsen" else 0
            lm.gram_skip = int(os.environ.get("RPH_LM_GRAM_SKIP", t.lm_gram_skip))  # (env: tuning sweeps)
            lm.leaf_blocks = leaf
            bufs["desc"] = lm
            return bufs
        return self._cache.get(("lm",) if not pin else ("lm", L.LOSS_PINBALL), make)

    def _lm_gram_mode(self, lm, data: DateData, allow_side: bool = True) -> bool:
        """Set the Gram subsample of ``lm`` for a fit on ``data``; returns True
        when every rank builds the same Gram matrix (the exchange then carries
        only the gradient region).  One rank reads the subsample from its shard
        (the shard is the whole range) unless simulated subsample data is given;
        data parallel, the simulated subsample is required for the small exchange
        (without it: this rank's part of the subsample, Gram summed over ranks)."""
        g = self._lm_buffers()["gram"]
        side = allow_side and data.gram_feats is not None and data.gram_prices_next is not None
        lm.gtarget = data.gram_target.data_ptr() if (side and data.gram_target is not None) else None
        if side:
            gw, blk, stride, inv = g["side"]
            if data.gram_feats[0].numel() != gw * L.LM_TILE:
                raise ValueError(f"Gram subsample data has {data.gram_feats[0].numel()} paths, expected {gw * L.LM_TILE}")
            for i, f in enumerate(data.gram_feats):
                lm.gfeat[i] = f.data_ptr()
            for i, p in enumerate(data.gram_prices_next):
                lm.gprice[i] = p.data_ptr()
        elif self.world <= 1:
            gw, blk, stride, inv = g["side"]
        else:
            gw, blk, stride, inv = g["local"]
        lm.gram_side = 1 if side else 0
        lm.gram_wgs, lm.gram_blk, lm.gram_blk_stride, lm.inv_ns = gw, blk, stride, inv
        ov = os.environ.get("RPH_LM_GRAM_OVERLAP")  # (env: A/B)
        auto = int(lm.leaf_blocks) > 0 if self.tcfg.lm_gram_overlap is None else bool(self.tcfg.lm_gram_overlap)
        ov = bool(int(ov)) if ov is not None else auto
        lm.gram_base = lm.num_wgs if (ov and int(lm.inst) == 1) else 0
        return side or self.world <= 1

    def lm_exchange_bytes(self) -> int:
        """Bytes one rank pushes to EACH peer per LM pass (the gradient region
        when the Gram is built redundantly, else the whole reduced block)."""
        if self.world <= 1:
            return 0
        P, _, nblk = self.native.lm_shape(self.spec.nin, self.spec.hidden, self.spec.nout, self.spec.head)
        return 8 * self._lm_greg(False) if self._lm_same_gram else 8 * (nblk * 1024 + lm_tpack_len(P, nblk) + L.LM_RED - L.LM_GBLK_MAX)

    def _lm_greg(self, og: bool) -> int:
        """Doubles of the gradient region a pass exchanges (even: 16-byte
        pushes): [g (LM_NPMAX) | stats (8)], + the packed output Gram in the
        passes that build it."""
        n = L.LM_RED_OUTG - L.LM_GBLK_MAX
        if og:
            nu = lm_out_nu(self.spec)
            n += nu * (nu + 1) // 2
        return n + (n & 1)

    def lm_exchange_bytes_run(self, passes_first: int, passes_rest: int, dates: int) -> int:
        """Bytes one rank pushes to each peer over a whole induction (the
        output-Gram passes carry the packed output Gram as well)."""
        if self.world <= 1:
            return 0
        if not self._lm_same_gram:
            return self.lm_exchange_bytes() * (passes_first + 1 + (dates - 1) * (passes_rest + 1))
        og = bool(_lm_out_n(self.spec, self.tcfg))
        tot = 0
        for n in [passes_first] + [passes_rest] * (dates - 1):
            k_og = min(L.LM_OUTG_TAIL, n + 1) if og else 0
            tot += 8 * ((n + 1 - k_og) * self._lm_greg(False) + k_og * self._lm_greg(True))
        return tot

    def _lm_fit(self, wts, opt, fit, data: DateData, fcfg: FitConfig):
        """Enqueue a full-batch Levenberg-Marquardt fit (MSE): ``fcfg.epochs``
        trial points after the start point, 3 launches each (pass, reduce,
        solve), graph-capturable; data parallel: the gradient region [g |
        stats | out-means] (2.1 KB) is all-reduced between reduce and solve
        (every rank builds the same Gram matrix from the simulated global
        subsample; without it the whole reduced block travels)."""
        pin = int(fcfg.loss) == L.LOSS_PINBALL
        if int(fcfg.loss) not in (L.LOSS_MSE, L.LOSS_PINBALL):
            raise ValueError(f"no Levenberg-Marquardt fit for loss {fcfg.loss}")
        if pin and int(fcfg.lm_starts) >= 1 and int(fcfg.lm_explore_passes) > 0:
            raise ValueError("pinball LM fits have no multi-start exploration")
        b = self._lm_buffers(fcfg.loss)
        lm = b["desc"]
        # (pinball: the IRLS Gram weights need the targets of the subsample
        # paths - the simulated subsample's own when the driver evaluated them
        # (DateData.gram_target), else the shard subsample)
        self._lm_same_gram = self._lm_gram_mode(lm, data, allow_side=(not pin or data.gram_target is not None))
        lm.q_delta = float(fcfg.lm_q_delta) if float(fcfg.lm_q_delta) > 0.0 else 1e-6
        lm.q_kappa = float(fcfg.lm_q_kappa)
        lm.passes = int(fcfg.epochs)
        lm.stop_tol, lm.stop_min = float(fcfg.lm_stop_tol), max(1, int(fcfg.lm_stop_min))
        lm.lam0 = float(self.tcfg.lm_lam0 if fcfg.lm_lam0 is None else fcfg.lm_lam0)
        d = self._train_desc(wts, opt, fit, data, fcfg, 0, None)
        d.batch, d.steps_per_epoch, d.shuffle = self.n_local, 1, 0
        d.inv_batch = 1.0 / float(self.n_local * max(self.world, 1))
        d.loss = int(fcfg.loss)
        d.quantile = float(fcfg.quantile)
        n = self.native
        lm.lam_carry = float(fcfg.lm_lam_carry)
        lm.renorm = 0
        if fcfg.lm_renorm is not None and data.fmu:
            mu, isd = fcfg.lm_renorm
            for i in range(len(mu)):
                lm.ren_mu[i], lm.ren_isd[i] = float(mu[i]), float(isd[i])
            lm.renorm = 1
        if int(fcfg.lm_starts) >= 1 and int(fcfg.lm_explore_passes) > 0:
            self._lm_explore(d, fcfg)
            lm.lam_carry = 1.0  # the polish starts at the chosen exploration's damping
        # data parallel on the shared Gram subsample with the xGMI mailbox: the
        # gradient region is summed inside k_lm_reduce (no extra launch per pass)
        fused = (self.world > 1 and self.lm_mailbox is not None and self._lm_same_gram
                 and not self.tcfg.lm_split)
        lm.dp_fused = 1 if fused else 0
        self.lm_last_fused = fused  # (transport probe record: which exchange this fit ran)
        if fused:
            lm.dp = self._cache.get(("lm_dp",), self.lm_mailbox.lm_desc)
        if (self.world <= 1 or fused) and not self.tcfg.lm_split:
            n.lm_fit(d, lm, b["red"], self.stream)
            return
        for k in range(lm.passes + 1):
            n.lm_eval(d, lm, b["red"], k, self.stream)
            og = bool(lm.out_gram) and k > lm.passes - L.LM_OUTG_TAIL
            self._lm_allreduce(b["red"], gram=not self._lm_same_gram, og=og)
            n.lm_solve(d, lm, b["red"], k, self.stream)

    def lm_explore_paths(self, fcfg: FitConfig) -> int:
        """Paths of a multi-start exploration: the global prefix (a multiple of
        256: one pass workgroup per 256 paths)."""
        have = int(fcfg.lm_explore_data.target.numel()) if fcfg.lm_explore_data is not None else self.n_local
        want = int(fcfg.lm_explore_paths) if int(fcfg.lm_explore_paths) > 0 else have
        return int(max(256, min(have, want) // 256 * 256))

    def _lm_explore(self, d_main, fcfg: FitConfig):
        """Multi-start exploration of a first date (graph-capturable): K
        independent LM fits in ONE launch per kernel (grid y = instance) on the
        global path prefix (FitConfig.lm_explore_data, or this rank's shard
        prefix when it is the global one); k_lm_select writes the winner into
        the NetWeights and its damping into the main LM state (the polish fit
        carries it).  Every rank runs the same fits on the same paths: the
        pick needs no exchange and does not depend on the world size."""
        b = self._lm_buffers()
        K = int(fcfg.lm_starts)
        xd = fcfg.lm_explore_data
        if self.world > 1 and xd is None:
            raise ValueError("data-parallel multi-start exploration needs lm_explore_data (the global prefix)")
        nsub = self.lm_explore_paths(fcfg)
        if K > L.LM_SEL_MAX:
            raise ValueError(f"{K} starts exceed the {L.LM_SEL_MAX} selection candidates")
        if fcfg.lm_w0s is None or len(fcfg.lm_w0s) < K:
            raise ValueError("multi-start exploration needs lm_w0s (one start point per instance)")
        P = self.P

        def make():
            _, R, nblk = self.native.lm_shape(self.spec.nin, self.spec.hidden, self.spec.nout, self.spec.head)
            t, dev = self.tcfg, self.device
            # K instances in one launch: at most 256 x wps / K pass workgroups
            # each, so the whole grid is co-resident (wps workgroups per CU) and
            # a pass costs one round of workgroups, not K
            wps = self.native.lm_pass_wps(self.spec.nin, self.spec.hidden, self.spec.nout, self.spec.head)
            wps = int(os.environ.get("RPH_LM_EXPLORE_WPS", wps))  # (env: A/B)
            nw, leaf = lm_pass_schedule(nsub, 0 if int(t.lm_leaf_paths) >= 0 else -1, wps)
            nw1 = lm_pass_schedule(nsub, 0 if int(t.lm_leaf_paths) >= 0 else -1)[0]
            if K > 1:
                nw = max(1, min(nw, 256 * wps // K))
                nw1 = max(1, min(nw1, 256 // K))
                if leaf > 0:
                    leaf = -(-((nsub + 127) // 128) // (4 * nw))
            # (the Gram subsample: one 64-path tile per workgroup of a one-per-CU
            # grid - the same subsample whatever wps)
            gw = int(max(1, min(max(L.LM_TILE, min(int(t.lm_gram_paths), nsub)) // L.LM_TILE, nw1)))
            w0 = torch.zeros(K, L.LM_NPMAX, dtype=torch.float32)
            rows = np.asarray(fcfg.lm_w0s, dtype=np.float32)[:K, :P]
            w0[:, :P] = torch.from_numpy(np.ascontiguousarray(rows))
            bufs = dict(state=torch.zeros(K, L.LMS_FLOATS, dtype=torch.float64, device=dev),
                        red=torch.zeros(K, L.LM_RED, dtype=torch.float64, device=dev),
                        slab_b=torch.zeros(K, nw, R, dtype=torch.float32, device=dev),
                        slab_g=torch.zeros(K, gw, nblk * 1024, dtype=torch.float32, device=dev),
                        w0=w0.to(dev), sel=torch.zeros(L.LM_RED, dtype=torch.float64, device=dev))
            lm = type(b["desc"]).from_buffer_copy(b["desc"])
            lm.state, lm.slab_b, lm.slab_g = (bufs[k].data_ptr() for k in ("state", "slab_b", "slab_g"))
            lm.w0 = bufs["w0"].data_ptr()
            lm.inst, lm.explore, lm.lam_carry, lm.weights_only, lm.stop_tol, lm.renorm = K, 1, 0.0, 0, 0.0, 0
            lm.out_n, lm.out_gram, lm.gram_side, lm.dp_fused = 0, 0, 0, 0  # (the prefix's own Gram subsample)
            lm.gram_base = 0
            bufs["w0_rows"] = np.ascontiguousarray(rows).tobytes()
            lm.num_wgs, lm.gram_wgs, lm.leaf_blocks = nw, gw, leaf
            lm.gram_blk, lm.gram_blk_stride = lm_gram_geometry(nsub, gw * L.LM_TILE, 1)
            lm.inv_ns, lm.inv_n = 1.0 / float(gw * L.LM_TILE), 1.0 / float(nsub)
            bufs["desc"] = lm
            return bufs
        x = self._cache.get(("lm_explore", K, nsub), make)
        # this call's start points: a cached buffer must not keep an earlier
        # fit's candidates (a new set is uploaded on the backend's stream, after
        # the work already queued there; not inside a graph capture)
        rows = np.ascontiguousarray(np.asarray(fcfg.lm_w0s, dtype=np.float32)[:K, :P])
        if rows.tobytes() != x["w0_rows"]:
            if self.device.type == "cuda" and torch.cuda.is_current_stream_capturing():
                raise RuntimeError("multi-start start points changed inside a graph capture")
            w0 = torch.zeros(K, L.LM_NPMAX, dtype=torch.float32)
            w0[:, :P] = torch.from_numpy(rows)
            if self.device.type == "cuda" and self.stream is not None:
                with torch.cuda.stream(self.stream):  # (the launches' stream: ordered after queued fits)
                    x["w0"].copy_(w0)
            else:
                x["w0"].copy_(w0)
            x["w0_rows"] = rows.tobytes()
        lm = x["desc"]
        lm.passes = int(fcfg.lm_explore_passes)
        lm.lam0 = float(self.tcfg.lm_lam0 if fcfg.lm_lam0 is None else fcfg.lm_lam0)
        d = type(d_main).from_buffer_copy(d_main)
        if xd is not None:
            for i, f in enumerate(xd.feats):
                d.feat[i] = f.data_ptr()
            for i, p in enumerate(xd.prices_next):
                d.price[i] = p.data_ptr()
            d.target = xd.target.data_ptr()
        d.n_local = d.batch = nsub
        d.inv_batch = 1.0 / float(nsub)
        n = self.native
        n.lm_fit(d, lm, x["red"], self.stream)
        n.lm_select(d, lm, x["sel"], b["state"], 1, 0, P, 0, self.stream)
        n.lm_select(d, lm, x["sel"], b["state"], 1, 0, P, 1, self.stream)
        self.lm_explore_last = x

    def _lm_allreduce(self, red: torch.Tensor, gram: bool = True, og: bool = False):
        """Sum the reduced LM block over the ranks: in-kernel exchange over the
        IPC mailboxes (xGMI transport) or one RCCL all-reduce.  ``gram=False``
        (every rank built the same Gram matrix): only the gradient region
        travels, [g | stats] = 200 doubles (1.6 KB), + the packed output Gram
        in the passes that build it (``og``)."""
        P, _, nblk = self.native.lm_shape(self.spec.nin, self.spec.hidden, self.spec.nout, self.spec.head)
        if self.lm_mailbox is not None:
            x = self._cache.get(("lm_dp",), self.lm_mailbox.lm_desc)
            if gram:
                self.native.lm_dp_exchange(x, red, nblk * 1024 + lm_tpack_len(P, nblk), P, self.stream)
            else:
                self.native.lm_dp_exchange(x, red, 0, self._lm_greg(og), self.stream)
            return
        if gram:
            self._lm_comm().allreduce_(red, self.stream)
        else:
            self._lm_comm().allreduce_(red[L.LM_GBLK_MAX:L.LM_GBLK_MAX + self._lm_greg(og)], self.stream)

    def bias_refit(self, wts, opt, fit, data: DateData, fcfg: FitConfig):
        """Exact refit of the bond holding's output bias after an Adam fit (one
        full-batch loss + gradient pass at the fitted weights, then the 1-D
        Newton step of the LM solver, FitState untouched): the residual's mean
        over all paths becomes zero, so no mean error drifts down the induction
        (V0 then sits on the paths' price instead of scattering with the
        minibatch noise of the last fits).  No-op for complement heads."""
        bi = _lm_bias_index(self.spec, self.tcfg)
        if bi < 0:
            return
        if not self.lm_supported():
            # nets without an LM solver (32-unit MFMA family): the eval kernel's
            # residual sum (res = target - prediction) gives the same step.
            # Every buffer is preallocated and every op writes into it (nothing
            # is allocated inside a graph capture); data parallel, the two sums
            # travel like an LM block: k_lm_dp_exchange over the LM mailbox
            # (xGMI) or the RCCL communicator chosen by select_transport
            c = self._cache.get(("refit",), self._refit_buffers)
            st, red = c["stats"], c["red"]
            G, S = L.LM_GBLK_MAX, L.LM_GBLK_MAX + L.LM_NPMAX
            self.eval(wts, data, st)
            torch.sum(st[:, L.ES_RES], dim=0, out=red[G])
            torch.sum(st[:, L.ES_COUNT], dim=0, out=red[S])
            if self.world > 1:
                if self.lm_mailbox is not None:
                    x = self._cache.get(("lm_dp",), self.lm_mailbox.lm_desc)
                    self.native.lm_dp_exchange(x, red, 0, L.LM_RED_OUTG - L.LM_GBLK_MAX, self.stream)
                else:
                    self._lm_comm().allreduce_(red[G:S + 1], self.stream)
            torch.clamp_min(red[S:S + 1], 1.0, out=c["cnt"])
            torch.div(red[G:G + 1], c["cnt"], out=c["delta"])
            c["delta"].mul_(1.0 / float(data.bond_next))
            wts[bi:bi + 1].add_(c["delta"])
            fit[L.F_WBEST + bi:L.F_WBEST + bi + 1].copy_(wts[bi:bi + 1])
            return
        b = self._lm_buffers()

        def make():
            src = b["desc"]
            lm = type(src).from_buffer_copy(src)
            lm.passes, lm.weights_only, lm.gram_wgs, lm.stop_tol, lm.out_n, lm.out_gram = 0, 1, 1, 0.0, 0, 0
            lm.renorm, lm.lam_carry, lm.gram_side, lm.dp_fused = 0, 0.0, 0, 0  # (not inherited from the main fit's desc)
            lm.gram_base = 0
            lm.gram_blk, lm.gram_blk_stride = lm_gram_geometry(self.n_local, L.LM_TILE, self.world)
            lm.inv_ns = 1.0 / float(L.LM_TILE * max(self.world, 1))
            return lm
        lm = self._cache.get(("lm_refit",), make)
        d = self._train_desc(wts, opt, fit, data, fcfg, 0, None)
        d.batch, d.steps_per_epoch, d.shuffle = self.n_local, 1, 0
        d.inv_batch = 1.0 / float(self.n_local * max(self.world, 1))
        d.loss = L.LOSS_MSE
        n = self.native
        if self.world <= 1:
            n.lm_fit(d, lm, b["red"], self.stream)
            return
        n.lm_eval(d, lm, b["red"], 0, self.stream)
        self._lm_allreduce(b["red"])
        n.lm_solve(d, lm, b["red"], 0, self.stream)

    def _refit_buffers(self) -> dict:
        dev = self.device
        return {"stats": self.new_stats(), "red": torch.zeros(L.LM_RED, dtype=torch.float64, device=dev),
                "cnt": torch.zeros(1, dtype=torch.float64, device=dev),
                "delta": torch.zeros(1, dtype=torch.float64, device=dev)}

    def _lm_comm(self):
        """RCCL communicator of the LM reduced block: the one select_transport
        created when the block's xGMI probe failed (``lm_comm``), else the
        backend's RCCL communicator.  Never created lazily here (it could be
        inside a graph capture)."""
        if self._lm_nccl is not None:
            return self._lm_nccl
        if self.comm is not None:
            return self.comm
        raise RuntimeError("LM reduced-block exchange without an xGMI mailbox or an RCCL communicator: build "
                           "data-parallel backends through rphedge.parallel.dist.select_transport (or pass lm_comm)")

    def lm_state(self) -> dict:
        """Host view of the last LM fit (accepted steps, Cholesky failures, damping)."""
        st = self._lm_buffers()["state"].cpu().numpy()
        return {"accepted": int(st[L.LMS_NACC]), "chol_failures": int(st[L.LMS_FAIL]), "lam": float(st[L.LMS_LAM]),
                "chol_failures_total": int(st[L.LMS_FAILTOT])}

    def step_mode(self, poll_every: int = 0) -> str:
        """Resolve TrainConfig.step_mode for this backend (see TrainConfig)."""
        t = self.tcfg
        atomic = not t.deterministic and not t.split_update
        dp_fused = self.mailbox is not None and self.comm is None
        if (t.step_mode == "persistent" and atomic and not poll_every and (self.world == 1 or dp_fused)
                and self.persistent_supported()):
            # (explicit only: needs every workgroup of every rank co-resident)
            return "persistent"
        shared = dp_fused and getattr(self.mailbox, "shared_device", False)
        if t.step_mode == "lag" and atomic and (self.world == 1 or dp_fused):
            return "lag"
        # small grids (the reference's batch 512 = 2 workgroups): the persistent
        # kernel's in-kernel barrier is cheaper than a kernel boundary below ~96
        # workgroups (profiles/r1/crossover_r1g.jsonl) and one launch per fit
        # removes the per-step host launch from eager runs
        if (t.step_mode == "auto" and atomic and self.world == 1 and not poll_every
                and self.spec.hidden == 8 and self.num_wgs <= PERSISTENT_MAX_WGS):
            return "persistent"
        if t.step_mode == "persistent" and atomic and (self.world == 1 or dp_fused):
            return "lag"  # shape without a persistent kernel (or host polling): lagged steps
        if t.step_mode == "auto" and atomic and (self.world == 1 or (dp_fused and not shared)):
            return "lag"
        return "ticket"

    def concurrent_with(self, other: "HipBackend") -> bool:
        """Whether a fit of this backend may run concurrently (another stream)
        with a fit of ``other`` without a co-residency deadlock: persistent
        kernels need every workgroup resident, so two of them must fit the
        device together (one workgroup per CU at one wave per SIMD)."""
        a, b = self.step_mode(), other.step_mode()
        cus = 256
        try:
            cus = int(torch.cuda.get_device_properties(self.device).multi_processor_count)
        except Exception:
            pass
        need = (self.num_wgs if a == "persistent" else 0) + (other.num_wgs if b == "persistent" else 0)
        if ("persistent" in (a, b)) and need > cus:
            return False
        return self.world == 1 and other.world == 1

    def persistent_supported(self) -> bool:
        """Shapes with a persistent per-fit kernel (csrc/hedge_fit.h): every
        8-unit net; the 32-unit nets up to 3 inputs (RPH_WIDE_FIT_SHAPES)."""
        return self.spec.hidden == 8 or self.spec.nin <= 3

    def check(self):
        """Raise if a persistent fit timed out waiting for co-resident workgroups."""
        if int(self.fit_ctl[1].item()) != 0:
            raise RuntimeError("persistent fit kernel: workgroups not co-resident (wait timed out); "
                               "use TrainConfig.step_mode='lag' or 'ticket'")

    def pnl_wgs(self) -> int:
        return (self.n_local + 256 * PNL_PPT - 1) // (256 * PNL_PPT)

    def new_pnl_stats(self):
        return torch.zeros(self.pnl_wgs(), L.EVAL_NSTAT, dtype=torch.float64, device=self.device)

    def pnl(self, snap, data: PnlData, stats, has_b: bool = False, hold_c: float = 0.0, pnl_out=None):
        """Enqueue the self-financing P&L scan (one k_hedge_pnl launch)."""
        n = self.native
        d = n.PnlDesc()
        f1 = data.features(1) if data.n_dates >= 1 else data.features(0)
        for i, f in enumerate(data.features(0)):
            d.feat[i] = f.data_ptr()
            d.feat_ts[i] = (f1[i].data_ptr() - f.data_ptr()) // 4
        p0, p1 = data.prices(0), data.prices(1)
        for k, p in enumerate(p0):
            d.price[k] = p.data_ptr()
            d.price_ts[k] = (p1[k].data_ptr() - p.data_ptr()) // 4
        d.snap = snap.data_ptr()
        d.fmu, d.fisd, d.bond = data.fmu.data_ptr(), data.fisd.data_ptr(), data.bond.data_ptr()
        d.w0, d.payoff = data.w0.data_ptr(), data.payoff.data_ptr()
        d.pnl_out = pnl_out.data_ptr() if pnl_out is not None else None
        d.stats = stats.data_ptr()
        d.alpha, d.hold_c, d.wealth0, d.has_b = float(self.spec.alpha), float(hold_c), 0.0, 1 if has_b else 0
        d.n_local, d.n_dates, d.num_wgs = self.n_local, int(data.n_dates), self.pnl_wgs()
        d.nin, d.h, d.nout, d.head = self.spec.nin, self.spec.hidden, self.spec.nout, self.spec.head
        assert stats.shape[0] == d.num_wgs and snap.shape[0] >= data.n_dates
        n.pnl(d, self.stream)

    def eval(self, wts, data: DateData, stats, wts_b=None, g_base=None, blend_c=0.0, hold_c=0.0,
             v_out=None, hold_out=None, resid_out=None, pred1_out=None, snap_a=None, snap_b=None,
             n_local: int | None = None):
        """k_hedge_eval over ``data`` (``n_local``: its path count when it is
        not this backend's shard, e.g. the Gram subsample)."""
        n = self.native
        d = n.EvalDesc()
        d.snap_a = snap_a.data_ptr() if snap_a is not None else None
        d.snap_b = snap_b.data_ptr() if snap_b is not None else None
        for i, f in enumerate(data.feats):
            d.feat[i] = f.data_ptr()
        for i, p in enumerate(data.prices_now):
            d.price_t[i] = p.data_ptr()
        for i, p in enumerate(data.prices_next):
            d.price_t1[i] = p.data_ptr()
        d.target = data.target.data_ptr() if data.target is not None else None
        d.wa = wts.data_ptr()
        d.wb = wts_b.data_ptr() if wts_b is not None else None
        d.g_base = g_base.data_ptr() if g_base is not None else None
        d.v_out = v_out.data_ptr() if v_out is not None else None
        if hold_out is not None:
            for k, h in enumerate(hold_out):
                d.hold_out[k] = h.data_ptr() if h is not None else None
        d.resid_out = resid_out.data_ptr() if resid_out is not None else None
        d.pred1_out = pred1_out.data_ptr() if pred1_out is not None else None
        d.stats = stats.data_ptr()
        d.bond_t, d.bond_t1 = float(data.bond_now), float(data.bond_next)
        d.alpha = float(self.spec.alpha)
        d.blend_c, d.hold_c = float(blend_c), float(hold_c)
        d.n_local = self.n_local if n_local is None else int(n_local)
        if d.n_local != int(data.feats[0].numel()):
            raise ValueError(f"eval over {data.feats[0].numel()} paths with n_local {d.n_local}")
        d.num_wgs = self.eval_wgs
        d.nin, d.h, d.nout, d.head = self.spec.nin, self.spec.hidden, self.spec.nout, self.spec.head
        _set_norm(d, data)
        n.eval_(d, self.stream)


# ---------------------------------------------------------------------------
# Torch reference backend (CPU oracle; gloo DP)
# ---------------------------------------------------------------------------
class TorchBackend:
    name = "torch"

    def __init__(self, spec: NetSpec, n_local: int, tcfg: TrainConfig, device="cpu", comm=None,
                 world: int = 1, rank: int = 0, dtype=torch.float32, stream=None):
        self.spec, self.n_local, self.tcfg = spec, int(n_local), tcfg
        self.device = torch.device(device)
        self.world, self.rank = world, rank
        self.dtype = dtype
        self.batch_local, self.steps_per_epoch = _steps(self.n_local, tcfg, world)
        self.eval_wgs = 1
        self._order_cache = {}
        self._lm_lam_last = {}  # loss -> the last LM fit's final damping (FitConfig.lm_lam_carry)

    new_weights = HipBackend.new_weights
    new_opt = HipBackend.new_opt

    def new_fit(self):
        return torch.zeros(L.FIT_FLOATS, dtype=torch.float32, device=self.device)

    def new_stats(self):
        return torch.zeros(1, L.EVAL_NSTAT, dtype=torch.float64, device=self.device)

    def _order(self, seed, epoch):
        from .ops.philox import epoch_order

        key = (seed, epoch)
        o = self._order_cache.get(key)
        if o is None:
            o = torch.from_numpy(epoch_order(self.n_local, self.tcfg.chunk_log2, seed, epoch,
                                             self.tcfg.shuffle)).to(self.device)
            if len(self._order_cache) > 64:
                self._order_cache.clear()
            self._order_cache[key] = o
        return o

    def _allreduce(self, t: torch.Tensor):
        if self.world > 1:
            import torch.distributed as dist

            dist.all_reduce(t)
        return t

    def _lm_fit(self, wts, fit, data: DateData, fcfg: FitConfig):
        """Reference semantics of the HIP Levenberg-Marquardt fit (hedge_lm.hip):
        same trial sequence, damping rule, Gram subsample (the first
        lm_gram_paths / world local paths) and bookkeeping, in float64; the
        multi-start exploration (k_lm_select) and the damping carry included."""
        from torch.func import jacrev, vmap

        spec, t = self.spec, self.tcfg
        P = spec.nparams
        dt = torch.float64
        pin = int(fcfg.loss) == L.LOSS_PINBALL
        q = float(np.float32(fcfg.quantile))
        q_delta = float(np.float32(fcfg.lm_q_delta if float(fcfg.lm_q_delta) > 0.0 else 1e-6))
        q_kappa = float(np.float32(fcfg.lm_q_kappa))
        X = _normalise(torch.stack([f.to(dt) for f in data.feats], dim=1), data)
        pr = torch.stack([p.to(dt) for p in data.prices_next] +
                         [torch.full_like(data.target, float(data.bond_next), dtype=dt)], dim=1)
        y = data.target.to(dt)
        W = max(self.world, 1)

        def v_one(w, x, p):
            return (torch_forward(spec, w, x[None])[0] * p).sum()

        side = None
        if data.gram_feats is not None and data.gram_prices_next is not None and (
                not pin or data.gram_target is not None):
            # the simulated global Gram subsample (identical on every rank; a
            # pinball fit also needs its targets for the IRLS weights)
            Xs = _normalise(torch.stack([f.to(dt) for f in data.gram_feats], dim=1), data)
            ps = torch.stack([p.to(dt) for p in data.gram_prices_next] +
                             [torch.full((Xs.shape[0],), float(data.bond_next), dtype=dt)], dim=1)
            side = (Xs, ps, data.gram_target.to(dt) if data.gram_target is not None else None)

        def make_eval(n_loc: int, world: int, main: bool = False):
            """evaluate(w) -> (G, g, stats) over the first n_loc local paths
            (all-reduced over the ranks when world > 1).  ``main``: the fit
            over every local path, whose Gram subsample is the global one of
            engine.gram_subsample (HipBackend._lm_gram_mode): from the
            simulated subsample data (the same G on every rank: only g and the
            statistics are summed) or, on one rank, from the shard."""
            Xn, prn, yn = X[:n_loc], pr[:n_loc], y[:n_loc]
            n_glob = float(n_loc * world)
            same_g = main and (side is not None or world == 1)
            if same_g:
                ns, blk, bstride = gram_subsample(n_loc * world, t.lm_gram_paths)
                inv_ns = 1.0 / float(ns)
                if side is not None:
                    Xg, pg, yg = side
                else:
                    sub = torch.tensor([(j // blk) * bstride + j % blk for j in range(ns)], dtype=torch.long)
                    Xg, pg, yg = Xn[sub], prn[sub], yn[sub]
            else:
                nw = lm_pass_wgs(n_loc)
                ns_local = max(L.LM_TILE, min(int(t.lm_gram_paths) // world, n_loc))
                gw = max(1, min(ns_local // L.LM_TILE, nw))
                ns = gw * L.LM_TILE
                inv_ns = 1.0 / float(ns * world)
                blk, bstride = lm_gram_geometry(n_loc, ns, world)
                sub = torch.tensor([(j // blk) * bstride + j % blk for j in range(ns)], dtype=torch.long)
                Xg, pg, yg = Xn[sub], prn[sub], yn[sub]

            def evaluate(w):
                wg = w.detach().clone().requires_grad_(True)
                e = (torch_forward(spec, wg, Xn) * prn).sum(1) - yn
                if pin:
                    # pinball loss of y - V (Replicating_Portfolio.py:138-145), its
                    # subgradient (path_loss), the IRLS Gram weights of its
                    # quadratic majoriser (k_lm_pass)
                    ed = e.detach()
                    pos = -q * ed >= (q - 1.0) * (-ed)
                    lvec = torch.where(pos, -q * ed, (q - 1.0) * (-ed))
                    lsum = lvec.sum()
                    dV = torch.where(pos, torch.full_like(ed, -q), torch.full_like(ed, 1.0 - q))
                    ((dV * (torch_forward(spec, wg, Xn) * prn).sum(1)).sum() / n_glob).backward()
                else:
                    lsum = (e * e).sum()
                    (lsum / n_glob).backward()
                J = vmap(jacrev(v_one), in_dims=(None, 0, 0))(w.detach(), Xg, pg)
                if pin:
                    rg = (torch_forward(spec, w.detach(), Xg) * pg).sum(1) - yg
                    ra = rg.abs()
                    # per 64-path tile: delta = max(q_delta, kappa x mean |r| of the tile)
                    dl = torch.clamp_min(q_kappa * ra.view(-1, L.LM_TILE).mean(1, keepdim=True), q_delta)
                    J = J * (0.5 / torch.sqrt(torch.maximum(ra.view(-1, L.LM_TILE), dl).reshape(-1)))[:, None]
                G = (J.T @ J).reshape(-1) * inv_ns
                rest = torch.cat([wg.grad.detach(),
                                  torch.stack([lsum.detach(), e.detach().abs().sum(),
                                               (e.detach().abs() / yn.abs().clamp_min(1e-7)).sum(),
                                               torch.tensor(float(len(yn)), dtype=dt)])])
                if world > 1:
                    if same_g:
                        self._allreduce(rest)  # (the gradient region only)
                    else:
                        red = torch.cat([G, rest])
                        self._allreduce(red)
                        G, rest = red[: P * P], red[P * P:]
                return G.reshape(P, P), rest[:P], rest[P:]
            return evaluate

        nielsen = str(t.lm_damping).lower() == "nielsen"

        def run(w_best, evaluate, passes, lam, tol=0.0, kmin=1):
            """The solve kernel's sequence: returns (w, G, g, stats, loss, lam, hist)."""
            nu = 2.0
            G, g, stb = evaluate(w_best)
            Lb = float(stb[0] / stb[3].clamp_min(1.0))
            hist = [Lb]
            self._lm_best_k = 0  # the evaluation the best point came from
            self._lm_last_eval = (w_best, g, Lb)
            for k in range(1, int(passes) + 1):
                Lb_old = Lb
                A = 2.0 * G
                dg = torch.diagonal(A).clone()
                dmp = torch.clamp_min(dg, float(np.float32(t.lm_diag_floor)) * float(dg.mean())) * lam + \
                    float(t.lm_ridge) * float(dg.mean())
                A = A + torch.diag(dmp)
                Lc, info = torch.linalg.cholesky_ex(A)
                pred = 0.0
                if int(info) != 0:
                    trial = w_best.clone()
                    lam = min(lam * t.lm_lam_up * t.lm_lam_up, t.lm_lam_max)
                else:
                    dlt = torch.cholesky_solve(-g[:, None], Lc)[:, 0]
                    trial = w_best + dlt
                    pred = float(0.5 * ((dmp * dlt * dlt).sum() - (g * dlt).sum()))
                Gt, gt, stt = evaluate(trial)
                Lt = float(stt[0] / stt[3].clamp_min(1.0))
                hist.append(Lt)
                self._lm_last_eval = (trial, gt, Lt)  # (the last trial: the final out step may start there)
                accepted = Lt == Lt and Lt < Lb
                if accepted:
                    if nielsen:
                        rho = (Lb - Lt) / pred if pred > 0.0 else 1.0
                        lam = max(lam * max(1.0 / 3.0, 1.0 - (2.0 * rho - 1.0) ** 3), t.lm_lam_min)
                        nu = 2.0
                    else:
                        lam = max(lam * t.lm_lam_down, t.lm_lam_min)
                    w_best, G, g, stb, Lb = trial, Gt, gt, stt, Lt
                    self._lm_best_k = k
                elif nielsen:
                    lam = min(lam * nu, t.lm_lam_max)
                    nu *= 2.0
                else:
                    lam = min(lam * t.lm_lam_up, t.lm_lam_max)
                # adaptive budget (the solve kernel's LSS_STOP rule, accepted
                # steps only; fp32 tolerance)
                if tol > 0.0 and k >= kmin and accepted and not (Lb_old - Lb > float(np.float32(tol)) * Lb):
                    break
            return w_best, G, g, stb, Lb, lam, hist

        cur = int(wts[L.W_CUR].item())
        w_best = wts[cur * L.PMAX: cur * L.PMAX + P].to(dt).clone()
        if fcfg.lm_renorm is not None and data.fmu:
            # the k_lm_pass start-point transform (fp64 from the fp32 weights, rounded once)
            o = spec.offsets
            f32 = lambda v: float(np.float32(v))  # noqa: E731
            w32 = wts[cur * L.PMAX: cur * L.PMAX + P].to(dt)
            mu_o, isd_o = fcfg.lm_renorm
            for j in range(spec.hidden):
                acc = float(w32[o["b1"] + j])
                for f in range(spec.nin):
                    acc += float(w32[o["W1"] + f * spec.hidden + j]) * f32(isd_o[f]) * (f32(data.fmu[f]) - f32(mu_o[f]))
                w_best[o["b1"] + j] = f32(acc)
            for f in range(spec.nin):
                r = f32(isd_o[f]) / f32(data.fisd[f])
                for j in range(spec.hidden):
                    w_best[o["W1"] + f * spec.hidden + j] = f32(float(w32[o["W1"] + f * spec.hidden + j]) * r)
        lam = float(t.lm_lam0 if fcfg.lm_lam0 is None else fcfg.lm_lam0)
        if float(fcfg.lm_lam_carry) > 0.0:
            lam = max(self._lm_lam_last.get(int(fcfg.loss), 0.0) * float(np.float32(fcfg.lm_lam_carry)),
                      float(np.float32(t.lm_lam_min)))
        K = int(fcfg.lm_starts)
        if K >= 1 and int(fcfg.lm_explore_passes) > 0:
            # multi-start exploration (k_lm_select): the same K fits on every
            # rank, on the global path prefix (FitConfig.lm_explore_data)
            xd = fcfg.lm_explore_data
            have = int(xd.target.numel()) if xd is not None else self.n_local
            want = int(fcfg.lm_explore_paths) if int(fcfg.lm_explore_paths) > 0 else have
            nsub = int(max(256, min(have, want) // 256 * 256))
            if xd is not None:
                Xs_ = _normalise(torch.stack([f.to(dt) for f in xd.feats], dim=1), data)
                ps_ = torch.stack([p.to(dt) for p in xd.prices_next] +
                                  [torch.full((Xs_.shape[0],), float(xd.bond_next), dtype=dt)], dim=1)
                X_main, pr_main, y_main = X, pr, y
                X, pr, y = Xs_, ps_, xd.target.to(dt)
            elif self.world > 1:
                raise ValueError("data-parallel multi-start exploration needs lm_explore_data (the global prefix)")
            ev = make_eval(nsub, 1)
            rows = np.asarray(fcfg.lm_w0s, dtype=np.float32)
            lam_x = float(t.lm_lam0 if fcfg.lm_lam0 is None else fcfg.lm_lam0)
            sel = torch.zeros(K, 2 + P, dtype=dt)
            for k in range(K):
                wk = torch.from_numpy(rows[k, :P].copy()).to(dt)
                wb, _, _, _, lb, lk, _ = run(wk, ev, int(fcfg.lm_explore_passes), lam_x)
                sel[k, 0], sel[k, 1], sel[k, 2:] = lb, lk, wb
            if xd is not None:
                X, pr, y = X_main, pr_main, y_main
            ls = sel[:, 0].clone()
            ls[torch.isnan(ls)] = float("inf")
            pick = int(torch.argmin(ls))  # (first index of the minimum)
            w_best = sel[pick, 2:].to(torch.float32).to(dt)
            lam = max(float(sel[pick, 1]), t.lm_lam_min)
            self.lm_explore_last = {"losses": sel[:, 0].tolist(), "pick": pick}
        tol, kmin = float(fcfg.lm_stop_tol), max(1, int(fcfg.lm_stop_min))
        w_best, G, g, stb, Lb, lam, hist = run(w_best, make_eval(self.n_local, W, main=True), int(fcfg.epochs), lam,
                                               tol, kmin)
        self._lm_lam_last[int(fcfg.loss)] = lam
        bi = -1 if pin else _lm_bias_index(spec, t)
        n_out, out_ok = (0 if pin else _lm_out_n(spec, t)), False

        def out_step(wp, gp):
            """lm_out_newton at point wp (gradient gp): the full-batch output-layer
            Gram G_oo = mean_p u u^T, u = dV/dtheta_o; (step, exact loss change) or None."""
            h = spec.hidden
            o = spec.offsets
            W1 = wp[o["W1"]:o["b1"]].view(spec.nin, h)
            a1 = torch.nn.functional.leaky_relu(X @ W1 + wp[o["b1"]:o["W2"]], spec.alpha)
            a2 = torch.nn.functional.leaky_relu(a1 @ wp[o["W2"]:o["b2"]].view(h, h) + wp[o["b2"]:o["W3"]], spec.alpha)
            c = pr if spec.head == L.HEAD_FREE else (pr[:, 0] - pr[:, 1])[:, None]
            u = torch.cat([(a2[:, :, None] * c[:, None, :]).reshape(len(c), -1), c], dim=1)
            Goo = u.T @ u
            if self.world > 1:
                self._allreduce(Goo)
            Goo = Goo / float(self.n_local * self.world)
            A = 2.0 * Goo
            dgA = torch.diagonal(A).clone()
            A = A + torch.diag(dgA * float(np.float32(t.lm_out_mu))) + \
                torch.eye(n_out, dtype=dt) * (float(np.float32(t.lm_ridge)) * float(dgA.sum()) / n_out)
            Lc, info = torch.linalg.cholesky_ex(A)
            if int(info) != 0:
                return None
            go = gp[P - n_out:]
            dlt = torch.cholesky_solve(-go[:, None], Lc)[:, 0]
            return dlt, float(go @ dlt + dlt @ Goo @ dlt)  # exact full-batch loss change

        # the solve kernel's final step: the last evaluation (k_lm_pass<BodyOG>,
        # LM_OUTG_TAIL = 1) built the output Gram; out step at the best point
        # when the last trial was accepted, else at the rejected last trial,
        # published when trial + step beats the best point; otherwise the bias step
        self.lm_out_dl = 0.0
        ran_all = len(hist) - 1 == int(fcfg.epochs)  # (an adaptive stop skips the output-Gram pass)
        if n_out and ran_all:
            if self._lm_best_k == int(fcfg.epochs):
                r = out_step(w_best, g)
                if r is not None:
                    w_best = w_best.clone()
                    w_best[P - n_out:] += r[0]
                    self.lm_out_dl, out_ok = r[1], True
            else:
                lw, lg, lL = self._lm_last_eval
                r = out_step(lw, lg) if (lL == lL and lL < 2.0 * Lb) else None
                if r is not None and lL + r[1] < Lb:
                    w_best = lw.clone()
                    w_best[P - n_out:] += r[0]
                    Lb, self.lm_out_dl, out_ok = lL, r[1], True
        # (the bond holding's bias: dV/db = B on every path, so G_bb = B^2
        # exactly - as k_lm_solve, independent of the subsample Gram's rounding)
        gbb = float(np.float32(data.bond_next)) ** 2
        if not out_ok and bi >= 0 and gbb > 0.0:
            w_best = w_best.clone()
            w_best[bi] -= g[bi] / (2.0 * gbb)
        w32 = w_best.to(torch.float32)
        wts[:P] = w32
        wts[L.PMAX:L.PMAX + P] = w32
        wts[L.W_CUR] = 0.0
        fit.zero_()
        fit[L.F_HIST:] = float("nan")  # (as k_lm_pass: passes never run stay NaN)
        fit[L.F_WBEST:L.F_WBEST + P] = w32
        c = max(float(stb[3]), 1.0)
        fit[L.F_BEST] = Lb + self.lm_out_dl
        fit[L.F_LAST_LOSS] = Lb + self.lm_out_dl
        fit[L.F_LAST_MAE] = float(stb[1]) / c
        fit[L.F_LAST_MAPE] = 100.0 * float(stb[2]) / c
        fit[L.F_EPOCH] = len(hist)
        fit[L.F_STOPPED] = 1.0
        fit[L.F_HASBEST] = 1.0
        k = min(len(hist), L.MAXHIST)
        fit[L.F_HIST:L.F_HIST + k] = torch.tensor(hist[:k], dtype=torch.float32)
        self.lm_last = {"lam": lam, "hist": hist}

    def bias_refit(self, wts, opt, fit, data: DateData, fcfg: FitConfig):
        """Reference semantics of HipBackend.bias_refit: b_psi -= mean(e) / B
        (e = fitted value - target over all paths, B = the bond price)."""
        spec = self.spec
        bi = _lm_bias_index(spec, self.tcfg)
        if bi < 0:
            return
        dt = torch.float64
        X = _normalise(torch.stack([f.to(dt) for f in data.feats], dim=1), data)
        pr = torch.stack([p.to(dt) for p in data.prices_next] +
                         [torch.full_like(data.target, float(data.bond_next), dtype=dt)], dim=1)
        cur = int(wts[L.W_CUR].item())
        w = wts[cur * L.PMAX: cur * L.PMAX + spec.nparams].to(dt)
        e = (torch_forward(spec, w, X) * pr).sum(1) - data.target.to(dt)
        es = self._allreduce(torch.stack([e.sum(), torch.tensor(float(e.numel()), dtype=dt)]))
        wb = float(w[bi] - es[0] / es[1] / float(data.bond_next))
        for k in range(2):
            wts[k * L.PMAX + bi] = wb
        fit[L.F_WBEST + bi] = wb

    def fit(self, wts, opt, fit, data: DateData, fcfg: FitConfig, seed: int, poll_every: int = 0):
        spec, dt = self.spec, self.dtype
        P = spec.nparams
        if fcfg.optimizer == "lm":
            if int(fcfg.loss) not in (L.LOSS_MSE, L.LOSS_PINBALL):
                raise ValueError(f"no Levenberg-Marquardt fit for loss {fcfg.loss}")
            return self._lm_fit(wts, fit, data, fcfg)
        fit.copy_(fit_template(fcfg, self.device))
        X = _normalise(torch.stack([f.to(dt) for f in data.feats], dim=1), data)
        pr = torch.stack([p.to(dt) for p in data.prices_next] +
                         [torch.full_like(data.target, float(data.bond_next), dtype=dt)], dim=1)
        y = data.target.to(dt)
        cur = int(wts[L.W_CUR].item())
        w = wts[cur * L.PMAX: cur * L.PMAX + P].to(dt).clone()
        m = opt[L.O_M:L.O_M + P].to(dt).clone()
        v = opt[L.O_V:L.O_V + P].to(dt).clone()
        t_it = float(opt[L.O_T].item())
        lr = float(opt[L.O_LR].item())
        b1, b2, eps = (float(opt[i].item()) for i in (L.O_B1, L.O_B2, L.O_EPS))
        inv_b = 1.0 / float(self.batch_local * self.world)
        best, wait, has_best = float("inf"), 0, False
        w_best = w.clone()
        patience = fcfg.patience if fcfg.early_stopping else 1 << 30
        restore = fcfg.restore_best and fcfg.early_stopping
        hist = []
        sums = torch.zeros(4, dtype=torch.float64)
        stopped = False
        nan_steps = 0
        epoch = 0
        q = fcfg.quantile
        for epoch in range(fcfg.epochs):
            if fcfg.lr_schedule is not None:
                l_ = fcfg.lr_schedule[epoch]
                if l_ == l_:
                    lr = float(l_)
            order = self._order(seed, epoch)
            for s in range(self.steps_per_epoch):
                idx = order[s * self.batch_local:(s + 1) * self.batch_local]
                wv = w.detach().requires_grad_(True)
                V = (torch_forward(spec, wv, X[idx]) * pr[idx]).sum(dim=1)
                e = V - y[idx]
                if fcfg.loss == L.LOSS_PINBALL:
                    ep = -e
                    lvec = torch.maximum(q * ep, (q - 1.0) * ep)
                else:
                    lvec = e * e
                (lvec.sum() * inv_b).backward()
                pkt = torch.zeros(P + 4, dtype=torch.float64)
                pkt[:P] = wv.grad.to(torch.float64)
                with torch.no_grad():
                    pkt[P] = lvec.sum().double()
                    pkt[P + 1] = e.abs().sum().double()
                    pkt[P + 2] = (e.abs() / y[idx].abs().clamp_min(1e-7)).sum().double()
                    pkt[P + 3] = float(len(idx))
                self._allreduce(pkt)
                g = pkt[:P].to(dt)
                if torch.isfinite(g).all():
                    t_it += 1.0
                    lr_t = lr * math.sqrt(1.0 - b2 ** t_it) / (1.0 - b1 ** t_it)
                    m = m + (g - m) * (1.0 - b1)
                    v = v + (g * g - v) * (1.0 - b2)
                    w = (w - lr_t * m / (torch.sqrt(v) + eps)).detach()
                else:
                    nan_steps += 1
                sums += pkt[P:P + 4]
            cnt = max(float(sums[3]), 1.0)
            Lval = float(sums[0]) / cnt
            hist.append(Lval)
            fit[L.F_LAST_MAE] = float(sums[1]) / cnt
            fit[L.F_LAST_MAPE] = 100.0 * float(sums[2]) / cnt
            sums.zero_()
            wait += 1
            if Lval < best or not has_best:
                if Lval < best:
                    best, wait = Lval, 0
                has_best = True
                w_best = w.clone()
            if wait >= patience and epoch > 0:
                stopped = True
                if restore:
                    w = w_best.clone()
                break
        else:
            if restore and fcfg.restore_at_end:
                w = w_best.clone()
        n_ep = epoch + 1
        wts[:P] = w.to(torch.float32)
        wts[L.PMAX:L.PMAX + P] = w.to(torch.float32)
        wts[L.W_CUR] = 0.0
        opt[L.O_M:L.O_M + P] = m.to(torch.float32)
        opt[L.O_V:L.O_V + P] = v.to(torch.float32)
        opt[L.O_T] = t_it
        opt[L.O_LR] = lr
        opt[L.O_NAN] += nan_steps
        fit[L.F_BEST] = best
        fit[L.F_WAIT] = wait
        fit[L.F_HASBEST] = 1.0 if has_best else 0.0
        fit[L.F_STOPPED] = 1.0
        fit[L.F_EPOCH] = n_ep
        fit[L.F_LAST_LOSS] = hist[-1] if hist else float("nan")
        fit[L.F_WBEST:L.F_WBEST + P] = w_best.to(torch.float32)
        k = min(len(hist), L.MAXHIST)
        fit[L.F_HIST:L.F_HIST + k] = torch.tensor(hist[:k], dtype=torch.float32)
        _ = stopped

    def pnl_wgs(self) -> int:
        return 1

    def new_pnl_stats(self):
        return torch.zeros(1, L.EVAL_NSTAT, dtype=torch.float64, device=self.device)

    def pnl(self, snap, data: PnlData, stats, has_b: bool = False, hold_c: float = 0.0, pnl_out=None):
        """Self-financing P&L scan (reference semantics of k_hedge_pnl)."""
        spec, dt = self.spec, torch.float32
        P = spec.nparams
        bond = data.bond.detach().cpu().double().numpy()
        fmu, fisd = data.fmu.detach().cpu(), data.fisd.detach().cpu()
        wealth = data.w0.to(dt).clone()
        with torch.no_grad():
            for t in range(data.n_dates):
                X = torch.stack([f.to(dt) for f in data.features(t)], dim=1)
                X = (X - fmu[t, : spec.nin].to(dt)) * fisd[t, : spec.nin].to(dt)
                hold = torch_forward(spec, snap[t, 0, :P].to(dt), X)
                if has_b:
                    hb = torch_forward(spec, snap[t, 1, :P].to(dt), X)
                    hold = hold + hold_c * (hb - hold)
                grow = float(bond[t + 1] / bond[t])
                w = wealth * grow
                for a, (s0, s1) in enumerate(zip(data.prices(t), data.prices(t + 1))):
                    w = w + hold[:, a] * (s1.to(dt) - s0.to(dt) * grow)
                wealth = w
            pnl = wealth - data.payoff.to(dt)
            if pnl_out is not None:
                pnl_out.copy_(pnl)
            st = torch.zeros(L.EVAL_NSTAT, dtype=torch.float64)
            wd, pd = wealth.double(), pnl.double()
            st[L.ES_V], st[L.ES_V2] = wd.sum(), (wd * wd).sum()
            st[L.ES_RES], st[L.ES_RES2], st[L.ES_ABSRES] = pd.sum(), (pd * pd).sum(), pd.abs().sum()
            st[L.ES_COUNT] = pd.numel()
            st[L.ES_RESMIN], st[L.ES_RESMAX] = pd.min(), pd.max()
            stats[0].copy_(st)

    def eval(self, wts, data: DateData, stats, wts_b=None, g_base=None, blend_c=0.0, hold_c=0.0,
             v_out=None, hold_out=None, resid_out=None, pred1_out=None, snap_a=None, snap_b=None,
             n_local: int | None = None):
        spec, dt = self.spec, torch.float32
        P = spec.nparams
        if snap_a is not None:
            snap_a.copy_(wts)
        if snap_b is not None:
            snap_b.copy_(wts_b if wts_b is not None else wts)
        X = _normalise(torch.stack([f.to(dt) for f in data.feats], dim=1), data)

        def cw(t):
            cur = int(t[L.W_CUR].item())
            return t[cur * L.PMAX: cur * L.PMAX + P].to(dt)

        with torch.no_grad():
            hold = torch_forward(spec, cw(wts), X)
            holdv = hold
            if wts_b is not None:
                holdv = torch_forward(spec, cw(wts_b), X)
                hold = hold + hold_c * (holdv - hold)
            n = X.shape[0]
            pr0 = torch.stack([p.to(dt) for p in data.prices_now] +
                              [torch.full((n,), float(data.bond_now), dtype=dt, device=X.device)], dim=1)
            V = (holdv * pr0).sum(dim=1)
            if g_base is not None:
                V = g_base + blend_c * (V - g_base)
            if data.prices_next:
                pr1 = torch.stack([p.to(dt) for p in data.prices_next] +
                                  [torch.full((n,), float(data.bond_next), dtype=dt, device=X.device)], dim=1)
                pred1 = (hold * pr1).sum(dim=1)
            else:
                pred1 = torch.zeros_like(V)
            res = (data.target.to(dt) - pred1) if data.target is not None else torch.zeros_like(V)
            if v_out is not None:
                v_out.copy_(V)
            if hold_out is not None:
                for k, h in enumerate(hold_out):
                    if h is not None:
                        h.copy_(hold[:, k])
            if resid_out is not None:
                resid_out.copy_(res)
            if pred1_out is not None:
                pred1_out.copy_(pred1)
            st = torch.zeros(L.EVAL_NSTAT, dtype=torch.float64)
            Vd, rd, hd = V.double(), res.double(), hold.double()
            st[L.ES_V] = Vd.sum()
            st[L.ES_V2] = (Vd * Vd).sum()
            st[L.ES_RES] = rd.sum()
            st[L.ES_RES2] = (rd * rd).sum()
            st[L.ES_ABSRES] = rd.abs().sum()
            if data.target is not None:
                st[L.ES_APE] = (rd.abs() / data.target.double().abs().clamp_min(1e-7)).sum()
            st[L.ES_PRED1] = pred1.double().sum()
            st[L.ES_COUNT] = n
            for k in range(spec.nhold):
                st[L.ES_HOLD + k] = hd[:, k].sum()
                st[L.ES_HOLD2 + k] = (hd[:, k] ** 2).sum()
            st[L.ES_RESMIN] = rd.min()
            st[L.ES_RESMAX] = rd.max()
            stats[0].copy_(st)


def make_backend(kind: str, spec: NetSpec, n_local: int, tcfg: TrainConfig, **kw):
    if kind == "hip":
        return HipBackend(spec, n_local, tcfg, **kw)
    kw.pop("stream", None)
    kw.pop("mailbox", None)
    kw.pop("lm_mailbox", None)
    kw.pop("lm_comm", None)
    return TorchBackend(spec, n_local, tcfg, **kw)


def reduce_stats(stats: torch.Tensor, world: int = 1) -> np.ndarray:
    """Sum per-workgroup eval partials (and across ranks) -> [EVAL_NSTAT] float64."""
    s = stats.sum(dim=0)
    mn = stats[:, L.ES_RESMIN].min()
    mx = stats[:, L.ES_RESMAX].max()
    if world > 1:
        from .parallel.dist import all_reduce_

        all_reduce_(s)
        all_reduce_(mn, "min")
        all_reduce_(mx, "max")
    s = s.detach().cpu().numpy().copy()
    s[L.ES_RESMIN] = float(mn)
    s[L.ES_RESMAX] = float(mx)
    return s
