"""Backward-induction replicating-portfolio driver (SURVEY C22–C27, L6).

For every rebalancing date ``t = n-2 … 0`` (RP:193-227):

1. fit the hedge MLP on ``X1 = [state_t, prices_{t+1}] -> V_{t+1}`` with MSE
   (first date: 500 epochs, Keras LR schedule, patience 50; later: 100 epochs,
   patience 7; warm start from date t+1 — Q17/Q18);
2. ``g_t = predict(X0)``; ``Errors += evaluate(X1)`` (mae, mape);
3. optionally refit with the 99% pinball loss (separate network by default,
   the reference's shared-weights quirk Q1 with ``parity``);
4. ``V_t = g_t + c (h_t - g_t)``; holdings, one-step residual ("VaR", Q24) and
   per-date statistics in one fused epilogue kernel.

Everything is enqueued on one stream without host synchronisation, so the
whole scan (simulation included, see :mod:`rphedge.api`) can be captured into a
single hipGraph and replayed (``bench.py``).
"""
from __future__ import annotations

import math
from dataclasses import dataclass, field

import numpy as np
import torch

from .engine import (MAXIN, DateData, FitConfig, PnlData, TrainConfig, fit_seed, fit_summary,
                     geometric_lr_schedule, keras_lr_schedule, reduce_stats)
from .models.hedge_mlp import NetSpec
from .ops import layout as L
from .ops.paths import Paths


@dataclass
class InductionConfig:
    epochs_first: int = 500
    epochs_rest: int = 100
    patience_first: int = 50
    patience_rest: int = 7
    early_stopping: bool = True
    lr_schedule_first: bool = True
    lr: float = 1e-3                     # first-date lr of the geometric schedule (lr_decay != 1)
    lr_rest: float = 0.0                 # later dates (0: keep the optimiser's current lr)
    lr_decay: float = 1.0                # geometric decay per date, last/first epoch
    q99: bool = True
    quantile: float = 0.99
    cost_of_capital: float = 0.1
    shared_q99_model: bool = False       # Q1
    holdings_blend_sign_rp: bool = False  # Q2
    warm_start: bool = True              # Q18
    carry_optimizer: bool = True         # Q18: Adam state persists across dates
    restore_best_at_end: bool = False
    keep_paths: bool = True              # values / holdings / residual arrays
    poll_every: int = 0                  # host early-stop polling (0 = async)
    seed: int = 1234
    # input standardisation (fused into the kernels' feature loads):
    # "none" = raw features (reference), "global" = one mean/std per feature
    # pooled over all fitted dates, "date" = per-date mean/std
    feature_norm: str = "none"
    feature_centers: tuple | None = None  # horizon mode: the payoff kink per price feature (None: date mean)
    feature_norm_floor: float = 0.0      # horizon mode: scale >= this x the date spread
    optimizer: str = "adam"              # MSE fits: adam | lm (engine.FitConfig.optimizer)
    q99_optimizer: str = "adam"          # pinball fits (two networks): adam | lm (IRLS Gauss-Newton LM)
    lm_q_passes_first: int = 40
    lm_q_passes_rest: int = 4
    lm_q_delta: float = 1e-4             # IRLS weight floor, relative to the mean |terminal value|
    lm_q_kappa: float = 3.0              # IRLS weight cap relative to the Gram tile's mean |r|
    lm_q_start: str = "mse"              # pinball LM start point: mse (the date's MSE net) | warm (Q18)
    lm_passes_first: int = 80
    lm_passes_rest: int = 3
    lm_stop_tol: float = 0.0             # later dates: adaptive LM pass budget (engine.FitConfig)
    lm_stop_min: int = 2
    lm_lam0_rest: float = 0.0            # later dates' initial LM damping (0: TrainConfig.lm_lam0)
    lm_lam0_first: float = 0.0           # first date's initial LM damping (0: TrainConfig.lm_lam0)
    lm_lam_carry: float = 0.0            # later dates: start at the previous fit's final damping x this (0: off)
    lm_renorm: bool = False              # later dates: warm start re-expressed for the date's standardisation
    # first date: multi-start exploration (engine.FitConfig.lm_starts): lm_starts
    # LM fits per rank of lm_explore_passes trial points on the first
    # 2^lm_explore_log2 local paths, the best over all ranks polished for
    # lm_passes_first passes on every path (1: off)
    lm_starts: int = 1
    lm_explore_passes: int = 45
    lm_explore_log2: int = 16
    # lm_starts = 1: still run the exploration machinery with the one start
    # (a first-date warm-up of lm_explore_passes on the path prefix)
    lm_explore_one: bool = False
    # the extra start points use the run's initialiser (TrainingParams.init,
    # ParityFlags.shared_initializer), so candidate 0 is not the odd one out
    init_spread: bool = False
    init_align: tuple | None = None      # init="aligned": first-layer direction (models.hedge_mlp.init_weights)
    init_shared_stream: bool = False
    # after each Adam MSE fit: exact refit of the bond holding's output bias
    # (engine bias_refit; LM fits do it in their last solve)
    mean_refit: bool = False


@dataclass
class DateResult:
    index: int
    time: float
    fit_mse: dict | None = None
    fit_q99: dict | None = None
    stats: np.ndarray | None = None
    stats_mse: np.ndarray | None = None

    @property
    def count(self) -> float:
        return float(self.stats[L.ES_COUNT])

    def mean_holdings(self, nhold: int) -> np.ndarray:
        return self.stats[L.ES_HOLD:L.ES_HOLD + nhold] / self.count

    @property
    def mean_value(self) -> float:
        return float(self.stats[L.ES_V] / self.count)

    @property
    def residual_mean(self) -> float:
        return float(self.stats[L.ES_RES] / self.count)

    @property
    def residual_std(self) -> float:
        n = self.count
        m = self.stats[L.ES_RES] / n
        return float(math.sqrt(max(self.stats[L.ES_RES2] / n - m * m, 0.0) * n / max(n - 1, 1)))

    @property
    def errors(self) -> tuple[float, float]:
        """(mae, mape) of model1.evaluate(X1, V_{t+1}) after the MSE fit (RP:215)."""
        s = self.stats_mse if self.stats_mse is not None else self.stats
        n = s[L.ES_COUNT]
        return float(s[L.ES_ABSRES] / n), float(100.0 * s[L.ES_APE] / n)


@dataclass
class InductionResult:
    dates: list = field(default_factory=list)     # DateResult, ordered t = n-2 .. 0
    values: torch.Tensor | None = None            # [n_coarse, n_local]
    holdings: torch.Tensor | None = None          # [n_coarse-1, nhold, n_local]
    residuals: torch.Tensor | None = None         # [n_coarse-1, n_local] (residual of date t at index t)
    weights_snapshots: torch.Tensor | None = None  # [n_coarse-1, 2, NETW]
    v0: float = float("nan")
    holdings0: np.ndarray | None = None
    terminal: DateResult | None = None             # one-step residual of the last date (Q24 "P&L")
    pnl: DateResult | None = None                  # self-financing P&L: stats in the eval layout (ES_RES = P&L)
    pnl_paths: torch.Tensor | None = None          # [n_local] per-path self-financing P&L (keep_paths)


class BackwardInduction:
    """Owns device buffers for one run; ``enqueue()`` is graph-capturable."""

    def __init__(self, paths: Paths, v_terminal: torch.Tensor, spec: NetSpec, w0: np.ndarray, backend,
                 icfg: InductionConfig, world: int = 1, rank: int = 0, backend_q=None, gram_paths: Paths | None = None,
                 explore_paths: tuple | None = None, gram_terminal: torch.Tensor | None = None):
        self.paths, self.spec, self.backend, self.cfg = paths, spec, backend, icfg
        # LM fits: the global Gram subsample simulated on this rank (engine.gram_subsample)
        self.gram_paths = gram_paths
        # LM multi-start exploration: (paths, terminal values) of the global path
        # prefix simulated on this rank (None: the shard prefix is the global one)
        self.explore_paths = explore_paths
        # independent-network model parallelism: with two networks (corrected
        # Q1 semantics) the pinball fit of a date does not depend on that date's
        # MSE fit, so it runs on its own backend (own buffers) on a side stream,
        # concurrently with the MSE fit + its eval; the blend joins them
        self.backend_q = backend_q if (backend_q is not None and icfg.q99 and not icfg.shared_q99_model) else None
        self._side = None
        self.world, self.rank = world, rank
        n, nc = paths.n_local, paths.n_coarse
        dev = paths.S.device
        self.n_dates = nc - 1
        self.values = torch.empty(nc, n, dtype=torch.float32, device=dev)
        self.values[nc - 1].copy_(v_terminal)
        self.v_terminal = v_terminal
        self.gbuf = torch.empty(n, dtype=torch.float32, device=dev)
        keep = icfg.keep_paths
        self.holdings = torch.empty(nc - 1, spec.nhold, n, dtype=torch.float32, device=dev) if keep else None
        self.residuals = torch.empty(nc - 1, n, dtype=torch.float32, device=dev) if keep else None
        self.w_mse = backend.new_weights(w0)
        self.opt_mse = backend.new_opt()
        if icfg.q99:
            self.w_q = self.w_mse if icfg.shared_q99_model else backend.new_weights(w0)
            self.opt_q = backend.new_opt()
        self.w_init = backend.new_weights(w0)
        # multi-start start points of the first LM fit: candidate 0 = the run's
        # initial weights, the others the reference initialiser at seeds
        # seed + 1000 c (same data-dependent output bias); every rank runs all
        # of them on the same global path prefix (the same set at every world size)
        self.lm_w0s = None
        if icfg.optimizer == "lm" and (icfg.lm_starts > 1 or icfg.lm_explore_one):
            from .models import hedge_mlp as hm
            o = spec.offsets
            b3 = np.asarray(w0, np.float32)[o["b3"]:o["P"]]
            rows = [np.asarray(w0, np.float32)] + [hm.init_weights(spec, b3, seed=icfg.seed + 1000 * c,
                                                                   spread=icfg.init_spread, align=icfg.init_align,
                                                                   shared_stream=icfg.init_shared_stream)
                                                   for c in range(1, icfg.lm_starts)]
            self.lm_w0s = np.stack(rows)
        self.opt_init = backend.new_opt()
        self.fits = [[backend.new_fit(), backend.new_fit()] for _ in range(self.n_dates)]
        self.stats = [[backend.new_stats(), backend.new_stats()] for _ in range(self.n_dates)]
        # per-date weights (written by the final eval of each date): saved-model
        # format and the self-financing P&L scan
        self.snap = torch.zeros(self.n_dates, 2, L.NETW_FLOATS, dtype=torch.float32, device=dev)
        if icfg.lr_schedule_first:
            self.lr_first = tuple(keras_lr_schedule(icfg.epochs_first))
        else:
            self.lr_first = geometric_lr_schedule(icfg.lr, icfg.epochs_first, icfg.lr_decay) \
                if icfg.lr_decay != 1.0 else None
        self.lr_rest = geometric_lr_schedule(icfg.lr_rest or icfg.lr, icfg.epochs_rest, icfg.lr_decay) \
            if (icfg.lr_rest > 0 or icfg.lr_decay != 1.0) else None
        self.norms = feature_norms(paths, icfg.feature_norm, world, centers=icfg.feature_centers,
                                   floor=icfg.feature_norm_floor)
        # pinball LM fits on the global Gram subsample: its values V_t at every
        # date (the two-network blend evaluated on the subsample paths at the
        # date boundary, like values[t] on the shard), so the IRLS weights need
        # no shard data - every rank builds the same pinball Gram and the fit
        # takes the fused exchange (world-invariant, no per-pass exchange launch)
        self.gvalues = None
        q_lm_side = (icfg.q99 and not icfg.shared_q99_model and str(icfg.q99_optimizer).lower() == "lm"
                     and gram_paths is not None and gram_terminal is not None)
        if q_lm_side:
            ns = gram_terminal.numel()
            self.gvalues = torch.empty(nc, ns, dtype=torch.float32, device=dev)
            self.gvalues[nc - 1].copy_(gram_terminal)
            self.g_terminal = gram_terminal
            self.ggbuf = torch.empty(ns, dtype=torch.float32, device=dev)
            # (per-workgroup statistics of the subsample evaluations: not reported)
            self.gstats = [backend.new_stats(), backend.new_stats()]
        # pinball LM fits: the IRLS floor in target units (one sync at build time)
        self.q_lm = icfg.q99 and not icfg.shared_q99_model and str(icfg.q99_optimizer).lower() == "lm"
        self.q_delta = 0.0
        if self.q_lm:
            vs = torch.stack([v_terminal.double().abs().sum(),
                              torch.tensor(float(v_terminal.numel()), dtype=torch.float64, device=dev)])
            if world > 1:
                from .parallel import dist as D

                D.all_reduce_(vs)
            vs = vs.cpu().numpy()
            self.q_delta = float(icfg.lm_q_delta) * float(vs[0] / max(vs[1], 1.0))
        # self-financing P&L scan inputs (device tables built once, outside any capture)
        nd, nin = self.n_dates, spec.nin
        fmu = np.zeros((nd, MAXIN), np.float32)
        fisd = np.ones((nd, MAXIN), np.float32)
        for t, (mu, isd) in enumerate(self.norms):
            fmu[t, :nin], fisd[t, :nin] = mu, isd
        self.pnl_data = PnlData(n_dates=nd, features=paths.features, prices=paths.prices,
                                bond=torch.tensor(np.asarray(paths.bond, np.float64), device=dev),
                                fmu=torch.from_numpy(fmu).to(dev), fisd=torch.from_numpy(fisd).to(dev),
                                w0=self.values[0], payoff=self.values[nc - 1])
        self.pnl_stats = backend.new_pnl_stats()
        self.pnl_paths = torch.empty(n, dtype=torch.float32, device=dev) if keep else None
        self.pnl_done = False

    @property
    def hold_c(self) -> float:
        """Reported holdings hA + hold_c (hB - hA) (get_phi_psi_VaR, RP:114-115; Q2 sign)."""
        c = self.cfg
        return -c.cost_of_capital if c.holdings_blend_sign_rp else c.cost_of_capital

    def _fcfg(self, first: bool, loss: int, t: int | None = None) -> FitConfig:
        c = self.cfg
        if loss == L.LOSS_PINBALL and self.q_lm:
            # IRLS Gauss-Newton LM on the pinball loss (engine / hedge_lm.hip)
            return FitConfig(epochs=c.lm_q_passes_first if first else c.lm_q_passes_rest, loss=loss,
                             quantile=c.quantile, optimizer="lm", early_stopping=False,
                             lm_lam0=(c.lm_lam0_first if (first and c.lm_lam0_first > 0) else None),
                             lm_lam_carry=0.0 if first else c.lm_lam_carry, lm_q_delta=self.q_delta,
                             lm_q_kappa=c.lm_q_kappa)
        if c.optimizer == "lm" and loss == L.LOSS_MSE:
            ms = first and (c.lm_starts > 1 or c.lm_explore_one)
            # the warm start was fitted at date t + 1 (its standardisation)
            ren = (self.norms[t + 1] if (c.lm_renorm and not first and c.warm_start and t is not None and self.norms
                                         and t + 1 < len(self.norms)) else None)
            return FitConfig(epochs=c.lm_passes_first if first else c.lm_passes_rest, loss=loss,
                             optimizer="lm", early_stopping=False, lm_stop_tol=0.0 if first else c.lm_stop_tol,
                             lm_stop_min=c.lm_stop_min,
                             lm_lam0=((c.lm_lam0_first if c.lm_lam0_first > 0 else None) if first else
                                      (c.lm_lam0_rest if c.lm_lam0_rest > 0 else None)),
                             lm_lam_carry=0.0 if first else c.lm_lam_carry,
                             lm_starts=c.lm_starts if ms else 1,
                             lm_explore_passes=c.lm_explore_passes if ms else 0,
                             lm_explore_paths=(1 << int(c.lm_explore_log2)) if ms else 0,
                             lm_w0s=self.lm_w0s if ms else None, lm_renorm=ren,
                             lm_explore_data=self.explore_data(t) if (ms and t is not None) else None)
        return FitConfig(epochs=c.epochs_first if first else c.epochs_rest,
                         patience=c.patience_first if first else c.patience_rest,
                         loss=loss, quantile=c.quantile, lr_schedule=self.lr_first if first else self.lr_rest,
                         restore_best=True, restore_at_end=c.restore_best_at_end, early_stopping=c.early_stopping)

    def explore_data(self, t: int) -> DateData | None:
        """The multi-start exploration's data at date t: the global path prefix
        simulated on this rank (FitConfig.lm_explore_data), or None when the
        shard prefix is the global one (one rank).  Only for the FIRST fitted
        date (t = n_coarse - 2): the prefix carries the terminal payoff as its
        target, which is V_{t+1} only there."""
        if self.explore_paths is None:
            return None
        if t != self.paths.n_coarse - 2:
            raise ValueError(f"explore_data(t={t}): the exploration prefix holds the terminal payoff, the target of "
                             f"the first fitted date t = {self.paths.n_coarse - 2} only")
        xp, xv = self.explore_paths
        mu, isd = self.norms[t] if self.norms else ((), ())
        return DateData(feats=xp.features(t), prices_next=xp.prices(t + 1), bond_next=float(xp.bond[t + 1]),
                        target=xv, prices_now=xp.prices(t), bond_now=float(xp.bond[t]), fmu=mu, fisd=isd)

    def date_data(self, t: int) -> DateData:
        p = self.paths
        mu, isd = self.norms[t] if self.norms else ((), ())
        gp = self.gram_paths
        return DateData(feats=p.features(t), prices_next=p.prices(t + 1), bond_next=float(p.bond[t + 1]),
                        target=self.values[t + 1], prices_now=p.prices(t), bond_now=float(p.bond[t]),
                        fmu=mu, fisd=isd, gram_feats=gp.features(t) if gp is not None else None,
                        gram_prices_next=gp.prices(t + 1) if gp is not None else None,
                        gram_target=self.gvalues[t + 1] if self.gvalues is not None else None)

    def gram_date_data(self, t: int) -> DateData:
        """The Gram subsample as a date's eval input (its V_t for the pinball fits)."""
        gp = self.gram_paths
        mu, isd = self.norms[t] if self.norms else ((), ())
        return DateData(feats=gp.features(t), prices_next=gp.prices(t + 1), bond_next=float(gp.bond[t + 1]),
                        target=self.gvalues[t + 1], prices_now=gp.prices(t), bond_now=float(gp.bond[t]),
                        fmu=mu, fisd=isd)

    def enqueue(self, start: int | None = None):
        """Enqueue dates ``start, start-1, ..., 0`` (default: all, from n-2).
        Resume restarts at ``start = i-1`` after loading the
        weights and ``values[i]`` of a saved date i."""
        c, be = self.cfg, self.backend
        nc = self.paths.n_coarse
        start = nc - 2 if start is None else int(start)
        self.ran = list(range(start, -1, -1))
        for t in self.ran:
            first = t == nc - 2
            data = self.date_data(t)
            if not c.carry_optimizer and c.warm_start and not first:
                self.opt_mse.copy_(self.opt_init)
                if c.q99:
                    self.opt_q.copy_(self.opt_init)
            if not c.warm_start and not first:
                self.w_mse.copy_(self.w_init)
                self.opt_mse.copy_(self.opt_init)
                if c.q99:
                    if not c.shared_q99_model:
                        self.w_q.copy_(self.w_init)
                    self.opt_q.copy_(self.opt_init)
            f_m, f_q = self.fits[t]
            s_m, s_q = self.stats[t]
            join = None
            q_from_mse = self.q_lm and str(c.lm_q_start).lower() == "mse"
            if self.backend_q is not None and not q_from_mse:  # fork: Q99 fit on the side stream
                main = torch.cuda.current_stream(self.values.device)
                if self._side is None:
                    self._side = torch.cuda.Stream(self.values.device)
                fork = torch.cuda.Event()
                fork.record(main)
                self._side.wait_event(fork)
                with torch.cuda.stream(self._side):
                    self.backend_q.fit(self.w_q, self.opt_q, f_q, data, self._fcfg(first, L.LOSS_PINBALL),
                                       seed=fit_seed(c.seed, t, 1), poll_every=0)
                    join = torch.cuda.Event()
                    join.record(self._side)
            be.fit(self.w_mse, self.opt_mse, f_m, data, self._fcfg(first, L.LOSS_MSE, t),
                   seed=fit_seed(c.seed, t, 0), poll_every=c.poll_every)
            if c.mean_refit and c.optimizer != "lm":
                be.bias_refit(self.w_mse, self.opt_mse, f_m, data, self._fcfg(first, L.LOSS_MSE))
            hold_out = [self.holdings[t, k] for k in range(self.spec.nhold)] if self.holdings is not None else None
            resid_out = self.residuals[t] if self.residuals is not None else None
            if c.q99:
                be.eval(self.w_mse, data, s_m, v_out=self.gbuf)
                if join is not None:
                    torch.cuda.current_stream(self.values.device).wait_event(join)
                else:
                    if q_from_mse:
                        self.w_q.copy_(self.w_mse)  # (the date's fitted MSE net: Q1's alternate training)
                    be.fit(self.w_q, self.opt_q, f_q, data, self._fcfg(first, L.LOSS_PINBALL),
                           seed=fit_seed(c.seed, t, 1), poll_every=c.poll_every)
                be.eval(self.w_mse, data, s_q, wts_b=self.w_q, g_base=self.gbuf, blend_c=c.cost_of_capital,
                        hold_c=self.hold_c, v_out=self.values[t], hold_out=hold_out, resid_out=resid_out,
                        snap_a=self.snap[t, 0], snap_b=self.snap[t, 1])
                if self.gvalues is not None and t > 0:
                    # the same blend on the Gram subsample: V_t there, the next
                    # date's pinball-fit targets
                    gd = self.gram_date_data(t)
                    ns = self.ggbuf.numel()
                    be.eval(self.w_mse, gd, self.gstats[0], v_out=self.ggbuf, n_local=ns)
                    be.eval(self.w_mse, gd, self.gstats[1], wts_b=self.w_q, g_base=self.ggbuf,
                            blend_c=c.cost_of_capital, hold_c=self.hold_c, v_out=self.gvalues[t], n_local=ns)
            else:
                be.eval(self.w_mse, data, s_q, v_out=self.values[t], hold_out=hold_out, resid_out=resid_out,
                        snap_a=self.snap[t, 0])
        # self-financing P&L of the reported holdings (needs every date's network)
        self.pnl_done = start == nc - 2
        if self.pnl_done:
            be.pnl(self.snap, self.pnl_data, self.pnl_stats, has_b=c.q99, hold_c=self.hold_c,
                   pnl_out=self.pnl_paths)

    def collect(self) -> InductionResult:
        c = self.cfg
        nc = self.paths.n_coarse
        dtc = self.paths.grid.dt_coarse
        res = InductionResult(values=self.values, holdings=self.holdings, residuals=self.residuals,
                              weights_snapshots=self.snap)
        for t in getattr(self, "ran", range(nc - 2, -1, -1)):
            f_m, f_q = self.fits[t]
            s_m, s_q = self.stats[t]
            d = DateResult(index=t, time=t * dtc, fit_mse=fit_summary(f_m),
                           fit_q99=fit_summary(f_q) if c.q99 else None,
                           stats=reduce_stats(s_q, self.world),
                           stats_mse=reduce_stats(s_m, self.world) if c.q99 else None)
            res.dates.append(d)
        d0 = res.dates[-1]
        res.terminal = res.dates[0]
        res.v0 = d0.mean_value
        res.holdings0 = d0.mean_holdings(self.spec.nhold)
        if self.pnl_done:
            res.pnl = DateResult(index=-1, time=float(self.paths.grid.times()[-1]),
                                 stats=reduce_stats(self.pnl_stats, self.world))
            res.pnl_paths = self.pnl_paths
        return res


def price_features(paths: Paths) -> list:
    """Indices of the features that are traded-asset prices (their hedge ratio
    has a payoff kink): every feature of a GBM / basket run, feature 0 of an
    SV / Heston / pension run (its other features are variance / survivors)."""
    nin = len(paths.features(0))
    return list(range(nin)) if paths.kind not in ("pension", "heston", "sv") else [0]


def feature_norms(paths: Paths, mode: str, world: int = 1, centers=None, floor: float = 0.0) -> list:
    """Per-date ``(fmu, fisd)`` tuples for :class:`DateData` (empty list = raw
    inputs).  Moments are pooled over ranks (one host sync at build time);
    a feature with (near-)zero spread at a date (e.g. S_0 on every path) keeps
    unit scale so it maps to the constant 0.

    ``mode="horizon"``: the price features are centred at the payoff kink
    (``centers[i]``; None: the date mean) and scaled by the REMAINING-horizon
    spread m_t * sd(log S_T - log S_t) (m_t the date mean; for GBM F_t sigma
    sqrt(T - t)), the width of the hedge ratio's transition at date t - so the
    kink the net draws has unit width at every date instead of narrowing like
    sqrt((T - t) / t) under the date spread (``date``: sigma sqrt(t)).  The
    scale is floored at ``floor`` x the date spread.  Other features keep the
    date standardisation."""
    mode = (mode or "none").lower()
    if mode == "none":
        return []
    if mode not in ("global", "date", "horizon"):
        raise ValueError(f"feature_norm must be none | global | date | horizon, got {mode!r}")
    nd = paths.n_coarse - 1
    nin = len(paths.features(0))
    # per (date, feature): fp64-accumulated full sums of x and x*x (fast full
    # reductions on MI355X: torch.var_mean ran ~10x slower, a [nin, n] dim-1
    # reduction ~100x; fp64 accumulation keeps the pooled DP moments equal to
    # the one-process ones), gathered with two stacks
    s1, s2 = [], []
    for t in range(nd):
        for x in paths.features(t):
            s1.append(x.sum(dtype=torch.float64))
            s2.append((x * x).sum(dtype=torch.float64))
    cnt = float(paths.features(0)[0].numel())
    mom = torch.stack([torch.stack(s1).view(nd, nin), torch.stack(s2).double().view(nd, nin),
                       torch.full((nd, nin), cnt, dtype=torch.float64, device=paths.S.device)], dim=-1)
    if world > 1:
        from .parallel import dist as D

        D.all_reduce_(mom)
    m = mom.cpu().numpy()
    if mode == "global":
        m = np.broadcast_to(m.sum(axis=0, keepdims=True), m.shape)
    out = []
    for t in range(nd):
        cnt = np.maximum(m[t, :, 2], 1.0)
        mu = m[t, :, 0] / cnt
        var = np.maximum(m[t, :, 1] / cnt - mu * mu, 0.0)
        sd = np.sqrt(var)
        ok = sd > 1e-6 * (np.abs(mu) + 1.0)
        isd = np.where(ok, 1.0 / np.where(ok, sd, 1.0), 1.0)
        out.append([mu, isd, sd])
    if mode == "horizon":
        _horizon_norms(paths, out, world, centers, floor)
    return [(tuple(float(v) for v in mu), tuple(float(v) for v in isd)) for mu, isd, _ in out]


def _horizon_norms(paths: Paths, out: list, world: int, centers, floor: float):
    """feature_norms(mode="horizon") for the price features, in place: per
    (date, price feature) sums of r = log S_T - log S_t and r^2 over the
    paths (pooled over ranks), one date at a time (no [dates x paths]
    temporary: basket5 holds 2^23 paths x 253 dates x 5 assets).  The sums are
    int64 fixed point (2^-32 units): exact, so the scales - and a data-parallel
    fit - do not depend on the summation order or the world size."""
    nd = paths.n_coarse - 1
    pf = price_features(paths)
    nin = len(paths.features(0))
    last = paths.features(nd)
    lT = [torch.log(last[i].double()) for i in pf]
    s = []
    q = float(2 ** 32)
    for t in range(nd):
        ft = paths.features(t)
        for k, i in enumerate(pf):
            r = lT[k] - torch.log(ft[i].double())
            s.append(torch.round(r * q).to(torch.int64).sum())
            s.append(torch.round(r * r * q).to(torch.int64).sum())
    mom = torch.stack(s).view(nd, len(pf), 2)
    if world > 1:
        from .parallel import dist as D

        D.all_reduce_(mom)
    m = mom.cpu().numpy().astype(np.float64) / q
    cnt = float(paths.features(0)[0].numel()) * world
    for t in range(nd):
        mu, isd, sd = out[t]
        mu, isd = np.array(mu, dtype=np.float64), np.array(isd, dtype=np.float64)
        for k, i in enumerate(pf):
            rm = m[t, k, 0] / cnt
            rsd = math.sqrt(max(m[t, k, 1] / cnt - rm * rm, 0.0))
            scale = max(abs(mu[i]) * rsd, float(floor) * float(sd[i]))
            if scale > 1e-12 * (abs(mu[i]) + 1.0):
                c = centers[i] if (centers is not None and i < len(centers) and centers[i] is not None) else mu[i]
                mu[i], isd[i] = float(c), 1.0 / scale
        out[t] = [mu, isd, sd]
    assert len(out) == nd and all(len(o[0]) == nin for o in out)


def expected_value_trajectory(result: InductionResult, e_payoff: float, mu: float, r: float, dt: float) -> np.ndarray:
    """P_E_Values (C27, RP:190, :227): [mean V_t, E_payoff e^{-mu dt its}, E_payoff e^{-r dt its}]."""
    rows = [[e_payoff, e_payoff, e_payoff]]
    for its, d in enumerate(result.dates, start=1):
        rows.append([d.mean_value, e_payoff * math.exp(-mu * dt * its), e_payoff * math.exp(-r * dt * its)])
    return np.asarray(rows)


def error_history(result: InductionResult) -> np.ndarray:
    """Errors (C26, RP:189, :215): rows [mae, mape], first row zeros like the reference."""
    rows = [[0.0, 0.0]] + [list(d.errors) for d in result.dates]
    return np.asarray(rows)
