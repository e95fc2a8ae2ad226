"""Public API — same names, dict keys and return values as the reference.

* ``Replicating_Portfolio(params) -> (phi, psi)``     (``Replicating_Portfolio.py:29-235``)
* ``Replicating_Portfolio_SV(params) -> (phi, psi)``  (``Replicating_Portfolio.py:237-459``)
* ``european_option(**kw) -> RunResult``              (``European Options.ipynb`` cells 3-20)

plus :class:`HedgeRun`, the reusable pipeline (simulate -> payoff -> backward
induction -> report) used by the CLI, the examples and ``bench.py``.  On a GPU
the whole pipeline runs on device (HIP kernels, optional hipGraph capture and
RCCL data parallelism); on CPU the torch reference backend runs the same
algorithm.
"""
from __future__ import annotations

import math
import time
from dataclasses import dataclass, field

import numpy as np
import torch

from . import risk
from .config import RunConfig, parse_params
from .driver import BackwardInduction, InductionConfig, InductionResult, error_history, expected_value_trajectory
from .engine import TrainConfig, gram_subsample, make_backend, set_weights
from .models import hedge_mlp as hm
from .ops import layout as L
from .ops import paths as P
from .parallel import dist as D
from .utils.logging import get_logger
from .utils.profiling import PhaseTimer


@dataclass
class RunResult:
    phi: float
    psi: float
    v0: float                              # scaled (EUR / option price)
    scale: float
    holdings0: np.ndarray
    induction: InductionResult
    errors: np.ndarray
    p_e_values: np.ndarray
    terminal_pnl: dict
    var: dict = field(default_factory=dict)
    summary: dict = field(default_factory=dict)
    timings: dict = field(default_factory=dict)
    config: dict = field(default_factory=dict)
    paths: object = None                   # ops.paths.Paths of this rank (plots, C32)
    terminal_residual: dict = field(default_factory=dict)   # one-step residual at the last date (Q24)
    self_financing_pnl: dict | None = None                   # W_T - liability of the reported hedge

    def as_tuple(self):
        return self.phi, self.psi


class HedgeRun:
    """One replicating-portfolio run, reusable for graph replay."""

    def __init__(self, cfg: RunConfig, dist_info: D.DistInfo | None = None, stream=None):
        self.cfg = cfg
        self.log = get_logger()
        if dist_info is None:
            dist_info = D.init(device=cfg.device) if D.env_world() > 1 else D.DistInfo(
                device=torch.device(cfg.device) if cfg.device else
                (torch.device("cuda", torch.cuda.current_device()) if torch.cuda.is_available() else
                 torch.device("cpu")))
        self.di = dist_info
        self.device = dist_info.device
        self.backend_kind = cfg.backend or ("hip" if self.device.type == "cuda" else "torch")
        if self.backend_kind == "hip" and self.device.type != "cuda":
            raise ValueError("hip backend needs a GPU device")
        self.stream = stream
        self.grid = P.Grid(cfg.T, cfg.dt, cfg.rebalancing)
        t_end = float(self.grid.times()[-1])
        if t_end - cfg.T > 1e-6 * max(cfg.T, 1.0):
            # ceil(T/dt) of the reference grid (C11) overshoots T when dt is a
            # truncated decimal (e.g. 0.0333333333333333 for 1/30); ending
            # short of T is the reference's own decimation (floor) convention
            import warnings

            warnings.warn(f"time grid ends at {t_end:.10g}, beyond T={cfg.T:g} (dt={cfg.dt!r}, "
                          f"rebalancing={cfg.rebalancing!r}); pass dt / rebalancing at full precision", stacklevel=2)
        self.n_total = 2 ** int(cfg.n_paths)
        self.offset, self.n_local = D.shard(self.n_total, dist_info.world, dist_info.rank)
        self.timer = PhaseTimer(enabled=True, device=self.device)
        self.kind = self._kind()
        self.spec = self._spec()
        self.paths = None
        self.gpaths = None  # LM Gram subsample paths (engine.gram_subsample), simulated on every rank
        self.gv_terminal = None  # ... their terminal values (pinball LM fits: the subsample's targets)
        self.xpaths = None  # LM multi-start exploration: (global prefix paths, their terminal values)
        self.induction = None
        self.graph = None

    # ------------------------------------------------------------------ setup
    def _kind(self) -> str:
        c = self.cfg
        if c.payoff in ("call", "put"):
            return "european"
        if c.payoff == "basket_call" or c.model == "basket":
            return "basket"
        return "pension"

    def _spec(self) -> hm.NetSpec:
        c = self.cfg
        alpha = c.train.leaky_alpha
        hid = int(c.train.hidden)
        if self.kind == "european":
            if c.model == "heston":
                return hm.NetSpec(nin=2, hidden=hid, nout=2, head=L.HEAD_FREE, alpha=alpha)
            if c.parity.complement_head:
                return hm.NetSpec(nin=1, hidden=hid, nout=1, head=L.HEAD_COMPLEMENT, alpha=alpha,
                                  layer_names=("LeakyReLU_1", "LeakyReLU_2", "Phi"))
            return hm.NetSpec(nin=1, hidden=hid, nout=2, head=L.HEAD_FREE, alpha=alpha)
        if self.kind == "basket":
            return hm.NetSpec(nin=c.n_assets, hidden=hid, nout=c.n_assets + 1, head=L.HEAD_FREE, alpha=alpha)
        if c.model in ("sv_ref", "heston") and not c.mortality:
            return hm.NetSpec(nin=2, hidden=hid, nout=2, head=L.HEAD_FREE, alpha=alpha)
        return hm.NetSpec(nin=3, hidden=hid, nout=2, head=L.HEAD_FREE, alpha=alpha)

    @property
    def scale(self) -> float:
        c = self.cfg
        return float(c.N * c.P) if self.kind == "pension" else float(c.Y)

    def simulate(self, into: P.Paths | None = None):
        """Paths (K1–K6) and terminal value V_T (K7) on the coarse grid.

        ``into``: re-simulate into the buffers of the existing paths and
        terminal value (no allocation, no host synchronisation), so the
        simulation can be captured into the run's hipGraph.  LM fits also get
        the global Gram subsample simulated on this rank (:meth:`gram_paths`)."""
        c = self.cfg
        vt_out = self.v_terminal if into is not None else None
        with self.timer.phase("simulate"):
            p = self._simulate_paths(self.n_local, self.offset, None, into)
            v_t = self._payoff(p, vt_out)
            tr = c.train
            if str(tr.optimizer).lower() == "lm":
                ns, blk, stride = gram_subsample(self.n_total, tr.lm_gram_paths)
                self.gpaths = self._simulate_paths(ns, 0, (blk, stride), self.gpaths if into is not None else None)
                if self._q_lm():
                    # pinball LM fits: the subsample's own terminal values (its
                    # later targets come from the date-boundary evaluations)
                    self.gv_terminal = self._payoff(self.gpaths, self.gv_terminal if into is not None else None)
                if self.di.world > 1 and (int(tr.lm_starts) > 1 or bool(getattr(tr, "lm_explore_one", False))):
                    # the multi-start exploration's global path prefix (every
                    # rank explores the same starts on the same paths)
                    nx = min(1 << int(tr.lm_explore_log2), self.n_total)
                    xp = self._simulate_paths(nx, 0, None, self.xpaths[0] if into is not None else None)
                    xv = self._payoff(xp, self.xpaths[1] if into is not None else None)
                    self.xpaths = (xp, xv)
        self.paths, self.v_terminal = p, v_t
        return p, v_t

    def _q_lm(self) -> bool:
        """Both networks with the pinball fit on Levenberg-Marquardt."""
        tr, pf = self.cfg.train, self.cfg.parity
        return bool(tr.q99) and not pf.shared_q99_model and str(getattr(tr, "q99_optimizer", "adam")).lower() == "lm"

    def _payoff(self, p: P.Paths, out=None) -> torch.Tensor:
        """Terminal value V_T of paths ``p`` (K7; ``out``: into that buffer)."""
        c = self.cfg
        if self.kind == "european":
            return P.payoff(c.option_type.lower(), p, c.K / c.Y, stream=self.stream, out=out)
        if self.kind == "basket":
            w = c.basket_weights or tuple([1.0 / c.n_assets] * c.n_assets)
            return P.payoff("basket_call", p, c.K / c.Y, weights=w, stream=self.stream, out=out)
        return P.payoff("guarantee", p, c.K, stream=self.stream, out=out)

    def _simulate_paths(self, n: int, offset: int, index_map, into: P.Paths | None) -> P.Paths:
        """One model's coarse-grid paths for ``n`` paths from global index
        ``offset`` (``index_map``: the Gram subsample's global blocks)."""
        c, g, dev = self.cfg, self.grid, self.device
        fp64 = c.dtype == "fp64"
        kw = dict(device=dev, offset=offset, stream=self.stream, out=into, index_map=index_map)
        if self.kind == "european":
            if c.model == "heston":
                p = P.simulate_sv(g, n, c.Y, c.r, c.v0, model="heston", kappa=c.kappa, theta=c.theta, xi=c.xi,
                                  rho=c.rho, norm=c.Y, fp64=fp64, scheme=c.heston_scheme,
                                  joint=not c.parity.paired_sobol, **kw)
            else:
                scheme = "arith" if c.model == "gbm" else "log"
                p = P.simulate_gbm(g, n, c.Y, c.r, c.sigma, scheme=scheme, norm=c.Y, fp64=fp64, **kw)
            # EO normalises BOTH prices by S0 (cell 13: _B_t = B/S0, so psi counts
            # unit bonds); the corrected default quotes the bond in S0 units.
            p.bond = g.bond(c.r, norm=c.Y if c.parity.complement_head else 1.0)
            return p
        if self.kind == "basket":
            na = c.n_assets
            corr = np.full((na, na), c.basket_corr) + np.eye(na) * (1 - c.basket_corr)
            s0 = [c.Y] * na
            p = P.simulate_basket(g, n, s0, [c.r] * na, [c.sigma] * na, corr, norm=s0, **kw)
            p.bond = g.bond(c.r)
            return p
        if c.model in ("sv_ref", "heston"):
            p = P.simulate_sv(g, n, c.Y, c.mu, c.s0, model=c.model, a=c.a, b=c.b, c=c.sv_c, kappa=c.kappa,
                              theta=c.theta, xi=c.xi, rho=c.rho, fp64=fp64, parity_nan=c.parity.sv_sqrt_nan,
                              scheme=c.heston_scheme,
                              sv_tscale=0.0 if c.parity.sv_reference_dynamics else c.sv_days_per_year,
                              joint=not c.parity.paired_sobol, **kw)
        else:
            p = P.simulate_gbm(g, n, c.Y, c.mu, c.sigma, scheme=("log" if c.model == "gbm_log" else "arith"),
                               fp64=fp64, **kw)
        if c.mortality:
            if into is not None and c.parity.numpy_binomial:
                raise NotImplementedError("numpy binomial (Q20 parity) runs on the host: not graph-safe")
            P.simulate_mortality(p, c.l0, c.c, c.ita, c.N, lambda_fine_index=c.parity.lambda_fine_index,
                                 fp64=fp64, numpy_binomial=c.parity.numpy_binomial, stream=self.stream)
        else:
            p.kind = "pension_nomort"
        p.bond = g.bond(c.r)
        if not c.parity.fine_terminal_payoff:
            if into is None:
                p.S_final = p.S[-1].clone()
            else:
                p.S_final.copy_(p.S[-1])
        if p.nfrac is not None:
            # the coarse terminal survivors are what the liability is paid on (RP:184)
            p.nfrac_final = p.nfrac[-1]
        return p

    def summary_stats(self) -> dict:
        """E[N_T], P(out of the money), E[payoff] (C10; global over ranks)."""
        c, p, w = self.cfg, self.paths, self.di.world
        n = float(self.n_total)
        yT = p.S_final if p.S_final.dim() == 1 else p.S_final[0]
        if self.kind == "pension":
            p_oom = D.all_reduce_scalar(float((yT < c.Y).double().sum()), device=self.device) / n if w > 1 else \
                float((yT < c.Y).double().mean())
        else:
            strike = c.K / c.Y
            p_oom = D.all_reduce_scalar(float((yT < strike).double().sum()), device=self.device) / n if w > 1 else \
                float((yT < strike).double().mean())
        e_pay = float(self.v_terminal.double().sum())
        e_pay = (D.all_reduce_scalar(e_pay, device=self.device) if w > 1 else e_pay) / n
        out = {"p_oom": p_oom, "E_payoff": e_pay}
        if p.nfrac_final is not None:
            en = float(p.nfrac_final.double().sum())
            out["E_N_T"] = (D.all_reduce_scalar(en, device=self.device) if w > 1 else en) / n * c.N
        out["mean_Y_T"] = (D.all_reduce_scalar(float(yT.double().sum()), device=self.device) if w > 1
                           else float(yT.double().sum())) / n * (c.Y if self.kind != "pension" else 1.0)
        return out

    def init_align(self) -> tuple | None:
        """init="aligned": the first layer's direction in the standardised
        input space - the basket weights (every asset input is standardised
        alike); None for single-price nets (aligned = spread there)."""
        c = self.cfg
        if str(getattr(c.train, "init", "reference")) != "aligned" or self.kind != "basket":
            return None
        return tuple(c.basket_weights or [1.0 / c.n_assets] * c.n_assets)

    def feature_centers(self) -> tuple | None:
        """The payoff kink of every price feature in the paths' units
        (feature_norm="horizon"): the strike K / Y of a call / put, K / Y per
        asset of the basket call (the normalised basket's kink level); None
        where the kink is not a fixed price level (the pension guarantee)."""
        c = self.cfg
        if self.kind == "pension" or c.payoff not in ("call", "put", "basket_call"):
            return None
        k = float(c.K) / float(c.Y)
        nin = self.spec.nin
        return tuple([k] * nin) if self.kind == "basket" else (k,) + (None,) * (nin - 1)

    def init_weights(self, stats: dict) -> np.ndarray:
        """Reference initialisers (RP:149-156): N(0,0.1) kernels + data-dependent output bias (Q11)."""
        c, spec = self.cfg, self.spec
        if self.kind == "pension":
            bias = [1.0 - stats["p_oom"], stats["p_oom"]]
        elif spec.head == L.HEAD_COMPLEMENT:
            bias = [stats["E_payoff"]]                      # mean(payoff)/S0  (EO cell 12)
        else:
            p_itm = 1.0 - stats["p_oom"]
            bias = [p_itm, stats["E_payoff"] - p_itm] + [0.0] * (spec.nout - 2)
            if self.kind == "basket":
                bias = [p_itm / c.n_assets] * c.n_assets + [stats["E_payoff"] - p_itm]
        return hm.init_weights(spec, bias[: spec.nout], seed=c.train.seed,
                               spread=str(getattr(c.train, "init", "reference")) in ("spread", "aligned"),
                               align=self.init_align(),
                               shared_stream=bool(c.parity.shared_initializer))

    def build(self, w0: np.ndarray | None = None):
        c = self.cfg
        if self.paths is None:
            self.simulate()
        self.stats0 = self.summary_stats()
        self.w0 = self.init_weights(self.stats0) if w0 is None else w0
        tr = c.train
        tcfg = TrainConfig(batch_size=tr.batch_size, shuffle=tr.shuffle, chunk_log2=tr.chunk_log2, seed=tr.seed,
                           lr=tr.lr, deterministic=tr.deterministic, max_wgs=tr.max_wgs,
                           mfma_fp32=str(tr.mfma_precision).lower() == "fp32", step_mode=tr.step_mode,
                           lm_gram_paths=int(tr.lm_gram_paths), lm_damping=str(tr.lm_damping),
                           lm_leaf_paths=int(getattr(tr, "lm_leaf_paths", -1)),
                           lm_lam0=float(tr.lm_lam0), lm_lam_up=float(tr.lm_lam_up),
                           lm_lam_down=float(tr.lm_lam_down), lm_out_fix=bool(tr.lm_out_fix),
                           lm_out_mu=float(tr.lm_out_mu), lm_out_tr=float(getattr(tr, "lm_out_tr", 0.0)),
                           lm_ridge=float(getattr(tr, "lm_ridge", 1e-10)),
                           lm_diag_floor=float(tr.lm_diag_floor))
        if int(tr.variant) >= 0:
            tcfg.variant = int(tr.variant)
        kw = {}
        if self.backend_kind == "hip" and self.di.world > 1:
            if self.di.probe is None and self.di.dp_mode == "xgmi":
                D.select_transport(self.di)  # once per process group (collective); may fall back to RCCL
            self.mailbox = D.make_mailbox(self.di, self.spec.red_width)
            kw["mailbox"] = self.mailbox
            # LM fits / mean refits: the reduced [G | g | stats] block travels
            # over its own mailbox (k_lm_dp_exchange) with the xGMI transport
            self.lm_mailbox = D.make_mailbox(self.di, L.LM_DP_PITCH, tag="rph_lmbox",
                                             mode=self.di.lm_dp_mode)
            kw["lm_mailbox"] = self.lm_mailbox
            kw["lm_comm"] = self.di.lm_comm
        self.backend = make_backend(self.backend_kind, self.spec, self.n_local, tcfg, device=self.device,
                                    comm=self.di.comm, world=self.di.world, rank=self.di.rank, stream=self.stream,
                                    **kw)
        pf = c.parity
        icfg = InductionConfig(epochs_first=tr.epochs_first, epochs_rest=tr.epochs_rest,
                               patience_first=tr.patience_first, patience_rest=tr.patience_rest,
                               early_stopping=tr.early_stopping,
                               lr_schedule_first=tr.lr_schedule_first and pf.lr_schedule_first_only,
                               lr=tr.lr, lr_rest=tr.lr_rest, lr_decay=tr.lr_decay,
                               q99=tr.q99, quantile=tr.quantile, cost_of_capital=tr.cost_of_capital,
                               shared_q99_model=pf.shared_q99_model,
                               holdings_blend_sign_rp=pf.holdings_blend_sign_rp, warm_start=pf.warm_start, carry_optimizer=pf.carry_optimizer,
                               restore_best_at_end=pf.restore_best_at_end, keep_paths=c.keep_paths,
                               poll_every=tr.poll_every, seed=tr.seed,
                               feature_norm="none" if pf.raw_features else tr.feature_norm,
                               feature_centers=self.feature_centers(),
                               feature_norm_floor=float(getattr(tr, "feature_norm_floor", 0.0)),
                               optimizer=str(tr.optimizer).lower(), lm_passes_first=int(tr.lm_passes_first),
                               q99_optimizer=str(getattr(tr, "q99_optimizer", "adam")).lower(),
                               lm_q_passes_first=int(getattr(tr, "lm_q_passes_first", 40)),
                               lm_q_passes_rest=int(getattr(tr, "lm_q_passes_rest", 4)),
                               lm_q_delta=float(getattr(tr, "lm_q_delta", 1e-4)),
                               lm_q_kappa=float(getattr(tr, "lm_q_kappa", 3.0)),
                               lm_q_start=str(getattr(tr, "lm_q_start", "mse")),
                               lm_passes_rest=int(tr.lm_passes_rest), lm_stop_tol=float(tr.lm_stop_tol),
                               lm_stop_min=int(tr.lm_stop_min), lm_lam0_rest=float(tr.lm_lam0_rest),
                               lm_lam0_first=float(tr.lm_lam0_first),
                               lm_lam_carry=float(tr.lm_lam_carry), lm_starts=int(tr.lm_starts),
                               lm_renorm=bool(tr.lm_renorm),
                               lm_explore_passes=int(tr.lm_explore_passes), lm_explore_log2=int(tr.lm_explore_log2),
                               lm_explore_one=bool(getattr(tr, "lm_explore_one", False)),
                               init_spread=str(getattr(tr, "init", "reference")) in ("spread", "aligned"),
                               init_align=self.init_align(),
                               init_shared_stream=bool(pf.shared_initializer),
                               mean_refit=bool(tr.mean_refit) and not pf.keras_fit_only)
        backend_q = None
        if (self.backend_kind == "hip" and self.di.world == 1 and icfg.q99 and not icfg.shared_q99_model
                and not icfg.poll_every and tr.concurrent_q99):
            # second backend (own accumulators / state slots) for the pinball
            # fit, run concurrently on a side stream (driver.BackwardInduction)
            backend_q = make_backend(self.backend_kind, self.spec, self.n_local, tcfg, device=self.device,
                                     world=1, rank=0, stream=None)
            if not backend_q.concurrent_with(self.backend):
                backend_q = None
        self.induction = BackwardInduction(self.paths, self.v_terminal, self.spec, self.w0, self.backend, icfg,
                                           world=self.di.world, rank=self.di.rank, backend_q=backend_q,
                                           gram_paths=self.gpaths, explore_paths=self.xpaths,
                                           gram_terminal=self.gv_terminal)
        return self

    # ------------------------------------------------------------------ run
    def enqueue(self, resimulate: bool = False):
        """Enqueue the run (graph-capturable when ``poll_every == 0``)."""
        ind = self.induction
        if resimulate:
            self.simulate()  # same buffers are re-created; only used outside capture
        ind.values[-1].copy_(self.v_terminal)
        if ind.gvalues is not None:
            ind.gvalues[-1].copy_(ind.g_terminal)
        ind.w_mse.copy_(ind.w_init)
        ind.opt_mse.copy_(ind.opt_init)
        if ind.cfg.q99:
            if not ind.cfg.shared_q99_model:
                ind.w_q.copy_(ind.w_init)
            ind.opt_q.copy_(ind.opt_init)
        with self.timer.phase("train"):
            ind.enqueue()

    def capture(self, include_simulation: bool = True):
        """Capture simulation + full backward induction into ONE hipGraph."""
        from .ops.native import Graph

        if self.backend_kind != "hip":
            raise RuntimeError("graph capture needs the hip backend")
        assert self.cfg.train.poll_every == 0, "graph capture requires fully asynchronous early stopping"
        # Capture must run on a non-default stream; torch ops inside enqueue()
        # follow torch's current stream, so make the side stream current.
        s = torch.cuda.Stream(self.device)
        s.wait_stream(torch.cuda.current_stream(self.device))
        g = Graph()
        timer_on, self.timer.enabled = self.timer.enabled, False  # no event records inside capture
        with torch.cuda.stream(s):
            # one eager pass first: populates every cached device constant (fit
            # templates, LR tables, Sobol tables) so the capture allocates nothing
            if include_simulation:
                self._enqueue_sim_into_existing()
            self.enqueue()
            s.synchronize()
            g.capture_begin(s)
            try:
                if include_simulation:
                    self._enqueue_sim_into_existing()
                self.enqueue()
            finally:
                g.capture_end()
        torch.cuda.current_stream(self.device).wait_stream(s)
        self.timer.enabled = timer_on
        self.graph = g
        return g

    def _enqueue_sim_into_existing(self):
        """Re-run the path and payoff kernels into the SAME buffers (graph-safe,
        no allocation) — every model family (GBM, SV/Heston, basket, mortality)."""
        if self.device.type != "cuda":
            raise RuntimeError("in-place re-simulation needs the GPU path kernels")
        self.simulate(into=self.paths)

    def replay(self):
        self.graph.replay(self.stream or torch.cuda.current_stream(self.device))

    def close(self):
        """Release the run's cross-rank resources (collective when data
        parallel: every rank's kernels finish before any mailbox is freed)."""
        for name in ("mailbox", "lm_mailbox"):
            mb = getattr(self, name, None)
            setattr(self, name, None)
            if mb is not None:
                D.close_mailbox(mb)

    def resume(self, out_dir: str, date: int) -> RunResult:
        """Restart the backward scan at ``date-1`` from a saved run directory
        (weights of ``date`` as the warm start, Q18, and ``values[date]``).
        Adam moments restart from zero (Keras does not persist them either)."""
        from .utils.model_io import load_date

        if self.induction is None:
            self.build()
        ind = self.induction
        _, spec, w, wq, vals = load_date(out_dir, date)
        assert spec.nparams == self.spec.nparams, "saved network shape differs from this configuration"
        # saved weights are raw-input; the warm start continues in this run's
        # standardised coordinates of the saved date
        if ind.norms:
            mu, isd = ind.norms[min(date, len(ind.norms) - 1)]
            w = hm.unfold_input_norm(self.spec, w, mu, isd)
            wq = hm.unfold_input_norm(self.spec, wq, mu, isd) if wq is not None else None
        set_weights(self.spec, ind.w_init, w)
        if wq is not None and ind.cfg.q99 and not ind.cfg.shared_q99_model:
            self._wq_resume = wq
        if vals is None:
            raise ValueError("values.npy missing: cannot resume the backward induction")
        # values.npy holds the GLOBAL path set (save_run gathers the shards):
        # every rank takes its own contiguous shard
        if vals.shape[0] == self.n_total:
            vals = vals[self.offset:self.offset + self.n_local]
        else:
            raise ValueError(f"values.npy has {vals.shape[0]} paths; this run has {self.n_total} "
                             f"({self.n_local} on this rank)")
        t0 = time.perf_counter()
        ind.values[date].copy_(torch.from_numpy(np.ascontiguousarray(vals)).to(ind.values.device))
        ind.w_mse.copy_(ind.w_init)
        ind.opt_mse.copy_(ind.opt_init)
        if ind.cfg.q99:
            if not ind.cfg.shared_q99_model:
                ind.w_q.copy_(ind.w_init)
                if getattr(self, "_wq_resume", None) is not None:
                    set_weights(self.spec, ind.w_q, self._wq_resume)
            ind.opt_q.copy_(ind.opt_init)
        # the first resumed date is NOT the reference's "first" date (no LR schedule)
        orig = ind._fcfg
        ind._fcfg = lambda first, loss, t=None: orig(False, loss, t)
        try:
            ind.enqueue(start=date - 1)
        finally:
            ind._fcfg = orig
        res = self.collect()
        res.timings["wall_s"] = time.perf_counter() - t0
        return res

    def run(self) -> RunResult:
        t0 = time.perf_counter()
        if self.induction is None:
            self.build()
        self.enqueue()
        res = self.collect()
        res.timings["wall_s"] = time.perf_counter() - t0
        return res

    def collect(self) -> RunResult:
        c, w = self.cfg, self.di.world
        if self.device.type == "cuda":
            torch.cuda.synchronize(self.device)
        for mb in (getattr(self, "mailbox", None), getattr(self, "lm_mailbox", None)):
            if mb is not None:
                mb.check()
        if hasattr(self.backend, "check"):
            self.backend.check()
        ind = self.induction.collect()
        scale = self.scale
        h0 = ind.holdings0
        if self.kind == "pension":
            phi, psi = float(h0[0] * scale), float(h0[1] * scale)
        else:
            # psi in unit bonds (B_0 = 1): parity head already counts unit bonds
            bond_unit = 1.0 if c.parity.complement_head else c.Y
            phi, psi = float(h0[0]), float(h0[-1] * bond_unit)
        def pnl_dict(dr):
            return {"mean": dr.residual_mean * scale, "std": dr.residual_std * scale,
                    "min": float(dr.stats[L.ES_RESMIN]) * scale, "max": float(dr.stats[L.ES_RESMAX]) * scale}

        # one-step residual of the last date (the reference's "P&L at T", Q24)
        # and the self-financing hedge P&L W_T - liability (corrected default)
        resid = pnl_dict(ind.terminal)
        sf = pnl_dict(ind.pnl) if ind.pnl is not None else None
        if sf is not None:
            sf["mean_terminal_wealth"] = ind.pnl.mean_value * scale
        tp = dict(resid) if (c.parity.local_residual_pnl or sf is None) else dict(sf)
        tp["kind"] = "one_step_residual" if (c.parity.local_residual_pnl or sf is None) else "self_financing"
        var = {}
        if ind.residuals is not None and c.keep_paths:
            var = risk.var_report(ind.residuals, scale=scale, world=w)
            if ind.pnl_paths is not None:
                q = risk.quantile(ind.pnl_paths, (0.01, 0.015, 0.02, 0.05), w)
                var["self_financing_pnl_quantiles"] = {"q": [0.01, 0.015, 0.02, 0.05],
                                                       "values": [float(x) * scale for x in q]}
        dtc = self.grid.dt_coarse
        pe = expected_value_trajectory(ind, self.stats0["E_payoff"], c.mu if self.kind == "pension" else c.r, c.r,
                                       dtc)
        summary = dict(self.stats0)
        summary.update({"V0": ind.v0 * scale, "phi0": phi, "psi0": psi, "n_paths": self.n_total,
                        "n_dates": self.paths.n_coarse - 1, "reduction": self.grid.reduction,
                        "epochs_mse": [d.fit_mse["epochs"] for d in ind.dates],
                        "terminal_pnl_std": tp["std"], "terminal_residual_std": resid["std"],
                        "self_financing_pnl_std": sf["std"] if sf is not None else None})
        if self.kind == "european":
            from .utils.reports import black_scholes

            bs = black_scholes(c.Y, c.K, c.r, c.sigma, c.T, c.option_type)
            summary["bs_price"], summary["bs_delta"] = bs
        return RunResult(phi=phi, psi=psi, v0=ind.v0 * scale, scale=scale, holdings0=h0, induction=ind,
                         errors=error_history(ind), p_e_values=pe, terminal_pnl=tp, var=var, summary=summary,
                         timings=self.timer.summary(), config=c.to_dict(), paths=self.paths,
                         terminal_residual=resid, self_financing_pnl=sf)


# ---------------------------------------------------------------------------
# reference-compatible entry points
# ---------------------------------------------------------------------------
def _print_dates(run: HedgeRun, res: RunResult):
    """Per-date log of the reference (RP:194, :122); ``verbose=2`` adds the
    Keras-style per-epoch training log of every fit (``fit(verbose=1)`` in
    "European Options.ipynb" cell 13) from the on-device epoch-loss history."""
    if not run.cfg.verbose:
        return
    ind = res.induction
    p = run.paths
    dtc = run.grid.dt_coarse
    w = run.di.world

    def gmean(x: torch.Tensor) -> float:
        s = float(x.double().sum())
        return (D.all_reduce_scalar(s, device=run.device) if w > 1 else s) / float(run.n_total)

    # collectives (global means, distributed quantiles) on EVERY rank, in the
    # same order; only the printing is rank 0's
    rows = []
    for d in ind.dates:
        t = d.index
        y = gmean(p.asset(t + 1)) * (1.0 if run.kind == "pension" else run.cfg.Y)
        nm = gmean(p.nfrac[t + 1]) if p.nfrac is not None else None
        q = risk.quantile(ind.residuals[t], (0.98, 0.99), w) if ind.residuals is not None else None
        rows.append((d, y, nm, q))
    if not run.di.is_main:
        return
    for d, y, nm, q in rows:
        t = d.index
        if int(run.cfg.verbose) >= 2:
            for name, fs in (("mse", d.fit_mse), ("q99", d.fit_q99)):
                if not fs:
                    continue
                hist = fs["history"]
                for e, loss in enumerate(hist):
                    print(f"[t={t * dtc:.4f} {name}] Epoch {e + 1}/{len(hist)} - loss: {loss:.4e}")
                print(f"[t={t * dtc:.4f} {name}] mae: {fs['mae']:.4e} - mape: {fs['mape']:.4f}"
                      f"{' - early stop' if fs['stopped'] and len(hist) else ''}")
        line = f">> Y_({(t + 1) * dtc:.2f}) = {y:.3f}"
        if nm is not None:
            line += f", N_({(t + 1) * dtc:.2f}) = {nm:.3f}"
        print(line)
        if q is not None:
            print(f"VaR: {q[0]:4f} (98%),  {q[1]:4f} (99%)  | epochs {d.fit_mse['epochs']}"
                  f"{'/' + str(d.fit_q99['epochs']) if d.fit_q99 else ''}  loss {d.fit_mse['last_loss']:.3e}")


def run_params(params: dict, sv: bool = False) -> RunResult:
    cfg = parse_params(params, sv=sv)
    run = HedgeRun(cfg)
    if cfg.verbose and run.di.is_main:
        print(f"reduction = {run.grid.reduction}")
    res = run.run()
    _print_dates(run, res)
    if cfg.save_dir:
        from .utils.model_io import save_run

        save_run(cfg.save_dir, run, res)
    run.close()
    return res


# Corrected-mode optimiser profile of the public entry points on the GPU: both
# fits of every date on Levenberg-Marquardt (MSE: a 16-start first date on the
# 2^15-path prefix + the exact output-layer step; Q99: IRLS Gauss-Newton, 200
# passes on the first date, 20 on later ones from the previous date's Q99 net).
# Measured against Keras-Adam on the MTS pension (BENCHMARKS.md round 5): 0.105
# vs 21.2 s per run, V0 / phi0 / psi0 inside the Adam seed band with 6x less
# V0 scatter, lower pinball loss, 1.01 % Q99 coverage.
LM_PROFILE = dict(optimizer="lm", q99_optimizer="lm", lm_starts=16, lm_explore_passes=40, lm_explore_log2=15,
                  lm_passes_first=60, lm_passes_rest=3, lm_lam_carry=3.0, lm_out_fix=True,
                  lm_q_passes_first=200, lm_q_passes_rest=20, lm_q_start="warm")


def default_params(params: dict, gpu: bool | None = None) -> dict:
    """The params a public entry point runs: in corrected mode on a GPU, the
    keys of :data:`LM_PROFILE` the caller did not set (unless the caller chose
    an ``optimizer``); ``parity=True`` keeps the reference's Keras-Adam fits,
    and so does the CPU torch oracle (plumbing)."""
    if gpu is None:
        dev = str(params.get("device") or ("cuda" if torch.cuda.is_available() else "cpu"))
        gpu = dev.startswith("cuda") and torch.cuda.is_available() and params.get("backend") != "torch"
    if params.get("parity") is True or not gpu or "optimizer" in params:
        return dict(params)
    return {**LM_PROFILE, **params}


def Replicating_Portfolio(params: dict):
    """Pension-guarantee replicating portfolio; returns ``(phi, psi)`` at t=0
    scaled by ``N*P`` (RP:29-235).  Corrected mode on a GPU fits both networks
    with Levenberg-Marquardt (:func:`default_params`); ``parity=True`` keeps
    the reference's Keras-Adam."""
    return run_params(default_params(params), sv=False).as_tuple()


def Replicating_Portfolio_SV(params: dict):
    """Stochastic-volatility variant (RP:237-459); returns ``(phi, psi)``
    (optimiser defaults as :func:`Replicating_Portfolio`)."""
    return run_params(default_params(params), sv=True).as_tuple()


EO_DEFAULTS = dict(S0=100.0, K=100.0, r=0.08, sigma=0.15, T=1.0, N_paths=3000, dt=1 / 365,
                   rebalancing_frequency=1 / 52, OPTION_TYPE="CALL")


def european_option(S0=100.0, K=100.0, r=0.08, sigma=0.15, T=1.0, N_paths=3000, dt=1 / 365,
                    rebalancing_frequency=1 / 52, OPTION_TYPE="CALL", parity: bool = False, model: str = "gbm_log",
                    **extra) -> RunResult:
    """European call/put replication (``European Options.ipynb``; C13, C16, C34).

    Defaults are the notebook's (cell 3).  The reference driver trains the MSE
    model only (the Q99 refit is commented out) and uses the ``psi = 1 - phi``
    head (Q13) — reproduced with ``parity=True``; the default corrected head
    learns (phi, psi) freely.
    """
    params = dict(Y=S0, K=K, T=T, mu=r, r=r, sigma=sigma, rebalancing=rebalancing_frequency, N=1, P=1.0, x=0.0,
                  l0=0.0, c=0.0, ita=0.0, dt=dt, n_paths=int(math.ceil(math.log2(N_paths))), payoff="call" if
                  OPTION_TYPE.upper() == "CALL" else "put", option_type=OPTION_TYPE.upper(), model=model,
                  mortality=False, q99=False)
    if parity:
        params["parity"] = True
    params.update(extra)
    return run_params(params, sv=False)
