"""Configuration: the reference dict API schema + extensions + parity flags.

The reference configures everything through a plain ``params`` dict whose keys
are read at ``Replicating_Portfolio.py:31-49`` (GBM) and ``:239-263`` (SV)
(SURVEY §5.6).  :func:`parse_params` validates exactly those keys (``n_paths``
is log2 of the path count, C03) and accepts optional extension keys with
defaults.  Parity flags reproduce the reference quirks Q1–Q24;
``parity=True`` switches all of them on, the default is corrected semantics.
"""
from __future__ import annotations

import math
from dataclasses import asdict, dataclass, field, fields

GBM_KEYS = ("Y", "K", "T", "mu", "r", "sigma", "rebalancing", "N", "P", "x", "l0", "c", "ita", "dt", "n_paths")
SV_KEYS = ("Y", "K", "T", "mu", "r", "s0", "a", "b", "c", "rebalancing", "N", "P", "x", "l0", "ita", "dt",
           "n_paths")


@dataclass
class ParityFlags:
    """Reference quirks.  True = reproduce the reference."""

    shared_q99_model: bool = False      # Q1/Q2: "model2" aliases model1's layers, two Adam instances
    holdings_blend_sign_rp: bool = False  # Q2: phi1 + c(phi1 - phi2) (RP) instead of phi1 + c(phi2 - phi1)
    lambda_fine_index: bool = False     # Q3: lambda not subsampled (fine index t_i)
    sv_c_overwrite: bool = False        # Q4: params['c'] is read twice (vol-of-vol := mortality c)
    sv_reference_dynamics: bool = False  # Q5: reference SV recursion (no dt on mean reversion, post-update vt
                                         # in the price step); False = CIR-on-sigma in calibration-day units
    sv_sqrt_nan: bool = False           # numpy sqrt(negative) -> NaN propagation
    fine_terminal_payoff: bool = True   # payoff from the last FINE point even if the coarse grid misses it
    lr_schedule_first_only: bool = True  # Q17: LR schedule + patience 50 only on the first date
    warm_start: bool = True             # Q18: one network refit at every date (weights + Adam persist)
    carry_optimizer: bool = True        # Q18: the Adam moments / step count persist across dates (False: reset per date)
    restore_best_at_end: bool = False   # Keras-2: restore best weights only on early stop
    numpy_binomial: bool = False        # Q20: numpy MT19937 reseeded 1234+t (CPU oracle only)
    local_residual_pnl: bool = False    # Q24: report the one-step residual as "the P&L at T" (reference);
                                        # False = the self-financing hedge P&L (driver k_hedge_pnl scan)
    complement_head: bool = False       # Q13: European psi = 1 - phi head
    eo_discount_artifact: bool = False  # Q14: report V0*e^{-rT} as "discounted E[V(T)]"
    raw_features: bool = False          # reference nets see raw (unstandardised) state features
    paired_sobol: bool = False          # Q25: SV price / vol shocks from two scrambled Sobol sequences of the
                                        # SAME dimensions (RP:274-275; dependent, not independent, shocks);
                                        # False = one sequence of 2 n_fine dimensions
    keras_fit_only: bool = False        # the Keras fit's weights are used as they are (no exact bias refit
                                        # after the Adam MSE fits, TrainingParams.mean_refit)
    shared_initializer: bool = False    # ONE seeded RandomNormal instance for every kernel (RP:149, :154-156):
                                        # with a stateless seeded generator each call restarts the same normal
                                        # stream, so W2 / W3 begin with W1's values (Keras >= 2.10); False: an
                                        # independent stream per kernel (what a stateful op seed gives)

    @classmethod
    def reference(cls) -> "ParityFlags":
        return cls(shared_q99_model=True, holdings_blend_sign_rp=True, lambda_fine_index=True,
                   sv_c_overwrite=True, sv_reference_dynamics=True, sv_sqrt_nan=True,
                   fine_terminal_payoff=True, lr_schedule_first_only=True, warm_start=True,
                   restore_best_at_end=False, numpy_binomial=True, local_residual_pnl=True,
                   complement_head=True, eo_discount_artifact=True, raw_features=True, paired_sobol=True,
                   keras_fit_only=True)


@dataclass
class TrainingParams:
    """Optimiser / schedule knobs (extension keys of the params dict)."""

    batch_size: int = 512
    epochs_first: int = 500
    epochs_rest: int = 100
    patience_first: int = 50
    patience_rest: int = 7
    lr: float = 1e-3
    lr_schedule_first: bool = True   # reference step schedule (RP:128-136) on the first date
    lr_rest: float = 0.0             # learning rate of the later dates (0: keep the optimiser's current lr)
    lr_decay: float = 1.0            # per-date geometric decay, last/first epoch (1: constant); applies to
                                     # lr on the first date when lr_schedule_first is off, and to lr_rest
    early_stopping: bool = True
    cost_of_capital: float = 0.1
    quantile: float = 0.99
    q99: bool = True                 # second (pinball) fit per date
    shuffle: bool = True
    chunk_log2: int = 0              # 0 = per-path shuffle (Keras); 6 = 64-path chunks (throughput)
    seed: int = 1234
    leaky_alpha: float = 0.3
    poll_every: int = 0              # host early-stop polling (0 = fully async / graph)
    deterministic: bool = False      # fixed-order gradient reduction (bitwise reproducible)
    max_wgs: int = 0                 # workgroups per training step (0: engine default per net family)
    hidden: int = 8                  # hidden width: 8 = reference nets (VALU kernel), 32 = MFMA kernel
    mfma_precision: str = "bf16"     # 32-unit nets: "bf16" (32x32x16 MFMA) or "fp32" (exact 32x32x2 MFMA)
    step_mode: str = "auto"          # GPU step schedule: auto | lag | ticket | persistent (engine.TrainConfig)
    variant: int = -1                # narrow lag-kernel variant (-1: engine default; see engine.TrainConfig)
    concurrent_q99: bool = True      # two networks: run the pinball fit concurrently with the MSE fit (GPU)
    optimizer: str = "adam"          # MSE fits: "adam" (Keras-Adam minibatches, the reference) | "lm" (full-batch
                                     # Levenberg-Marquardt on the GPU: csrc/hedge_lm.hip)
    q99_optimizer: str = "adam"      # pinball (Q99) fits: "adam" | "lm" (IRLS Gauss-Newton in the same LM
                                     # kernels: Gram weighted by 1 / (2 max(|r|, delta)), exact pinball loss
                                     # for the accept test; two networks only - the shared Q1 net stays Adam)
    lm_q_passes_first: int = 40      # pinball LM trial points, first date
    lm_q_passes_rest: int = 4        # ... later dates
    lm_q_delta: float = 1e-4         # IRLS weight floor, relative to the mean |terminal value|
    lm_q_kappa: float = 3.0          # IRLS weight cap: |r| below lm_q_kappa x the mean |r| of its 64-path Gram
                                     # tile counts as that (a near-zero residual would dominate the step)
    lm_q_start: str = "mse"          # each pinball LM fit starts from: "mse" (the date's fitted MSE net, the
                                     # reference's alternate training of one net, Q1) | "warm" (the previous
                                     # date's Q99 net, Q18)
    lm_passes_first: int = 80        # LM trial points on the first date (from the random init)
    lm_passes_rest: int = 3          # LM trial points on later dates (warm start, Q18)
    lm_stop_tol: float = 0.0         # later dates: adaptive pass budget, lm_passes_rest = the cap; an accepted
                                     # pass that lowers the best loss by < lm_stop_tol (relative) ends the
                                     # fit; rejections never do (0: off)
    lm_stop_min: int = 2             # ... never before this pass
    init: str = "reference"          # weight init: reference (N(0, 0.1) kernels, zero hidden biases) | spread
                                     # (first-layer breakpoints spread over the standardised inputs)
    lm_lam0_rest: float = 0.0        # later dates' initial LM damping (0: lm_lam0; warm starts take smaller steps
                                     # with a larger value)
    lm_lam_carry: float = 0.0        # later dates: initial LM damping = the previous fit's final one x this
                                     # (0: off, lm_lam0 / lm_lam0_rest)
    lm_out_fix: bool = False         # LM fits end with the exact Newton step on the whole output layer (linear
                                     # in the value) instead of the bond bias alone
    lm_out_mu: float = 1e-5          # ... its relative Marquardt damping: directions of the output Gram below
                                     # ~1e-5 of its scale are rounding noise of the bf16 hi/lo products - and
                                     # the net's own collinear directions (an exact fp32 Gram at 1e-7 blew up
                                     # basket5 seeds: BENCHMARKS.md round 5)
    lm_out_tr: float = 0.0           # ... its trust region: ||d|| <= lm_out_tr x max(||w_o||, 1e-3 sqrt(n_o)) (0: off)
    lm_ridge: float = 1e-10          # LM systems (the fit's and the output step's): + this x the mean diagonal
    lm_renorm: bool = False          # later dates: the warm start's first layer re-expressed for the date's input
                                     # standardisation (the previous hedge as a function of the raw state)
    lm_starts: int = 1               # first date: multi-start LM exploration, starts per rank (1: off)
    lm_explore_passes: int = 45      # ... trial points of every exploration fit
    lm_explore_log2: int = 16        # ... on the first 2^this local paths; the best start over all ranks is
                                     # then polished for lm_passes_first passes on every path
    lm_explore_one: bool = False     # lm_starts = 1: the one start still explores first (a warm-up of
                                     # lm_explore_passes on the 2^lm_explore_log2 path prefix)
    lm_gram_paths: int = 4096        # Gram-matrix subsample (global paths, 64-path MFMA tiles)
    lm_leaf_paths: int = -1          # LM pass schedule: -1 cyclic path blocks (fastest); > 0 contiguous leaves of
                                     # this many paths per wave - with the same value at every world size the
                                     # data-parallel fit over the same global paths is bitwise the 1-rank fit
    lm_damping: str = "simple"       # LM damping update: simple (x1/3 / x4) | nielsen (gain ratio)
    lm_lam0: float = 1e-3            # LM initial damping of every fit
    lm_lam_up: float = 4.0           # simple rule: damping x lam_up on a rejected trial
    lm_lam_down: float = 1.0 / 3.0   #              x lam_down on an accepted one
    lm_lam0_first: float = 0.0       # first date's initial LM damping (0: lm_lam0)
    lm_diag_floor: float = 0.0       # LM damping diagonal floor, relative to mean diag 2G (0: Marquardt scaling)
    mean_refit: bool = True          # after each Adam MSE fit: exact refit of the bond holding's bias (the
                                     # residual mean over all paths -> 0; no mean error drifts into V0)
    feature_norm: str = "date"       # input standardisation: none | global | date | horizon (driver.feature_norms);
                                     # ParityFlags.raw_features forces none (reference)
    feature_norm_floor: float = 0.0  # horizon mode: the remaining-horizon scale >= this x the date spread


@dataclass
class RunConfig:
    """Normalised configuration of one replicating-portfolio run."""

    # financial (reference names kept in the dict API)
    Y: float = 1.0
    K: float = 1.0
    T: float = 10.0
    mu: float = 0.08
    r: float = 0.03
    sigma: float = 0.15
    rebalancing: float = 0.25
    N: int = 10_000
    P: float = 100.0
    x: float = 55.0                  # age (read but unused in the reference, Q19)
    l0: float = 0.01
    c: float = 0.075
    ita: float = 0.000597
    dt: float = 1 / 100
    n_paths: int = 12                # log2 (C03)
    # SV
    s0: float = 0.15965
    a: float = 0.0033566
    b: float = 0.15431
    sv_c: float = 0.015833
    # Heston (corrected SV model)
    kappa: float = 2.0
    theta: float = 0.0256
    xi: float = 0.3
    rho: float = -0.7
    v0: float = 0.0256
    heston_scheme: str = "qe"        # qe (Andersen QE, martingale-corrected) | euler (full truncation)
    sv_days_per_year: float = 252.0  # corrected CIR-on-sigma: calibration steps per year (daily data)
    # extensions
    model: str = "gbm"               # gbm | gbm_log | sv_ref | heston | basket
    payoff: str = "guarantee"        # guarantee | call | put | basket_call
    option_type: str = "CALL"
    mortality: bool = True
    n_assets: int = 1
    basket_weights: tuple = ()
    basket_corr: float = 0.5
    device: str | None = None
    backend: str | None = None       # hip | torch (default: hip when a GPU is present)
    world_size: int | None = None
    dtype: str = "fp32"              # recursion precision on device (fp32 | fp64)
    verbose: bool = True
    save_dir: str | None = None
    keep_paths: bool = True          # keep per-date holdings/residuals for reports
    train: TrainingParams = field(default_factory=TrainingParams)
    parity: ParityFlags = field(default_factory=ParityFlags)

    # derived grid (RP:51, :92-96)
    @property
    def n_fine(self) -> int:
        return int(math.ceil(self.T / self.dt) + 1)

    @property
    def reduction(self) -> int:
        return max(1, int(math.floor((self.n_fine - 1) / (self.T / self.rebalancing))))

    @property
    def n_coarse(self) -> int:
        return int(math.ceil(self.n_fine / self.reduction))

    @property
    def dt_coarse(self) -> float:
        return self.dt * self.reduction

    @property
    def paths(self) -> int:
        return 2 ** int(self.n_paths)

    def to_dict(self) -> dict:
        d = asdict(self)
        return d


_TRAIN_KEYS = {f.name for f in fields(TrainingParams)}
_PARITY_KEYS = {f.name for f in fields(ParityFlags)}
_RUN_KEYS = {f.name for f in fields(RunConfig)} - {"train", "parity"}


def parse_params(params: dict, sv: bool = False) -> RunConfig:
    """Validate a reference-style params dict and build a :class:`RunConfig`.

    Required keys are exactly the reference's (``GBM_KEYS``/``SV_KEYS``);
    unknown keys raise.  Extension keys (``batch_size``, ``epochs_first`` …,
    ``parity``/``parity_flags``, ``model``, ``payoff``, ``device`` …) are optional.
    """
    req = SV_KEYS if sv else GBM_KEYS
    missing = [k for k in req if k not in params]
    if missing:
        raise KeyError(f"params missing required keys: {missing}")
    cfg = RunConfig()
    tr = TrainingParams()
    pf = ParityFlags()
    parity = params.get("parity", False)
    if parity is True:
        pf = ParityFlags.reference()
    flags = params.get("parity_flags") or {}
    for k, v in params.items():
        if k in ("parity", "parity_flags"):
            continue
        if k in _TRAIN_KEYS:
            setattr(tr, k, v)
        elif k in _RUN_KEYS:
            setattr(cfg, k, v)
        elif k in _PARITY_KEYS:
            setattr(pf, k, v)
        else:
            raise KeyError(f"unknown params key {k!r}")
    for k, v in dict(flags).items():
        if k not in _PARITY_KEYS:
            raise KeyError(f"unknown parity flag {k!r}")
        setattr(pf, k, v)
    if sv:
        # Q4: the reference reads params['c'] for BOTH the SV vol-of-vol and the
        # mortality drift; the caller's dict (with its duplicate key) has c=0.075.
        if "sv_c" not in params and pf.sv_c_overwrite:
            cfg.sv_c = float(params["c"])
        if "model" not in params:
            cfg.model = "sv_ref"
    cfg.train = tr
    cfg.parity = pf
    int(cfg.n_paths)
    return cfg
