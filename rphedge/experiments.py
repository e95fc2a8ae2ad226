"""Experiment drivers of the reference notebooks (C33, C35–C37, C44).

* :func:`single_time_step` — ``Single Time Step.ipynb`` (C33): one fit pair
  over [0, T] (8192 paths, reduction 120), MSE holdings (Res1) vs
  cost-of-capital blended holdings (Res2); cost of capital ``0.1*dt`` = 1.0
  after the reduction (Q12) under ``parity``.
* :func:`volatility_sweep` — σ ∈ {.05,.10,.15,.20,.30} of full
  ``Replicating_Portfolio`` runs (C36, "Multi Time Step.ipynb":2299-2306).
* :func:`sv_experiment` — the SV parameter dict of "Multi Time Step.ipynb":2612-2646 (C37).
* :func:`mts_parameters` / :func:`sv_parameters` — the notebooks' param dicts (C35).
* :func:`sanity_checks` — the implicit acceptance checks printed by the
  notebooks (C44): MC mean vs analytic, grid shape, survivors, param counts.
"""
from __future__ import annotations

import math

import numpy as np
import torch

from . import risk
from .api import HedgeRun, run_params
from .config import parse_params
from .ops import layout as L


def mts_parameters(**over) -> dict:
    """``parameters`` dict of "Multi Time Step.ipynb":1329-1351 (μ, σ from the SV cell, Q16)."""
    p = dict(Y=1, K=1, T=10, mu=0.09464, r=0.03, sigma=0.15965, rebalancing=0.25, N=10_000, P=100, x=55,
             l0=0.01, c=0.075, ita=0.000597, dt=1 / 100, n_paths=int(math.ceil(math.log2(3000))))
    p.update(over)
    return p


def mts_lm_parameters(**over) -> dict:
    """:func:`mts_parameters` (corrected two-network semantics) with BOTH fits
    of every date on Levenberg-Marquardt (MSE fits and the Q99 pinball fits,
    ``q99_optimizer="lm"``): a 16-start first date on the 2^15-path prefix, the
    exact output-layer step after every MSE fit, 200 IRLS passes for the first
    pinball fit and 20 for the later ones, each starting from the previous
    date's Q99 net.  At 2^20 paths the whole 40-date induction takes ~0.1 s on
    one MI355X vs 10-23 s with Keras-Adam, with V0 / phi0 / psi0 inside the
    Adam seed band and a lower pinball loss on every date (BENCHMARKS.md round 5,
    profiles/r5/pension_lm_vs_adam.jsonl)."""
    from .api import LM_PROFILE

    p = mts_parameters(**LM_PROFILE)
    p.update(over)
    return p


def mts_notebook_parameters(**over) -> dict:
    """The paths behind the "Multi Time Step.ipynb" HEADLINE numbers (Q15):
    cell 9 ("SV - Version", exec 94) overwrote ``Y_paths`` after the GBM cell -
    log-Euler fund paths with vol s0 = sigma_0 = 0.15965 held CONSTANT (Q6:
    ``vt[:,t]`` is read before it is written, so it is the fill value) and
    mu = 0.09464, dt = 1/365 (3651 fine steps), Sobol seed 1235 ("Multi Time
    Step.ipynb":218-248); mortality and the quarterly induction as in the
    notebook's training cells (shared Q99 model, c = 0.1, Keras LR schedule,
    ``parity=True``).  Published: V0 = 981,038.213, phi0 / psi0 = 643,687 /
    350,888, overall residual VaR 98.5 / 99 / 99.5 % = -121.96 / 54.38 /
    1,160.76 EUR (":1039", ":987-988", ":954-956")."""
    p = mts_parameters(dt=1 / 365, model="gbm_log", mu=0.09464, sigma=0.15965, parity=True)
    p.update(over)
    return p


MTS_NOTEBOOK_PUBLISHED = {"V0": 981_038.213, "phi0": 643_687.0, "psi0": 350_888.0,
                          "VaR": (-121.96, 54.38, 1_160.76)}


def mts_notebook(**over) -> dict:
    """Run :func:`mts_notebook_parameters` and report the notebook's headline
    quantities next to the published ones."""
    res = run_params(mts_notebook_parameters(**over))
    out = {"V0": res.v0, "phi0": res.phi, "psi0": res.psi, "published": MTS_NOTEBOOK_PUBLISHED,
           "epochs_mse": res.summary.get("epochs_mse"), "result": res}
    if res.var:
        out["VaR"] = [res.var[k] for k in ("VaR(98.5%)", "VaR(99.0%)", "VaR(99.5%)") if k in res.var]
    return out


def sv_parameters(**over) -> dict:
    """``sv_parameters`` of "Multi Time Step.ipynb":2612-2639 (duplicate 'c' key: later value wins, Q4)."""
    p = dict(Y=1, K=1, T=10, mu=0.09464, r=0.03, s0=0.15965, a=0.0033566, b=0.15431, c=0.075,
             rebalancing=0.25, N=10_000, P=100, x=55, l0=0.01, ita=0.000597, dt=1 / 100,
             n_paths=int(math.ceil(math.log2(3000))))
    p.update(over)
    return p


def volatility_sweep(base: dict | None = None, sigmas=(0.05, 0.10, 0.15, 0.20, 0.30), **over) -> list[dict]:
    """Rows [sigma, Phi, Psi, Phi+Psi] like "Multi Time Step.ipynb":2397-2403."""
    base = dict(mts_parameters(**over) if base is None else base)
    rows = []
    for s in sigmas:
        p = dict(base, sigma=s)
        res = run_params(p)
        rows.append({"sigma": s, "Phi": res.phi, "Psi": res.psi, "sum": res.phi + res.psi, "V0": res.v0})
    return rows


def sv_experiment(**over) -> tuple[float, float]:
    from .api import Replicating_Portfolio_SV

    return Replicating_Portfolio_SV(sv_parameters(**over))


def single_time_step(parity: bool = True, **over) -> dict:
    """One-step pension hedge (C33).  Returns VaRs of Res1 (MSE holdings) and
    Res2 (blended), phi0/psi0 and V0 (all in EUR)."""
    p = dict(Y=1, K=1, T=10, mu=0.08, r=0.03, sigma=0.15, rebalancing=10, N=10_000, P=100, x=55, l0=0.01,
             c=0.075, ita=0.000597, dt=1 / 12, n_paths=int(math.ceil(math.log2(8000))), parity=parity)
    p.update(over)
    cfg = parse_params(p)
    if parity and "cost_of_capital" not in over:
        cfg.train.cost_of_capital = 0.1 * cfg.dt_coarse   # Q12: 0.1*dt after dt *= reduction -> 1.0
    cfg.parity.shared_q99_model = parity and cfg.parity.shared_q99_model
    run = HedgeRun(cfg)
    run.build()
    ind = run.induction
    # STS evaluates the MSE holdings BEFORE the pinball fit (Res1) -> keep that residual too
    res1 = torch.empty(run.n_local, dtype=torch.float32, device=run.device)
    orig_eval = run.backend.eval

    def eval_hook(wts, data, stats, **kw):
        if kw.get("v_out") is ind.gbuf and kw.get("wts_b") is None:
            kw["resid_out"] = res1
        return orig_eval(wts, data, stats, **kw)

    run.backend.eval = eval_hook
    res = run.run()
    scale = res.scale
    r1 = risk.quantile(res1, (0.985, 0.99, 0.995), run.di.world)
    r2 = risk.quantile(res.induction.residuals[0], (0.985, 0.99, 0.995), run.di.world)
    return {"phi0": res.phi, "psi0": res.psi, "V0": res.v0, "VaR_Res1": (r1 * scale).tolist(),
            "VaR_Res2": (r2 * scale).tolist(), "VaR_Res1_unit": r1.tolist(), "VaR_Res2_unit": r2.tolist(),
            "result": res}


def sanity_checks(cfg_or_params, sv: bool = False) -> dict:
    """Implicit notebook checks on freshly simulated paths."""
    cfg = parse_params(cfg_or_params, sv=sv) if isinstance(cfg_or_params, dict) else cfg_or_params
    run = HedgeRun(cfg)
    p, vt = run.simulate()
    st = run.summary_stats()
    out = {"grid": {"n_fine": run.grid.n_fine, "reduction": run.grid.reduction, "n_coarse": run.grid.n_coarse,
                    "dt_coarse": run.grid.dt_coarse, "shape": [run.n_total, p.n_coarse]}}
    drift = cfg.mu if run.kind == "pension" else cfg.r
    analytic = cfg.Y * math.exp(drift * cfg.T)
    out["mean_Y_T"] = st["mean_Y_T"] * (cfg.Y if run.kind == "pension" else 1.0)
    out["analytic_Y_T"] = analytic
    out["diff"] = out["mean_Y_T"] - analytic
    if "E_N_T" in st:
        nT = p.nfrac_final.double() * cfg.N
        out["N_T"] = {"mean": float(nT.mean()), "std": float(nT.std())}
    out["p_oom"] = st["p_oom"]
    out["E_payoff"] = st["E_payoff"]
    out["nparams"] = run.spec.nparams
    return out
