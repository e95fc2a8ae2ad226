"""Host-side reports (SURVEY C28–C32): valuation, holdings, residuals, plots.

Plotting is optional (matplotlib/seaborn are not needed by the engine) and off
the hot path; every report also returns its numbers as a dict/DataFrame.
"""
from __future__ import annotations

import math

import numpy as np

from ..ops import layout as L


def norm_cdf(x: float) -> float:
    return 0.5 * math.erfc(-x / math.sqrt(2.0))


def black_scholes(S0: float, K: float, r: float, sigma: float, T: float, option_type: str = "CALL"):
    """Closed-form price and delta (the BASELINE comparison 10.3896 / 0.7285)."""
    d1 = (math.log(S0 / K) + (r + 0.5 * sigma * sigma) * T) / (sigma * math.sqrt(T))
    d2 = d1 - sigma * math.sqrt(T)
    if option_type.upper() == "CALL":
        return S0 * norm_cdf(d1) - K * math.exp(-r * T) * norm_cdf(d2), norm_cdf(d1)
    return K * math.exp(-r * T) * norm_cdf(-d2) - S0 * norm_cdf(-d1), norm_cdf(d1) - 1.0


def pension_closed_form(N0: float, P: float, T: float, r: float, sigma: float, E_N_T_frac: float):
    """Q-measure value of N P max(1, Y_T) = N P E[N_T]/N (e^{-rT} + BS call(K=1))."""
    call, delta = black_scholes(1.0, 1.0, r, sigma, T, "CALL")
    v = N0 * P * E_N_T_frac * (math.exp(-r * T) + call)
    return v, N0 * P * E_N_T_frac * delta, v - N0 * P * E_N_T_frac * delta


def valuation_report(res, discount_rate: float, T: float, eo_artifact: bool = False) -> dict:
    """V0 of the replicating portfolio vs discounted expected payoff (C29)."""
    scale = res.scale
    e_pay = res.summary["E_payoff"] * scale
    disc = e_pay * math.exp(-discount_rate * T)
    v0 = res.v0
    if eo_artifact:  # Q14: the EO notebook discounts values[:,0] instead of the payoff
        disc = v0 * math.exp(-discount_rate * T)
    return {"V0": v0, "discounted_E_payoff": disc, "difference": v0 - disc,
            "difference_pct": 100.0 * (v0 - disc) / disc if disc else float("nan")}


def holdings_over_time(res) -> dict:
    """Mean phi/psi per date (C30) -> {time: [phi, psi, ...]} (unscaled)."""
    nh = res.induction.dates[0].stats is not None and res.holdings0.shape[0]
    out = {}
    for d in res.induction.dates:
        out[round(d.time, 10)] = d.mean_holdings(nh).tolist()
    return dict(sorted(out.items()))


def value_fan(values, qs=(0.99, 0.95, 0.9, 0.1, 0.05, 0.01), scale: float = 1.0) -> np.ndarray:
    """Quantiles of V_t per date (fan chart, C29)."""
    import torch

    v = values.detach().float().cpu()
    return (torch.quantile(v.T.contiguous(), torch.tensor(qs, dtype=torch.float32), dim=0).numpy() * scale)


def residual_summary(res) -> dict:
    """Terminal residual describe() (C31)."""
    return dict(res.terminal_pnl)


def plot_run(res, paths=None, out_prefix: str = "rphedge_run"):
    """Optional matplotlib reports (C32/C43 style: bmh, 20x7, font 13)."""
    try:
        import matplotlib

        matplotlib.use("Agg")
        import matplotlib.pyplot as plt
    except Exception:  # pragma: no cover
        return []
    plt.rcParams["figure.figsize"] = (20, 7)
    plt.rcParams["font.size"] = 13
    plt.style.use("bmh")
    files = []
    hot = holdings_over_time(res)
    t = list(hot.keys())
    arr = np.asarray(list(hot.values()))
    fig, ax = plt.subplots()
    for k in range(arr.shape[1]):
        ax.plot(t, arr[:, k], marker="o", label=["Phi", "Psi"][k] if k < 2 else f"h{k}")
    ax.set_title("Phi / Psi over time")
    ax.legend()
    f = f"{out_prefix}_holdings.png"
    fig.savefig(f)
    files.append(f)
    plt.close(fig)
    if res.induction.residuals is not None:
        r = res.induction.residuals[0].detach().float().cpu().numpy() * res.scale
        fig, ax = plt.subplots()
        ax.hist(r, bins=100)
        ax.set_title("Distribution of residuals at T")
        f = f"{out_prefix}_residuals.png"
        fig.savefig(f)
        files.append(f)
        plt.close(fig)
    return files
