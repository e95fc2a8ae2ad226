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


def _plt():
    """matplotlib with the reference notebooks' style (C43: bmh, 20x7, font 13)."""
    import matplotlib

    matplotlib.use("Agg")
    import matplotlib.pyplot as plt

    plt.style.use("bmh")
    plt.rcParams["figure.figsize"] = (20, 7)
    plt.rcParams["font.size"] = 13
    return plt


def _np(x, limit: int | None = None):
    a = x.detach().float().cpu().numpy() if hasattr(x, "detach") else np.asarray(x)
    return a[..., :limit] if limit is not None else a


def _save(plt, fig, files, path):
    fig.savefig(path, bbox_inches="tight")
    plt.close(fig)
    files.append(path)


def plot_paths(paths, out_prefix: str = "rphedge", n_show: int = 50, scale: float = 1.0) -> list:
    """C32: sampled paths of the traded asset / fund, lambda and N(t) paths, and
    terminal-distribution histograms ("Multi Time Step.ipynb":169-171, :258-270,
    :346-358, :390-420; "European Options.ipynb" path cells)."""
    try:
        plt = _plt()
    except Exception:  # pragma: no cover
        return []
    files = []
    t = paths.grid.times()[: paths.n_coarse]
    S = _np(paths.S)
    S0 = S[:, 0, :] if S.ndim == 3 else S
    fig, ax = plt.subplots()
    ax.plot(t, S0[:, :n_show] * paths.norm * scale, lw=0.8)
    ax.set_title(f"{n_show} simulated paths")
    ax.set_xlabel("t")
    _save(plt, fig, files, f"{out_prefix}_paths.png")
    if paths.lam is not None:
        fig, ax = plt.subplots()
        ax.plot(t, _np(paths.lam)[:, :n_show], lw=0.8)
        ax.set_title("mortality intensity lambda_t")
        _save(plt, fig, files, f"{out_prefix}_lambda.png")
    if paths.nfrac is not None:
        fig, ax = plt.subplots()
        ax.plot(t, _np(paths.nfrac)[:, :n_show], lw=0.8)
        ax.set_title("survivors N_t / N")
        _save(plt, fig, files, f"{out_prefix}_survivors.png")
    if paths.vol is not None:
        fig, ax = plt.subplots()
        ax.plot(t, _np(paths.vol)[:, :n_show], lw=0.8)
        ax.set_title("stochastic volatility paths")
        _save(plt, fig, files, f"{out_prefix}_vol.png")
    ncols = 1 + (paths.nfrac_final is not None)
    fig, axs = plt.subplots(1, ncols)
    axs = np.atleast_1d(axs)
    sf = _np(paths.S_final)
    sf = sf[0] if sf.ndim == 2 else sf
    axs[0].hist(sf * paths.norm * scale, bins=100)
    axs[0].set_title("terminal value distribution")
    if paths.nfrac_final is not None:
        axs[1].hist(_np(paths.nfrac_final), bins=100)
        axs[1].set_title("N_T / N distribution")
    _save(plt, fig, files, f"{out_prefix}_terminal_hist.png")
    return files


def plot_run(res, paths=None, out_prefix: str = "rphedge_run", max_points: int = 20000) -> list:
    """Report figures of a finished run (C26, C27, C29–C31; C32 with ``paths``):

    * holdings over time: violin of phi / psi per rebalancing date + mean lines
      ("Multi Time Step.ipynb":1005-1023);
    * terminal residual vs terminal asset value coloured by sign, and its
      histogram (:921-930);
    * value fan chart (quantiles .99/.95/.9/.1/.05/.01 of V_t, :1086-1110);
    * expected-value trajectory P_E_Values and the mae/mape error history
      (:1112-1119).
    """
    try:
        plt = _plt()
    except Exception:  # pragma: no cover
        return []
    files = []
    ind = res.induction
    scale = res.scale
    if paths is None:
        paths = getattr(res, "paths", None)
    hot = holdings_over_time(res)
    times = np.asarray(list(hot.keys()))
    means = np.asarray(list(hot.values()))
    names = ["Phi", "Psi"] + [f"h{k}" for k in range(2, means.shape[1])]
    if ind.holdings is not None:
        H = _np(ind.holdings, max_points)          # [dates, nhold, n]
        fig, axs = plt.subplots(1, min(2, H.shape[1]))
        axs = np.atleast_1d(axs)
        tt = np.arange(H.shape[0]) * (times[1] - times[0] if len(times) > 1 else 1.0)
        width = 0.8 * (tt[1] - tt[0]) if len(tt) > 1 else 0.5
        for k, ax in enumerate(axs):
            ax.violinplot([H[i, k] for i in range(H.shape[0])], positions=tt, widths=width, showmeans=True)
            ax.plot(times, means[:, k], color="k", marker="o", lw=1)
            ax.set_title(f"{names[k]} over time")
            ax.set_xlabel("T")
        _save(plt, fig, files, f"{out_prefix}_holdings.png")
    else:
        fig, ax = plt.subplots()
        for k in range(means.shape[1]):
            ax.plot(times, means[:, k], marker="o", label=names[k])
        ax.set_title("Phi / Psi over time")
        ax.legend()
        _save(plt, fig, files, f"{out_prefix}_holdings.png")
    if ind.residuals is not None:
        r = _np(ind.residuals[0], max_points) * scale
        fig, axs = plt.subplots(1, 2)
        if paths is not None:
            sT = _np(paths.asset(paths.n_coarse - 1, 0), max_points) * paths.norm
            axs[0].scatter(sT[r >= 0], r[r >= 0], s=2, color="tab:green", label="residual >= 0")
            axs[0].scatter(sT[r < 0], r[r < 0], s=2, color="tab:red", label="residual < 0")
            axs[0].set_xlabel("terminal asset value")
            axs[0].legend()
        else:
            axs[0].plot(np.sort(r))
        axs[0].set_title("residual at T")
        axs[1].hist(r, bins=100)
        axs[1].set_title("distribution of residuals at T")
        _save(plt, fig, files, f"{out_prefix}_residuals.png")
    if ind.values is not None:
        fan = value_fan(ind.values, scale=scale)      # [6, n_coarse]
        tv = np.arange(fan.shape[1]) * (times[1] - times[0] if len(times) > 1 else 1.0)
        fig, ax = plt.subplots()
        for q, row in zip((0.99, 0.95, 0.9, 0.1, 0.05, 0.01), fan):
            ax.plot(tv, row, label=f"q{q}")
        ax.plot(tv, _np(ind.values).mean(axis=1) * scale, color="k", lw=2, label="mean")
        ax.set_title("value of the replicating portfolio (fan chart)")
        ax.legend()
        _save(plt, fig, files, f"{out_prefix}_value_fan.png")
    if res.p_e_values is not None and len(res.p_e_values):
        pe = np.asarray(res.p_e_values)
        fig, axs = plt.subplots(1, 2)
        axs[0].plot(pe[:, 0], label="mean V_t")
        axs[0].plot(pe[:, 1], label="E payoff e^{-mu dt its}")
        axs[0].plot(pe[:, 2], label="E payoff e^{-r dt its}")
        axs[0].legend()
        axs[0].set_title("expected value trajectory")
        er = np.asarray(res.errors)
        if er.size:
            axs[1].plot(er[:, 0], label="mae")
            ax2 = axs[1].twinx()
            ax2.plot(er[:, 1], color="tab:orange", label="mape")
            axs[1].legend(loc="upper left")
            ax2.legend(loc="upper right")
        axs[1].set_title("fit error per backward step")
        _save(plt, fig, files, f"{out_prefix}_trajectory.png")
    if paths is not None:
        files += plot_paths(paths, out_prefix=out_prefix)
    return files
