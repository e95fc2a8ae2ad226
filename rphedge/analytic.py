"""Closed-form / semi-closed-form option prices used as quality anchors.

* Black–Scholes price and delta (the European anchor 10.3896 / 0.7285,
  BASELINE.md; re-exported from :mod:`rphedge.utils.reports`).
* Heston (1993) European call price and delta by Fourier inversion
  (Albrecher et al. "little Heston trap" characteristic function, Gil-Pelaez
  probabilities P1/P2) — the anchor for the BASELINE.json Heston config
  ("Heston stochastic-vol, 30 steps, 1M paths"), which the reference does not
  cover (its SV model is the CIR-on-sigma recursion of
  ``Replicating_Portfolio.py:273-289``).
* Margrabe-free basket bounds are not closed-form; the basket anchor is the
  discounted Monte-Carlo payoff mean the run itself reports (``E_payoff``).

Host-only numpy/scipy code: nothing here is on a hot path.
"""
from __future__ import annotations

import math

import numpy as np

from .utils.reports import black_scholes, norm_cdf  # noqa: F401  (re-export)


def _heston_cf(u, T, kappa, theta, xi, rho, v0, r, x0, j):
    """Characteristic function of ln S_T under the measure of P_j (j = 1, 2)."""
    u = np.asarray(u, dtype=np.complex128)
    if j == 1:
        uu, b = 0.5, kappa - rho * xi
    else:
        uu, b = -0.5, kappa
    a = kappa * theta
    d = np.sqrt((rho * xi * 1j * u - b) ** 2 - xi * xi * (2.0 * uu * 1j * u - u * u))
    g = (b - rho * xi * 1j * u - d) / (b - rho * xi * 1j * u + d)
    e = np.exp(-d * T)
    C = r * 1j * u * T + a / (xi * xi) * ((b - rho * xi * 1j * u - d) * T - 2.0 * np.log((1.0 - g * e) / (1.0 - g)))
    D = (b - rho * xi * 1j * u - d) / (xi * xi) * (1.0 - e) / (1.0 - g * e)
    return np.exp(C + D * v0 + 1j * u * x0)


def _heston_p(j, S0, K, T, kappa, theta, xi, rho, v0, r, umax=200.0, n=4001):
    x0, lk = math.log(S0), math.log(K)
    # integrand is smooth and decays like exp(-c u): composite Simpson on (0, umax]
    u = np.linspace(1e-8, umax, n)
    f = np.real(np.exp(-1j * u * lk) * _heston_cf(u, T, kappa, theta, xi, rho, v0, r, x0, j) / (1j * u))
    h = u[1] - u[0]
    integral = h / 3.0 * (f[0] + f[-1] + 4.0 * f[1:-1:2].sum() + 2.0 * f[2:-1:2].sum())
    return 0.5 + integral / math.pi


def heston_call(S0: float, K: float, r: float, T: float, kappa: float, theta: float, xi: float, rho: float,
                v0: float) -> tuple[float, float]:
    """Heston European call price and delta (= P1).  Put via parity."""
    p1 = _heston_p(1, S0, K, T, kappa, theta, xi, rho, v0, r)
    p2 = _heston_p(2, S0, K, T, kappa, theta, xi, rho, v0, r)
    price = S0 * p1 - K * math.exp(-r * T) * p2
    return float(price), float(p1)


def heston_price(S0, K, r, T, kappa, theta, xi, rho, v0, option_type: str = "CALL") -> tuple[float, float]:
    c, d = heston_call(S0, K, r, T, kappa, theta, xi, rho, v0)
    if option_type.upper() == "CALL":
        return c, d
    return c - S0 + K * math.exp(-r * T), d - 1.0


def _moments(x, world: int = 1):
    import torch

    m = torch.stack([x.sum(), (x * x).sum(), torch.tensor(float(x.numel()), dtype=x.dtype, device=x.device)])
    if world > 1:
        from .parallel.dist import all_reduce_

        all_reduce_(m)
    s1, s2, n = (float(v) for v in m.cpu())
    mean = s1 / n
    return mean, math.sqrt(max(s2 / n - mean * mean, 0.0) * n / max(n - 1.0, 1.0))


def bs_delta_hedge(S, bond, strike: float, r: float, sigma: float, T: float, times,
                   option_type: str = "CALL", payoff=None, world: int = 1) -> dict:
    """Black–Scholes delta hedge of a European option on the SAME simulated
    coarse grid — the analytic anchor for the learnt hedge's P&L.

    ``S``: [n_coarse, n] normalised prices (S/S0, any torch device), ``bond``
    [n_coarse] B_t, ``strike`` normalised K/S0, ``times`` [n_coarse].  Wealth
    starts at the BS price, holds Δ_BS(t, S_t) stocks and the rest in the
    bank account (self-financing), P&L_T = W_T - payoff(S_T).  Also returns the
    one-step residual of the last date (the reference's "P&L", Q24) of the
    BS replicating portfolio (Δ S + (V - Δ S)/B B).  Values are normalised
    (multiply by S0).  float64 throughout; moments pooled over ranks."""
    import torch

    S = S.double()
    n_c = S.shape[0]
    B = torch.as_tensor(np.asarray(bond, np.float64), device=S.device)
    tt = np.asarray(times, np.float64)
    put = option_type.upper() != "CALL"
    if payoff is None:
        payoff = (strike - S[-1]).clamp_min(0) if put else (S[-1] - strike).clamp_min(0)
    payoff = payoff.double()

    def price_delta(s, tau):
        if tau <= 0:
            itm = (s < strike) if put else (s > strike)
            return ((strike - s).clamp_min(0) if put else (s - strike).clamp_min(0)), \
                (-itm.double() if put else itm.double())
        sq = sigma * math.sqrt(tau)
        d1 = (torch.log(s / strike) + (r + 0.5 * sigma * sigma) * tau) / sq
        d2 = d1 - sq
        Nd1 = 0.5 * torch.erfc(-d1 / math.sqrt(2.0))
        Nd2 = 0.5 * torch.erfc(-d2 / math.sqrt(2.0))
        disc = math.exp(-r * tau)
        if put:
            return strike * disc * (1 - Nd2) - s * (1 - Nd1), Nd1 - 1.0
        return s * Nd1 - strike * disc * Nd2, Nd1

    v0, _ = price_delta(S[0], T - tt[0])
    w = v0.clone()
    for t in range(n_c - 1):
        _, dl = price_delta(S[t], T - tt[t])
        g = float(B[t + 1] / B[t])
        w = w * g + dl * (S[t + 1] - S[t] * g)
    pnl = w - payoff
    vl, dl = price_delta(S[n_c - 2], T - tt[n_c - 2])
    resid = payoff - (dl * S[-1] + (vl - dl * S[n_c - 2]) / B[n_c - 2] * B[-1])
    pm, ps = _moments(pnl, world)
    _, rs = _moments(resid, world)
    return {"price": float(v0.mean()), "pnl_mean": pm, "pnl_std": ps, "residual_std_last": rs, "n_dates": n_c - 1}
