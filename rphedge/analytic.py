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
