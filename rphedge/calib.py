"""Offline stochastic-volatility calibration (C38–C41).

The reference downloads 10 years of S&P500 closes with yfinance
("Extra: Stochastic Volatility.ipynb":132-140).  There is no network here, so
:func:`load_prices` reads a local CSV (Date, Close) instead — or any array of
prices — and the rest is the notebook's pipeline:

* daily log returns, 40-day rolling std x sqrt(252) (``HV40D``, :208-217);
* drift ``mu = log(P_end / P_0) / years`` (:215);
* CIR OLS on the volatility series (``estimate_CIR_params``, :76-98):
  ``y = dsigma/sqrt(sigma)`` regressed on ``[1/sqrt(sigma), sqrt(sigma)]`` without
  intercept; ``a = -beta1``, ``b = beta0/a``, ``c = std(residuals)``.

The notebook's Feller check raises when ``2ab < c^2`` but its message says the
opposite (Q22); :class:`CIRParams` raises with the correct message unless
``parity_message=True``.
"""
from __future__ import annotations

import csv
import math
from dataclasses import dataclass

import numpy as np


@dataclass
class CIRParams:
    """CIR parameters; the Feller condition 2ab >= c^2 must hold (C40)."""

    a: float  # mean reversion speed
    b: float  # long-run mean
    c: float  # diffusion scale
    parity_message: bool = False

    def __post_init__(self):
        if 2 * self.a * self.b < self.c ** 2:
            msg = ("2ab has to be less than or equal to c^2." if self.parity_message
                   else f"Feller condition violated: 2ab={2 * self.a * self.b:.3g} < c^2={self.c ** 2:.3g}")
            raise ValueError(msg)

    def as_sv_params(self) -> dict:
        """Keys of the ``Replicating_Portfolio_SV`` params dict."""
        return {"a": self.a, "b": self.b, "sv_c": self.c}


def estimate_CIR_params(sigma_t, check_feller: bool = True) -> CIRParams:
    """OLS estimate (C41) — identical regression to the notebook, no sklearn."""
    s = np.asarray(sigma_t, dtype=np.float64)
    sq = np.sqrt(s[:-1])
    y = np.diff(s) / sq
    X = np.stack([1.0 / sq, sq], axis=1)
    beta, *_ = np.linalg.lstsq(X, y, rcond=None)
    ab, a = beta[0], -beta[1]
    b = ab / a
    c = float(np.std(y - X @ beta))
    if not check_feller:
        obj = CIRParams.__new__(CIRParams)
        obj.a, obj.b, obj.c, obj.parity_message = float(a), float(b), c, False
        return obj
    return CIRParams(float(a), float(b), c)


def load_prices(path: str, column: str = "Close") -> np.ndarray:
    """Read closing prices from a CSV with a header (offline replacement of yfinance)."""
    with open(path, newline="") as f:
        rows = list(csv.DictReader(f))
    return np.asarray([float(r[column]) for r in rows if r.get(column) not in (None, "")], dtype=np.float64)


def log_returns(prices) -> np.ndarray:
    p = np.asarray(prices, dtype=np.float64)
    return np.diff(np.log(p))


def historic_volatility(prices, window: int = 40, annualise: int = 252) -> np.ndarray:
    """Rolling std of daily log returns x sqrt(252) (C39, "HV40D"), NaNs dropped."""
    r = log_returns(prices)
    if len(r) < window:
        return np.empty(0)
    c = np.cumsum(np.insert(r, 0, 0.0))
    c2 = np.cumsum(np.insert(r * r, 0, 0.0))
    n = window
    s = c[n:] - c[:-n]
    s2 = c2[n:] - c2[:-n]
    var = (s2 - s * s / n) / (n - 1)  # pandas rolling std uses ddof=1
    return np.sqrt(np.maximum(var, 0.0)) * math.sqrt(annualise)


def drift(prices, years: float = 10.0) -> float:
    p = np.asarray(prices, dtype=np.float64)
    return float(math.log(p[-1] / p[0]) / years)


def acf(x, nlags: int = 40) -> np.ndarray:
    """Sample autocorrelation (the notebook plots ACF of returns and squared returns)."""
    x = np.asarray(x, dtype=np.float64) - np.mean(x)
    d = np.dot(x, x)
    return np.asarray([1.0] + [float(np.dot(x[:-k], x[k:]) / d) for k in range(1, nlags + 1)])


def calibrate(prices, window: int = 40, years: float | None = None) -> dict:
    """Full SVN pipeline: mu, vol_0 and CIR(a, b, c) from a price history."""
    p = np.asarray(prices, dtype=np.float64)
    years = years if years is not None else len(p) / 252.0
    vol = historic_volatility(p, window)
    cir = estimate_CIR_params(vol, check_feller=False)
    return {"mu": drift(p, years), "vol0": float(vol[-1]), "a": cir.a, "b": cir.b, "c": cir.c,
            "volatility": vol}


def synthetic_prices(n_days: int = 2520, mu: float = 0.09, seed: int = 0, s0: float = 2000.0,
                     a: float = 0.0034, b: float = 0.155, c: float = 0.0158) -> np.ndarray:
    """Offline stand-in for the S&P500 download: daily prices with CIR-on-sigma
    volatility (used by tests/examples; no network)."""
    rng = np.random.default_rng(seed)
    v = b
    lp = math.log(s0)
    out = [s0]
    dt = 1 / 252
    for _ in range(n_days):
        v = max(v + a * (b - v) + c * math.sqrt(max(v, 1e-12)) * rng.standard_normal(), 1e-4)
        lp += (mu - 0.5 * v * v) * dt + v * math.sqrt(dt) * rng.standard_normal()
        out.append(math.exp(lp))
    return np.asarray(out)
