"""Host twins of the device inverse-normal-CDF approximations (K2).

* :func:`ndtri_u30_f32` — Giles' single-precision erfinv in the
  ``w = -log(4u(1-u))`` form evaluated from the raw 30-bit Sobol integer
  (no cancellation near u=0 or u=1).
* :func:`ndtri_u30_f64` — Acklam's rational approximation plus one Halley step
  on ``erfc``; matches ``scipy.stats.norm.ppf`` (reference
  ``Replicating_Portfolio.py:57``) to ~1e-15 relative.
"""
from __future__ import annotations

import numpy as np
from scipy.special import erfc

_GILES_C = [2.81022636e-08, 3.43273939e-07, -3.5233877e-06, -4.39150654e-06, 0.00021858087,
            -0.00125372503, -0.00417768164, 0.246640727, 1.50140941]
_GILES_T = [-0.000200214257, 0.000100950558, 0.00134934322, -0.00367342844, 0.00573950773,
            -0.0076224613, 0.00943887047, 1.00167406, 2.83297682]

_A = [-3.969683028665376e+01, 2.209460984245205e+02, -2.759285104469687e+02, 1.383577518672690e+02,
      -3.066479806614716e+01, 2.506628277459239e+00]
_B = [-5.447609879822406e+01, 1.615858368580409e+02, -1.556989798598866e+02, 6.680131188771972e+01,
      -1.328068155288572e+01]
_C = [-7.784894002430293e-03, -3.223964580411365e-01, -2.400758277161838e+00, -2.549732539343734e+00,
      4.374664141464968e+00, 2.938163982698783e+00]
_D = [7.784695709041462e-03, 3.224671290700398e-01, 2.445134137142996e+00, 3.754408661907416e+00]

S30 = 2.0 ** -30


def ndtri_u30_f32(x) -> np.ndarray:
    x = np.asarray(x, dtype=np.int64)
    x = np.where(x == 0, 1, x)
    a = (x.astype(np.float32) * np.float32(S30)).astype(np.float32)
    b = ((2 ** 30 - x).astype(np.float32) * np.float32(S30)).astype(np.float32)
    y = ((2 * x - 2 ** 30).astype(np.float32) * np.float32(S30)).astype(np.float32)
    w = (-np.log(np.float32(4.0) * a * b)).astype(np.float32)
    central = w < 5.0
    wc = w - np.float32(2.5)
    wt = np.sqrt(w) - np.float32(3.0)
    pc = np.full_like(w, _GILES_C[0])
    pt = np.full_like(w, _GILES_T[0])
    for c in _GILES_C[1:]:
        pc = (pc * wc + np.float32(c)).astype(np.float32)
    for c in _GILES_T[1:]:
        pt = (pt * wt + np.float32(c)).astype(np.float32)
    p = np.where(central, pc, pt)
    return (np.float32(1.41421356237309505) * p * y).astype(np.float32)


def ndtri_acklam(p, q=None) -> np.ndarray:
    p = np.asarray(p, dtype=np.float64)
    q = 1.0 - p if q is None else np.asarray(q, dtype=np.float64)
    plow = 0.02425
    z = np.empty_like(p)
    lo = p < plow
    hi = (~lo) & (q < plow)
    mid = ~(lo | hi)
    with np.errstate(divide="ignore", invalid="ignore"):
        t = np.sqrt(-2.0 * np.log(np.where(lo, p, 0.5)))
        z_lo = (((((_C[0] * t + _C[1]) * t + _C[2]) * t + _C[3]) * t + _C[4]) * t + _C[5]) / \
               ((((_D[0] * t + _D[1]) * t + _D[2]) * t + _D[3]) * t + 1.0)
        t = np.sqrt(-2.0 * np.log(np.where(hi, q, 0.5)))
        z_hi = -(((((_C[0] * t + _C[1]) * t + _C[2]) * t + _C[3]) * t + _C[4]) * t + _C[5]) / \
            ((((_D[0] * t + _D[1]) * t + _D[2]) * t + _D[3]) * t + 1.0)
        r0 = p - 0.5
        r = r0 * r0
        z_mid = (((((_A[0] * r + _A[1]) * r + _A[2]) * r + _A[3]) * r + _A[4]) * r + _A[5]) * r0 / \
                (((((_B[0] * r + _B[1]) * r + _B[2]) * r + _B[3]) * r + _B[4]) * r + 1.0)
    z = np.where(lo, z_lo, np.where(hi, z_hi, z_mid))
    e = np.where(p < 0.5, 0.5 * erfc(-z / np.sqrt(2.0)) - p, q - 0.5 * erfc(z / np.sqrt(2.0)))
    u = e * np.sqrt(2.0 * np.pi) * np.exp(0.5 * z * z)
    return z - u / (1.0 + 0.5 * z * u)


def ndtri_u30_f64(x) -> np.ndarray:
    x = np.asarray(x, dtype=np.int64)
    with np.errstate(divide="ignore", invalid="ignore"):
        z = ndtri_acklam(x * S30, (2 ** 30 - x) * S30)
    return np.where(x == 0, -np.inf, z)
