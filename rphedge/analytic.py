"""Closed-form / semi-closed-form option prices used as quality anchors.

* Black–Scholes price and delta (the European anchor 10.3896 / 0.7285,
  BASELINE.md; re-exported from :mod:`rphedge.utils.reports`).
* Heston (1993) European call price and delta by Fourier inversion
  (Albrecher et al. "little Heston trap" characteristic function, Gil-Pelaez
  probabilities P1/P2) — the anchor for the BASELINE.json Heston config
  ("Heston stochastic-vol, 30 steps, 1M paths"), which the reference does not
  cover (its SV model is the CIR-on-sigma recursion of
  ``Replicating_Portfolio.py:273-289``).
* Hedge anchors on the SAME simulated grid and paths as the learnt hedge
  (self-financing P&L std, the quantity the bench reports):
  Black-Scholes delta (GBM), the Heston delta and the Heston minimum-variance
  hedge Delta + (rho xi / S) dC/dv (per-path Fourier quadrature, torch on the
  paths' device), and the basket's per-asset deltas of a moment-matched
  lognormal (Levy) basket.  The reference's only quality anchor is its
  terminal P&L ("European Options.ipynb":3672-3678).

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


# ---------------------------------------------------------------------------
# Heston hedges on simulated paths
# ---------------------------------------------------------------------------
def _heston_cd(u, tau, kappa, theta, xi, rho, r, j):
    """C_j(u), D_j(u) of the Heston characteristic function (little-trap
    form): phi_j(u; x, v) = exp(C_j + D_j v + i u x), torch complex128."""
    import torch

    i = torch.complex(torch.zeros((), dtype=torch.float64), torch.ones((), dtype=torch.float64)).to(u.device)
    uu, b = (0.5, kappa - rho * xi) if j == 1 else (-0.5, kappa)
    a = kappa * theta
    iu = i * u
    bm = b - rho * xi * iu
    d = torch.sqrt(bm * bm - xi * xi * (2.0 * uu * iu - u * u))
    g = (bm - d) / (bm + d)
    e = torch.exp(-d * tau)
    C = r * iu * tau + a / (xi * xi) * ((bm - d) * tau - 2.0 * torch.log((1.0 - g * e) / (1.0 - g)))
    D = (bm - d) / (xi * xi) * (1.0 - e) / (1.0 - g * e)
    return C, D


def heston_greeks(S, v, strike: float, r: float, tau: float, kappa: float, theta: float, xi: float, rho: float,
                  n_quad: int = 3001, chunk: int = 4096):
    """Per-path Heston call price, delta dC/dS (= P1) and dC/dv at spot S,
    variance v (torch tensors, float64 on their device), time to maturity tau.

    Gil-Pelaez P_j = 1/2 + (1/pi) int_0^inf Re[e^{-iu ln K} phi_j / (iu)] du
    (and d/dv: an extra factor D_j) by composite Simpson in s = u sd with a
    per-path scale sd = sqrt(v_bar tau) (v_bar: expected mean variance to
    maturity), s in (0, 60]: near maturity and at small variance the
    integrand decays only at u ~ 1 / sd.  Paths more than 8 sd in or out of
    the money take the limits (P = 0 or 1, no vega)."""
    import torch

    S = S.double()
    v = v.double().clamp_min(0.0)
    dev = S.device
    x = torch.log(S)
    lk = math.log(strike)
    ekt = math.exp(-kappa * tau)
    vbar = theta + (v - theta) * ((1.0 - ekt) / (kappa * tau))
    sd = torch.sqrt((vbar * tau).clamp_min(1e-10))
    m = (x - lk) / sd
    far = m.abs() > 8.0
    nq = n_quad if n_quad % 2 == 1 else n_quad + 1
    s = torch.linspace(0.0, 60.0, nq, dtype=torch.float64, device=dev)
    s[0] = 1e-8
    w = torch.ones(nq, dtype=torch.float64, device=dev)
    w[1:-1:2], w[2:-1:2] = 4.0, 2.0
    w *= (s[2] - s[1]) / 3.0
    P = [torch.empty_like(S), torch.empty_like(S)]
    Pv = [torch.empty_like(S), torch.empty_like(S)]
    for lo in range(0, S.numel(), chunk):
        hi = min(S.numel(), lo + chunk)
        u = s[None, :] / sd[lo:hi, None]                         # [c, nq]
        for j in (1, 2):
            C, D = _heston_cd(u, tau, kappa, theta, xi, rho, r, j)
            ph = torch.exp(C + D * v[lo:hi, None] + 1j * u * (x[lo:hi, None] - lk))
            base = ph / (1j * u)
            f = torch.real(base)
            fv = torch.real(base * D)
            jac = 1.0 / sd[lo:hi, None]                          # du = ds / sd
            P[j - 1][lo:hi] = 0.5 + (f * jac * w).sum(1) / math.pi
            Pv[j - 1][lo:hi] = (fv * jac * w).sum(1) / math.pi
    itm = (x > lk).double()
    P1 = torch.where(far, itm, P[0].clamp(0.0, 1.0))
    P2 = torch.where(far, itm, P[1].clamp(0.0, 1.0))
    disc = math.exp(-r * tau)
    price = S * P1 - strike * disc * P2
    vega_v = torch.where(far, torch.zeros_like(S), S * Pv[0] - strike * disc * Pv[1])
    return price, P1, vega_v


def _sf_pnl(prices_fn, hedge_fn, bond, n_c: int, w0, payoff):
    """Self-financing wealth: start w0, hold hedge_fn(t) units of every risky
    asset (list), the rest in the bank account; P&L = W_T - payoff."""
    w = w0
    for t in range(n_c - 1):
        g = float(bond[t + 1] / bond[t])
        h = hedge_fn(t)
        s0, s1 = prices_fn(t), prices_fn(t + 1)
        w = w * g
        for a in range(len(h)):
            w = w + h[a] * (s1[a] - s0[a] * g)
    return w - payoff


def heston_hedge_anchor(S, V, bond, strike: float, r: float, T: float, times, kappa: float, theta: float,
                        xi: float, rho: float, payoff=None, world: int = 1, max_paths: int = 1 << 16,
                        option_type: str = "CALL") -> dict:
    """Self-financing P&L of the Heston delta hedge and of the minimum-
    variance hedge Delta + (rho xi / S) dC/dv on the simulated coarse grid
    (``S``, ``V`` [n_coarse, n] normalised price and variance; the first
    ``max_paths`` paths of this rank), started from the Heston price.  Moments
    pooled over ranks; values normalised (x S0)."""
    import torch

    m = min(int(S.shape[1]), int(max_paths))
    S = S[:, :m].double()
    V = V[:, :m].double()
    n_c = S.shape[0]
    tt = np.asarray(times, np.float64)
    put = option_type.upper() != "CALL"
    if payoff is None:
        payoff = (strike - S[-1]).clamp_min(0) if put else (S[-1] - strike).clamp_min(0)
    payoff = payoff[:m].double()
    hd, hm = [], []
    price0 = None
    for t in range(n_c - 1):
        pr, dl, cv = heston_greeks(S[t], V[t], strike, r, T - tt[t], kappa, theta, xi, rho)
        if put:
            dl = dl - 1.0
            pr = pr - S[t] + strike * math.exp(-r * (T - tt[t]))
        if t == 0:
            price0 = pr
        hd.append(dl)
        hm.append(dl + rho * xi * cv / S[t])
    out = {"price": float(price0.mean()), "paths": m * world}
    for name, h in (("delta", hd), ("min_variance", hm)):
        pnl = _sf_pnl(lambda t: [S[t]], lambda t, h=h: [h[t]], bond, n_c, price0, payoff)
        pm, ps = _moments(pnl, world)
        out[name] = {"pnl_mean": pm, "pnl_std": ps}
    return out


# ---------------------------------------------------------------------------
# Basket: moment-matched lognormal (Levy) deltas
# ---------------------------------------------------------------------------
def levy_basket_call(S, weights, strike: float, r: float, sigma: float, corr: float, tau: float):
    """Basket call price of a lognormal matched to the basket's first two
    moments (equal vols, one pairwise correlation).  S: [na, n] float64."""
    import torch

    w = torch.as_tensor(np.asarray(weights, np.float64), device=S.device)[:, None]
    ws = w * S
    F = ws.sum(0) * math.exp(r * tau)
    tot = ws.sum(0)
    sq = (ws * ws).sum(0)
    # E[B_T^2] = sum_ij w_i w_j S_i S_j e^{(2r + rho_ij sigma^2) tau}
    m2 = math.exp(2 * r * tau) * (math.exp(corr * sigma * sigma * tau) * (tot * tot - sq)
                                  + math.exp(sigma * sigma * tau) * sq)
    s2 = torch.log(m2 / (F * F)).clamp_min(1e-14)
    sb = torch.sqrt(s2)
    d1 = (torch.log(F / strike) + 0.5 * s2) / sb
    d2 = d1 - sb
    N = lambda z: 0.5 * torch.erfc(-z / math.sqrt(2.0))  # noqa: E731
    return math.exp(-r * tau) * (F * N(d1) - strike * N(d2))


def basket_hedge_anchor(S, bond, weights, strike: float, r: float, sigma: float, corr: float, T: float, times,
                        payoff=None, world: int = 1, max_paths: int = 1 << 16) -> dict:
    """Self-financing P&L of the per-asset Levy-basket deltas dC/dS_i
    (autograd) on the simulated grid (``S`` [n_coarse, na, n] normalised),
    started from the Levy price; the first ``max_paths`` paths of this rank."""
    import torch

    m = min(int(S.shape[2]), int(max_paths))
    S = S[:, :, :m].double()
    n_c = S.shape[0]
    tt = np.asarray(times, np.float64)
    w = np.asarray(weights, np.float64)
    if payoff is None:
        payoff = ((torch.as_tensor(w, device=S.device)[:, None] * S[-1]).sum(0) - strike).clamp_min(0)
    payoff = payoff[:m].double()
    hs = []
    price0 = None
    for t in range(n_c - 1):
        x = S[t].clone().requires_grad_(True)
        c = levy_basket_call(x, w, strike, r, sigma, corr, T - tt[t])
        (g,) = torch.autograd.grad(c.sum(), x)
        hs.append([g[a].detach() for a in range(S.shape[1])])
        if t == 0:
            price0 = c.detach()
    pnl = _sf_pnl(lambda t: [S[t, a] for a in range(S.shape[1])], lambda t: hs[t], bond, n_c, price0, payoff)
    pm, ps = _moments(pnl, world)
    return {"price": float(price0.mean()), "paths": m * world, "levy_delta": {"pnl_mean": pm, "pnl_std": ps}}
