"""Heston QE scheme and the corrected CIR-on-sigma SV dynamics (numpy oracles,
the twins of the k_sim_scan branches; GPU parity in test_gpu_kernels.py)."""
import math

import numpy as np
import pytest

from rphedge.ops import paths as P


def _heston_grid():
    return P.Grid(T=1.0, dt=1.0 / 300, rebalancing=1.0 / 30)


HP = dict(kappa=2.0, theta=0.04, xi=0.5, rho=-0.7)


def test_qe_matches_analytic_heston_price():
    """Andersen QE at 10 steps per date: the MC call price sits within 3
    standard errors of the semi-closed-form price (full-truncation Euler is
    biased by about +1.3 % at the same step, BENCHMARKS.md)."""
    from rphedge.analytic import heston_call

    g = _heston_grid()
    n = 1 << 14
    S, V, fin = P._cpu_sv(g, n, 100.0, 0.05, 0.04, "heston", 0, 0, 0, HP["kappa"], HP["theta"], HP["xi"],
                          HP["rho"], 0, False, P.SEED_W1, P.SEED_W2, scheme="qe")
    pay = np.maximum(fin - 100.0, 0.0) * math.exp(-0.05)
    ref, _ = heston_call(100.0, 100.0, 0.05, 1.0, HP["kappa"], HP["theta"], HP["xi"], HP["rho"], 0.04)
    se = pay.std() / math.sqrt(n)
    assert abs(pay.mean() - ref) < 3 * se, (pay.mean(), ref, se)
    # martingale correction: the discounted price is a martingale to MC accuracy
    assert abs(fin.mean() * math.exp(-0.05) - 100.0) < 4 * fin.std() / math.sqrt(n)
    assert (V >= 0).all() and np.isfinite(S).all()


def test_qe_moments_of_the_variance():
    """E[v_T] = theta + (v0 - theta) e^{-kappa T} (exact CIR mean)."""
    g = _heston_grid()
    n = 1 << 14
    _, V, _ = P._cpu_sv(g, n, 100.0, 0.05, 0.09, "heston", 0, 0, 0, HP["kappa"], HP["theta"], HP["xi"],
                        HP["rho"], 0, False, P.SEED_W1, P.SEED_W2, scheme="qe")
    ev = HP["theta"] + (0.09 - HP["theta"]) * math.exp(-HP["kappa"] * float(g.times()[-1]))
    assert V[-1].mean() == pytest.approx(ev, rel=0.01)


def test_corrected_cir_sigma_units():
    """sv_tscale > 0: the calibrated daily (a, b, c) act per calibration day,
    so over 10 years sigma mean-reverts to b; the reference recursion (Q5)
    reverts per fine step regardless of dt."""
    g = P.Grid(T=10.0, dt=0.01, rebalancing=0.25)
    n = 1 << 11
    a, b, c = 0.0033566, 0.15431, 0.015833
    _, Vc, _ = P._cpu_sv(g, n, 1.0, 0.09, 0.30, "sv_ref", a, b, c, 0, 0, 0, 0, 0, False, P.SEED_W1, P.SEED_W2,
                         sv_tscale=252.0)
    # days elapsed after 1 year = 252: E[v] = b + (v0 - b)(1 - a)^252 (drift exact in expectation up to truncation)
    k1 = int(round(1.0 / g.dt_coarse))
    exp1 = b + (0.30 - b) * (1 - a) ** 252
    assert Vc[k1].mean() == pytest.approx(exp1, rel=0.03)
    assert Vc[-1].mean() == pytest.approx(b + (0.30 - b) * (1 - a) ** 2520, rel=0.05)
    _, Vr, _ = P._cpu_sv(g, n, 1.0, 0.09, 0.30, "sv_ref", a, b, c, 0, 0, 0, 0, 0, False, P.SEED_W1, P.SEED_W2)
    # reference: 100 fine steps per year, each reverting by a
    assert Vr[k1].mean() == pytest.approx(b + (0.30 - b) * (1 - a) ** 100, rel=0.03)


def test_config_wires_sv_flags():
    from rphedge.config import ParityFlags, parse_params

    base = dict(Y=1.0, K=1.0, T=10.0, mu=0.09, r=0.03, s0=0.16, a=0.0034, b=0.154, c=0.075, rebalancing=0.25,
                N=10000, P=100, x=55, l0=0.01, ita=0.0006, dt=0.01, n_paths=10)
    assert parse_params(dict(base), sv=True).parity.sv_reference_dynamics is False
    assert parse_params(dict(base, parity=True), sv=True).parity.sv_reference_dynamics is True
    assert ParityFlags.reference().sv_reference_dynamics is True
    assert parse_params(dict(base, heston_scheme="euler"), sv=True).heston_scheme == "euler"
