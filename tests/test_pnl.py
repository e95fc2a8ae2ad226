"""Self-financing hedge P&L: the driver's P&L scan
(TorchBackend.pnl here; k_hedge_pnl on the GPU, test_gpu_kernels.py) against
an independent numpy oracle, and the Black-Scholes delta-hedge anchor."""
import math

import numpy as np
import pytest
import torch


def _np_forward(spec, w, X, alpha):
    t = spec.unflatten(w)
    n1, n2, n3 = spec.layer_names
    a = X @ t[f"{n1}/kernel"] + t[f"{n1}/bias"]
    a = np.where(a > 0, a, alpha * a)
    a = a @ t[f"{n2}/kernel"] + t[f"{n2}/bias"]
    a = np.where(a > 0, a, alpha * a)
    o = a @ t[f"{n3}/kernel"] + t[f"{n3}/bias"]
    if spec.nhold != spec.nout:  # psi = 1 - phi head
        o = np.concatenate([o, 1.0 - o], axis=1)
    return o


def _run(q99=False, parity=False):
    from rphedge.api import european_option, run_params
    from rphedge.experiments import mts_parameters

    if q99:
        return run_params(mts_parameters(n_paths=12, dt=0.1, rebalancing=1.0, epochs_first=30, epochs_rest=6,
                                         verbose=False, device="cpu", batch_size=1024))
    return european_option(N_paths=4096, dt=1 / 52, rebalancing_frequency=1 / 13, epochs_first=40, epochs_rest=8,
                           batch_size=1024, verbose=False, device="cpu", parity=parity)


def oracle_pnl(res, complement_head=False, hold_c=0.0, raw=False):
    """Independent numpy recursion of the self-financing P&L of a finished run:
    wealth starts at V_0, holds phi_t of date t's network, rest in the bank."""
    from rphedge.driver import feature_norms
    from rphedge.engine import current_weights
    import rphedge.models.hedge_mlp as hm
    from rphedge.ops import layout as L

    ind, p = res.induction, res.paths
    nd = p.n_coarse - 1
    nin, nhold = len(p.features(0)), len(p.prices(0)) + 1
    head = L.HEAD_COMPLEMENT if complement_head else L.HEAD_FREE
    spec = hm.NetSpec(nin=nin, hidden=8, nout=1 if complement_head else nhold, head=head)
    norms = feature_norms(p, "none" if raw else "date") or [((0.0,) * nin, (1.0,) * nin)] * nd
    bond = np.asarray(p.bond, np.float64)
    snap = ind.weights_snapshots.cpu()
    W = ind.values[0].double().cpu().numpy().copy()
    for t in range(nd):
        X = np.stack([f.double().cpu().numpy() for f in p.features(t)], axis=1)
        mu, isd = norms[t]
        X = (X - np.asarray(mu)) * np.asarray(isd)
        h = _np_forward(spec, current_weights(spec, snap[t, 0]).astype(np.float64), X, spec.alpha)
        if hold_c:
            hb = _np_forward(spec, current_weights(spec, snap[t, 1]).astype(np.float64), X, spec.alpha)
            h = h + hold_c * (hb - h)
        g = bond[t + 1] / bond[t]
        S0 = np.stack([s.double().cpu().numpy() for s in p.prices(t)], axis=1)
        S1 = np.stack([s.double().cpu().numpy() for s in p.prices(t + 1)], axis=1)
        W = W * g + (h[:, :S0.shape[1]] * (S1 - S0 * g)).sum(axis=1)
    return W, W - ind.values[nd].double().cpu().numpy()


def check_against_oracle(res, **kw):
    W, pnl = oracle_pnl(res, **kw)
    ind = res.induction
    np.testing.assert_allclose(ind.pnl_paths.double().cpu().numpy(), pnl, rtol=0,
                               atol=2e-5 * max(1.0, np.abs(W).max()))
    sf = res.self_financing_pnl
    assert sf["std"] == pytest.approx(pnl.std(ddof=1) * res.scale, rel=1e-4)
    assert sf["mean"] == pytest.approx(pnl.mean() * res.scale, abs=1e-4 * res.scale * max(pnl.std(), 1e-3))


@pytest.mark.parametrize("case", ["euro", "euro_parity_head", "pension_q99"])
def test_self_financing_pnl_matches_numpy_oracle(case):
    res = _run(q99=case == "pension_q99", parity=case == "euro_parity_head")
    check_against_oracle(res, complement_head=case == "euro_parity_head",
                         hold_c=0.1 if case == "pension_q99" else 0.0, raw=case == "euro_parity_head")
    # the default reports it; the parity flag keeps the reference's one-step residual
    assert res.terminal_pnl["kind"] == ("one_step_residual" if case == "euro_parity_head" else "self_financing")
    assert res.terminal_residual["std"] > 0


def test_bs_delta_anchor_converges():
    """The BS delta hedge on the simulated grid: P&L std shrinks ~ 1/sqrt(dates),
    its mean is near zero, and its price is the BS price."""
    from rphedge import analytic
    from rphedge.ops import paths as P

    out = []
    for nd in (13, 52):
        g = P.Grid(1.0, 1.0 / nd, 1.0 / nd)
        p = P.simulate_gbm(g, 1 << 14, 100.0, 0.08, 0.15, scheme="log", norm=100.0, device="cpu")
        a = analytic.bs_delta_hedge(p.S, g.bond(0.08), 1.0, 0.08, 0.15, 1.0, g.times())
        out.append(a)
        assert a["price"] * 100 == pytest.approx(10.3896, abs=1e-3)
        assert abs(a["pnl_mean"] * 100) < 0.05
    assert out[1]["pnl_std"] < 0.6 * out[0]["pnl_std"]
    assert 0.4 < out[1]["pnl_std"] * 100 < 0.9   # ~ sqrt(pi/4)/sqrt(52) * vega scale


def test_pnl_config_flag():
    from rphedge.config import ParityFlags

    assert ParityFlags().local_residual_pnl is False
    assert ParityFlags.reference().local_residual_pnl is True
