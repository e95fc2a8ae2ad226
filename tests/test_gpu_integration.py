"""GPU integration: the reference experiments end to end on the HIP backend."""
import json
import math
import os

import numpy as np
import pytest
import torch

pytestmark = pytest.mark.gpu

OUT = os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "gpurun_out")


def _record(name, payload):
    os.makedirs(OUT, exist_ok=True)
    with open(os.path.join(OUT, "integration.jsonl"), "a") as f:
        f.write(json.dumps({"test": name, **payload}, default=float) + "\n")


@pytest.mark.parametrize("parity", [True, False])
def test_pension_reference_config(parity):
    """RP module config ("Multi Time Step.ipynb":1329-1351): 4096 paths, dt=1/100,
    quarterly, 500/100 epochs with early stopping, batch 512.  Reference
    (unknown hardware, TF): phi0=634,349 psi0=350,176."""
    from rphedge.api import run_params
    from rphedge.experiments import mts_parameters

    p = mts_parameters(verbose=False, parity=parity, poll_every=10)
    res = run_params(p)
    _record(f"pension_parity={parity}", {"phi0": res.phi, "psi0": res.psi, "V0": res.v0,
                                         "epochs": res.summary["epochs_mse"], "var": res.var})
    assert 4.5e5 < res.phi < 8.5e5
    assert 1.5e5 < res.psi < 5.5e5
    assert 8.8e5 < res.phi + res.psi < 1.1e6
    assert 8.5e5 < res.v0 < 1.1e6


def test_sv_reference_config():
    """Replicating_Portfolio_SV with the notebook dict (Q4: c overwritten to 0.075).
    Reference: phi0=626,123 psi0=371,854."""
    from rphedge.api import Replicating_Portfolio_SV
    from rphedge.experiments import sv_parameters

    phi, psi = Replicating_Portfolio_SV(sv_parameters(verbose=False, parity=True, poll_every=10))
    _record("sv_parity", {"phi0": phi, "psi0": psi})
    assert math.isfinite(phi) and math.isfinite(psi)
    assert 8.0e5 < phi + psi < 1.2e6


@pytest.mark.parametrize("sv", [False, True])
def test_public_entry_points_run_lm_by_default(sv, monkeypatch):
    """Corrected mode: Replicating_Portfolio(_SV)(notebook dict) on the GPU fits
    BOTH networks with Levenberg-Marquardt (api.LM_PROFILE) - the run's
    config says so - and lands in the same holdings band as the Keras-Adam
    reference config (test_pension_reference_config; RP:29-235, :237-459)."""
    from rphedge import api
    from rphedge.experiments import mts_parameters, sv_parameters

    seen = {}
    orig = api.HedgeRun.build

    def spy(self, *a, **kw):
        seen["opt"] = (self.cfg.train.optimizer, self.cfg.train.q99_optimizer, self.backend_kind)
        return orig(self, *a, **kw)

    monkeypatch.setattr(api.HedgeRun, "build", spy)
    fn = api.Replicating_Portfolio_SV if sv else api.Replicating_Portfolio
    phi, psi = fn((sv_parameters if sv else mts_parameters)(verbose=False))
    _record(f"default_lm_sv={sv}", {"phi0": phi, "psi0": psi})
    assert seen["opt"] == ("lm", "lm", "hip")
    assert math.isfinite(phi) and math.isfinite(psi)
    assert 8.0e5 < phi + psi < 1.2e6
    if not sv:
        assert 4.5e5 < phi < 8.5e5 and 1.5e5 < psi < 5.5e5


def test_european_eo_parity_head():
    """EO notebook config with the psi = 1 - phi head (Q13): reference V0 = 11.352."""
    import rphedge

    res = rphedge.european_option(parity=True, verbose=False, poll_every=10)
    _record("eo_parity", {"V0": res.v0, "phi0": res.phi, "psi0": res.psi, "pnl": res.terminal_pnl})
    assert 9.5 < res.v0 < 13.0


def test_european_eo_corrected():
    import rphedge

    res = rphedge.european_option(verbose=False, poll_every=10)
    _record("eo_corrected", {"V0": res.v0, "phi0": res.phi, "psi0": res.psi, "pnl": res.terminal_pnl,
                             "var": res.var})
    assert abs(res.v0 - 10.3896) < 0.5
    # like-for-like with the reference's "P&L" (the one-step residual at T, Q24)
    assert res.terminal_residual["std"] < 1.7504
    assert res.terminal_pnl["kind"] == "self_financing" and math.isfinite(res.terminal_pnl["std"])


@pytest.mark.parametrize("optimizer", ["adam", "lm"])
def test_heston_and_basket_runs(optimizer):
    """Heston (QE) and basket-of-5 calls through the dict API.  Anchors: the
    semi-analytic Heston price 10.1546 (analytic.heston_call) and, for both, the
    discounted MC payoff of the run's own paths; the LM fits' exact bias step
    keeps V0 on the paths' MC price."""
    from rphedge.analytic import heston_call
    from rphedge.api import run_params

    base = dict(K=100, mu=0.05, r=0.05, sigma=0.2, N=1, P=1, x=0, l0=0, c=0, ita=0, mortality=False, q99=False,
                chunk_log2=6, lr_schedule_first=False, early_stopping=False, verbose=False, option_type="CALL",
                optimizer=optimizer)
    h = run_params(dict(base, Y=100, T=1.0, dt=1 / 300, rebalancing=1 / 30, n_paths=16, payoff="call",
                        model="heston", kappa=2.0, theta=0.04, xi=0.5, rho=-0.7, v0=0.04, batch_size=1 << 14,
                        epochs_first=40, epochs_rest=8, lr=1e-2))
    b = run_params(dict(base, Y=100, T=1.0, dt=1 / 30, rebalancing=1 / 30, n_paths=16, payoff="basket_call",
                        model="basket", n_assets=5, basket_corr=0.5, batch_size=1 << 14, epochs_first=40,
                        epochs_rest=8, lr=1e-2))
    mc_h = h.summary["E_payoff"] * h.scale * math.exp(-0.05)
    mc_b = b.summary["E_payoff"] * b.scale * math.exp(-0.05)
    ref_h, _ = heston_call(100.0, 100.0, 0.05, 1.0, 2.0, 0.04, 0.5, -0.7, 0.04)
    _record(f"heston_{optimizer}", {"V0": h.v0, "mc": mc_h, "analytic": ref_h, "pnl": h.terminal_pnl})
    _record(f"basket5_{optimizer}", {"V0": b.v0, "mc": mc_b, "pnl": b.terminal_pnl, "holdings0": b.holdings0.tolist()})
    assert abs(mc_h / ref_h - 1) < 0.01          # QE paths: MC price on the analytic one (2^16 paths)
    tol = 0.003 if optimizer == "lm" else 0.035  # Adam: no exact-mean step, the per-date mean error drifts
    assert abs(h.v0 / mc_h - 1) < tol and math.isfinite(h.terminal_pnl["std"])
    assert abs(b.v0 / mc_b - 1) < tol and len(b.holdings0) == 6


def test_async_and_polled_early_stopping_agree():
    from rphedge.api import run_params
    from rphedge.experiments import mts_parameters

    p = mts_parameters(verbose=False, n_paths=11, dt=0.1, rebalancing=1.0, epochs_first=60, epochs_rest=20,
                       patience_first=5, patience_rest=3, deterministic=True)
    a = run_params(dict(p, poll_every=0))
    b = run_params(dict(p, poll_every=4))
    assert a.summary["epochs_mse"] == b.summary["epochs_mse"]
    assert a.phi == pytest.approx(b.phi, rel=1e-3)


def test_concurrent_q99_fit_matches_sequential():
    """Corrected semantics (two networks): the pinball fit runs on a side
    stream concurrently with the MSE fit; the result equals the sequential
    schedule (the fits are independent), in eager mode and replayed from a graph."""
    import time

    from rphedge.api import HedgeRun
    from rphedge.config import parse_params
    from rphedge.experiments import mts_parameters

    out = {}
    for conc in (False, True):
        p = mts_parameters(verbose=False, concurrent_q99=conc, keep_paths=False)
        run = HedgeRun(parse_params(p))
        run.build()
        assert (run.induction.backend_q is not None) == conc
        run.run()  # warm (tables, templates)
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        res = run.run()
        out[conc] = (res, time.perf_counter() - t0)
        if conc:
            run.capture(include_simulation=False)
            run.replay()
            rg = run.collect()
            assert rg.phi == pytest.approx(res.phi, rel=1e-5)
    (rs, ts), (rc, tc) = out[False], out[True]
    _record("concurrent_q99", {"seq_s": ts, "conc_s": tc, "phi_seq": rs.phi, "phi_conc": rc.phi})
    assert rc.phi == pytest.approx(rs.phi, rel=1e-5)
    assert rc.psi == pytest.approx(rs.psi, rel=1e-5)
    assert rc.v0 == pytest.approx(rs.v0, rel=1e-5)
