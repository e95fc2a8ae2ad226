"""API / feature coverage on CPU: pension + SV dict API, parity flags, saved-model
format, CLI, experiments, calibration, Brownian helpers, reports."""
import json
import math
import os
import subprocess
import sys

import numpy as np
import pytest
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _small(**kw):
    from rphedge.experiments import mts_parameters

    p = mts_parameters(n_paths=9, dt=0.1, rebalancing=1.0, epochs_first=20, epochs_rest=5, verbose=False,
                       device="cpu")
    p.update(kw)
    return p


def test_replicating_portfolio_returns_two_floats():
    from rphedge import Replicating_Portfolio

    phi, psi = Replicating_Portfolio(_small())
    assert isinstance(phi, float) and isinstance(psi, float)
    # holdings of a N*P=1e6 guarantee: phi + psi of the order of the liability value
    assert 4e5 < phi + psi < 1.6e6


def test_public_entry_points_default_optimizer_per_mode():
    """Replicating_Portfolio(_SV) defaults (api.default_params): corrected mode
    on a GPU fits both networks with Levenberg-Marquardt (LM_PROFILE);
    parity=True keeps the reference's Keras-Adam (RP:149-175); the CPU torch
    oracle keeps Adam; a caller's own optimizer always wins."""
    from rphedge.api import LM_PROFILE, default_params
    from rphedge.config import parse_params
    from rphedge.experiments import mts_parameters, sv_parameters

    for sv, base in ((False, mts_parameters()), (True, sv_parameters())):
        tr = parse_params(default_params(base, gpu=True), sv=sv).train
        assert (tr.optimizer, tr.q99_optimizer) == ("lm", "lm")
        assert tr.lm_starts == LM_PROFILE["lm_starts"] and tr.lm_out_fix
        tr = parse_params(default_params(dict(base, parity=True), gpu=True), sv=sv).train
        assert (tr.optimizer, tr.q99_optimizer) == ("adam", "adam")
        tr = parse_params(default_params(base, gpu=False), sv=sv).train
        assert (tr.optimizer, tr.q99_optimizer) == ("adam", "adam")
        tr = parse_params(default_params(dict(base, optimizer="adam"), gpu=True), sv=sv).train
        assert tr.optimizer == "adam"
    # explicit device="cpu" on a GPU machine: the CPU oracle, Adam
    assert "optimizer" not in default_params(dict(mts_parameters(), device="cpu"))


def test_replicating_portfolio_sv_parity():
    from rphedge import Replicating_Portfolio_SV
    from rphedge.experiments import sv_parameters

    p = sv_parameters(n_paths=9, dt=0.1, rebalancing=1.0, epochs_first=20, epochs_rest=5, verbose=False,
                      device="cpu", parity=True)
    phi, psi = Replicating_Portfolio_SV(p)
    assert math.isfinite(phi) and math.isfinite(psi)


def test_parity_shared_model_has_identical_nets():
    from rphedge.api import HedgeRun
    from rphedge.config import parse_params

    cfg = parse_params(_small(parity=True))
    run = HedgeRun(cfg)
    run.build()
    assert run.induction.w_q is run.induction.w_mse           # Q1 alias
    assert run.induction.opt_q is not run.induction.opt_mse   # two Adam instances
    cfg2 = parse_params(_small())
    run2 = HedgeRun(cfg2)
    run2.build()
    assert run2.induction.w_q is not run2.induction.w_mse


def test_lr_rest_and_decay_schedules_through_dict_api():
    """lr / lr_rest / lr_decay build the per-epoch schedules of every date's fit
    (the throughput presets of bench.py use them); defaults keep the reference
    behaviour (step schedule on the first date, current lr afterwards)."""
    from rphedge.api import HedgeRun
    from rphedge.config import parse_params
    from rphedge.engine import geometric_lr_schedule, keras_lr_schedule

    g = geometric_lr_schedule(5e-2, 5, 0.1)
    np.testing.assert_allclose(g, [5e-2 * 0.1 ** (e / 4) for e in range(5)], rtol=1e-12)
    assert geometric_lr_schedule(1e-3, 3) == (1e-3,) * 3
    run = HedgeRun(parse_params(_small(lr=5e-2, lr_rest=4e-3, lr_decay=0.1, lr_schedule_first=False)))
    run.build()
    ind = run.induction
    assert ind._fcfg(True, 0).lr_schedule == geometric_lr_schedule(5e-2, 20, 0.1)
    assert ind._fcfg(False, 0).lr_schedule == geometric_lr_schedule(4e-3, 5, 0.1)
    ref = HedgeRun(parse_params(_small()))
    ref.build()
    assert list(ref.induction._fcfg(True, 0).lr_schedule) == keras_lr_schedule(20)
    assert ref.induction._fcfg(False, 0).lr_schedule is None


def test_example_configs_end_their_grid_at_maturity():
    """Every shipped config's coarse grid ends at T (a truncated 1/30 once made
    the reference-convention grid overshoot by one date)."""
    import glob

    from rphedge.ops.paths import Grid

    for p in sorted(glob.glob(os.path.join(ROOT, "examples", "*.json"))):
        d = json.load(open(p))
        g = Grid(d["T"], d["dt"], d["rebalancing"])
        assert abs(float(g.times()[-1]) - d["T"]) < 1e-9 * d["T"], p


def test_lambda_fine_index_quirk():
    """Q3: with parity the lambda feature at coarse index i is lambda on the fine grid at i."""
    from rphedge.ops import paths as P

    g = P.Grid(10.0, 0.1, 1.0)
    a = P.simulate_gbm(g, 512, 1.0, 0.08, 0.15, device="cpu")
    P.simulate_mortality(a, 0.01, 0.075, 0.000597, 10000, lambda_fine_index=True)
    b = P.simulate_gbm(g, 512, 1.0, 0.08, 0.15, device="cpu")
    P.simulate_mortality(b, 0.01, 0.075, 0.000597, 10000, lambda_fine_index=False)
    # fine index 1 vs coarse index 1 (= fine 10)
    assert not torch.allclose(a.lam[1], b.lam[1])
    assert torch.allclose(a.lam[0], b.lam[0])


def test_saved_model_roundtrip(tmp_path):
    from rphedge.api import HedgeRun
    from rphedge.config import parse_params
    from rphedge.engine import current_weights
    from rphedge.models.hedge_mlp import fold_input_norm, torch_forward, unfold_input_norm
    from rphedge.utils.model_io import load_date, save_run

    cfg = parse_params(_small())
    run = HedgeRun(cfg)
    res = run.run()
    save_run(str(tmp_path), run, res)
    files = sorted(os.listdir(tmp_path))
    assert "config.json" in files and "report.json" in files and "values.npy" in files
    assert sum(f.startswith("weights_t") for f in files) == run.paths.n_coarse - 1
    meta, spec, w, wq, vals = load_date(str(tmp_path), 0)
    mu0, isd0 = run.induction.norms[0]
    np.testing.assert_allclose(w, fold_input_norm(spec, current_weights(spec, res.induction.weights_snapshots[0, 0]),
                                                  mu0, isd0), rtol=1e-6, atol=1e-7)
    assert wq is not None and vals.shape == (run.n_local,)
    # saved weights are raw-input: same network outputs as the standardised
    # weights on standardised features (last date, non-degenerate spread)
    t = run.paths.n_coarse - 2
    _, _, wt, _, _ = load_date(str(tmp_path), t)
    mu, isd = run.induction.norms[t]
    assert any(s != 1.0 for s in isd)
    X = torch.stack(run.paths.features(t), dim=1).float()
    wn = torch.from_numpy(current_weights(spec, res.induction.weights_snapshots[t, 0]))
    raw = torch_forward(spec, torch.from_numpy(wt), X)
    std = torch_forward(spec, wn, (X - torch.tensor(mu).float()) * torch.tensor(isd).float())
    torch.testing.assert_close(raw, std, rtol=1e-4, atol=1e-5)
    np.testing.assert_allclose(unfold_input_norm(spec, wt, mu, isd), wn.numpy(), rtol=1e-4, atol=1e-6)
    from safetensors.numpy import load_file

    t = load_file(str(tmp_path / "weights_t0000.safetensors"))
    assert t["LeakyReLU_1/kernel"].shape == (3, 8) and t["Phi_Psi/bias"].shape == (2,)
    rep = json.load(open(tmp_path / "report.json"))
    assert abs(rep["phi0"] - res.phi) < 1e-6


def test_single_time_step_cpu():
    from rphedge.experiments import single_time_step

    out = single_time_step(parity=True, n_paths=9, epochs_first=30, device="cpu", verbose=False)
    assert len(out["VaR_Res1"]) == 3 and len(out["VaR_Res2"]) == 3
    # Q12: cost of capital 0.1*dt = 1.0 -> the blended (Res2) holdings are the Q99 holdings,
    # whose 99% VaR is below the MSE holdings' (the hedge sign condition of the notebook)
    assert out["VaR_Res2_unit"][1] <= out["VaR_Res1_unit"][1] + 1e-3


def test_volatility_sweep_rows():
    from rphedge.experiments import volatility_sweep

    rows = volatility_sweep(sigmas=(0.1, 0.3), n_paths=8, dt=0.1, rebalancing=2.0, epochs_first=10, epochs_rest=3,
                            verbose=False, device="cpu")
    assert [r["sigma"] for r in rows] == [0.1, 0.3]
    assert all(math.isfinite(r["Phi"]) and math.isfinite(r["Psi"]) for r in rows)


def test_sanity_checks_match_notebook_values():
    from rphedge.experiments import mts_parameters, sanity_checks

    out = sanity_checks(mts_parameters(device="cpu", verbose=False))
    assert out["grid"]["shape"] == [4096, 41]
    assert abs(out["diff"]) < 0.03                  # "Multi Time Step.ipynb":122-124 (diff 0.0016)
    assert 8550 < out["N_T"]["mean"] < 8680         # mean 8,615-8,617
    assert 110 < out["N_T"]["std"] < 160            # std 132-133
    assert out["nparams"] == 122


def test_cir_calibration_recovers_parameters():
    from rphedge import calib

    rng = np.random.default_rng(3)
    a, b, c = 0.02, 0.16, 0.01
    v = [b]
    for _ in range(20000):
        v.append(max(v[-1] + a * (b - v[-1]) + c * math.sqrt(v[-1]) * rng.standard_normal(), 1e-4))
    est = calib.estimate_CIR_params(np.asarray(v))
    assert est.a == pytest.approx(a, rel=0.3) and est.b == pytest.approx(b, rel=0.05)
    assert est.c == pytest.approx(c, rel=0.05)
    with pytest.raises(ValueError):
        calib.CIRParams(0.001, 0.1, 0.5)     # Feller violated (Q22: message corrected)
    out = calib.calibrate(calib.synthetic_prices(1500))
    assert set(out) >= {"mu", "vol0", "a", "b", "c"}
    assert len(calib.acf(np.random.default_rng(0).standard_normal(500), 10)) == 11


def test_brownian_helpers():
    from rphedge.brownian_motion import get_W, get_dW

    dW = get_dW(50, 1)
    W = get_W(50, 1)
    assert dW.shape == (50,) and W[0] == 0.0
    np.testing.assert_allclose(W[1:], np.cumsum(dW)[:-1])
    # the reference's draws: np.random.seed(1); np.random.normal(0, 1, T)
    # (legacy MT19937 stream; pinned values of seed 1)
    np.testing.assert_allclose(dW[:3], [1.6243453636632417, -0.6117564136500754, -0.5281717522634557], rtol=0,
                               atol=1e-15)
    np.testing.assert_allclose(W[:3], [0.0, 1.6243453636632417, 1.0125889500131663], rtol=0, atol=1e-14)
    # reseeds the global stream like the reference (side effect included)
    get_dW(5, 7)
    a = np.random.normal()
    np.random.seed(7)
    np.random.normal(0.0, 1.0, 5)
    assert a == np.random.normal()


def test_cli_calibrate_and_info():
    env = dict(os.environ, PYTHONPATH=ROOT)
    out = subprocess.run([sys.executable, "-m", "rphedge", "calibrate", "--synthetic"], capture_output=True,
                         text=True, cwd=ROOT, env=env, timeout=120)
    assert out.returncode == 0, out.stderr
    assert "vol0" in json.loads(out.stdout)
    out = subprocess.run([sys.executable, "-m", "rphedge", "info"], capture_output=True, text=True, cwd=ROOT,
                         env=env, timeout=120)
    assert out.returncode == 0 and json.loads(out.stdout)["native_loaded"]


def test_cli_run_config(tmp_path):
    cfg = dict(json.load(open(os.path.join(ROOT, "examples", "pension_mts.json"))), n_paths=8, dt=0.1,
               rebalancing=2.0, epochs_first=5, epochs_rest=2, device="cpu", verbose=False)
    p = tmp_path / "c.json"
    p.write_text(json.dumps(cfg))
    env = dict(os.environ, PYTHONPATH=ROOT)
    out = subprocess.run([sys.executable, "-m", "rphedge", "run", "--config", str(p), "--out", str(tmp_path / "o")],
                         capture_output=True, text=True, cwd=ROOT, env=env, timeout=300)
    assert out.returncode == 0, out.stderr
    res = json.loads(out.stdout)
    assert math.isfinite(res["phi0"]) and (tmp_path / "o" / "report.json").exists()


def test_reports():
    import rphedge
    from rphedge.utils import reports

    res = rphedge.european_option(N_paths=512, rebalancing_frequency=0.25, epochs_first=10, epochs_rest=3,
                                  verbose=False, device="cpu")
    v = reports.valuation_report(res, 0.08, 1.0)
    assert set(v) == {"V0", "discounted_E_payoff", "difference", "difference_pct"}
    h = reports.holdings_over_time(res)
    assert len(h) == 4
    fan = reports.value_fan(res.induction.values)
    assert fan.shape == (6, 5)
    cf = reports.pension_closed_form(10000, 100, 10, 0.03, 0.15, 0.8617)
    assert 8.5e5 < cf[0] < 1.0e6  # SURVEY: ~917,112 EUR


def test_report_figures(tmp_path):
    """C26-C32 figures (Agg backend): holdings violins, residual scatter/hist,
    value fan, trajectory/errors, sampled paths incl. lambda/N for the pension."""
    from rphedge import Replicating_Portfolio  # noqa: F401
    from rphedge.api import run_params
    from rphedge.utils import reports

    res = run_params(_small(), sv=False)
    files = reports.plot_run(res, out_prefix=str(tmp_path / "mts"))
    names = {os.path.basename(f) for f in files}
    for want in ("mts_holdings.png", "mts_residuals.png", "mts_value_fan.png", "mts_trajectory.png",
                 "mts_paths.png", "mts_lambda.png", "mts_survivors.png", "mts_terminal_hist.png"):
        assert want in names, (want, names)
    for f in files:
        assert os.path.getsize(f) > 1000


def test_resume_from_saved_date(tmp_path):
    """Checkpoint/resume: a run restarted at date i from the saved weights and
    values reproduces the dates < i of the uninterrupted run (CPU backend is
    deterministic)."""
    from rphedge.api import HedgeRun
    from rphedge.config import parse_params
    from rphedge.utils.model_io import save_run

    p = _small(rebalancing=2.0, shuffle=False, q99=False)
    run = HedgeRun(parse_params(p))
    full = run.run()
    save_run(str(tmp_path), run, full)
    i = 3
    run2 = HedgeRun(parse_params(p))
    res = run2.resume(str(tmp_path), i)
    assert [d.index for d in res.induction.dates] == list(range(i - 1, -1, -1))
    assert math.isfinite(res.phi) and math.isfinite(res.v0)
    assert res.v0 == pytest.approx(full.v0, rel=0.05)


def test_nan_gradient_guard_cpu():
    """Fault injection: a NaN target poisons the gradient -> the update is
    skipped and counted, weights stay finite."""
    from rphedge.engine import DateData, FitConfig, TorchBackend, TrainConfig, current_weights
    from rphedge.models.hedge_mlp import NetSpec, init_weights
    from rphedge.ops import layout as L

    spec = NetSpec(nin=1, hidden=8, nout=2, head=0)
    n = 1024
    x = torch.linspace(0.8, 1.2, n)
    y = torch.relu(x - 1)
    y[5] = float("nan")
    be = TorchBackend(spec, n, TrainConfig(batch_size=256, shuffle=False))
    w, o, f = be.new_weights(init_weights(spec, [0.5, 0.0])), be.new_opt(), be.new_fit()
    be.fit(w, o, f, DateData(feats=[x], prices_next=[x], bond_next=1.0, target=y, prices_now=[x]),
           FitConfig(epochs=3, patience=100, early_stopping=False), seed=1)
    assert np.all(np.isfinite(current_weights(spec, w)))
    assert float(o[L.O_NAN]) == 3.0   # one poisoned batch per epoch


def test_verbose_epoch_log(capsys):
    """verbose=2: Keras-style per-epoch loss lines for every fit (EO cell 13 log)."""
    from rphedge.api import run_params

    p = _small(verbose=2, epochs_first=4, epochs_rest=2, early_stopping=False)
    run_params(p)
    out = capsys.readouterr().out
    assert "Epoch 4/4 - loss:" in out and "mse]" in out and "q99]" in out
    assert "mae:" in out and "reduction =" in out


@pytest.mark.parametrize("mode", ["none", "global", "date"])
def test_feature_norm_modes_through_dict_api(mode):
    """`feature_norm` is a dict-API key; every mode runs end to end, parity
    forces raw inputs, and an unknown mode is rejected at build time."""
    from rphedge.api import HedgeRun
    from rphedge.config import parse_params

    run = HedgeRun(parse_params(_small(feature_norm=mode)))
    res = run.run()
    assert np.isfinite(res.phi) and np.isfinite(res.psi)
    assert (run.induction.norms == []) == (mode == "none")
    if mode == "global":
        assert all(n == run.induction.norms[0] for n in run.induction.norms)
    par = HedgeRun(parse_params(_small(feature_norm=mode, parity=True)))
    par.build()
    assert par.induction.norms == []
    with pytest.raises(ValueError):
        HedgeRun(parse_params(_small(feature_norm="bogus"))).build()


def test_phase_timer_does_not_leak():
    import gc

    from rphedge.utils import profiling

    gc.collect()
    n0 = profiling.live_timers()
    for _ in range(20):
        t = profiling.PhaseTimer(enabled=True, device="cpu")
        with t.phase("x"):
            pass
    del t
    gc.collect()
    assert profiling.live_timers() == n0


def test_cli_lm_example_config(tmp_path):
    """examples/euro_call_30_lm.json (full-batch Levenberg-Marquardt fits)
    through the CLI on the CPU oracle, at a reduced size."""
    cfg = dict(json.load(open(os.path.join(ROOT, "examples", "euro_call_30_lm.json"))), n_paths=11,
               rebalancing=0.25, dt=0.25, batch_size=2048, lm_passes_first=20, lm_passes_rest=2, device="cpu",
               verbose=False)
    p = tmp_path / "c.json"
    p.write_text(json.dumps(cfg))
    env = dict(os.environ, PYTHONPATH=ROOT)
    out = subprocess.run([sys.executable, "-m", "rphedge", "run", "--config", str(p)], capture_output=True, text=True,
                         cwd=ROOT, env=env, timeout=300)
    assert out.returncode == 0, out.stderr
    res = json.loads(out.stdout)
    assert abs(res["V0"] - 10.3896) < 0.6, res
