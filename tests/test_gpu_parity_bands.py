"""Published reference numbers pinned by multi-seed bands (GPU, parity mode).

Every reference headline is ONE TensorFlow run (one random init, one shuffle
order), so the honest band is the scatter over training seeds of the same
configuration: the published value must lie within 3 seed standard deviations
of our multi-seed mean, and the scatter itself is bounded (so a broken run
cannot widen its own band).  Measured scatter (profiles/r3/parity_seed_bands_r3b.jsonl,
relative seed standard deviation): headline V0 2.5 %, phi0 / psi0 4.2 / 11.0 %;
RP module 4.0 / 12.1 % (sum 1.1 %); SV 2.5 / 6.5 % (sum 1.0 %); single time
step 0.4 / 2.3 %.  Each scatter cap sits just above its measurement (the runs
are deterministic per seed), so a regression that widens the seed scatter
fails the test instead of widening the band.

Sources: "Multi Time Step.ipynb":1039 / :987-988 (headline), :1329-1351 (RP
module, 634,349 / 350,176), :2384-2385 (sigma sweep), :2612-2639 (SV,
626,123 / 371,854); "Single Time Step.ipynb" (819,539 / 257,308).
"""
import json
import math
import os

import numpy as np
import pytest

pytestmark = pytest.mark.gpu

OUT = os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "gpurun_out")
SEEDS = [1234 + k for k in range(6)]


def _record(name, payload):
    os.makedirs(OUT, exist_ok=True)
    with open(os.path.join(OUT, "parity_seed_bands.jsonl"), "a") as f:
        f.write(json.dumps({"test": name, **payload}, default=float) + "\n")


def _band(values, published, k=3.0, max_rel_scatter=0.12, rel_floor=0.01):
    v = np.asarray(values, dtype=np.float64)
    mean, sd = float(v.mean()), float(v.std(ddof=1))
    assert sd <= max_rel_scatter * abs(mean), (mean, sd)
    assert abs(mean - published) <= k * sd + rel_floor * abs(published), (mean, sd, published)
    return mean, sd


def _robust_band(values, published, k=3.0, max_rel_scatter=0.02, rel_floor=0.01):
    """_band on the median and the MAD scale (1.4826 MAD): one diverged seed
    (the reference's Adam + early-stopping fits on 4,096 paths occasionally
    land a run several % off) neither widens nor shifts the band."""
    v = np.asarray(values, dtype=np.float64)
    med = float(np.median(v))
    sd = 1.4826 * float(np.median(np.abs(v - med)))
    assert sd <= max_rel_scatter * abs(med), (med, sd)
    assert abs(med - published) <= k * sd + rel_floor * abs(published), (med, sd, published)
    return med, sd


def test_mts_notebook_headline_seed_band():
    """The "Multi Time Step.ipynb" headline run (Q15 paths, dt = 1/365, 4096
    paths, shared Q99 model): V0 981,038.213, phi0 / psi0 643,687 / 350,888."""
    from rphedge.experiments import MTS_NOTEBOOK_PUBLISHED as PUB
    from rphedge.experiments import mts_notebook

    runs = [mts_notebook(verbose=False, poll_every=10, seed=s) for s in SEEDS + [1240, 1241]]
    v0, phi, psi = ([r[k] for r in runs] for k in ("V0", "phi0", "psi0"))
    _record("mts_notebook", {"V0": v0, "phi0": phi, "psi0": psi, "VaR": [r.get("VaR") for r in runs],
                             "published": PUB})
    assert abs(np.mean(v0) / PUB["V0"] - 1) < 0.015, np.mean(v0)
    _band(v0, PUB["V0"], max_rel_scatter=0.035)
    _band(phi, PUB["phi0"], max_rel_scatter=0.06)
    _band(psi, PUB["psi0"], max_rel_scatter=0.115)
    # the published (phi0, psi0) pair as one draw of the seed distribution:
    # squared Mahalanobis distance under the 8-seed covariance within the 99 %
    # chi-square(2) quantile (GPU: 1.56, z = -1.19 / +1.02; the CPU oracle's
    # 13-variant sweep puts the reference semantics at 1.7,
    # profiles/r5/mts_variants_cpu_8seeds.jsonl: the split is seed scatter of
    # an early-stopped Adam endpoint, psi0 sd 11 % of its mean)
    d = np.array([PUB["phi0"] - np.mean(phi), PUB["psi0"] - np.mean(psi)])
    md2 = float(d @ np.linalg.solve(np.cov(np.vstack([phi, psi])), d))
    assert md2 <= 9.21, md2
    # the total t = 0 hedge value phi0 + psi0 is far tighter than its split
    # (8 seeds: 7 within 3 % of each other, seed 1235 +6.7 %: robust band)
    _robust_band(np.add(phi, psi), PUB["phi0"] + PUB["psi0"], max_rel_scatter=0.02)
    # overall residual VaR 98.5 / 99 / 99.5 % (":954-956"; EUR, near zero, so
    # the scatter bound is absolute: 0.1 % of N P = 1,000 EUR)
    var = np.asarray([r["VaR"] for r in runs], dtype=np.float64)
    for k, pub in enumerate(PUB["VaR"]):
        mean, sd = float(var[:, k].mean()), float(var[:, k].std(ddof=1))
        assert sd <= 1_000.0, (k, mean, sd)
        assert abs(mean - pub) <= 3.0 * sd + 50.0, (k, mean, sd, pub)


def test_pension_rp_module_seed_band():
    """RP-module run of the pension (dt = 1/100, quarterly, 4096 paths):
    phi0 / psi0 = 634,349 / 350,176."""
    from rphedge.api import run_params
    from rphedge.experiments import mts_parameters

    res = [run_params(mts_parameters(verbose=False, parity=True, poll_every=10, seed=s)) for s in SEEDS]
    phi, psi = [r.phi for r in res], [r.psi for r in res]
    _record("pension_rp", {"phi0": phi, "psi0": psi, "V0": [r.v0 for r in res]})
    _band(phi, 634_349.0, max_rel_scatter=0.06)
    _band(psi, 350_176.0, max_rel_scatter=0.135)
    _band(np.add(phi, psi), 634_349.0 + 350_176.0, max_rel_scatter=0.02)


def test_sv_seed_band():
    """Replicating_Portfolio_SV with the notebook dict (Q4): 626,123 / 371,854."""
    from rphedge.api import Replicating_Portfolio_SV
    from rphedge.experiments import sv_parameters

    out = [Replicating_Portfolio_SV(sv_parameters(verbose=False, parity=True, poll_every=10, seed=s)) for s in SEEDS]
    phi, psi = [o[0] for o in out], [o[1] for o in out]
    _record("sv", {"phi0": phi, "psi0": psi})
    _band(phi, 626_123.0, max_rel_scatter=0.04)
    _band(psi, 371_854.0, max_rel_scatter=0.08)
    _band(np.add(phi, psi), 626_123.0 + 371_854.0, max_rel_scatter=0.02)


def test_single_time_step_seed_band():
    """"Single Time Step.ipynb": phi0 / psi0 = 819,539 / 257,308."""
    from rphedge.experiments import single_time_step

    out = [single_time_step(parity=True, verbose=False, seed=s) for s in SEEDS]
    phi, psi = [o["phi0"] for o in out], [o["psi0"] for o in out]
    _record("sts", {"phi0": phi, "psi0": psi, "VaR_Res1": [o["VaR_Res1"] for o in out]})
    _band(phi, 819_539.0, max_rel_scatter=0.01)
    _band(psi, 257_308.0, max_rel_scatter=0.04)


SWEEP_PUB = {0.05: (896_236.240864, 14_488.995075), 0.10: (892_169.296741, 18_210.105598),
             0.15: (635_912.120342, 331_816.464663), 0.20: (574_618.518353, 479_856.312275),
             0.30: (687_849.521637, 534_581.005573)}


def test_sigma_sweep_parity_seed_band():
    """sigma sweep ("Multi Time Step.ipynb":2384-2385) in parity mode: Phi and
    Phi + Psi per sigma within the seed band (Psi too where it is not ~0).  The
    round-1 drift (sigma = 0.05: 847k vs 896k) came from running the sweep in
    the corrected mode (separate Q99 network, normalised features), not the
    reference's shared-model semantics."""
    from rphedge.experiments import volatility_sweep

    rows = np.array([[[r["sigma"], r["Phi"], r["Psi"], r["sum"]]
                      for r in volatility_sweep(parity=True, seed=s, verbose=False, poll_every=10)] for s in SEEDS])
    _record("sigma_sweep_parity", {"rows": rows.tolist()})
    for j in range(rows.shape[1]):
        sig = round(float(rows[0, j, 0]), 2)
        ph, ps = SWEEP_PUB[sig]
        _band(rows[:, j, 1], ph, max_rel_scatter=0.06)
        _band(rows[:, j, 3], ph + ps, max_rel_scatter=0.05)
        if ps > 1e5:
            _band(rows[:, j, 2], ps, max_rel_scatter=0.15)
    assert math.isfinite(float(rows.sum()))


def test_corrected_pension_matches_closed_form():
    """Corrected semantics, pure MSE hedge (no capital-charge blend, no Q99
    fit), LM fits: V0 against the closed form of SURVEY §6.1 (N·P·max(1, Y_T)
    under Q with independent mortality ≈ 917,112 EUR).  Measured 909,987 ±
    3,625 over 4 seeds at 4096 paths (profiles/r2/pension_corrected_vs_closed_form.jsonl)."""
    from rphedge.api import run_params
    from rphedge.experiments import mts_parameters

    v0 = [run_params(mts_parameters(verbose=False, poll_every=10, seed=s, optimizer="lm", cost_of_capital=0.0,
                                    q99=False)).v0 for s in SEEDS[:4]]
    _record("pension_corrected_mse", {"V0": v0})
    assert abs(np.mean(v0) / 917_112.0 - 1) < 0.02, v0
    assert np.std(v0) < 0.01 * np.mean(v0)
