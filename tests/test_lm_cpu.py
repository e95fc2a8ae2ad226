"""Levenberg-Marquardt fits (engine.FitConfig.optimizer = "lm"): reference
semantics on the torch backend (the oracle of the HIP kernels in
test_gpu_lm.py) and end-to-end quality vs Keras-Adam."""
import math

import numpy as np
import pytest
import torch


def _teacher_problem(spec, n, seed=0):
    from rphedge.models.hedge_mlp import init_weights, torch_forward

    g = torch.Generator().manual_seed(seed)
    x = torch.rand(n, spec.nin, generator=g) * 2 - 1
    pr = [1.0 + 0.1 * torch.randn(n, generator=g) for _ in range(spec.nhold - 1)]
    wt = torch.tensor(init_weights(spec, [0.3] * spec.nout, seed=99), dtype=torch.float32) * 3
    P = torch.stack(pr + [torch.full((n,), 1.01)], 1)
    y = (torch_forward(spec, wt, x) * P).sum(1)
    return [x[:, f].contiguous() for f in range(spec.nin)], pr, y


@pytest.mark.parametrize("shape", [(1, 8, 2, 0), (3, 8, 2, 0)])
def test_lm_recovers_teacher_network(shape):
    """Same-architecture teacher -> student: LM drives the MSE down by four
    orders of magnitude in 60 passes; the best loss never increases."""
    from rphedge.engine import DateData, FitConfig, TorchBackend, TrainConfig
    from rphedge.models.hedge_mlp import NetSpec, init_weights

    spec = NetSpec(*shape)
    n = 1 << 12
    feats, pr, y = _teacher_problem(spec, n)
    data = DateData(feats=feats, prices_next=pr, bond_next=1.01, target=y, prices_now=pr)
    be = TorchBackend(spec, n, TrainConfig(batch_size=n, shuffle=False, lm_gram_paths=1024))
    w, o, f = be.new_weights(init_weights(spec, [0.5] * spec.nout, seed=1)), be.new_opt(), be.new_fit()
    be.fit(w, o, f, data, FitConfig(epochs=60, optimizer="lm", early_stopping=False), seed=0)
    hist = be.lm_last["hist"]
    assert min(hist) < 1e-4 * hist[0], hist[-5:]
    assert all(b <= a for a, b in zip(np.minimum.accumulate(hist)[:-1], np.minimum.accumulate(hist)[1:]))
    assert float(f[2048 + 12]) == pytest.approx(min(hist), rel=1e-6)   # F_LAST_LOSS = best loss


def test_lm_diag_floor_escapes_degenerate_subsample_curvature():
    """A 2048-path Gram subsample of the 1-8-8-2 teacher problem gives one
    parameter (almost) no curvature: with plain Marquardt scaling its step
    never shrinks, every trial is rejected and the damping runs to lam_max
    (the fit stalls at 2.6e-3 of the start loss); the damping floor
    (TrainConfig.lm_diag_floor) makes growing damping shorten every step."""
    from rphedge.engine import DateData, FitConfig, TorchBackend, TrainConfig
    from rphedge.models.hedge_mlp import NetSpec, init_weights

    spec = NetSpec(1, 8, 2, 0)
    n = 1 << 12
    feats, pr, y = _teacher_problem(spec, n)
    data = DateData(feats=feats, prices_next=pr, bond_next=1.01, target=y, prices_now=pr)
    out = {}
    for floor in (0.0, 1e-6):
        be = TorchBackend(spec, n, TrainConfig(batch_size=n, shuffle=False, lm_gram_paths=2048, lm_diag_floor=floor))
        w, o, f = be.new_weights(init_weights(spec, [0.5] * spec.nout, seed=1)), be.new_opt(), be.new_fit()
        be.fit(w, o, f, data, FitConfig(epochs=60, optimizer="lm", early_stopping=False), seed=0)
        out[floor] = (min(be.lm_last["hist"]) / be.lm_last["hist"][0], be.lm_last["lam"])
    assert out[0.0][0] > 1e-3 and out[0.0][1] >= 1e9          # stalled at the damping ceiling
    assert out[1e-6][0] < 1e-6                                 # converges with the floor


def test_lm_adaptive_budget_stops_early_and_equals_fixed_budget():
    """lm_stop_tol: from pass lm_stop_min on, the first ACCEPTED pass that
    lowers the best loss by less than the tolerance ends the fit (rejections
    never stop it).  The stopped fit is the fixed-budget fit of that many
    passes (same weights, same history)."""
    from rphedge.engine import DateData, FitConfig, TorchBackend, TrainConfig
    from rphedge.models.hedge_mlp import NetSpec, init_weights
    from rphedge.ops import layout as L

    spec = NetSpec(1, 8, 2, 0)
    n = 1 << 11
    feats, pr, y = _teacher_problem(spec, n)
    data = DateData(feats=feats, prices_next=pr, bond_next=1.01, target=y, prices_now=pr)
    w0 = init_weights(spec, [0.5] * spec.nout, seed=1)

    def run(**kw):
        be = TorchBackend(spec, n, TrainConfig(batch_size=n, shuffle=False, lm_gram_paths=1024))
        w, o, f = be.new_weights(w0), be.new_opt(), be.new_fit()
        be.fit(w, o, f, data, FitConfig(optimizer="lm", early_stopping=False, **kw), seed=0)
        return w.clone(), f.clone(), be.lm_last["hist"]

    w_s, f_s, h_s = run(epochs=60, lm_stop_tol=0.05, lm_stop_min=3)
    k = len(h_s) - 1                      # passes run
    assert 3 <= k < 60
    # the stopping pass was accepted and gained < 5 %; every earlier accepted
    # pass from lm_stop_min on gained more
    best = np.minimum.accumulate(h_s)
    assert h_s[k] < best[k - 1] and not (best[k - 1] - best[k] > 0.05 * best[k])
    assert all(best[j - 1] - best[j] > np.float32(0.05) * best[j] for j in range(3, k) if h_s[j] < best[j - 1])
    w_f, f_f, h_f = run(epochs=k)
    assert h_f == h_s
    assert torch.equal(w_s, w_f)
    assert int(f_s[L.F_EPOCH]) == k + 1


def test_lm_pinball_fit_reaches_the_conditional_quantile():
    """Pinball (Q99) LM fit (IRLS Gauss-Newton: Gram weighted by 1 / (2 max(|r|,
    delta)), exact pinball loss in the accept test; the reference's second fit,
    Replicating_Portfolio.py:138-145, :217): teacher values + N(0, 0.05^2)
    noise, so the 99 % conditional quantile is the teacher shifted by
    2.326 x 0.05 in the bond holding.  From the MSE-fitted net the fit
    reaches the quantile's loss and ~1 % of the targets lie above it; the best
    loss never increases."""
    from rphedge.engine import DateData, FitConfig, TorchBackend, TrainConfig
    from rphedge.models.hedge_mlp import NetSpec, init_weights, torch_forward
    from rphedge.ops import layout as L

    spec = NetSpec(1, 8, 2, 0)
    n = 1 << 13
    feats, pr, y0 = _teacher_problem(spec, n)
    g = torch.Generator().manual_seed(5)
    y = y0 + 0.05 * torch.randn(n, generator=g)
    data = DateData(feats=feats, prices_next=pr, bond_next=1.01, target=y, prices_now=pr)
    be = TorchBackend(spec, n, TrainConfig(batch_size=n, shuffle=False, lm_gram_paths=2048))
    w, o, f = be.new_weights(init_weights(spec, [0.5] * spec.nout, seed=1)), be.new_opt(), be.new_fit()
    be.fit(w, o, f, data, FitConfig(epochs=40, optimizer="lm", early_stopping=False), seed=0)  # MSE start point
    be.fit(w, o, f, data, FitConfig(epochs=40, optimizer="lm", loss=L.LOSS_PINBALL, quantile=0.99,
                                    early_stopping=False, lm_q_delta=1e-4), seed=0)
    hist = be.lm_last["hist"]
    assert all(b <= a for a, b in zip(np.minimum.accumulate(hist)[:-1], np.minimum.accumulate(hist)[1:]))
    X = torch.stack(feats, 1)
    P = torch.stack(pr + [torch.full((n,), 1.01)], 1)
    V = (torch_forward(spec, w[:spec.nparams], X) * P).sum(1)
    above = float((y > V).double().mean())
    assert 0.004 < above < 0.02, above

    def pinball(v):
        e = (y - v).double()
        return float(torch.maximum(0.99 * e, -0.01 * e).mean())

    l_q = pinball(y0 + 2.326 * 0.05)  # the true conditional quantile
    assert pinball(V) < 1.05 * l_q, (pinball(V), l_q)
    assert float(f[L.F_BEST]) == pytest.approx(pinball(V), rel=1e-4)


def test_lm_induction_beats_adam_on_cpu():
    """30-date European call on 2^13 paths: LM (60 / 3 passes) reaches the
    least-squares hedge: one-step residual and self-financing P&L well below
    the Adam fit at a comparable budget, V0 near Black-Scholes."""
    from rphedge.api import european_option

    kw = dict(N_paths=1 << 13, dt=1 / 30, rebalancing_frequency=1 / 30, epochs_first=100, epochs_rest=8,
              batch_size=2048, lr=5e-2, lr_rest=4e-3, lr_decay=0.1, lr_schedule_first=False, verbose=False,
              device="cpu", early_stopping=False, q99=False, chunk_log2=6, lm_passes_first=60, lm_passes_rest=3)
    a = european_option(optimizer="adam", **kw)
    m = european_option(optimizer="lm", **kw)
    assert abs(m.v0 - 10.3896) < 0.25
    assert m.terminal_residual["std"] < 0.5 and m.terminal_residual["std"] < 0.6 * a.terminal_residual["std"]
    assert m.terminal_pnl["std"] < 1.1 and m.terminal_pnl["std"] < 0.6 * a.terminal_pnl["std"]
    assert m.induction.dates[0].fit_mse["epochs"] == 61


@pytest.mark.parametrize("shape", [(1, 8, 2, 0), (3, 8, 2, 0)])
def test_bias_refit_zeroes_mean_residual(shape):
    """engine bias_refit (after an Adam fit): the bond holding's output bias
    moves by -mean(e) / B, the full-batch residual mean becomes zero and the
    loss can only drop (exact 1-D least squares); complement heads untouched."""
    from rphedge.engine import DateData, FitConfig, TorchBackend, TrainConfig
    from rphedge.models.hedge_mlp import NetSpec, init_weights, torch_forward
    from rphedge.ops import layout as L

    spec = NetSpec(*shape)
    n = 1 << 11
    feats, pr, y = _teacher_problem(spec, n)
    y = y + 0.05   # a mean offset the Adam fit below does not remove
    data = DateData(feats=feats, prices_next=pr, bond_next=1.01, target=y, prices_now=pr)
    be = TorchBackend(spec, n, TrainConfig(batch_size=256))
    w, o, f = be.new_weights(init_weights(spec, [0.5] * spec.nout, seed=1)), be.new_opt(), be.new_fit()
    fc = FitConfig(epochs=3, early_stopping=False)
    be.fit(w, o, f, data, fc, seed=0)

    def resid(wv):
        X = torch.stack(feats, 1).double()
        P = torch.stack(pr + [torch.full((n,), 1.01)], 1).double()
        return (torch_forward(spec, wv.double(), X) * P).sum(1) - y.double()

    cur = int(w[L.W_CUR].item())
    e0 = resid(w[cur * L.PMAX: cur * L.PMAX + spec.nparams])
    be.bias_refit(w, o, f, data, fc)
    e1 = resid(w[cur * L.PMAX: cur * L.PMAX + spec.nparams])
    assert abs(float(e0.mean())) > 1e-3
    assert abs(float(e1.mean())) < 1e-5
    assert float((e1 ** 2).mean()) <= float((e0 ** 2).mean())
    assert torch.allclose(e1, e0 - e0.mean(), atol=1e-5)

    eo = NetSpec(1, 8, 1, L.HEAD_COMPLEMENT)
    be2 = TorchBackend(eo, n, TrainConfig(batch_size=256))
    w2 = be2.new_weights(init_weights(eo, [0.5], seed=1))
    before = w2.clone()
    be2.bias_refit(w2, be2.new_opt(), be2.new_fit(), DateData(feats=feats[:1], prices_next=pr[:1], bond_next=1.01,
                                                              target=y, prices_now=pr[:1]), fc)
    assert torch.equal(w2, before)


def test_mean_refit_keeps_v0_on_price_cpu():
    """30-date European call through the API with Adam fits: mean_refit (the
    corrected default) puts V0 on the paths' discounted MC payoff; the parity
    flag keras_fit_only switches it off."""
    from rphedge.api import run_params

    base = dict(Y=100, K=100, T=1.0, mu=0.08, r=0.08, sigma=0.15, N=1, P=1, x=0, l0=0, c=0, ita=0,
                mortality=False, q99=False, dt=1 / 12, rebalancing=1 / 12, n_paths=12, payoff="call",
                option_type="CALL", model="gbm_log", batch_size=1 << 10, epochs_first=30, epochs_rest=4,
                lr=1e-2, lr_schedule_first=False, early_stopping=False, verbose=False, device="cpu")
    on = run_params(base)
    off = run_params(dict(base, mean_refit=False))
    mc = on.summary["E_payoff"] * on.scale * math.exp(-0.08)
    assert abs(on.v0 / mc - 1) < 2e-3, (on.v0, mc)
    assert abs(on.v0 - off.v0) > 1e-4   # the refit is active in the default run


def test_pension_lm_preset_cpu():
    """experiments.mts_lm_parameters (both fits of every date on LM, the Q99
    fits as IRLS Gauss-Newton warm-started from the previous date's Q99 net)
    through the API on the torch oracle, shrunk to 10 annual dates and 2^10
    paths: finite results in the range of the Adam runs and every pinball fit
    lowers its loss."""
    from rphedge import experiments
    from rphedge.api import run_params

    p = experiments.mts_lm_parameters(n_paths=10, dt=0.1, rebalancing=1.0, device="cpu", verbose=False, lm_starts=4,
                                      lm_explore_passes=10, lm_explore_log2=9, lm_passes_first=20,
                                      lm_q_passes_first=30, lm_q_passes_rest=5)
    r = run_params(p)
    assert 0.8e6 < r.v0 < 1.2e6 and 0.3e6 < r.phi < 0.9e6 and 0.0 < r.psi < 0.6e6, (r.v0, r.phi, r.psi)
    for d in r.induction.dates:
        h = d.fit_q99["history"]
        assert len(h) > 1 and math.isfinite(d.fit_q99["best_loss"]) and d.fit_q99["best_loss"] <= h[0]


def test_lm_pass_grid_sizes():
    """LM pass grid (engine.lm_pass_wgs / lm_pass_schedule): one workgroup per
    CU (256), or two (512) for the bodies that fit twice (native.lm_pass_wps),
    at most one per 256 local paths; contiguous leaves keep 4 per workgroup,
    a power-of-two workgroup count and whole leaves per shard."""
    import pytest

    from rphedge.engine import lm_pass_schedule, lm_pass_wgs

    assert lm_pass_wgs(1 << 20) == 256 and lm_pass_wgs(1 << 20, 2) == 512
    assert lm_pass_wgs(1 << 16, 2) == 256 and lm_pass_wgs(1 << 10, 2) == 4 and lm_pass_wgs(100, 2) == 1
    assert lm_pass_wgs(1 << 20, 4) == 512  # (capped at LM_PASS_WGS_MAX)
    assert lm_pass_schedule(1 << 20, -1, 2) == (512, 0)       # cyclic
    assert lm_pass_schedule(1 << 20, 0, 2) == (512, 4)        # auto leaves: 512 paths
    assert lm_pass_schedule(1 << 20, 1024, 2) == (256, 8)     # fixed leaves: 1024 paths
    assert lm_pass_schedule(1 << 20, 512, 2) == (512, 4)
    assert lm_pass_schedule(1 << 19, 256, 2) == (512, 2)
    with pytest.raises(ValueError):
        lm_pass_schedule(1 << 20, 256, 2)  # 1024 workgroups needed
    with pytest.raises(ValueError):
        lm_pass_schedule(1 << 20, 256, 1)
    with pytest.raises(ValueError):
        lm_pass_schedule(3 * (1 << 16), 1024, 2)  # 48 workgroups: not a power of two
