"""GPU numerics: every HIP kernel vs a plain fp32/fp64 PyTorch/numpy reference."""
import math

import numpy as np
import pytest
import torch

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def dev():
    from rphedge.ops import native

    native.load(required=True)
    return torch.device("cuda", 0)


def test_native_is_loaded(dev):
    from rphedge.ops import native

    assert native._lib is not None
    info = native.device_info(0)
    assert info["cus"] > 0
    assert info["arch"].startswith("gfx9")


@pytest.mark.parametrize("d,m,seed", [(7, 10, 1235), (31, 12, 1234), (3, 8, 42)])
def test_sobol_fp64_matches_scipy(dev, d, m, seed):
    from scipy.stats import norm, qmc

    from rphedge.ops.sobol import sobol_norm

    ref = norm.ppf(qmc.Sobol(d, scramble=True, seed=seed).random_base2(m))
    got = sobol_norm(m, d, seed, device=dev, dtype=torch.float64).cpu().numpy()
    fin = np.isfinite(ref)
    assert np.array_equal(fin, np.isfinite(got))
    np.testing.assert_allclose(got[fin], ref[fin], rtol=1e-12, atol=1e-13)


def test_sobol_raw_bit_exact(dev):
    from scipy.stats import qmc

    from rphedge.ops import native
    from rphedge.ops.sobol import device_table

    d, m, seed = 9, 11, 1235
    ref = qmc.Sobol(d, scramble=True, seed=seed).random_base2(m)
    out = torch.empty(2 ** m, d, dtype=torch.float64, device=dev)
    native.sobol_normal(out, device_table(d, seed, dev), raw=True)
    assert np.array_equal(out.cpu().numpy(), ref)


def test_sobol_fp32_accuracy(dev):
    from scipy.stats import norm, qmc

    from rphedge.ops.sobol import sobol_norm

    d, m = 5, 14
    ref = norm.ppf(qmc.Sobol(d, scramble=True, seed=1235).random_base2(m))
    got = sobol_norm(m, d, 1235, device=dev, dtype=torch.float32).cpu().numpy().astype(np.float64)
    core = np.abs(ref) < 5
    np.testing.assert_allclose(got[core], ref[core], rtol=2e-6, atol=2e-6)
    assert np.max(np.abs(got[~core & np.isfinite(ref)] - ref[~core & np.isfinite(ref)]), initial=0) < 1e-3


@pytest.mark.parametrize("scheme", ["arith", "log"])
def test_gbm_paths_vs_numpy(dev, scheme):
    from rphedge.ops import paths as P

    g = P.Grid(T=1.0, dt=1 / 100, rebalancing=1 / 20)
    n = 4096
    gp = P.simulate_gbm(g, n, 1.0, 0.08, 0.15, scheme=scheme, device=dev, fp64=True)
    cp = P.simulate_gbm(g, n, 1.0, 0.08, 0.15, scheme=scheme, device="cpu")
    torch.cuda.synchronize()
    np.testing.assert_allclose(gp.S.cpu().numpy(), cp.S.numpy(), rtol=2e-6)
    np.testing.assert_allclose(gp.S_final.cpu().numpy(), cp.S_final.numpy(), rtol=2e-6)
    g32 = P.simulate_gbm(g, n, 1.0, 0.08, 0.15, scheme=scheme, device=dev, fp64=False)
    np.testing.assert_allclose(g32.S.cpu().numpy(), cp.S.numpy(), rtol=5e-5)


def test_gbm_offset_shard_consistency(dev):
    """Sharded generation (DP) reproduces the same global path set."""
    from rphedge.ops import paths as P

    g = P.Grid(T=1.0, dt=1 / 30, rebalancing=1 / 30)
    full = P.simulate_gbm(g, 8192, 100.0, 0.08, 0.15, scheme="log", norm=100.0, device=dev)
    a = P.simulate_gbm(g, 4096, 100.0, 0.08, 0.15, scheme="log", norm=100.0, device=dev, offset=0)
    b = P.simulate_gbm(g, 4096, 100.0, 0.08, 0.15, scheme="log", norm=100.0, device=dev, offset=4096)
    torch.testing.assert_close(torch.cat([a.S, b.S], 1), full.S)


def test_gbm_moments(dev):
    from rphedge.ops import paths as P

    g = P.Grid(T=1.0, dt=1 / 30, rebalancing=1 / 30)
    p = P.simulate_gbm(g, 1 << 20, 100.0, 0.08, 0.15, scheme="log", norm=100.0, device=dev)
    m = float(p.S_final.double().mean()) * 100
    assert abs(m - 100 * math.exp(0.08)) < 0.02


def test_sv_and_heston_vs_numpy(dev):
    from rphedge.ops import paths as P

    g = P.Grid(T=2.0, dt=1 / 50, rebalancing=0.25)
    for model, kw in [("sv_ref", dict(a=0.0034, b=0.154, c=0.0158)),
                      ("sv_ref", dict(a=0.0034, b=0.154, c=0.0158, sv_tscale=252.0)),
                      ("heston", dict(kappa=2.0, theta=0.04, xi=0.3, rho=-0.7, scheme="euler")),
                      ("heston", dict(kappa=2.0, theta=0.04, xi=0.3, rho=-0.7, scheme="qe")),
                      ("heston", dict(kappa=1.0, theta=0.04, xi=0.9, rho=-0.5, scheme="qe"))]:  # QE exp. branch
        gp = P.simulate_sv(g, 2048, 1.0, 0.09, 0.16 if model == "sv_ref" else 0.04, model=model, device=dev,
                           fp64=True, **kw)
        cp = P.simulate_sv(g, 2048, 1.0, 0.09, 0.16 if model == "sv_ref" else 0.04, model=model, device="cpu",
                           **kw)
        np.testing.assert_allclose(gp.S.cpu().numpy(), cp.S.numpy(), rtol=1e-5, atol=1e-6)
        np.testing.assert_allclose(gp.vol.cpu().numpy(), cp.vol.numpy(), rtol=1e-5, atol=1e-6)


def test_heston_qe_price_matches_semi_analytic(dev):
    """BASELINE config #3 quality anchor: the heston30 paths (30 dates x 10
    substeps, 2^20 Sobol paths, fp32, Andersen QE) price the call within 3
    standard errors of the semi-closed-form Heston price 10.1546 (full-
    truncation Euler sat 1.3 % above it)."""
    from rphedge.analytic import heston_call
    from rphedge.ops import paths as P

    g = P.Grid(T=1.0, dt=1 / 300, rebalancing=1 / 30)
    kw = dict(kappa=2.0, theta=0.04, xi=0.5, rho=-0.7)
    ref, _ = heston_call(100.0, 100.0, 0.05, 1.0, kw["kappa"], kw["theta"], kw["xi"], kw["rho"], 0.04)
    p = P.simulate_sv(g, 1 << 20, 100.0, 0.05, 0.04, model="heston", norm=100.0, device=dev, scheme="qe", **kw)
    pay = (p.S_final.double() * 100.0 - 100.0).clamp_min(0.0) * math.exp(-0.05)
    se = float(pay.std()) / math.sqrt(pay.numel())
    assert abs(float(pay.mean()) - ref) < 3 * se, (float(pay.mean()), ref, se)
    assert abs(ref - 10.1546) < 1e-3


def test_basket_vs_numpy(dev):
    from rphedge.ops import paths as P

    g = P.Grid(T=1.0, dt=1 / 20, rebalancing=1 / 10)
    na = 5
    corr = np.full((na, na), 0.5) + np.eye(na) * 0.5
    gp = P.simulate_basket(g, 2048, [100.0] * na, [0.05] * na, [0.2] * na, corr, device=dev)
    cp = P.simulate_basket(g, 2048, [100.0] * na, [0.05] * na, [0.2] * na, corr, device="cpu")
    np.testing.assert_allclose(gp.S.cpu().numpy(), cp.S.numpy(), rtol=2e-4)


def test_mortality_statistics(dev):
    from rphedge.ops import paths as P

    g = P.Grid(T=10.0, dt=1 / 100, rebalancing=0.25)
    p = P.simulate_gbm(g, 8192, 1.0, 0.08, 0.15, device=dev)
    P.simulate_mortality(p, 0.01, 0.075, 0.000597, 10000)
    cp = P.simulate_gbm(g, 2048, 1.0, 0.08, 0.15, device="cpu")
    P.simulate_mortality(cp, 0.01, 0.075, 0.000597, 10000)
    # lambda is deterministic given the Sobol draws
    np.testing.assert_allclose(p.lam[:, :2048].cpu().numpy(), cp.lam.numpy(), rtol=1e-5)
    nT = p.nfrac_final.double().cpu().numpy() * 10000
    # SURVEY: E[N_T] = 8615-8617, std 132-133
    assert abs(nT.mean() - 8616) < 15
    assert 110 < nT.std() < 160


def _fit_pair(dev, spec, n, batch, epochs, loss, chunk_log2=0, lr=1e-2, norm=None, **tkw):
    from rphedge.engine import DateData, FitConfig, HipBackend, TorchBackend, TrainConfig, current_weights
    from rphedge.models.hedge_mlp import init_weights
    from rphedge.ops import layout as L

    g = torch.Generator().manual_seed(0)
    feats = [torch.rand(n, generator=g) * 0.5 + 0.75 for _ in range(spec.nin)]
    prices = [f.clone() * (1 + 0.05 * torch.randn(n, generator=g)) for f in feats[: spec.nhold - 1]]
    target = torch.relu(prices[0] - 1.0) if spec.nhold > 1 else torch.rand(n)
    w0 = init_weights(spec, ([0.5] + [-0.4] * (spec.nout - 1)) if spec.head == 0 else [0.1])
    tc = TrainConfig(batch_size=batch, chunk_log2=chunk_log2, lr=lr, **tkw)
    fc = FitConfig(epochs=epochs, patience=1000, loss=loss, early_stopping=False)
    out = []
    for be_cls, d in ((TorchBackend, torch.device("cpu")), (HipBackend, dev)):
        be = be_cls(spec, n, tc, device=d)
        data = DateData(feats=[f.to(d) for f in feats], prices_next=[p.to(d) for p in prices], bond_next=1.02,
                        target=target.to(d), prices_now=[f.to(d) for f in feats[: spec.nhold - 1]], bond_now=1.0)
        if norm is not None:
            data.fmu, data.fisd = norm(spec.nin)
        w, o, f = be.new_weights(w0), be.new_opt(), be.new_fit()
        be.fit(w, o, f, data, fc, seed=7)
        st = be.new_stats()
        vo = torch.empty(n, device=d)
        ro = torch.empty(n, device=d)
        be.eval(w, data, st, v_out=vo, resid_out=ro)
        if d.type == "cuda":
            torch.cuda.synchronize()
        out.append((current_weights(spec, w), o.cpu().numpy(), f.cpu().numpy(), vo.cpu().numpy(), ro.cpu().numpy(),
                    st.sum(0).cpu().numpy()))
    return out


@pytest.mark.parametrize("mode", ["lag", "ticket", "persistent"])
@pytest.mark.parametrize("shape", [(1, 8, 2, 0), (3, 8, 2, 0), (1, 8, 1, 1), (2, 8, 2, 0), (5, 8, 6, 0)])
def test_train_step_matches_torch(dev, shape, mode):
    """Fused HIP training (fwd+bwd+reduce+Adam, several steps) vs torch autograd
    + Keras-Adam — lagged-update step kernels, ticketed step kernels and the
    persistent one-launch-per-fit kernel."""
    from rphedge.models.hedge_mlp import NetSpec
    from rphedge.ops import layout as L

    nin, h, nout, head = shape
    spec = NetSpec(nin=nin, hidden=h, nout=nout, head=head)
    (wc, oc, fc, vc, rc, sc), (wg, og, fg, vg, rg, sg) = _fit_pair(dev, spec, 4096, 512, 2, L.LOSS_MSE,
                                                                   step_mode=mode)
    np.testing.assert_allclose(wg, wc, rtol=2e-3, atol=2e-4)
    assert og[L.O_T] == oc[L.O_T] == 16
    # Adam moments: m, v are linear / quadratic in the gradient, so (unlike the
    # weights) they expose a mis-scaled gradient packet
    P = spec.nparams
    for off in (L.O_M, L.O_V):
        ref = oc[off:off + P]
        np.testing.assert_allclose(og[off:off + P], ref, rtol=0, atol=5e-3 * np.abs(ref).max())
        assert abs(np.linalg.norm(og[off:off + P]) / np.linalg.norm(ref) - 1.0) < 5e-3
    np.testing.assert_allclose(fg[L.F_HIST:L.F_HIST + 2], fc[L.F_HIST:L.F_HIST + 2], rtol=1e-3)
    np.testing.assert_allclose(vg, vc, rtol=1e-3, atol=1e-4)
    np.testing.assert_allclose(rg, rc, rtol=1e-3, atol=1e-4)


@pytest.mark.parametrize("variant", [0, 1, 2, 3, 4, 5])
@pytest.mark.parametrize("shape", [(1, 8, 2, 0), (3, 8, 2, 0), (5, 8, 6, 0)])
def test_narrow_lag_variants_match_torch(dev, shape, variant):
    """Every narrow lagged-step variant (weights in registers / re-read from
    LDS, 1 or 2 waves per SIMD, prefetch depth 1 or 3) vs torch, on a grid of
    several workgroups (batch 2^13 -> 32 WGs, 512 WGs requested)."""
    from rphedge.models.hedge_mlp import NetSpec
    from rphedge.ops import layout as L

    nin, h, nout, head = shape
    spec = NetSpec(nin=nin, hidden=h, nout=nout, head=head)
    (wc, oc, fc, vc, rc, sc), (wg, og, fg, vg, rg, sg) = _fit_pair(dev, spec, 1 << 14, 1 << 13, 2, L.LOSS_MSE,
                                                                   chunk_log2=6, step_mode="lag", variant=variant,
                                                                   max_wgs=512)
    np.testing.assert_allclose(wg, wc, rtol=2e-3, atol=2e-4)
    np.testing.assert_allclose(fg[L.F_HIST:L.F_HIST + 2], fc[L.F_HIST:L.F_HIST + 2], rtol=1e-3)
    np.testing.assert_allclose(vg, vc, rtol=1e-3, atol=1e-4)


def _norm(nin):
    return tuple(1.0 - 0.01 * f for f in range(nin)), tuple(7.0 + f for f in range(nin))


@pytest.mark.parametrize("mode", ["lag", "ticket", "persistent"])
@pytest.mark.parametrize("shape", [(1, 8, 2, 0), (3, 8, 2, 0), (1, 32, 2, 0), (2, 32, 2, 0)])
def test_feature_norm_matches_torch(dev, shape, mode):
    """Input standardisation fused into the kernels' feature loads (train and
    eval, narrow VALU and wide fp32-MFMA bodies) vs torch on standardised X."""
    from rphedge.models.hedge_mlp import NetSpec
    from rphedge.ops import layout as L

    nin, h, nout, head = shape
    spec = NetSpec(nin=nin, hidden=h, nout=nout, head=head)
    (wc, oc, fc, vc, rc, sc), (wg, og, fg, vg, rg, sg) = _fit_pair(dev, spec, 4096, 512, 2, L.LOSS_MSE,
                                                                   step_mode=mode, norm=_norm, mfma_fp32=True)
    np.testing.assert_allclose(wg, wc, rtol=2e-3, atol=3e-4)
    np.testing.assert_allclose(fg[L.F_HIST:L.F_HIST + 2], fc[L.F_HIST:L.F_HIST + 2], rtol=1e-3)
    np.testing.assert_allclose(vg, vc, rtol=1e-3, atol=2e-4)
    np.testing.assert_allclose(rg, rc, rtol=1e-3, atol=2e-4)


@pytest.mark.parametrize("det,split", [(False, False), (True, False), (False, True)])
def test_train_pinball_multi_wg(dev, det, split):
    """Large batch -> many workgroups + last-arriver reduction (float-atomic or
    deterministic slab), standalone update kernel (the DP path); pinball loss;
    64-path chunk shuffle."""
    from rphedge.models.hedge_mlp import NetSpec
    from rphedge.ops import layout as L

    spec = NetSpec(nin=3, hidden=8, nout=2, head=0)
    (wc, oc, fc, *_), (wg, og, fg, *_) = _fit_pair(dev, spec, 1 << 17, 1 << 16, 3, L.LOSS_PINBALL, chunk_log2=6,
                                                   deterministic=det, split_update=split)
    np.testing.assert_allclose(wg, wc, rtol=2e-3, atol=2e-4)
    np.testing.assert_allclose(fg[L.F_HIST:L.F_HIST + 3], fc[L.F_HIST:L.F_HIST + 3], rtol=1e-3)


@pytest.mark.parametrize("mode", ["lag", "ticket", "persistent"])
def test_early_stopping_device_matches_torch(dev, mode):
    from rphedge.engine import DateData, FitConfig, HipBackend, TorchBackend, TrainConfig, current_weights
    from rphedge.models.hedge_mlp import NetSpec, init_weights
    from rphedge.ops import layout as L

    spec = NetSpec(nin=1, hidden=8, nout=2, head=0)
    n = 2048
    x = torch.linspace(0.7, 1.3, n)
    data_c = DateData(feats=[x], prices_next=[x * 1.01], bond_next=1.0, target=torch.relu(x - 1), prices_now=[x])
    data_g = DateData(feats=[x.to(dev)], prices_next=[(x * 1.01).to(dev)], bond_next=1.0,
                      target=torch.relu(x - 1).to(dev), prices_now=[x.to(dev)])
    fc = FitConfig(epochs=40, patience=3, loss=L.LOSS_MSE, lr_schedule=tuple([0.05] * 40))
    res = []
    for be, dd in ((TorchBackend(spec, n, TrainConfig(batch_size=512), device="cpu"), data_c),
                   (HipBackend(spec, n, TrainConfig(batch_size=512, step_mode=mode), device=dev), data_g)):
        w, o, f = be.new_weights(init_weights(spec, [0.5, 0.0])), be.new_opt(), be.new_fit()
        be.fit(w, o, f, dd, fc, seed=3)
        res.append((int(f[L.F_EPOCH].item()), current_weights(spec, w), f.cpu().numpy(), o.cpu().numpy()))
    assert res[0][0] == res[1][0]
    fc_, fg_ = res[0][2], res[1][2]
    for k in (L.F_STOPPED, L.F_WAIT, L.F_HASBEST):
        assert fc_[k] == fg_[k], k
    # (lr 0.05 for ~20 epochs amplifies fp32 summation-order differences)
    np.testing.assert_allclose(fg_[L.F_BEST], fc_[L.F_BEST], rtol=2e-2)
    np.testing.assert_allclose(fg_[L.F_HIST:L.F_HIST + res[0][0]], fc_[L.F_HIST:L.F_HIST + res[0][0]], rtol=2e-2)
    assert res[0][3][L.O_T] == res[1][3][L.O_T]
    np.testing.assert_allclose(res[1][1], res[0][1], rtol=5e-2, atol=1e-2)


def test_radix_quantile_matches_numpy(dev):
    from rphedge import risk

    x = torch.randn(100_003, generator=torch.Generator().manual_seed(1)) ** 3
    qs = (0.0, 0.01, 0.5, 0.98, 0.99, 0.995, 1.0)
    got = risk.quantile(x.to(dev), qs)
    ref = np.quantile(x.numpy().astype(np.float64), qs)
    np.testing.assert_allclose(got, ref, rtol=1e-6, atol=1e-6)


def test_graph_replay_equals_eager(dev):
    from rphedge.config import ParityFlags, RunConfig, TrainingParams
    from rphedge.api import HedgeRun

    tr = TrainingParams(batch_size=4096, epochs_first=4, epochs_rest=2, early_stopping=False, q99=False,
                        lr_schedule_first=False, chunk_log2=6)
    cfg = RunConfig(Y=100.0, K=100.0, T=1.0, mu=0.08, r=0.08, sigma=0.15, rebalancing=0.1, dt=0.1, n_paths=14,
                    payoff="call", option_type="CALL", model="gbm_log", mortality=False, N=1, P=1.0,
                    keep_paths=False, verbose=False, train=tr, parity=ParityFlags())
    run = HedgeRun(cfg)
    run.build()
    r_eager = run.run()
    run.capture(include_simulation=True)
    run.replay()
    r_graph = run.collect()
    assert r_graph.v0 == pytest.approx(r_eager.v0, rel=1e-6)
    assert r_graph.terminal_pnl["std"] == pytest.approx(r_eager.terminal_pnl["std"], rel=1e-6)


@pytest.mark.parametrize("family", ["heston", "basket", "pension"])
def test_graph_resimulation_all_models(dev, family):
    """The captured graph re-simulates every path family into the SAME buffers:
    bitwise-identical paths/terminal values and the same run as eager."""
    from rphedge.config import ParityFlags, RunConfig, TrainingParams
    from rphedge.api import HedgeRun

    tr = TrainingParams(batch_size=4096, epochs_first=3, epochs_rest=2, early_stopping=False,
                        q99=family == "pension", lr_schedule_first=False, chunk_log2=6, deterministic=False)
    kw = dict(Y=100.0, K=100.0, T=1.0, mu=0.05, r=0.05, sigma=0.2, rebalancing=0.25, dt=0.05, n_paths=13,
              N=1, P=1.0, keep_paths=False, verbose=False, train=tr, parity=ParityFlags())
    if family == "heston":
        kw.update(payoff="call", option_type="CALL", model="heston", mortality=False)
    elif family == "basket":
        kw.update(payoff="basket_call", model="basket", n_assets=5, mortality=False)
    else:
        kw.update(Y=1.0, K=1.0, T=2.0, payoff="guarantee", model="gbm", mortality=True, N=10000, P=100.0)
    run = HedgeRun(RunConfig(**kw))
    run.build()
    r_eager = run.run()
    s0 = run.paths.S.clone()
    v0 = run.v_terminal.clone()
    nf0 = run.paths.nfrac.clone() if run.paths.nfrac is not None else None
    run.paths.S.zero_()
    run.v_terminal.zero_()
    run.capture(include_simulation=True)
    run.replay()
    r_graph = run.collect()
    assert torch.equal(run.paths.S, s0)
    assert torch.equal(run.v_terminal, v0)
    if nf0 is not None:
        assert torch.equal(run.paths.nfrac, nf0)
    assert r_graph.v0 == pytest.approx(r_eager.v0, rel=2e-3)


def test_european_converges_to_black_scholes(dev):
    """Integration: corrected replication at 2^18 paths lands near BS 10.3896."""
    from rphedge.config import ParityFlags, RunConfig, TrainingParams
    from rphedge.api import HedgeRun

    tr = TrainingParams(batch_size=1 << 14, epochs_first=60, epochs_rest=15, early_stopping=False, q99=False,
                        lr_schedule_first=False, chunk_log2=6, lr=5e-3)
    cfg = RunConfig(Y=100.0, K=100.0, T=1.0, mu=0.08, r=0.08, sigma=0.15, rebalancing=1 / 12, dt=1 / 12,
                    n_paths=18, payoff="call", option_type="CALL", model="gbm_log", mortality=False, N=1, P=1.0,
                    keep_paths=True, verbose=False, train=tr, parity=ParityFlags())
    res = HedgeRun(cfg).run()
    assert abs(res.v0 - 10.3896) < 0.35
    assert abs(res.phi - 0.7285) < 0.06


def test_deterministic_mode_is_bitwise_reproducible(dev):
    from rphedge.models.hedge_mlp import NetSpec
    from rphedge.ops import layout as L

    spec = NetSpec(nin=1, hidden=8, nout=2, head=0)
    a = _fit_pair(dev, spec, 1 << 16, 1 << 15, 2, L.LOSS_MSE, chunk_log2=6, deterministic=True)[1]
    b = _fit_pair(dev, spec, 1 << 16, 1 << 15, 2, L.LOSS_MSE, chunk_log2=6, deterministic=True)[1]
    assert np.array_equal(a[0], b[0])


def test_rccl_comm_split_update_and_graph_capture(dev):
    """The DP hot path on one rank: step kernel -> native RCCL all-reduce ->
    standalone update kernel, eager and captured in a hipGraph."""
    import os
    import socket

    import torch.distributed as dist
    from torch.distributed import distributed_c10d as c10d

    from rphedge.engine import DateData, FitConfig, HipBackend, TorchBackend, TrainConfig, current_weights
    from rphedge.models.hedge_mlp import NetSpec, init_weights
    from rphedge.ops import layout as L
    from rphedge.ops.native import Graph, NcclComm

    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("nccl", rank=0, world_size=1, device_id=dev)
    try:
        comm = NcclComm(0, 1, c10d._get_default_store(), tag="test_rccl")
        spec = NetSpec(nin=3, hidden=8, nout=2, head=0)
        n = 1 << 15
        gen = torch.Generator().manual_seed(5)
        feats = [torch.rand(n, generator=gen) * 0.5 + 0.75 for _ in range(3)]
        prices = [feats[0] * 1.02]
        target = torch.relu(prices[0] - 1.0)
        w0 = init_weights(spec, [0.5, -0.4])
        tc = TrainConfig(batch_size=1 << 13, chunk_log2=6, lr=1e-2, split_update=True)
        fc = FitConfig(epochs=3, patience=100, early_stopping=False)
        out = {}
        for name, be, d in (("cpu", TorchBackend(spec, n, tc, device="cpu"), torch.device("cpu")),
                            ("gpu", HipBackend(spec, n, tc, device=dev, comm=comm, world=1), dev)):
            data = DateData(feats=[f.to(d) for f in feats], prices_next=[p.to(d) for p in prices],
                            bond_next=1.0, target=target.to(d), prices_now=[feats[0].to(d)])
            w, o, f = be.new_weights(w0), be.new_opt(), be.new_fit()
            be.fit(w, o, f, data, fc, seed=9)
            out[name] = current_weights(spec, w)
            if name == "gpu":
                torch.cuda.synchronize()
                # capture the same fit (RCCL all-reduce nodes included) and replay it
                w2, o2, f2 = be.new_weights(w0), be.new_opt(), be.new_fit()
                be.fit(w2, o2, f2, data, fc, seed=9)  # eager warm-up populates caches
                torch.cuda.synchronize()
                w2.copy_(be.new_weights(w0))
                o2.copy_(be.new_opt())
                st = torch.cuda.Stream(dev)
                st.wait_stream(torch.cuda.current_stream())
                g = Graph()
                with torch.cuda.stream(st):
                    g.capture_begin(st)
                    be.fit(w2, o2, f2, data, fc, seed=9)
                    g.capture_end()
                    g.replay(st)
                st.synchronize()
                out["graph"] = current_weights(spec, w2)
                assert float(f2[L.F_EPOCH].item()) == 3
        np.testing.assert_allclose(out["gpu"], out["cpu"], rtol=2e-3, atol=2e-4)
        np.testing.assert_allclose(out["graph"], out["gpu"], rtol=1e-4, atol=1e-5)
        comm.close()
    finally:
        dist.destroy_process_group()


def test_nan_gradient_guard_gpu(dev):
    """Fault injection on device: NaN gradients -> update skipped + counted."""
    from rphedge.engine import DateData, FitConfig, HipBackend, TrainConfig, current_weights
    from rphedge.models.hedge_mlp import NetSpec, init_weights
    from rphedge.ops import layout as L

    spec = NetSpec(nin=1, hidden=8, nout=2, head=0)
    n = 1 << 14
    x = torch.linspace(0.8, 1.2, n, device=dev)
    y = torch.relu(x - 1)
    y[5] = float("nan")
    be = HipBackend(spec, n, TrainConfig(batch_size=4096, shuffle=False), device=dev)
    w, o, f = be.new_weights(init_weights(spec, [0.5, 0.0])), be.new_opt(), be.new_fit()
    be.fit(w, o, f, DateData(feats=[x], prices_next=[x], bond_next=1.0, target=y, prices_now=[x]),
           FitConfig(epochs=3, patience=100, early_stopping=False), seed=1)
    torch.cuda.synchronize()
    assert np.all(np.isfinite(current_weights(spec, w)))
    assert float(o[L.O_NAN].item()) == 3.0
    assert float(o[L.O_T].item()) == 9.0   # 12 steps, 3 skipped


@pytest.mark.parametrize("mode", ["lag", "persistent"])
def test_step_modes_match_ticket_kernels(dev, mode):
    """Lagged-update / one-launch-per-fit kernels == ticketed per-step kernels
    (same math; float-atomic summation order only), many workgroups, pinball
    loss, lr schedule, early stopping."""
    from rphedge.engine import DateData, FitConfig, HipBackend, TrainConfig, current_weights
    from rphedge.models.hedge_mlp import NetSpec, init_weights
    from rphedge.ops import layout as L

    spec = NetSpec(nin=3, hidden=8, nout=2, head=0)
    n = 1 << 18
    g = torch.Generator().manual_seed(5)
    feats = [(torch.rand(n, generator=g) * 0.5 + 0.75).to(dev) for _ in range(3)]
    prices = [feats[0] * 1.02]
    data = DateData(feats=feats, prices_next=prices, bond_next=1.01, target=torch.relu(prices[0] - 1.0),
                    prices_now=feats[:1])
    fc = FitConfig(epochs=12, patience=4, loss=L.LOSS_PINBALL, lr_schedule=tuple([1e-2] * 6 + [1e-3] * 6))
    out = []
    for m in (mode, "ticket"):
        be = HipBackend(spec, n, TrainConfig(batch_size=1 << 15, chunk_log2=6, step_mode=m), device=dev)
        assert be.step_mode() == m
        w, o, f = be.new_weights(init_weights(spec, [0.5, 0.1])), be.new_opt(), be.new_fit()
        be.fit(w, o, f, data, fc, seed=11)
        torch.cuda.synchronize()
        be.check()
        out.append((current_weights(spec, w), o.cpu().numpy(), f.cpu().numpy()))
    (wp, op, fp), (ws, os_, fs) = out
    assert fp[L.F_EPOCH] == fs[L.F_EPOCH] and op[L.O_T] == os_[L.O_T]
    np.testing.assert_allclose(fp[L.F_HIST:L.F_HIST + 12], fs[L.F_HIST:L.F_HIST + 12], rtol=1e-4)
    np.testing.assert_allclose(wp, ws, rtol=1e-3, atol=1e-5)
    np.testing.assert_allclose(op[L.O_M:L.O_M + spec.nparams], os_[L.O_M:L.O_M + spec.nparams], rtol=1e-2, atol=1e-7)


@pytest.mark.parametrize("mode", ["lag", "ticket"])
def test_k10_first_step_matches_torch_optim_adam(dev, mode):
    """K10 vs torch.optim.Adam: one full-batch step from the same
    weights.  Keras' Adam adds eps to sqrt(v) before bias correction, so the
    matching torch eps at step t is eps / sqrt(1 - beta2^t)."""
    from rphedge.engine import DateData, FitConfig, HipBackend, TrainConfig, current_weights
    from rphedge.models.hedge_mlp import NetSpec, init_weights

    spec = NetSpec(nin=3, hidden=8, nout=2, head=0)
    n = 4096
    g = torch.Generator().manual_seed(9)
    feats = [torch.rand(n, generator=g) * 0.5 + 0.75 for _ in range(3)]
    price = feats[0] * 1.02
    target = torch.relu(price - 1.0)
    w0 = init_weights(spec, [0.5, 0.1])
    lr, eps, b2 = 1e-2, 1e-7, 0.999
    be = HipBackend(spec, n, TrainConfig(batch_size=n, lr=lr, eps=eps, shuffle=False, step_mode=mode), device=dev)
    data = DateData(feats=[f.to(dev) for f in feats], prices_next=[price.to(dev)], bond_next=1.03,
                    target=target.to(dev), prices_now=[feats[0].to(dev)])
    w, o, f = be.new_weights(w0), be.new_opt(), be.new_fit()
    be.fit(w, o, f, data, FitConfig(epochs=1, patience=10 ** 6, early_stopping=False), seed=1)
    torch.cuda.synchronize()
    wg = current_weights(spec, w)

    # torch reference: fp64 autograd of the same MSE, torch.optim.Adam step
    o_ = spec.offsets
    p = torch.tensor(w0, dtype=torch.float64, requires_grad=True)
    X = torch.stack(feats, 1).double()
    W1 = p[o_["W1"]:o_["b1"]].view(3, 8); b1 = p[o_["b1"]:o_["W2"]]
    W2 = p[o_["W2"]:o_["b2"]].view(8, 8); b2_ = p[o_["b2"]:o_["W3"]]
    W3 = p[o_["W3"]:o_["b3"]].view(8, 2); b3 = p[o_["b3"]:o_["P"]]
    a = torch.nn.functional.leaky_relu(X @ W1 + b1, 0.3)
    a = torch.nn.functional.leaky_relu(a @ W2 + b2_, 0.3)
    h = a @ W3 + b3
    V = h[:, 0] * price.double() + h[:, 1] * 1.03
    loss = ((V - target.double()) ** 2).mean()
    opt = torch.optim.Adam([p], lr=lr, betas=(0.9, b2), eps=eps / math.sqrt(1 - b2))
    loss.backward()
    opt.step()
    np.testing.assert_allclose(wg, p.detach().numpy(), rtol=1e-4, atol=2e-6)


@pytest.mark.parametrize("case", ["euro", "pension_q99"])
def test_pnl_scan_kernel_vs_numpy(dev, case):
    """k_hedge_pnl (self-financing P&L over the per-date networks written by
    the eval kernels' snapshots) against the numpy recursion."""
    from test_pnl import check_against_oracle

    from rphedge.api import european_option, run_params
    from rphedge.experiments import mts_parameters

    if case == "euro":
        res = european_option(N_paths=1 << 14, dt=1 / 52, rebalancing_frequency=1 / 13, epochs_first=40,
                              epochs_rest=8, batch_size=4096, verbose=False, device=dev)
        check_against_oracle(res)
    else:
        res = run_params(mts_parameters(n_paths=13, dt=0.1, rebalancing=1.0, epochs_first=30, epochs_rest=6,
                                        verbose=False, device=dev, batch_size=2048))
        check_against_oracle(res, hold_c=0.1)
    assert res.induction.pnl_paths.is_cuda
