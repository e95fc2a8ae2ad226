"""CPU tests: host twins of the device math, config/API plumbing, CPU engine."""
import math

import numpy as np
import pytest
import torch


def test_philox_known_answer():
    from rphedge.ops.philox import philox4x32_10

    r = philox4x32_10(0, 0, 0, 0, 0, 0)
    assert [int(v) for v in r] == [0x6627E8D5, 0xE169C58D, 0xBC57AC4C, 0x9B00DBD8]
    m = 0xFFFFFFFF
    r = philox4x32_10(m, m, m, m, m, m)
    assert [int(v) for v in r] == [0x408F276D, 0x41C83B0E, 0xA20BC7C6, 0x6D5451FD]


@pytest.mark.parametrize("n", [1, 7, 64, 100, 4096])
def test_chunk_perm_is_bijection(n):
    from rphedge.ops.philox import ChunkPerm

    p = ChunkPerm(n, seed=11, epoch=3)
    y = p(np.arange(n))
    assert sorted(y.tolist()) == list(range(n))


def test_epoch_order_chunks():
    from rphedge.ops.philox import epoch_order

    o = epoch_order(4096, 6, 5, 0)
    assert sorted(o.tolist()) == list(range(4096))
    # chunks of 64 stay contiguous
    assert np.all(np.diff(o.reshape(-1, 64), axis=1) == 1)


def test_ndtri_twins_vs_scipy():
    from scipy.special import ndtri

    from rphedge.ops.ndtri import ndtri_u30_f32, ndtri_u30_f64

    rng = np.random.default_rng(0)
    x = np.concatenate([rng.integers(1, 2 ** 30, 50000), np.arange(1, 500), 2 ** 30 - np.arange(1, 500)])
    ref = ndtri(x * 2.0 ** -30)
    np.testing.assert_allclose(ndtri_u30_f64(x), ref, rtol=1e-12, atol=1e-13)
    core = np.abs(ref) < 5
    np.testing.assert_allclose(ndtri_u30_f32(x)[core], ref[core], rtol=1e-6, atol=1e-6)


@pytest.mark.parametrize("d,m,seed", [(5, 8, 1235), (40, 10, 1234)])
def test_sobol_cpu_bit_exact(d, m, seed):
    from scipy.stats import qmc

    from rphedge.ops.sobol import sobol_uniform_cpu

    ref = qmc.Sobol(d, scramble=True, seed=seed).random_base2(m)
    assert np.array_equal(sobol_uniform_cpu(m, d, seed), ref)


def test_sobol_norm_api_cpu():
    from scipy.stats import norm, qmc

    from rphedge import sobol_norm

    z = sobol_norm(6, 3, 1235, device="cpu").numpy()
    ref = norm.ppf(qmc.Sobol(3, scramble=True, seed=1235).random_base2(6))
    np.testing.assert_allclose(z, ref, rtol=1e-12, atol=1e-13)


def test_native_layout_loads_without_gpu():
    from rphedge.ops import native

    lib = native.load(required=False)
    assert lib is not None
    assert native.net_nparams(3, 8, 2, 0) == (122, 128)
    assert native.net_nparams(1, 8, 1, 1) == (97, 128)


def test_param_counts_match_reference():
    from rphedge.models import EUROPEAN_REF, PENSION

    assert PENSION.nparams == 122       # "Multi Time Step.ipynb":617
    assert EUROPEAN_REF.nparams == 97   # "European Options.ipynb":451


def test_grid_matches_reference():
    from rphedge.ops.paths import Grid

    g = Grid(10.0, 1 / 100, 0.25)
    assert (g.n_fine, g.reduction, g.n_coarse) == (1001, 25, 41)
    g = Grid(10.0, 1 / 365, 0.25)
    assert (g.n_fine, g.reduction, g.n_coarse) == (3651, 91, 41)
    g = Grid(1.0, 1 / 365, 1 / 52)
    assert (g.n_fine, g.reduction, g.n_coarse) == (366, 7, 53)


def test_parse_params_keys():
    from rphedge.config import parse_params

    base = dict(Y=1, K=1, T=10, mu=0.09464, r=0.03, sigma=0.15965, rebalancing=0.25, N=10000, P=100, x=55,
                l0=0.01, c=0.075, ita=0.000597, dt=1 / 100, n_paths=12)
    cfg = parse_params(base)
    assert cfg.paths == 4096 and cfg.n_coarse == 41
    with pytest.raises(KeyError):
        parse_params({k: v for k, v in base.items() if k != "ita"})
    with pytest.raises(KeyError):
        parse_params(dict(base, bogus=1))
    sv = dict(base)
    sv.pop("sigma")
    sv.update(s0=0.15965, a=0.0033566, b=0.15431)
    cfg = parse_params(dict(sv, parity=True), sv=True)
    assert cfg.sv_c == 0.075 and cfg.model == "sv_ref"   # Q4


def test_gbm_cpu_moments():
    from rphedge.ops import paths as P

    g = P.Grid(10.0, 1 / 100, 0.25)
    p = P.simulate_gbm(g, 4096, 1.0, 0.09464, 0.15965, device="cpu")
    # MTS sanity check: mean Y_T ~ e^{mu T}
    assert abs(float(p.S_final.double().mean()) - math.exp(0.9464)) < 0.03


def test_black_scholes_reference_numbers():
    from rphedge.utils.reports import black_scholes

    price, delta = black_scholes(100, 100, 0.08, 0.15, 1.0)
    assert price == pytest.approx(10.3896, abs=1e-3)
    assert delta == pytest.approx(0.7285, abs=1e-3)


def test_cpu_quantile_exact():
    from rphedge import risk

    x = torch.randn(5001, generator=torch.Generator().manual_seed(3))
    qs = (0.0, 0.1, 0.5, 0.985, 1.0)
    np.testing.assert_allclose(risk.quantile(x, qs), np.quantile(x.double().numpy(), qs), rtol=1e-6, atol=1e-7)


def test_european_cpu_end_to_end():
    import rphedge

    res = rphedge.european_option(N_paths=4096, rebalancing_frequency=1 / 12, epochs_first=60, epochs_rest=15,
                                  verbose=False, batch_size=512)
    assert abs(res.v0 - 10.39) < 0.6
    assert abs(res.phi - 0.7285) < 0.08
    assert res.terminal_pnl["std"] < 3.5


def test_launcher_rejects_bad_descriptors():
    """Host-side validation in the native launchers (csrc/hedge_core.h
    validate_train): a malformed descriptor never reaches the GPU — checked
    here on CPU, where the library loads but no kernel may run."""
    from rphedge.ops import native

    native.load(required=True)
    d = native.TrainDesc()
    d.nin, d.h, d.nout, d.head = 1, 8, 2, 0
    d.num_wgs, d.batch, d.n_local, d.steps_per_epoch = 0, 512, 4096, 8
    with pytest.raises(RuntimeError, match="num_wgs"):
        native.train_step(d, 0, 0, stream=0)
    d.num_wgs = 16
    d.steps_per_epoch = 2  # 2 x 512 < 4096
    with pytest.raises(RuntimeError, match="batch"):
        native.train_lag_step(d, 0, 0, stream=0)
    d.steps_per_epoch = 8
    d.alpha = 1.5  # the kernels compute LeakyReLU as max(z, alpha z)
    with pytest.raises(RuntimeError, match="slope"):
        native.train_lag_fit(d, 1, stream=0)
    d.alpha = 0.3
    with pytest.raises(RuntimeError, match="null state"):
        native.train_fit(d, 1, stream=0)
    # dummy (never dereferenced) pointers past the null checks
    d.wts = d.opt = d.fit = d.target = d.feat[0] = 4096
    d.fisd[0] = 0.0
    with pytest.raises(RuntimeError, match="standardisation"):
        native.train_fit(d, 1, stream=0)
    d.fisd[0], d.fmu[0] = 1.0, float("nan")
    with pytest.raises(RuntimeError, match="standardisation"):
        native.train_lag_fit(d, 1, stream=0)


def test_feature_norms_modes():
    """driver.feature_norms: per-date / pooled moments; degenerate spread
    (every path at S_0 on date 0) keeps unit scale; parity forces raw."""
    from rphedge.driver import feature_norms
    from rphedge.ops import paths as P

    g = P.Grid(1.0, 0.1, 0.1)
    p = P.simulate_gbm(g, 1 << 12, 1.0, 0.08, 0.2, device="cpu", scheme="log")
    assert feature_norms(p, "none") == []
    nd = feature_norms(p, "date")
    assert len(nd) == p.n_coarse - 1
    assert nd[0] == ((pytest.approx(1.0),), (1.0,))
    t = p.n_coarse - 2
    x = p.features(t)[0].double()
    assert nd[t][0][0] == pytest.approx(float(x.mean()), rel=1e-6)  # (fp32 Welford)
    assert nd[t][1][0] == pytest.approx(1.0 / float(x.std(unbiased=False)), rel=1e-6)
    gl = feature_norms(p, "global")
    assert all(v == gl[0] for v in gl) and gl[0][1][0] > 1.0
    with pytest.raises(ValueError):
        feature_norms(p, "bogus")
    from rphedge.config import ParityFlags

    assert ParityFlags.reference().raw_features and not ParityFlags().raw_features


def test_feature_norms_horizon():
    """feature_norm="horizon": price inputs centred at the kink, scaled by the
    remaining-horizon spread m_t sd(log S_T - log S_t) (GBM: F_t sigma
    sqrt(T - t)) floored at floor x the date spread; the fixed-point moment
    sums make the scales independent of the path order (hence of the world
    size); Heston's variance input keeps the date scale."""
    from rphedge.driver import feature_norms
    from rphedge.ops import paths as P

    g = P.Grid(1.0, 0.1, 0.1)
    sig = 0.2
    p = P.simulate_gbm(g, 1 << 14, 1.0, 0.08, sig, device="cpu", scheme="log")
    nd = p.n_coarse - 1
    hz = feature_norms(p, "horizon", centers=(1.0,))
    dt = feature_norms(p, "date")
    tt = g.times()
    for t in range(nd):
        mu, isd = hz[t][0][0], hz[t][1][0]
        assert mu == 1.0                                     # the strike
        m = float(p.features(t)[0].double().mean())
        want = m * sig * math.sqrt(1.0 - tt[t])              # F_t sigma sqrt(T - t)
        assert 1.0 / isd == pytest.approx(want, rel=0.03), (t, 1.0 / isd, want)
    # the floor binds late: scale >= 0.5 x the date spread
    fl = feature_norms(p, "horizon", centers=(1.0,), floor=0.5)
    t = nd - 1
    assert 1.0 / fl[t][1][0] == pytest.approx(max(1.0 / hz[t][1][0], 0.5 / dt[t][1][0]), rel=1e-12)
    # order-independent (exact int64 sums): a permuted path set gives the same bits
    perm = torch.randperm(1 << 14, generator=torch.Generator().manual_seed(3))
    q = P.simulate_gbm(g, 1 << 14, 1.0, 0.08, sig, device="cpu", scheme="log")
    q.S = q.S[:, perm].contiguous()
    assert feature_norms(q, "horizon", centers=(1.0,)) == hz
    # Heston: the variance input keeps the date standardisation
    h = P.simulate_sv(g, 1 << 12, 1.0, 0.05, 0.04, model="heston", kappa=2.0, theta=0.04, xi=0.5, rho=-0.7,
                      device="cpu")
    hh, hd = feature_norms(h, "horizon", centers=(1.0, None)), feature_norms(h, "date")
    assert all(hh[t][0][1] == hd[t][0][1] and hh[t][1][1] == hd[t][1][1] for t in range(h.n_coarse - 1))
    assert hh[3][0][0] == 1.0 and hh[3][1][0] != hd[3][1][0]


def test_keras_adam_matches_torch_optim_adam_cpu():
    """Torch reference backend's Keras-Adam (K10 semantics) vs torch.optim.Adam
    for 3 full-batch steps; the per-step matching torch eps is eps/sqrt(1-b2^t)."""
    from rphedge.engine import DateData, FitConfig, TorchBackend, TrainConfig, current_weights
    from rphedge.models.hedge_mlp import NetSpec, init_weights

    spec = NetSpec(nin=1, hidden=8, nout=2, head=0)
    n = 1024
    x = torch.linspace(0.7, 1.3, n)
    w0 = init_weights(spec, [0.5, 0.0])
    lr, eps, b2 = 5e-3, 1e-7, 0.999
    be = TorchBackend(spec, n, TrainConfig(batch_size=n, lr=lr, eps=eps, shuffle=False), device="cpu",
                      dtype=torch.float64)
    data = DateData(feats=[x], prices_next=[x * 1.01], bond_next=1.0, target=torch.relu(x - 1), prices_now=[x])
    w, o, f = be.new_weights(w0), be.new_opt(), be.new_fit()
    be.fit(w, o, f, data, FitConfig(epochs=3, patience=10 ** 6, early_stopping=False), seed=1)
    wk = current_weights(spec, w)

    o_ = spec.offsets
    p = torch.tensor(w0, dtype=torch.float64, requires_grad=True)
    X = x.double()[:, None]
    opt = torch.optim.Adam([p], lr=lr, betas=(0.9, b2), eps=eps)
    for t in range(1, 4):
        for gr in opt.param_groups:
            gr["eps"] = eps / math.sqrt(1 - b2 ** t)
        opt.zero_grad()
        a = torch.nn.functional.leaky_relu(X @ p[o_["W1"]:o_["b1"]].view(1, 8) + p[o_["b1"]:o_["W2"]], 0.3)
        a = torch.nn.functional.leaky_relu(a @ p[o_["W2"]:o_["b2"]].view(8, 8) + p[o_["b2"]:o_["W3"]], 0.3)
        h = a @ p[o_["W3"]:o_["b3"]].view(8, 2) + p[o_["b3"]:o_["P"]]
        V = h[:, 0] * (x.double() * 1.01) + h[:, 1]
        ((V - torch.relu(x.double() - 1)) ** 2).mean().backward()
        opt.step()
    np.testing.assert_allclose(wk, p.detach().numpy(), rtol=1e-5, atol=1e-7)
