"""Multi-start first-date LM fits (LmDesc.inst / explore, k_lm_select) and the
damping carry (LmDesc.lam_carry) on the GPU: every exploration instance of the
one-launch-per-kernel grid is bitwise the single fit from its start point, the
selection writes the lowest-loss candidate, the whole explore + polish fit
graph-captures and replays bitwise, and it follows the fp64 torch oracle."""
import numpy as np
import pytest
import torch

from test_gpu_lm import _setup

pytestmark = pytest.mark.gpu


def _starts(spec, w0, k):
    from rphedge.models.hedge_mlp import init_weights

    o = spec.offsets
    return np.stack([w0] + [init_weights(spec, w0[o["b3"]:o["P"]], seed=77 + 13 * c) for c in range(1, k)])


@pytest.mark.parametrize("shape", [(1, 8, 2, 0), (3, 8, 2, 0)])
def test_explore_instances_equal_single_fits_and_pick_the_best(shape):
    from rphedge.engine import DateData, FitConfig, HipBackend, TrainConfig, current_weights
    from rphedge.ops import layout as L

    dev = torch.device("cuda", 0)
    n, nsub, K, n1 = 1 << 14, 1 << 12, 3, 10
    spec, feats, pr, y, data, w0 = _setup(shape, n, dev, seed=5)
    w0s = _starts(spec, w0, K)
    tc = TrainConfig(batch_size=n, lm_gram_paths=1024)
    be = HipBackend(spec, n, tc, device=dev)
    w, o, f = be.new_weights(w0), be.new_opt(), be.new_fit()
    fc = FitConfig(epochs=0, optimizer="lm", early_stopping=False, lm_starts=K, lm_explore_passes=n1,
                   lm_explore_paths=nsub, lm_w0s=w0s)
    be.fit(w, o, f, data, fc, seed=0)
    torch.cuda.synchronize()
    x = be.lm_explore_last
    st = x["state"].cpu().numpy()
    sel = x["sel"].cpu().numpy()
    # every instance == the single-instance fit of its start point on the prefix
    sub = DateData(feats=[t[:nsub] for t in data.feats], prices_next=[t[:nsub] for t in data.prices_next],
                   bond_next=data.bond_next, target=data.target[:nsub], prices_now=[t[:nsub] for t in data.prices_now],
                   fmu=data.fmu, fisd=data.fisd)
    losses = []
    for k in range(K):
        b1 = HipBackend(spec, nsub, TrainConfig(batch_size=nsub, lm_gram_paths=1024), device=dev)
        w1, o1, f1 = b1.new_weights(w0s[k]), b1.new_opt(), b1.new_fit()
        b1.fit(w1, o1, f1, sub, FitConfig(epochs=n1, optimizer="lm", early_stopping=False), seed=0)
        torch.cuda.synchronize()
        s1 = b1._lm_buffers()["state"].cpu().numpy()
        best = int(s1[L.LMS_BEST])
        assert int(st[k, L.LMS_BEST]) == best
        np.testing.assert_array_equal(st[k, L.LMS_W + best * L.LM_NPMAX:][:spec.nparams],
                                      s1[L.LMS_W + best * L.LM_NPMAX:][:spec.nparams])
        assert st[k, L.LMS_LFIN] == s1[L.LMS_LFIN]
        assert st[k, L.LMS_LAM] == s1[L.LMS_LAM]
        losses.append(s1[L.LMS_LFIN])
        # the packed selection block
        assert sel[k * L.LM_SEL_W] == s1[L.LMS_LFIN] and sel[k * L.LM_SEL_W + 1] == s1[L.LMS_LAM]
    pick = int(np.argmin(losses))
    bp = int(st[pick, L.LMS_BEST])
    want = st[pick, L.LMS_W + bp * L.LM_NPMAX:][:spec.nparams].astype(np.float32)
    # epochs = 0 polish: the start point is published (+ the bias Newton step)
    got = current_weights(spec, w)
    bi = spec.nparams - 1 if spec.head == L.HEAD_FREE else -1
    keep = [i for i in range(spec.nparams) if i != bi]
    np.testing.assert_array_equal(got[keep], want[keep])
    assert int(f[L.F_EPOCH]) == 1 and np.isnan(float(f[L.F_HIST + 1]))


def test_multistart_fit_graph_replays_and_follows_torch():
    from rphedge.engine import DateData, FitConfig, HipBackend, TorchBackend, TrainConfig, current_weights
    from rphedge.ops import layout as L
    from rphedge.ops.native import Graph

    dev = torch.device("cuda", 0)
    n, K = 1 << 14, 4
    spec, feats, pr, y, data, w0 = _setup((1, 8, 2, 0), n, dev, seed=3)
    w0s = _starts(spec, w0, K)
    tc = TrainConfig(batch_size=n, lm_gram_paths=1024)
    fc = FitConfig(epochs=8, optimizer="lm", early_stopping=False, lm_starts=K, lm_explore_passes=12,
                   lm_explore_paths=1 << 12, lm_w0s=w0s)
    be = HipBackend(spec, n, tc, device=dev)
    w, o, f = be.new_weights(w0), be.new_opt(), be.new_fit()
    be.fit(w, o, f, data, fc, seed=0)
    torch.cuda.synchronize()
    w_e, f_e = current_weights(spec, w), f.cpu().numpy()
    s = torch.cuda.Stream()
    s.wait_stream(torch.cuda.current_stream())
    outs = []
    with torch.cuda.stream(s):
        g = Graph()
        g.capture_begin(s)
        try:
            # (the exploration reads its start points from LmDesc.w0 and the
            # selection overwrites the NetWeights: nothing to reset per replay)
            be.fit(w, o, f, data, fc, seed=0)
        finally:
            g.capture_end()
        for _ in range(2):
            g.replay(s)
            s.synchronize()
            outs.append((current_weights(spec, w), f.cpu().numpy()))
    for wg, fg in outs:
        np.testing.assert_array_equal(wg, w_e)
        np.testing.assert_array_equal(fg[L.F_HIST:L.F_HIST + 9], f_e[L.F_HIST:L.F_HIST + 9])
    # torch oracle: same candidates picked, polish best loss close
    cd = DateData(feats=feats, prices_next=pr, bond_next=1.01, target=y, prices_now=pr, fmu=data.fmu, fisd=data.fisd)
    tb = TorchBackend(spec, n, tc)
    tb.fit(tb.new_weights(w0), tb.new_opt(), tb.new_fit(), cd, fc, seed=0)
    xs = be.lm_explore_last["sel"].cpu().numpy()
    lg = [xs[c * L.LM_SEL_W] for c in range(K)]
    lc = tb.lm_explore_last["losses"]
    np.testing.assert_allclose(lg, lc, rtol=2e-2)
    assert int(np.argmin(lg)) == tb.lm_explore_last["pick"]
    hist_g = np.minimum.accumulate(f_e[L.F_HIST:L.F_HIST + 9])
    hist_c = np.minimum.accumulate(tb.lm_last["hist"])
    np.testing.assert_allclose(hist_g[:4], hist_c[:4], rtol=5e-3)


def test_lam_carry_starts_at_the_previous_fit_damping():
    """lam_carry: a fit's first trial uses max(previous final damping x carry,
    lam_min): two consecutive fits == the torch oracle's carried sequence."""
    from rphedge.engine import FitConfig, HipBackend, TrainConfig
    from rphedge.ops import layout as L

    dev = torch.device("cuda", 0)
    n = 1 << 13
    spec, feats, pr, y, data, w0 = _setup((1, 8, 2, 0), n, dev, seed=4)
    tc = TrainConfig(batch_size=n, lm_gram_paths=1024)
    be = HipBackend(spec, n, tc, device=dev)
    w, o, f = be.new_weights(w0), be.new_opt(), be.new_fit()
    be.fit(w, o, f, data, FitConfig(epochs=6, optimizer="lm", early_stopping=False), seed=0)
    torch.cuda.synchronize()
    lam1 = float(be._lm_buffers()["state"][L.LMS_LAM])
    # second fit, carry x 3, 0 trial points: the damping after its (start-only)
    # final solve is the carried start damping
    be.fit(w, o, f, data, FitConfig(epochs=0, optimizer="lm", early_stopping=False, lm_lam_carry=3.0), seed=0)
    torch.cuda.synchronize()
    lam2 = float(be._lm_buffers()["state"][L.LMS_LAM])
    assert lam2 == pytest.approx(max(lam1 * 3.0, tc.lm_lam_min), rel=1e-12)


def test_renorm_reexpresses_the_warm_start():
    """lm_renorm: the start point's first layer is re-expressed for the new
    standardisation, so the network is the same function of the raw state
    (before any trial), and the HIP transform equals the torch oracle's."""
    from rphedge.engine import DateData, FitConfig, HipBackend, TorchBackend, TrainConfig, current_weights
    from rphedge.models.hedge_mlp import torch_forward

    dev = torch.device("cuda", 0)
    n = 1 << 12
    spec, feats, pr, y, data, w0 = _setup((2, 8, 2, 0), n, dev, seed=6)
    old = ((0.3, -0.2), (0.8, 1.7))  # (mu, isd) the start weights were fitted with
    tc = TrainConfig(batch_size=n, lm_gram_paths=1024)
    fc = FitConfig(epochs=0, optimizer="lm", early_stopping=False, lm_renorm=old)
    be = HipBackend(spec, n, tc, device=dev)
    w, o, f = be.new_weights(w0), be.new_opt(), be.new_fit()
    be.fit(w, o, f, data, fc, seed=0)
    torch.cuda.synchronize()
    got = current_weights(spec, w)
    raw = torch.stack([t.double() for t in feats], 1)
    x_old = (raw - torch.tensor(old[0], dtype=torch.float64)) * torch.tensor(old[1], dtype=torch.float64)
    x_new = (raw - torch.tensor(data.fmu, dtype=torch.float64)) * torch.tensor(data.fisd, dtype=torch.float64)
    h_old = torch_forward(spec, torch.tensor(w0, dtype=torch.float64), x_old)[:, 0]
    h_new = torch_forward(spec, torch.tensor(got, dtype=torch.float64), x_new)[:, 0]
    np.testing.assert_allclose(h_new.numpy(), h_old.numpy(), rtol=1e-5, atol=1e-6)
    cd = DateData(feats=feats, prices_next=pr, bond_next=1.01, target=y, prices_now=pr, fmu=data.fmu, fisd=data.fisd)
    tb = TorchBackend(spec, n, tc)
    wc = tb.new_weights(w0)
    tb.fit(wc, tb.new_opt(), tb.new_fit(), cd, fc, seed=0)
    o_ = spec.offsets
    np.testing.assert_array_equal(got[o_["W1"]:o_["W2"]], current_weights(spec, wc)[o_["W1"]:o_["W2"]])


@pytest.mark.parametrize("shape,fitted,n", [((1, 8, 2, 0), True, 1 << 13), ((5, 8, 6, 0), True, 1 << 13),
                                            ((2, 8, 2, 0), True, 1 << 13), ((1, 8, 1, 1), True, 1 << 13),
                                            ((3, 8, 2, 0), True, 1 << 13), ((1, 8, 2, 0), False, 1 << 13),
                                            ((2, 8, 2, 0), False, 1 << 13),
                                            # 512 pass workgroups: the 512-row output-Gram reduction
                                            ((1, 8, 2, 0), True, 1 << 17)])
def test_output_newton_step_matches_torch(shape, fitted, n):
    """lm_out_fix: the last solve's Newton step on the output layer with the
    FULL-BATCH output Gram matrix (built on the matrix cores by the pass,
    bf16 operands, fp32 accumulation): only the output layer moves, the
    full-batch loss drops (also from the random init, where the Gram
    subsample's output block is near-singular), by the fp64 torch oracle's
    amount, the full-batch mean residual vanishes, and FitState.best_loss
    reports the full-batch loss of the published weights."""
    from rphedge.engine import DateData, FitConfig, HipBackend, TorchBackend, TrainConfig, current_weights, lm_out_nu
    from rphedge.models.hedge_mlp import torch_forward
    from rphedge.ops import layout as L

    dev = torch.device("cuda", 0)
    spec, feats, pr, y, data, w_init = _setup(shape, n, dev, seed=7)
    w0 = w_init
    if fitted:
        b0 = HipBackend(spec, n, TrainConfig(batch_size=n, lm_gram_paths=2048), device=dev)
        w1 = b0.new_weights(w_init)
        b0.fit(w1, b0.new_opt(), b0.new_fit(), data, FitConfig(epochs=20, optimizer="lm", early_stopping=False),
               seed=0)
        torch.cuda.synchronize()
        w0 = current_weights(spec, w1)
    tc = TrainConfig(batch_size=n, lm_gram_paths=2048, lm_out_fix=True)
    fc = FitConfig(epochs=0, optimizer="lm", early_stopping=False)
    be = HipBackend(spec, n, tc, device=dev)
    w, fit = be.new_weights(w0), be.new_fit()
    be.fit(w, be.new_opt(), fit, data, fc, seed=0)
    torch.cuda.synchronize()
    got = current_weights(spec, w)
    cd = DateData(feats=feats, prices_next=pr, bond_next=1.01, target=y, prices_now=pr, fmu=data.fmu, fisd=data.fisd)
    tb = TorchBackend(spec, n, tc)
    wc = tb.new_weights(w0)
    tb.fit(wc, tb.new_opt(), tb.new_fit(), cd, fc, seed=0)
    want = current_weights(spec, wc)
    n_out = lm_out_nu(spec)
    np.testing.assert_array_equal(got[:-n_out], w0[:-n_out])
    assert not np.array_equal(got[-n_out:], w0[-n_out:])
    X = (torch.stack([f.double() for f in feats], 1) - torch.tensor(data.fmu, dtype=torch.float64)) * \
        torch.tensor(data.fisd, dtype=torch.float64)
    if spec.head == L.HEAD_FREE:
        Pm = torch.stack([p.double() for p in pr] + [torch.full((n,), 1.01, dtype=torch.float64)], 1)
    else:
        Pm = torch.stack([pr[0].double(), torch.full((n,), 1.01, dtype=torch.float64)], 1)

    def res(wv):
        out = torch_forward(spec, torch.tensor(wv, dtype=torch.float64), X)
        return (out * Pm).sum(1) - y.double()

    l0, lg, lt = [float((res(v) ** 2).mean()) for v in (w0, got, want)]
    assert lg < l0 and lt < l0
    # the same step (bf16 hi/lo split Gram vs fp64): the GPU's reduction is the
    # oracle's within 2 % (more is fine: the damped step of an ill-conditioned
    # output Gram (cond 1e9+) differs in its near-null directions)
    assert lg - lt <= 2e-2 * (l0 - lt) and lt - lg <= 5e-2 * (l0 - lt), (l0, lg, lt)
    # full-batch optimum of the output layer: the mean residual vanishes
    assert abs(float(res(got).mean())) < 1e-3 * float(y.double().abs().mean()) + 1e-6
    # FitState: the full-batch loss after the step (predicted exactly from the quadratic)
    fb = float(fit[L.F_BEST].item())
    # (5 %: the published weights are the fp32 rounding of best + d, and d is
    # long in the Gram's near-null directions)
    assert abs(fb - lg) <= 5e-2 * (l0 - lg) + 1e-6 * l0, (fb, lg, l0)


def test_output_newton_step_every_lm_shape():
    """The full-batch output Gram needs no packet room: every 8-unit LM net
    (complement head and 1-6 inputs included) takes the output-layer step."""
    from rphedge.engine import TrainConfig, _lm_out_n, lm_out_nu
    from rphedge.models.hedge_mlp import NetSpec

    tc = TrainConfig(lm_out_fix=True)
    for shp in [(1, 8, 2, 0), (5, 8, 6, 0), (1, 8, 1, 1), (2, 8, 2, 0), (3, 8, 2, 0), (4, 8, 2, 0), (6, 8, 7, 0)]:
        sp = NetSpec(*shp)
        assert _lm_out_n(sp, tc) == lm_out_nu(sp) == (9 if shp[3] == 1 else 8 * shp[2] + shp[2])


def test_out_step_from_rejected_last_trial():
    """LM_OUTG_TAIL = 1: only the last evaluation builds the output Gram.  When
    the last trial is rejected (and within 2x the best loss), the final solve
    still takes the out step at that trial (its own exact Gram and gradient)
    and publishes trial + step if it beats the best point.  Warm-started
    2-pass fits (as the later dates) at two dampings take both branches, as
    the torch oracle does; every published point's fp64 full-batch loss equals
    FitState.best_loss and is no worse than the best LM point's."""
    from rphedge.engine import DateData, FitConfig, HipBackend, TorchBackend, TrainConfig, current_weights
    from rphedge.models.hedge_mlp import torch_forward
    from rphedge.ops import layout as L

    dev = torch.device("cuda", 0)
    n = 1 << 13
    branches = set()
    for k in range(3):
        spec, feats, pr, y, data, w0 = _setup((1, 8, 2, 0), n, dev, seed=20 + k)
        b0 = HipBackend(spec, n, TrainConfig(batch_size=n, lm_gram_paths=2048), device=dev)
        w = b0.new_weights(w0)
        b0.fit(w, b0.new_opt(), b0.new_fit(), data, FitConfig(epochs=12, optimizer="lm", early_stopping=False), seed=0)
        torch.cuda.synchronize()
        w1 = current_weights(spec, w)
        X = (torch.stack([f.double() for f in feats], 1) - torch.tensor(data.fmu, dtype=torch.float64)) * \
            torch.tensor(data.fisd, dtype=torch.float64)
        Pm = torch.stack([p.double() for p in pr] + [torch.full((n,), 1.01, dtype=torch.float64)], 1)

        def loss(wv):
            e = (torch_forward(spec, torch.tensor(np.asarray(wv, np.float64)), X) * Pm).sum(1) - y.double()
            return float((e ** 2).mean())

        for lam0 in (1.2, 2.0):
            tc = TrainConfig(batch_size=n, lm_gram_paths=2048, lm_out_fix=True, lm_lam0=lam0)
            fc = FitConfig(epochs=2, optimizer="lm", early_stopping=False)
            be = HipBackend(spec, n, tc, device=dev)
            w, fit = be.new_weights(w1), be.new_fit()
            be.fit(w, be.new_opt(), fit, data, fc, seed=0)
            torch.cuda.synchronize()
            got = current_weights(spec, w)
            st = be._lm_buffers()["state"].cpu().numpy()
            best = int(st[L.LMS_BEST])
            wb = st[L.LMS_W + best * L.LM_NPMAX:][:spec.nparams]
            hidden = spec.offsets["W3"]
            from_trial = not np.allclose(got[:hidden], wb[:hidden].astype(np.float32))
            branches.add(from_trial)
            lg, lb = loss(got), loss(wb)
            assert lg <= lb * (1 + 1e-6), (k, lam0, lg, lb)
            assert abs(float(fit[L.F_BEST].item()) - lg) <= 0.05 * max(lb - lg, 0.0) + 1e-5 * lb, \
                (k, lam0, fit[L.F_BEST], lg, lb)
            # the oracle takes the same branch and lands at the same loss
            cd = DateData(feats=feats, prices_next=pr, bond_next=1.01, target=y, prices_now=pr, fmu=data.fmu,
                          fisd=data.fisd)
            tb = TorchBackend(spec, n, tc)
            wc = tb.new_weights(w1)
            tb.fit(wc, tb.new_opt(), tb.new_fit(), cd, fc, seed=0)
            want = current_weights(spec, wc)
            wt = st[L.LMS_W + (1 - best) * L.LM_NPMAX:][:spec.nparams]  # the GPU's last trial
            near_trial = np.abs(want[:hidden] - wt[:hidden]).max() < np.abs(want[:hidden] - wb[:hidden]).max()
            assert near_trial == from_trial, (k, lam0)
            assert loss(want) == pytest.approx(lg, rel=5e-2)
    assert branches == {False, True}, branches
