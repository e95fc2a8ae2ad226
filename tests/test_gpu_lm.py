"""Levenberg-Marquardt kernels (csrc/hedge_lm.hip) vs fp64 torch: one pass's
reduced block [G | g | stats] (the Gram matrix on the matrix cores), whole
fits vs the torch reference, run-to-run determinism, and the 30-date
induction quality."""
import math

import numpy as np
import pytest
import torch

from test_lm_cpu import _teacher_problem

pytestmark = pytest.mark.gpu

SHAPES = [(1, 8, 2, 0), (1, 8, 1, 1), (2, 8, 2, 0), (3, 8, 2, 0), (4, 8, 2, 0), (5, 8, 6, 0), (6, 8, 7, 0)]


def _lm_row(q, h):
    return (q & 3) + 8 * (q >> 2) + 4 * h


def decode_gram(red, P):
    """Dense G from the upper-triangular 32x32 blocks in MFMA register order."""
    NP = (P + 31) // 32 * 32
    NB = NP // 32
    G = np.zeros((NP, NP))
    b = 0
    for mb in range(NB):
        for nb in range(mb, NB):
            blk = red[b * 1024:(b + 1) * 1024]
            for q in range(16):
                for lane in range(64):
                    i = mb * 32 + _lm_row(q, lane >> 5)
                    j = nb * 32 + (lane & 31)
                    G[i, j] = G[j, i] = blk[q * 64 + lane]
            b += 1
    return G[:P, :P]


def _setup(shape, n, dev, seed=0):
    from rphedge.engine import DateData, HipBackend, TrainConfig
    from rphedge.models.hedge_mlp import NetSpec, init_weights

    spec = NetSpec(*shape)
    feats, pr, y = _teacher_problem(spec, n, seed)
    y = y + 0.05 * torch.sin(7 * feats[0])  # not exactly representable
    data = DateData(feats=[f.to(dev) for f in feats], prices_next=[p.to(dev) for p in pr], bond_next=1.01,
                    target=y.to(dev), prices_now=[p.to(dev) for p in pr], fmu=tuple([0.1] * spec.nin),
                    fisd=tuple([1.5] * spec.nin))
    w0 = init_weights(spec, [0.5] * spec.nout, seed=1)
    return spec, feats, pr, y, data, w0


@pytest.mark.parametrize("shape,n", [(s, 1 << 15) for s in SHAPES] + [((1, 8, 2, 0), 1 << 17), ((2, 8, 2, 0), 1 << 18)])
def test_lm_pass_block_matches_fp64(shape, n):
    """(2^17+ paths on the nets with two pass workgroups per CU: a 512-row
    packet reduction)"""
    from rphedge.engine import FitConfig, HipBackend, TrainConfig
    from rphedge.models.hedge_mlp import torch_forward
    from rphedge.ops import layout as L

    dev = torch.device("cuda", 0)
    spec, feats, pr, y, data, w0 = _setup(shape, n, dev)
    be = HipBackend(spec, n, TrainConfig(batch_size=n, lm_gram_paths=4096), device=dev)
    b = be._lm_buffers()
    w, o, f = be.new_weights(w0), be.new_opt(), be.new_fit()
    d = be._train_desc(w, o, f, data, FitConfig(), 0, None)
    d.batch, d.steps_per_epoch, d.shuffle, d.inv_batch = n, 1, 0, 1.0 / n
    lm = b["desc"]
    lm.passes = 1
    if n >= 1 << 17:
        wps = be.native.lm_pass_wps(*shape)
        assert wps == 2 and lm.num_wgs == 512
    be.native.lm_eval(d, lm, b["red"], 0, None)
    torch.cuda.synchronize()
    red = b["red"].cpu().numpy()
    P = spec.nparams
    ns = lm.gram_wgs * 64
    assert ns == 4096
    # fp64 reference
    X = (torch.stack(feats, 1).double() - 0.1) * 1.5
    Pm = torch.stack([p.double() for p in pr] + [torch.full((n,), 1.01, dtype=torch.float64)], 1)
    wt = torch.tensor(np.asarray(w0, np.float64), requires_grad=True)
    e = (torch_forward(spec, wt, X) * Pm).sum(1) - y.double()
    ((e * e).sum() / n).backward()
    from torch.func import jacrev, vmap

    sub = torch.tensor([(j // lm.gram_blk) * lm.gram_blk_stride + j % lm.gram_blk for j in range(ns)])
    assert lm.gram_blk == ns // 8 and lm.gram_blk_stride == n // 8
    J = vmap(jacrev(lambda ww, x, p: (torch_forward(spec, ww, x[None])[0] * p).sum()), in_dims=(None, 0, 0))(
        wt.detach(), X[sub], Pm[sub])
    G_ref = (J.T @ J).numpy() / ns
    G = decode_gram(red, P)
    assert np.linalg.norm(G - G_ref) / np.linalg.norm(G_ref) < 2e-5
    g = red[L.LM_GBLK_MAX:L.LM_GBLK_MAX + P]
    g_ref = wt.grad.numpy()
    assert np.linalg.norm(g - g_ref) / np.linalg.norm(g_ref) < 2e-5
    st = red[L.LM_GBLK_MAX + L.LM_NPMAX:L.LM_GBLK_MAX + L.LM_NPMAX + 4]
    assert st[0] == pytest.approx(float((e * e).sum()), rel=1e-5) and st[3] == n


@pytest.mark.parametrize("shape,damping", [((1, 8, 2, 0), "simple"), ((3, 8, 2, 0), "simple"),
                                           ((5, 8, 6, 0), "simple"), ((1, 8, 2, 0), "nielsen"),
                                           # padded tile grids (16 NT > PB: P = 97, 114, 130)
                                           ((1, 8, 1, 1), "simple"), ((2, 8, 2, 0), "simple"),
                                           ((4, 8, 2, 0), "simple"),
                                           ((3, 8, 2, 0), "nielsen")])
def test_lm_fit_matches_torch_and_is_deterministic(shape, damping):
    """HIP LM fit == fp64 torch reference (same accept / reject sequence and
    damping rule: simple x1/3 / x4, or Nielsen's gain-ratio update with the
    solve kernel's predicted reduction), bitwise run to run."""
    from rphedge.engine import FitConfig, HipBackend, TorchBackend, TrainConfig, current_weights

    dev = torch.device("cuda", 0)
    n = 1 << 14
    spec, feats, pr, y, data, w0 = _setup(shape, n, dev, seed=3)
    tc = TrainConfig(batch_size=n, lm_gram_paths=2048, lm_damping=damping)
    fc = FitConfig(epochs=12, optimizer="lm", early_stopping=False)
    outs = []
    for _ in range(2):
        be = HipBackend(spec, n, tc, device=dev)
        w, o, f = be.new_weights(w0), be.new_opt(), be.new_fit()
        be.fit(w, o, f, data, fc, seed=0)
        torch.cuda.synchronize()
        outs.append((current_weights(spec, w), f.cpu().numpy(), be.lm_state()))
    assert np.array_equal(outs[0][0], outs[1][0])           # bitwise reproducible (no float atomics)
    assert outs[0][2]["chol_failures"] == 0
    from rphedge.engine import DateData

    cd = DateData(feats=feats, prices_next=pr, bond_next=1.01, target=y, prices_now=pr, fmu=data.fmu, fisd=data.fisd)
    tb = TorchBackend(spec, n, tc)
    wc, oc, fcs = tb.new_weights(w0), tb.new_opt(), tb.new_fit()
    tb.fit(wc, oc, fcs, cd, fc, seed=0)
    hist_g = outs[0][1][2048 + 16:2048 + 16 + 13]
    hist_c = np.asarray(tb.lm_last["hist"])
    # the best-so-far losses follow the fp64 reference (same accept / reject
    # decisions; rejected trials far from the best point amplify the fp32 /
    # fp64 step difference, so they are not compared)
    np.testing.assert_allclose(np.minimum.accumulate(hist_g)[:8], np.minimum.accumulate(hist_c)[:8], rtol=2e-3)
    assert min(hist_g) == pytest.approx(min(hist_c), rel=2e-2)


@pytest.mark.parametrize("graph", [False, True])
def test_lm_adaptive_budget_matches_fixed_budget(graph):
    """Device-side adaptive pass budget (LmDesc.stop_tol, slot LSS_STOP): the
    fit stops at the pass the torch oracle stops at, the remaining launches
    return at once, and the result is BITWISE the fixed-budget fit of that
    many passes (weights, FitState epoch and loss history); eager and
    hipGraph-captured."""
    from rphedge.engine import FitConfig, HipBackend, TorchBackend, TrainConfig, current_weights, DateData
    from rphedge.ops import layout as L
    from rphedge.ops.native import Graph

    dev = torch.device("cuda", 0)
    n = 1 << 14
    spec, feats, pr, y, data, w0 = _setup((1, 8, 2, 0), n, dev, seed=3)
    tc = TrainConfig(batch_size=n, lm_gram_paths=2048)

    def fit(fc):
        be = HipBackend(spec, n, tc, device=dev)
        w, o, f = be.new_weights(w0), be.new_opt(), be.new_fit()
        if not graph:
            be.fit(w, o, f, data, fc, seed=0)
        else:
            s = torch.cuda.Stream()
            s.wait_stream(torch.cuda.current_stream())
            with torch.cuda.stream(s):
                be.fit(w, o, f, data, fc, seed=0)
                s.synchronize()
                w.copy_(be.new_weights(w0))
                f.zero_()
                g = Graph()
                g.capture_begin(s)
                try:
                    be.fit(w, o, f, data, fc, seed=0)
                finally:
                    g.capture_end()
                g.replay(s)
                s.synchronize()
        torch.cuda.synchronize()
        return current_weights(spec, w), f.cpu().numpy()

    fc_s = FitConfig(epochs=40, optimizer="lm", early_stopping=False, lm_stop_tol=0.02, lm_stop_min=3)
    w_s, f_s = fit(fc_s)
    k = int(f_s[L.F_EPOCH]) - 1
    assert 3 <= k < 40, k
    cd = DateData(feats=feats, prices_next=pr, bond_next=1.01, target=y, prices_now=pr, fmu=data.fmu, fisd=data.fisd)
    tb = TorchBackend(spec, n, tc)
    tb.fit(tb.new_weights(w0), tb.new_opt(), tb.new_fit(), cd, fc_s, seed=0)
    assert len(tb.lm_last["hist"]) - 1 == k
    w_f, f_f = fit(FitConfig(epochs=k, optimizer="lm", early_stopping=False))
    np.testing.assert_array_equal(w_s, w_f)
    np.testing.assert_array_equal(f_s[L.F_HIST:L.F_HIST + k + 1], f_f[L.F_HIST:L.F_HIST + k + 1])
    assert f_s[L.F_EPOCH] == f_f[L.F_EPOCH] and f_s[L.F_BEST] == f_f[L.F_BEST]


def test_lm_unsupported_shape_rejected_cleanly():
    """The 32-unit nets (P = 1,153) have no LM solver (the system does not fit
    one workgroup's LDS; every 8-unit net up to the 6-asset P = 191 does):
    lm_supported() is False, an LM fit raises ValueError before any launch,
    and the runtime is left without a pending HIP error."""
    from rphedge.engine import FitConfig, HipBackend, TrainConfig

    dev = torch.device("cuda", 0)
    n = 1 << 12
    spec, feats, pr, y, data, w0 = _setup((1, 32, 2, 0), n, dev)
    be = HipBackend(spec, n, TrainConfig(batch_size=n), device=dev)
    assert not be.lm_supported()
    with pytest.raises(ValueError):
        be.fit(be.new_weights(w0), be.new_opt(), be.new_fit(), data,
               FitConfig(epochs=2, optimizer="lm", early_stopping=False), seed=0)
    torch.zeros(8, device=dev).sum().item()  # no stale error surfaces here


def test_lm_induction_quality_on_gpu():
    """30-date European call, 2^18 paths, LM 80 / 3 passes: V0 at Black-
    Scholes, the last date's residual at the BS-delta floor (0.304) and a
    self-financing P&L near the BS delta hedge's (0.875)."""
    from rphedge.api import european_option

    r = european_option(N_paths=1 << 18, dt=1 / 30, rebalancing_frequency=1 / 30, batch_size=1 << 16,
                        verbose=False, device="cuda", early_stopping=False, q99=False, chunk_log2=6,
                        optimizer="lm", lm_passes_first=80, lm_passes_rest=3, keep_paths=False)
    assert abs(r.v0 - 10.3896) < 0.1, r.v0
    assert r.terminal_residual["std"] < 0.33, r.terminal_residual
    assert r.terminal_pnl["kind"] == "self_financing" and r.terminal_pnl["std"] < 1.0, r.terminal_pnl


@pytest.mark.parametrize("shape", [(1, 8, 2, 0), (3, 8, 2, 0), (5, 8, 6, 0)])
def test_bias_refit_matches_torch(shape):
    """HipBackend.bias_refit (k_lm_pass + k_lm_reduce + k_lm_solve with passes
    = 0, weights only) after a few Adam steps equals the torch reference
    refit (b_psi -= mean(e) / B); the full-batch residual mean is ~0 after it
    and the FitState record of the Adam fit is untouched."""
    from rphedge.engine import FitConfig, HipBackend, TorchBackend, TrainConfig
    from rphedge.models.hedge_mlp import torch_forward
    from rphedge.ops import layout as L

    dev = torch.device("cuda", 0)
    n = 1 << 14
    spec, feats, pr, y, data, w0 = _setup(shape, n, dev)
    be = HipBackend(spec, n, TrainConfig(batch_size=1 << 12), device=dev)
    w, o, f = be.new_weights(w0), be.new_opt(), be.new_fit()
    fc = FitConfig(epochs=2, early_stopping=False)
    be.fit(w, o, f, data, fc, seed=0)
    torch.cuda.synchronize()
    P = spec.nparams
    w_fit = w[:P].double().cpu()
    f_before = f.clone()
    be.bias_refit(w, o, f, data, fc)
    torch.cuda.synchronize()
    w_hip = w[:P].double().cpu()
    # torch reference on the same fitted weights
    tb = TorchBackend(spec, n, TrainConfig(batch_size=1 << 12))
    wt = tb.new_weights(w_fit.float().numpy())
    datac = type(data)(feats=[x.cpu() for x in data.feats], prices_next=[p.cpu() for p in data.prices_next],
                       bond_next=data.bond_next, target=data.target.cpu(), prices_now=None, fmu=data.fmu,
                       fisd=data.fisd)
    tb.bias_refit(wt, tb.new_opt(), tb.new_fit(), datac, fc)
    assert torch.equal(w_hip[:-1], w_fit[:-1])
    assert float(w_hip[-1]) == pytest.approx(float(wt[P - 1]), abs=2e-5)
    X = (torch.stack(feats, 1).double() - 0.1) * 1.5
    Pm = torch.stack([p.double() for p in pr] + [torch.full((n,), 1.01, dtype=torch.float64)], 1)
    e = (torch_forward(spec, w_hip, X) * Pm).sum(1) - y.double()
    assert abs(float(e.mean())) < 2e-5
    skip = set(range(L.F_WBEST, L.F_WBEST + P))
    fb, fa = f_before.cpu().view(torch.int32), f.cpu().view(torch.int32)   # bitwise (NaN-filled history)
    diff = [i for i in range(f.numel()) if i not in skip and int(fa[i]) != int(fb[i])]
    assert not diff, diff[:10]
