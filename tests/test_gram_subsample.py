"""The world-invariant LM Gram subsample (engine.gram_subsample): every rank
simulates the same global subsample paths (SimDesc.map_blk / map_stride,
ops.paths.path_indices) and builds the same Gram matrix, so the data-parallel
exchange carries only the gradient region (2.1 KB).  CPU: the numpy twins of
the mapped simulation equal a gather of the full simulation, for every model
family; the geometry is world-invariant; the torch LM oracle's 2-rank gloo fit
sees the same Gram matrix as the 1-rank fit."""
import numpy as np
import pytest
import torch

from rphedge.engine import gram_subsample
from rphedge.ops import paths as P


@pytest.mark.parametrize("n_total,want", [(1 << 20, (4096, 512, 1 << 17)), (1 << 12, (4096, 512, 512)),
                                          (1 << 10, (1024, 128, 128)), (3 << 10, (3072, 384, 384))])
def test_gram_subsample_geometry(n_total, want):
    ns, blk, stride = gram_subsample(n_total, 4096)
    assert (ns, blk, stride) == want
    idx = P.path_indices(ns, 0, (blk, stride))
    assert len(np.unique(idx)) == ns and idx.max() < n_total        # distinct global paths inside the run
    assert blk % 64 == 0 or ns < 512                                 # aligned blocks (sim kernel fast path)


def test_gram_subsample_is_world_invariant():
    """Aligned global blocks: rank r of W holds blocks [8r/W, 8(r+1)/W) whole,
    so the subsample is the union of the ranks' local prefixes at every W."""
    n_total = 1 << 16
    ns, blk, stride = gram_subsample(n_total, 4096)
    idx = set(P.path_indices(ns, 0, (blk, stride)).tolist())
    for W in (1, 2, 4, 8):
        per = n_total // W
        local = set()
        for r in range(W):
            local |= {i for i in idx if r * per <= i < (r + 1) * per}
        assert local == idx


def _gather(full, idx):
    return full[..., torch.as_tensor(idx.astype(np.int64))]


def test_mapped_simulation_equals_gather_gbm_heston_basket():
    g = P.Grid(1.0, 1 / 20, 1 / 5)
    n_total = 1 << 10
    ns, blk, stride = gram_subsample(n_total, 256)
    idx = P.path_indices(ns, 0, (blk, stride))
    for scheme in ("log", "arith"):
        full = P.simulate_gbm(g, n_total, 100.0, 0.08, 0.2, scheme=scheme, norm=100.0, device="cpu")
        sub = P.simulate_gbm(g, ns, 100.0, 0.08, 0.2, scheme=scheme, norm=100.0, device="cpu",
                             index_map=(blk, stride))
        assert torch.equal(sub.S, _gather(full.S, idx)) and torch.equal(sub.S_final, _gather(full.S_final, idx))
    kw = dict(model="heston", kappa=2.0, theta=0.04, xi=0.5, rho=-0.7, norm=100.0, device="cpu")
    full = P.simulate_sv(g, n_total, 100.0, 0.08, 0.04, **kw)
    sub = P.simulate_sv(g, ns, 100.0, 0.08, 0.04, index_map=(blk, stride), **kw)
    assert torch.equal(sub.S, _gather(full.S, idx)) and torch.equal(sub.vol, _gather(full.vol, idx))
    corr = np.full((3, 3), 0.5) + 0.5 * np.eye(3)
    full = P.simulate_basket(g, n_total, [100.0] * 3, [0.08] * 3, [0.2] * 3, corr, device="cpu")
    sub = P.simulate_basket(g, ns, [100.0] * 3, [0.08] * 3, [0.2] * 3, corr, device="cpu", index_map=(blk, stride))
    assert torch.equal(sub.S, _gather(full.S, idx))


def test_mapped_simulation_equals_gather_mortality():
    """Binomial deaths: the Philox counter is the GLOBAL path index."""
    g = P.Grid(2.0, 1 / 50, 1 / 4)
    n_total = 1 << 10
    ns, blk, stride = gram_subsample(n_total, 256)
    idx = P.path_indices(ns, 0, (blk, stride))
    full = P.simulate_mortality(P.simulate_gbm(g, n_total, 1.0, 0.08, 0.15, device="cpu"), 0.01, 0.075,
                                0.000597, 10000)
    sub = P.simulate_mortality(P.simulate_gbm(g, ns, 1.0, 0.08, 0.15, device="cpu", index_map=(blk, stride)),
                               0.01, 0.075, 0.000597, 10000)
    assert torch.equal(sub.nfrac, _gather(full.nfrac, idx)) and torch.equal(sub.lam, _gather(full.lam, idx))


def test_lm_oracle_same_gram_every_world_size():
    """TorchBackend LM fit with the simulated subsample: the Gram matrix does
    not depend on the shard (every rank gets the same G from the same paths),
    so a 1-rank fit with subsample data equals the 1-rank fit that reads the
    subsample from its shard, bit for bit."""
    from rphedge.engine import DateData, FitConfig, TorchBackend, TrainConfig
    from rphedge.models.hedge_mlp import NetSpec, init_weights

    spec = NetSpec(1, 8, 2, 0)
    g = P.Grid(1.0, 1 / 10, 1 / 10)
    n = 1 << 12
    p = P.simulate_gbm(g, n, 100.0, 0.08, 0.15, scheme="log", norm=100.0, device="cpu")
    ns, blk, stride = gram_subsample(n, 2048)
    gp = P.simulate_gbm(g, ns, 100.0, 0.08, 0.15, scheme="log", norm=100.0, device="cpu", index_map=(blk, stride))
    y = (p.S[-1] - 1.0).clamp_min(0)
    t = g.n_coarse - 2
    kw = dict(feats=p.features(t), prices_next=p.prices(t + 1), bond_next=1.0, target=y, prices_now=p.prices(t))
    res = []
    for side in (False, True):
        data = DateData(**kw, gram_feats=gp.features(t) if side else None,
                        gram_prices_next=gp.prices(t + 1) if side else None)
        be = TorchBackend(spec, n, TrainConfig(batch_size=n, shuffle=False, lm_gram_paths=2048))
        w, o, f = be.new_weights(init_weights(spec, [0.5, 0.0], seed=3)), be.new_opt(), be.new_fit()
        be.fit(w, o, f, data, FitConfig(epochs=8, optimizer="lm", early_stopping=False), seed=0)
        res.append((w.clone(), list(be.lm_last["hist"])))
    assert torch.equal(res[0][0], res[1][0]) and res[0][1] == res[1][1]
