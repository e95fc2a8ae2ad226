"""The world-invariant LM Gram subsample on the GPU: the path kernels with a
global index map (SimDesc.map_blk / map_stride) reproduce the shard's paths
bit for bit, and a pass grid with Gram-only workgroups (Gram subsample larger
than 64 x the path grid) builds the fp64 reference Gram matrix."""
import numpy as np
import pytest
import torch

from test_gpu_lm import decode_gram, _setup

pytestmark = pytest.mark.gpu


def _idx(ns, blk, stride, dev):
    from rphedge.ops.paths import path_indices

    return torch.as_tensor(path_indices(ns, 0, (blk, stride)).astype(np.int64), device=dev)


def test_mapped_path_kernels_are_the_shard_paths():
    from rphedge.engine import gram_subsample
    from rphedge.ops import paths as P

    dev = torch.device("cuda", 0)
    g = P.Grid(1.0, 1 / 60, 1 / 30)
    n = 1 << 16
    ns, blk, stride = gram_subsample(n, 4096)
    idx = _idx(ns, blk, stride, dev)
    full = P.simulate_gbm(g, n, 100.0, 0.08, 0.15, scheme="log", norm=100.0, device=dev)
    sub = P.simulate_gbm(g, ns, 100.0, 0.08, 0.15, scheme="log", norm=100.0, device=dev, index_map=(blk, stride))
    assert torch.equal(sub.S, full.S[:, idx]) and torch.equal(sub.S_final, full.S_final[idx])
    kw = dict(model="heston", kappa=2.0, theta=0.04, xi=0.5, rho=-0.7, norm=100.0, device=dev)
    full = P.simulate_sv(g, n, 100.0, 0.05, 0.04, **kw)
    sub = P.simulate_sv(g, ns, 100.0, 0.05, 0.04, index_map=(blk, stride), **kw)
    assert torch.equal(sub.S, full.S[:, idx]) and torch.equal(sub.vol, full.vol[:, idx])
    corr = np.full((5, 5), 0.5) + 0.5 * np.eye(5)
    full = P.simulate_basket(g, n, [100.0] * 5, [0.05] * 5, [0.2] * 5, corr, device=dev)
    sub = P.simulate_basket(g, ns, [100.0] * 5, [0.05] * 5, [0.2] * 5, corr, device=dev, index_map=(blk, stride))
    assert torch.equal(sub.S, full.S[:, :, idx])
    gm = P.Grid(2.0, 1 / 100, 1 / 4)
    full = P.simulate_mortality(P.simulate_gbm(gm, n, 1.0, 0.08, 0.15, device=dev), 0.01, 0.075, 0.000597, 10000)
    sub = P.simulate_mortality(P.simulate_gbm(gm, ns, 1.0, 0.08, 0.15, device=dev, index_map=(blk, stride)),
                               0.01, 0.075, 0.000597, 10000)
    assert torch.equal(sub.nfrac, full.nfrac[:, idx]) and torch.equal(sub.lam, full.lam[:, idx])


@pytest.mark.parametrize("side", [False, True])
def test_gram_only_workgroups_match_fp64(side):
    """n = 2^12 local paths: 16 path workgroups, a 4096-path Gram subsample =
    64 Gram workgroups (48 of them Gram-only).  G vs fp64 over the subsample,
    read from the shard or from the subsample data."""
    from rphedge.engine import FitConfig, HipBackend, TrainConfig, gram_subsample
    from rphedge.models.hedge_mlp import torch_forward
    from torch.func import jacrev, vmap

    dev = torch.device("cuda", 0)
    n = 1 << 12
    spec, feats, pr, y, data, w0 = _setup((1, 8, 2, 0), n, dev)
    ns, blk, stride = gram_subsample(n, 4096)
    idx = _idx(ns, blk, stride, dev)
    if side:
        data.gram_feats = [f.to(dev)[idx].contiguous() for f in feats]
        data.gram_prices_next = [p.to(dev)[idx].contiguous() for p in pr]
    be = HipBackend(spec, n, TrainConfig(batch_size=n, lm_gram_paths=4096), device=dev)
    b = be._lm_buffers()
    w, o, f = be.new_weights(w0), be.new_opt(), be.new_fit()
    d = be._train_desc(w, o, f, data, FitConfig(), 0, None)
    d.batch, d.steps_per_epoch, d.shuffle, d.inv_batch = n, 1, 0, 1.0 / n
    lm = b["desc"]
    be._lm_gram_mode(lm, data)
    lm.passes = 1
    assert lm.num_wgs == 16 and lm.gram_wgs == 64 and lm.gram_side == int(side)
    be.native.lm_eval(d, lm, b["red"], 0, None)
    torch.cuda.synchronize()
    red = b["red"].cpu().numpy()
    X = (torch.stack(feats, 1).double() - 0.1) * 1.5
    Pm = torch.stack([p.double() for p in pr] + [torch.full((n,), 1.01, dtype=torch.float64)], 1)
    wt = torch.tensor(np.asarray(w0, np.float64))
    J = vmap(jacrev(lambda ww, x, p: (torch_forward(spec, ww, x[None])[0] * p).sum()), in_dims=(None, 0, 0))(
        wt, X[idx.cpu()], Pm[idx.cpu()])
    G_ref = (J.T @ J).numpy() / ns
    G = decode_gram(red, spec.nparams)
    assert np.linalg.norm(G - G_ref) / np.linalg.norm(G_ref) < 2e-5
