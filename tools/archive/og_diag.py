"""GPU diagnostic of the full-batch output-layer Gram (k_lm_pass<BodyOG> +
k_lm_reduce): one output-Gram pass at several path counts, the packed Gram
matrix and the gradient against fp64 torch on the same data.

    python tools/archive/og_diag.py [log2 ...]
"""
import os
import sys

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tests"))

from rphedge.engine import FitConfig, HipBackend, TrainConfig, lm_out_nu  # noqa: E402
from rphedge.models.hedge_mlp import torch_forward  # noqa: E402
from rphedge.ops import layout as L  # noqa: E402
from test_gpu_lm import _setup  # noqa: E402

F64 = torch.float64


def one(shape, n, dev):
    spec, feats, pr, y, data, w0 = _setup(shape, n, dev, seed=7)
    be = HipBackend(spec, n, TrainConfig(batch_size=n, lm_gram_paths=4096, lm_out_fix=True), device=dev)
    b = be._lm_buffers()
    w, o, f = be.new_weights(w0), be.new_opt(), be.new_fit()
    d = be._train_desc(w, o, f, data, FitConfig(), 0, None)
    d.batch, d.steps_per_epoch, d.shuffle, d.inv_batch = n, 1, 0, 1.0 / n
    lm = b["desc"]
    be._lm_gram_mode(lm, data)
    lm.passes = 1
    be.native.lm_eval(d, lm, b["red"], 0, None)
    torch.cuda.synchronize()
    red = b["red"].cpu().numpy()
    NU = lm_out_nu(spec)
    pk = red[L.LM_RED_OUTG:L.LM_RED_OUTG + NU * (NU + 1) // 2]
    G = np.zeros((NU, NU))
    e = 0
    for i in range(NU):
        for j in range(i, NU):
            G[i, j] = G[j, i] = pk[e]
            e += 1
    X = ((torch.stack([f.double() for f in feats], 1) - torch.tensor(data.fmu, dtype=F64)) *
         torch.tensor(data.fisd, dtype=F64)).to(dev)
    bond = torch.full((n,), 1.01, dtype=F64, device=dev)
    Pm = torch.stack([p.double().to(dev) for p in pr] + [bond], 1) if spec.head == L.HEAD_FREE else \
        torch.stack([pr[0].double().to(dev), bond], 1)
    wt = torch.tensor(np.asarray(w0, np.float64), device=dev)
    o_, h = spec.offsets, spec.hidden
    a1 = torch.nn.functional.leaky_relu(X @ wt[o_["W1"]:o_["b1"]].view(spec.nin, h) + wt[o_["b1"]:o_["W2"]], spec.alpha)
    a2 = torch.nn.functional.leaky_relu(a1 @ wt[o_["W2"]:o_["b2"]].view(h, h) + wt[o_["b2"]:o_["W3"]], spec.alpha)
    c = Pm if spec.head == L.HEAD_FREE else (Pm[:, 0] - Pm[:, 1])[:, None]
    u = torch.cat([(a2[:, :, None] * c[:, None, :]).reshape(n, -1), c], 1)
    Gr = (u.T @ u / n).cpu().numpy()
    err = np.abs(G - Gr) / np.sqrt(np.outer(np.diag(Gr), np.diag(Gr)))
    i, j = np.unravel_index(np.argmax(err), err.shape)
    res = (torch_forward(spec, wt, X) * Pm).sum(1) - y.double().to(dev)
    go = (2 * (u * res[:, None]).mean(0)).cpu().numpy()
    g = red[L.LM_GBLK_MAX:L.LM_GBLK_MAX + spec.nparams][-NU:]
    print(f"{shape} n=2^{int(np.log2(n))}: OG marker {red[L.LM_RED_OUTG]:.3g}  max rel err {err.max():.2e} at ({i},{j}) "
          f"got {G[i, j]:.6g} want {Gr[i, j]:.6g}  median {np.median(err):.2e}  |g_o err| {np.abs(g - go).max():.2e} "
          f"(|g_o| {np.abs(go).max():.2e})", flush=True)


def main(argv):
    dev = torch.device("cuda", 0)
    logs = [int(a) for a in argv] or [13, 16, 18, 20]
    for shape in [(1, 8, 2, 0), (5, 8, 6, 0), (1, 8, 1, 1)]:
        for k in logs:
            one(shape, 1 << k, dev)


if __name__ == "__main__":
    main(sys.argv[1:])
