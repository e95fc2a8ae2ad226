"""Diagnostic: one LM pass (pass 0) on n paths vs fp64 torch: relative error
of the gradient, the loss sum and the path count of the reduced block.
usage: python tools/archive/pass_check.py [n_log2]"""
import json
import sys

import numpy as np
import torch

sys.path.insert(0, ".")
sys.path.insert(0, "tests")
from test_gpu_lm import _setup  # noqa: E402

from rphedge.engine import FitConfig, HipBackend, TrainConfig  # noqa: E402
from rphedge.models.hedge_mlp import torch_forward  # noqa: E402
from rphedge.ops import layout as L  # noqa: E402


def main(n_log2=20):
    dev = torch.device("cuda", 0)
    n = 1 << n_log2
    for shape in [(1, 8, 2, 0), (3, 8, 2, 0), (1, 8, 1, 1)]:
        spec, feats, pr, y, data, w0 = _setup(shape, n, dev)
        be = HipBackend(spec, n, TrainConfig(batch_size=n, lm_gram_paths=4096), device=dev)
        b = be._lm_buffers()
        w, o, f = be.new_weights(w0), be.new_opt(), be.new_fit()
        d = be._train_desc(w, o, f, data, FitConfig(), 0, None)
        d.batch, d.steps_per_epoch, d.shuffle, d.inv_batch = n, 1, 0, 1.0 / n
        lm = b["desc"]
        lm.passes = 1
        be.native.lm_eval(d, lm, b["red"], 0, None)
        torch.cuda.synchronize()
        red = b["red"].cpu().numpy()
        P = spec.nparams
        X = ((torch.stack(feats, 1).double() - 0.1) * 1.5).to(dev)
        Pm = torch.stack([p.double() for p in pr] + [torch.full((n,), 1.01, dtype=torch.float64)], 1).to(dev)
        wt = torch.tensor(np.asarray(w0, np.float64), requires_grad=True, device=dev)
        e = (torch_forward(spec, wt, X) * Pm).sum(1) - y.double().to(dev)
        ((e * e).sum() / n).backward()
        g = red[L.LM_GBLK_MAX:L.LM_GBLK_MAX + P]
        g_ref = wt.grad.cpu().numpy()
        st = red[L.LM_GBLK_MAX + L.LM_NPMAX:L.LM_GBLK_MAX + L.LM_NPMAX + 4]
        print(json.dumps({"shape": shape, "n": n, "nwgs": lm.num_wgs,
                          "g_rel": float(np.linalg.norm(g - g_ref) / np.linalg.norm(g_ref)),
                          "g_maxrel_entry": int(np.argmax(np.abs(g - g_ref))),
                          "loss_rel": float(st[0] / float((e * e).sum()) - 1), "count": float(st[3])}), flush=True)


if __name__ == "__main__":
    main(int(sys.argv[1]) if len(sys.argv) > 1 else 20)
