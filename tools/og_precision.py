"""Precision of the full-batch output-layer Gram matrix (k_lm_pass<BodyOG>,
csrc/hedge_narrow.h): the output-layer Newton step of lm_out_fix from a Gram
matrix built with bf16 operands, with the bf16 hi + lo split the kernel uses
(hi hi^T + hi lo^T + lo hi^T, fp32 accumulation), and in fp64.  CPU only.

    python tools/og_precision.py

Prints, per LM net shape, the condition number of the output Gram matrix and
the loss after the step (fp64 / bf16 / split) relative to the loss reduction
of the fp64 step.  Measured: bf16 operands alone leave 0.2-1.3 % of the
reduction on the table from the random init and move the step by 25-250x its
length (cond 1e9-1e18); the split matches fp64 to 1e-5."""
import os
import sys

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tests"))

from rphedge.models.hedge_mlp import torch_forward  # noqa: E402
from rphedge.ops import layout as L  # noqa: E402
from test_gpu_lm import _setup  # noqa: E402

F64 = torch.float64


def main(n=1 << 13):
    for shape in [(1, 8, 2, 0), (2, 8, 2, 0), (5, 8, 6, 0), (1, 8, 1, 1)]:
        spec, feats, pr, y, data, w0 = _setup(shape, n, "cpu", seed=7)
        X = (torch.stack([f.double() for f in feats], 1) - torch.tensor(data.fmu, dtype=F64)) * \
            torch.tensor(data.fisd, dtype=F64)
        bond = torch.full((n,), 1.01, dtype=F64)
        Pm = torch.stack([p.double() for p in pr] + [bond], 1) if spec.head == L.HEAD_FREE else \
            torch.stack([pr[0].double(), bond], 1)
        w = torch.tensor(np.asarray(w0, np.float64))
        o, h = spec.offsets, spec.hidden
        a1 = torch.nn.functional.leaky_relu(X @ w[o["W1"]:o["b1"]].view(spec.nin, h) + w[o["b1"]:o["W2"]], spec.alpha)
        a2 = torch.nn.functional.leaky_relu(a1 @ w[o["W2"]:o["b2"]].view(h, h) + w[o["b2"]:o["W3"]], spec.alpha)
        c = Pm if spec.head == L.HEAD_FREE else (Pm[:, 0] - Pm[:, 1])[:, None]
        u = torch.cat([(a2[:, :, None] * c[:, None, :]).reshape(n, -1), c], 1)

        def res(wv):
            return (torch_forward(spec, wv, X) * Pm).sum(1) - y.double()

        e = res(w)
        g = 2 * (u * e[:, None]).mean(0)

        def step(G):  # lm_out_newton's system: 2 G (1 + mu) + ridge
            A = 2 * G
            dg = torch.diagonal(A).clone()
            nu = A.shape[0]
            A = A + torch.diag(dg * 1e-6) + torch.eye(nu, dtype=F64) * (1e-10 * dg.sum() / nu)
            d = torch.linalg.solve(A, -g)
            wn = w.clone()
            wn[-nu:] += d
            return float((res(wn) ** 2).mean()), float(d.norm())

        uf = u.float()
        hi = uf.to(torch.bfloat16)
        lo = (uf - hi.float()).to(torch.bfloat16)
        hd, ld = hi.double(), lo.double()
        G64 = u.T @ u / n
        Gb = hd.T @ hd / n
        Gs = (hd.T @ hd + hd.T @ ld + ld.T @ hd) / n
        ev = torch.linalg.eigvalsh(G64).abs()
        l0 = float((e ** 2).mean())
        (l64, d64), (lb, db), (ls, ds) = step(G64), step(Gb), step(Gs)
        print(f"{shape}: cond {float(ev.max() / ev.min()):.2e}  loss {l0:.5g} -> fp64 {l64:.5g} | "
              f"bf16 {lb:.5g} (gap {(lb - l64) / (l0 - l64):.2e}, |d| x{db / d64:.0f}) | "
              f"split {ls:.5g} (gap {(ls - l64) / (l0 - l64):.2e}, |d| x{ds / d64:.3f})")


if __name__ == "__main__":
    main()
