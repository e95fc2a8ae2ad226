"""Risk & diagnostics (C23, C28–C31; kernel K13).

* :func:`quantile` — exact ``np.quantile(x, q)`` ('linear' interpolation) via
  a 3-pass radix select over monotone float keys.  On the GPU each pass is one
  HIP histogram kernel (LDS histogram + one atomic per bin); with data
  parallelism the 2048-bin histogram (8 KB) is all-reduced instead of
  gathering residuals (§2.5: 16 KB class messages, latency-bound).
* :func:`var_report` — per-date and overall residual VaR (RP:122,
  "Multi Time Step.ipynb":961-968).
"""
from __future__ import annotations

import math

import numpy as np
import torch

_PASSES = ((21, 2048), (10, 2048), (0, 1024))


def _key_to_float(k: int) -> float:
    k &= 0xFFFFFFFF
    b = (k & 0x7FFFFFFF) if (k & 0x80000000) else (~k & 0xFFFFFFFF)
    return float(np.array([b], dtype=np.uint32).view(np.float32)[0])


def _hist_pass(x: torch.Tensor, pmask: int, prefix: int, shift: int, nbins: int, world: int) -> np.ndarray:
    if x.is_cuda:
        from .ops import native

        h = torch.zeros(nbins, dtype=torch.int32, device=x.device)
        native.radix_hist(x, pmask, prefix, shift, nbins, h)
    else:
        b = x.detach().contiguous().view(torch.int32).numpy().view(np.uint32)
        k = np.where(b & 0x80000000, ~b, b | 0x80000000).astype(np.uint32)
        sel = (k & np.uint32(pmask)) == np.uint32(prefix)
        h = torch.from_numpy(np.bincount(((k[sel] >> np.uint32(shift)) & np.uint32(nbins - 1)).astype(np.int64),
                                         minlength=nbins).astype(np.int32))
    if world > 1:
        from .parallel.dist import all_reduce_

        all_reduce_(h)
    return h.cpu().numpy().astype(np.int64)


def kth_smallest_many(x: torch.Tensor, ks, world: int = 1) -> list[float]:
    """Exact k-th smallest (0-based) float32 values over all ranks for several
    k at once: per radix pass one histogram per DISTINCT key prefix (the first
    pass is shared by every k; neighbouring order statistics usually share
    all three), so a 3-level VaR report costs a handful of histogram passes
    instead of 3 per order statistic.  Every rank derives the same prefixes
    from the all-reduced histograms, so the collective sequence matches."""
    st = [[0, 0, int(k)] for k in ks]  # pmask, prefix, remaining rank
    for shift, nbins in _PASSES:
        cache = {}
        for e in st:
            key = (e[0], e[1])
            if key not in cache:
                cache[key] = np.cumsum(_hist_pass(x, e[0], e[1], shift, nbins, world))
            c = cache[key]
            b = int(np.searchsorted(c, e[2] + 1))
            e[2] -= int(c[b - 1]) if b > 0 else 0
            e[1] |= b << shift
            e[0] |= (nbins - 1) << shift
    return [_key_to_float(e[1]) for e in st]


def kth_smallest(x: torch.Tensor, k: int, world: int = 1) -> float:
    """Exact k-th smallest (0-based) float32 value over all ranks."""
    return kth_smallest_many(x, [k], world)[0]


def quantile(x: torch.Tensor, qs, world: int = 1, n_total: int | None = None) -> np.ndarray:
    """np.quantile(x, qs) with linear interpolation, exact for float32 data
    (all order statistics selected together, :func:`kth_smallest_many`)."""
    x = x.reshape(-1).float()
    n = int(n_total) if n_total is not None else x.numel() * world
    plan = []
    for q in np.atleast_1d(qs):
        h = (n - 1) * float(q)
        lo = int(math.floor(h))
        plan.append((h, lo, lo + 1 < n and h > lo))
    ks = sorted({lo for _, lo, _ in plan} | {lo + 1 for _, lo, two in plan if two})
    val = dict(zip(ks, kth_smallest_many(x, ks, world)))
    out = []
    for h, lo, two in plan:
        a = val[lo]
        out.append(a + (h - lo) * (val[lo + 1] - a) if two else a)
    return np.asarray(out)


def var_report(residuals: torch.Tensor, scale: float = 1.0, qs=(0.985, 0.99, 0.995), world: int = 1) -> dict:
    """Overall VaR over all dates' residuals (EO :3733-3740, MTS :961-968)."""
    v = quantile(residuals, qs, world) * scale
    return {f"VaR({q * 100:.1f}%)": float(x) for q, x in zip(qs, v)}


def describe(x: torch.Tensor, scale: float = 1.0, world: int = 1) -> dict:
    """pandas-like describe() of a residual vector (C31)."""
    xd = x.reshape(-1).double()
    n = torch.tensor([xd.numel()], dtype=torch.float64, device=xd.device)
    s = torch.stack([xd.sum(), (xd * xd).sum()])
    mn, mx = xd.min().reshape(1), xd.max().reshape(1)
    if world > 1:
        from .parallel.dist import all_reduce_

        all_reduce_(n)
        all_reduce_(s)
        all_reduce_(mn, "min")
        all_reduce_(mx, "max")
    N = float(n.item())
    mean = float(s[0].item()) / N
    var = max(float(s[1].item()) / N - mean * mean, 0.0) * N / max(N - 1, 1)
    q = quantile(x, (0.25, 0.5, 0.75), world)
    return {"count": N, "mean": mean * scale, "std": math.sqrt(var) * scale, "min": float(mn.item()) * scale,
            "25%": q[0] * scale, "50%": q[1] * scale, "75%": q[2] * scale, "max": float(mx.item()) * scale}
