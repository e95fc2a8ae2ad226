"""Saved-model format — the reference has no checkpointing.

A run directory holds::

    config.json                 params + parity flags
    weights_t{i:04d}.safetensors per backward date i, Keras layer names
                                (LeakyReLU_1/kernel [nin,8] ... Phi_Psi/bias [2]);
                                the Q99 network under the prefix "q99/"
    values.npy (optional)       V_t on the coarse grid
    report.json                 phi0, psi0, V0, VaRs, Errors, P_E_Values, epochs

Resume = reload the weights of the last finished date i (warm start, Q18) and
``values[i]`` and restart the backward scan at i-1 (:func:`load_date`).
"""
from __future__ import annotations

import json
import os

import numpy as np
import torch

from ..engine import current_weights
from ..models.hedge_mlp import fold_input_norm
from ..ops import layout as L


def _save_tensors(path: str, tensors: dict):
    from safetensors.numpy import save_file

    save_file({k: np.ascontiguousarray(v, dtype=np.float32) for k, v in tensors.items()}, path)


def _load_tensors(path: str) -> dict:
    from safetensors.numpy import load_file

    return load_file(path)


def save_weights(path: str, spec, w: np.ndarray, prefix: str = ""):
    _save_tensors(path, {prefix + k: v for k, v in spec.unflatten(w).items()})


def load_weights(path: str, spec, prefix: str = "") -> np.ndarray:
    t = _load_tensors(path)
    return spec.flatten({k: t[prefix + k] for k, _ in spec.shapes()})


def _gather_values(run, values: torch.Tensor) -> np.ndarray:
    """[n_coarse, n_total] on rank 0 from every rank's contiguous shard
    (collective when data parallel; shards are equal-sized, rank-ordered)."""
    w = run.di.world
    if w <= 1:
        return values.detach().cpu().numpy()
    import torch.distributed as dist

    v = values.detach().contiguous()
    if dist.get_backend() == "gloo":
        v = v.cpu()
    parts = [torch.empty_like(v) for _ in range(w)]
    dist.all_gather(parts, v)
    return torch.cat([p.cpu() for p in parts], dim=1).numpy()


def save_run(out_dir: str, run, res, save_values: bool = True):
    """Write the run directory (rank 0).  Collective when data parallel: the
    per-rank value shards are gathered so ``values.npy`` holds every path."""
    vals = None
    if save_values and res.induction.values is not None:
        vals = _gather_values(run, res.induction.values)
    if run.di.rank != 0:
        return
    os.makedirs(out_dir, exist_ok=True)
    spec = run.spec
    cfg = res.config
    with open(os.path.join(out_dir, "config.json"), "w") as f:
        json.dump({"config": cfg, "spec": {"nin": spec.nin, "hidden": spec.hidden, "nout": spec.nout,
                                           "head": spec.head, "alpha": spec.alpha,
                                           "layer_names": list(spec.layer_names)}}, f, indent=1, default=str)
    snap = res.induction.weights_snapshots
    norms = getattr(run.induction, "norms", None) or []
    if snap is not None:
        s = snap.detach().cpu()
        for i in range(s.shape[0]):
            mu, isd = norms[i] if norms else ((), ())  # fold input standardisation: raw-input weights

            def raw(k):
                return spec.unflatten(fold_input_norm(spec, current_weights(spec, s[i, k]), mu, isd))

            tensors = dict(raw(0))
            if run.cfg.train.q99:
                tensors.update({"q99/" + k: v for k, v in raw(1).items()})
            _save_tensors(os.path.join(out_dir, f"weights_t{i:04d}.safetensors"), tensors)
    if vals is not None:
        np.save(os.path.join(out_dir, "values.npy"), vals)
    rep = {"phi0": res.phi, "psi0": res.psi, "V0": res.v0, "VaR": res.var, "terminal_pnl": res.terminal_pnl,
           "Errors": res.errors.tolist(), "P_E_Values": res.p_e_values.tolist(), "summary": res.summary,
           "dates": [{"index": d.index, "time": d.time, "fit_mse": {k: v for k, v in d.fit_mse.items()
                                                                     if k != "history"},
                      "fit_q99": ({k: v for k, v in d.fit_q99.items() if k != "history"} if d.fit_q99 else None),
                      "mean_holdings": d.mean_holdings(spec.nhold).tolist(), "mean_value": d.mean_value,
                      "residual_std": d.residual_std} for d in res.induction.dates]}
    with open(os.path.join(out_dir, "report.json"), "w") as f:
        json.dump(rep, f, indent=1, default=float)


def load_date(out_dir: str, i: int):
    """(config dict, mse weights, q99 weights|None, values[i]|None) for resume."""
    from ..models.hedge_mlp import NetSpec

    with open(os.path.join(out_dir, "config.json")) as f:
        meta = json.load(f)
    sp = meta["spec"]
    spec = NetSpec(nin=sp["nin"], hidden=sp["hidden"], nout=sp["nout"], head=sp["head"], alpha=sp["alpha"],
                   layer_names=tuple(sp["layer_names"]))
    t = _load_tensors(os.path.join(out_dir, f"weights_t{i:04d}.safetensors"))
    w = spec.flatten({k: t[k] for k, _ in spec.shapes()})
    wq = spec.flatten({k: t["q99/" + k] for k, _ in spec.shapes()}) if ("q99/" + spec.shapes()[0][0]) in t else None
    vals = None
    vp = os.path.join(out_dir, "values.npy")
    if os.path.exists(vp):
        vals = np.load(vp, allow_pickle=False)[i]
    return meta, spec, w, wq, vals
