"""CPU oracle of the reference semantics (SURVEY §4 test plan, item 1).

Everything the GPU computes has a host twin with the same algorithm:

* Sobol points: :func:`rphedge.ops.sobol.sobol_uniform_cpu` (bit-exact scipy),
  inverse normal :mod:`rphedge.ops.ndtri`;
* path recursions: ``rphedge.ops.paths._cpu_*`` (fp64 numpy, same Sobol
  columns as the kernels, Q20 numpy binomial under parity);
* training: :class:`rphedge.engine.TorchBackend` (same Philox chunk
  permutation, Keras-Adam, EarlyStopping, device-state layout);
* the full pipeline: :func:`run_reference` = the public API on the torch
  backend.
"""
from __future__ import annotations

from ..api import RunResult, run_params


def run_reference(params: dict, sv: bool = False, parity: bool = True, dtype: str = "fp32") -> RunResult:
    """Run a params dict through the CPU oracle (torch backend, numpy paths)."""
    p = dict(params)
    p.setdefault("device", "cpu")
    p.setdefault("backend", "torch")
    if parity:
        p["parity"] = True
    return run_params(p, sv=sv)


def sobol_norm(m: int, d: int = 1, seed: int = 1234):
    """``sobol_norm`` of the reference (RP:54-57) on the host (float64 ndarray)."""
    from ..ops.sobol import sobol_norm_cpu

    return sobol_norm_cpu(m, d, seed)
