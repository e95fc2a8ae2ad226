"""Hedge-ratio MLP family.

Reference architecture (``Replicating_Portfolio.py:149-161``):

    state(nin) -> Dense(8, LeakyReLU) -> Dense(8, LeakyReLU) -> Dense(nout) 'Phi_Psi'
    V = Dot([holdings, prices])                                  'V_t'

* pension: nin=3 ``[Y_t, N_t/N, lambda_t]``, nout=2 ``(phi, psi)`` -> 122 params
* European (EO cell 12): nin=1, Dense(1) 'Phi', ``psi = 1 - phi`` -> 97 params
  (``HEAD_COMPLEMENT``; quirk Q13) — corrected default is the free 2-output head.
* Heston (nin=2: S, v), basket-of-5 (nin=5, nout=6: 5 stocks + bond).

Parameters are stored as ONE flat float32 vector in Keras ``get_weights()``
order ``[W1(nin,h), b1, W2(h,h), b2, W3(h,nout), b3]`` — exactly the layout the
HIP kernels read (``csrc/hedge_mlp.hip::NetShape``) and the saved-model format
writes with Keras layer names (``rphedge/utils/model_io.py``).
"""
from __future__ import annotations

from dataclasses import dataclass, field

import numpy as np
import torch

from ..ops import layout as L
from ..ops.ndtri import ndtri_u30_f64
from ..ops.philox import philox4x32_10


@dataclass(frozen=True)
class NetSpec:
    nin: int = 3
    hidden: int = 8
    nout: int = 2
    head: int = L.HEAD_FREE
    alpha: float = 0.3                    # Keras-2 LeakyReLU default
    layer_names: tuple = ("LeakyReLU_1", "LeakyReLU_2", "Phi_Psi")

    @property
    def nhold(self) -> int:
        return 2 if self.head == L.HEAD_COMPLEMENT else self.nout

    @property
    def offsets(self) -> dict:
        h, nin, no = self.hidden, self.nin, self.nout
        o = {}
        o["W1"] = 0
        o["b1"] = o["W1"] + nin * h
        o["W2"] = o["b1"] + h
        o["b2"] = o["W2"] + h * h
        o["W3"] = o["b2"] + h
        o["b3"] = o["W3"] + h * no
        o["P"] = o["b3"] + no
        return o

    @property
    def nparams(self) -> int:
        return self.offsets["P"]

    @property
    def red_width(self) -> int:
        n = self.nparams + 4  # mirrors NetShape::R (csrc/hedge_core.h)
        return 128 if n <= 128 else 256 if n <= 256 else ((n + 255) // 256) * 256

    def shapes(self) -> list[tuple[str, tuple]]:
        h, nin, no = self.hidden, self.nin, self.nout
        n1, n2, n3 = self.layer_names
        return [(f"{n1}/kernel", (nin, h)), (f"{n1}/bias", (h,)), (f"{n2}/kernel", (h, h)),
                (f"{n2}/bias", (h,)), (f"{n3}/kernel", (h, no)), (f"{n3}/bias", (no,))]

    def unflatten(self, w) -> dict:
        w = np.asarray(w, dtype=np.float32)
        out, off = {}, 0
        for name, shp in self.shapes():
            n = int(np.prod(shp))
            out[name] = w[off:off + n].reshape(shp).copy()
            off += n
        return out

    def flatten(self, tensors: dict) -> np.ndarray:
        return np.concatenate([np.asarray(tensors[name], np.float32).reshape(-1) for name, _ in self.shapes()])


def fold_input_norm(spec: NetSpec, w, fmu, fisd) -> np.ndarray:
    """Weights on standardised inputs ``x' = (x - fmu) * fisd`` -> the same
    function on raw inputs (first layer only): ``W1r = diag(fisd) W1``,
    ``b1r = b1 - (fmu * fisd) @ W1``.  Saved models are always raw-input."""
    if not len(fmu):
        return np.asarray(w, np.float32).copy()
    o, h, nin = spec.offsets, spec.hidden, spec.nin
    w = np.asarray(w, np.float64).copy()
    W1 = w[o["W1"]:o["b1"]].reshape(nin, h)
    mu, isd = np.asarray(fmu, np.float64), np.asarray(fisd, np.float64)
    b1 = w[o["b1"]:o["W2"]] - (mu * isd) @ W1
    w[o["W1"]:o["b1"]] = (W1 * isd[:, None]).reshape(-1)
    w[o["b1"]:o["W2"]] = b1
    return w.astype(np.float32)


def unfold_input_norm(spec: NetSpec, w, fmu, fisd) -> np.ndarray:
    """Inverse of :func:`fold_input_norm` (raw-input weights -> standardised)."""
    if not len(fmu):
        return np.asarray(w, np.float32).copy()
    o, h, nin = spec.offsets, spec.hidden, spec.nin
    w = np.asarray(w, np.float64).copy()
    W1r = w[o["W1"]:o["b1"]].reshape(nin, h)
    mu, isd = np.asarray(fmu, np.float64), np.asarray(fisd, np.float64)
    w[o["b1"]:o["W2"]] = w[o["b1"]:o["W2"]] + mu @ W1r
    w[o["W1"]:o["b1"]] = (W1r / isd[:, None]).reshape(-1)
    return w.astype(np.float32)


PENSION = NetSpec(nin=3, hidden=8, nout=2, head=L.HEAD_FREE)
EUROPEAN_REF = NetSpec(nin=1, hidden=8, nout=1, head=L.HEAD_COMPLEMENT,
                       layer_names=("LeakyReLU_1", "LeakyReLU_2", "Phi"))
EUROPEAN = NetSpec(nin=1, hidden=8, nout=2, head=L.HEAD_FREE)
HESTON = NetSpec(nin=2, hidden=8, nout=2, head=L.HEAD_FREE)


def basket_spec(n_assets: int) -> NetSpec:
    return NetSpec(nin=n_assets, hidden=8, nout=n_assets + 1, head=L.HEAD_FREE)


def philox_normal(n: int, seed: int, stream: int = 0) -> np.ndarray:
    """Deterministic N(0,1) draws (host) — stand-in for Keras RandomNormal(seed)
    (TF's stateless RNG is not reproducible here: parity unpinned)."""
    i = np.arange(n, dtype=np.uint32)
    r = philox4x32_10(i, np.uint32(stream), 0x1A1A, 0, seed, 0xBEEF)
    x = (r[0] >> np.uint32(2)).astype(np.int64)  # 30-bit
    x = np.clip(x, 1, 2 ** 30 - 1)
    return ndtri_u30_f64(x)


def init_weights(spec: NetSpec, out_bias, seed: int = 1234, stddev: float = 0.1,
                 spread: bool = False, shared_stream: bool = False, align=None) -> np.ndarray:
    """Reference initialisation: kernels ~ N(0, 0.1) (seed 1234), hidden biases 0,
    output bias data-dependent (Q11: ``[1-p_oom, p_oom]`` pension,
    ``mean(payoff)/S0`` European).

    ``spread``: the first layer's breakpoints are spread over the
    standardised input range instead of all sitting at 0 (b1_j = -c_j |W1_j|,
    c_j evenly spaced in [-1.5, 1.5]), so a kinked target has hidden units
    near its kink from the start (an LM-mode option; the reference keeps
    zero biases).

    ``shared_stream``: every kernel is a prefix of ONE normal stream (the
    reference's single seeded initializer instance reused for all layers,
    RP:149 / :154-156, under a stateless seeded generator): W2 and W3 begin
    with W1's values (ParityFlags.shared_initializer).

    ``align`` (a direction in the standardised input space, e.g. the basket
    weights): every first-layer kernel column is turned towards +-align (its
    norm kept, 0.3 of its random direction left so the units stay distinct),
    so the hidden units start as functions of the payoff's own coordinate
    (the basket level) instead of random asset combinations; implies
    ``spread``."""
    o = spec.offsets
    w = np.zeros(spec.nparams, dtype=np.float32)
    for k, (name, shp) in enumerate(spec.shapes()):
        if name.endswith("kernel"):
            n = int(np.prod(shp))
            start = {0: o["W1"], 2: o["W2"], 4: o["W3"]}[k]
            w[start:start + n] = (stddev * philox_normal(n, seed, stream=0 if shared_stream else k)).astype(np.float32)
    if align is not None and spec.nin > 1:
        u = np.asarray(align, dtype=np.float64)[: spec.nin]
        u = u / np.linalg.norm(u)
        W1 = w[o["W1"]:o["b1"]].reshape(spec.nin, spec.hidden).astype(np.float64)
        nrm = np.linalg.norm(W1, axis=0)
        r = W1 / np.where(nrm > 0, nrm, 1.0)
        sg = np.where(u @ r >= 0.0, 1.0, -1.0)
        d = sg[None, :] * u[:, None] + 0.3 * r
        W1 = d / np.linalg.norm(d, axis=0) * nrm
        w[o["W1"]:o["b1"]] = W1.reshape(-1).astype(np.float32)
        spread = True
    if spread and spec.hidden > 1:
        W1 = w[o["W1"]:o["b1"]].reshape(spec.nin, spec.hidden).astype(np.float64)
        c = np.linspace(-1.5, 1.5, spec.hidden)
        w[o["b1"]:o["W2"]] = (-c * np.linalg.norm(W1, axis=0)).astype(np.float32)
    ob = np.broadcast_to(np.asarray(out_bias, dtype=np.float32), (spec.nout,))
    w[o["b3"]:o["b3"] + spec.nout] = ob
    return w


# ---------------------------------------------------------------------------
# torch reference forward (CPU oracle / tests)
# ---------------------------------------------------------------------------
def torch_forward(spec: NetSpec, w: torch.Tensor, x: torch.Tensor):
    """Holdings for states ``x`` [n, nin] with flat weights ``w``."""
    o = spec.offsets
    h, nin, no = spec.hidden, spec.nin, spec.nout
    W1 = w[o["W1"]:o["b1"]].view(nin, h)
    b1 = w[o["b1"]:o["W2"]]
    W2 = w[o["W2"]:o["b2"]].view(h, h)
    b2 = w[o["b2"]:o["W3"]]
    W3 = w[o["W3"]:o["b3"]].view(h, no)
    b3 = w[o["b3"]:o["P"]]
    a1 = torch.nn.functional.leaky_relu(x @ W1 + b1, spec.alpha)
    a2 = torch.nn.functional.leaky_relu(a1 @ W2 + b2, spec.alpha)
    out = a2 @ W3 + b3
    if spec.head == L.HEAD_COMPLEMENT:
        return torch.cat([out[:, :1], 1.0 - out[:, :1]], dim=1)
    return out


def torch_value(spec: NetSpec, w: torch.Tensor, x: torch.Tensor, prices: torch.Tensor):
    """V = holdings(x) . prices  (Keras Dot 'V_t')."""
    hold = torch_forward(spec, w, x)
    return (hold * prices).sum(dim=1), hold


@dataclass
class HedgeNet:
    """A network on a device: flat weights + spec (host convenience wrapper)."""

    spec: NetSpec
    weights: np.ndarray = field(default=None)

    def state_dict(self) -> dict:
        return self.spec.unflatten(self.weights)
