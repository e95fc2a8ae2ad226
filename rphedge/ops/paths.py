"""Path simulation (K3–K7) on the device, plus a numpy oracle.

Output is a :class:`Paths` object holding ONLY the coarse rebalancing grid,
time-major ``[n_coarse, n_local]`` float32 (per asset for baskets), normalised
prices, the deterministic bank account ``B_t`` (C07, RP:67-69) and the
terminal fine-grid values used for the payoff (RP:88 computes the payoff
before subsampling).

Reference call sites: fund GBM RP:59-65 (C04), EO log-GBM (C05), SV RP:273-289
(C06), mortality RP:71-84 (C08, C09), decimation RP:91-97 (C11).
"""
from __future__ import annotations

import math
from dataclasses import dataclass, field

import numpy as np
import torch

from . import layout as L
from .sobol import sobol_table, device_table
from .ndtri import ndtri_u30_f64, ndtri_u30_f32
from .philox import philox4x32_10, u01d

SEED_W1 = 1235   # fund / stock shocks (RP:60)
SEED_W2 = 1234   # mortality shocks (RP:72) — also W_SV in the SV model (Q7)


@dataclass
class Grid:
    T: float
    dt: float
    rebalancing: float

    @property
    def n_fine(self) -> int:
        return int(math.ceil(self.T / self.dt) + 1)

    @property
    def reduction(self) -> int:
        return max(1, int(math.floor((self.n_fine - 1) / (self.T / self.rebalancing))))

    @property
    def n_coarse(self) -> int:
        return int(math.ceil(self.n_fine / self.reduction))

    @property
    def dt_coarse(self) -> float:
        return self.dt * self.reduction

    def times(self) -> np.ndarray:
        return np.arange(self.n_coarse) * self.dt * self.reduction

    def bond(self, r: float, norm: float = 1.0) -> np.ndarray:
        """B_t = exp(r t) on the fine linspace, subsampled (RP:68, :94)."""
        fine = np.exp(r * np.linspace(0, self.T, self.n_fine))
        return (fine[:: self.reduction] / norm).astype(np.float64)


@dataclass
class Paths:
    kind: str
    grid: Grid
    n_local: int
    path_offset: int
    S: torch.Tensor                      # [n_coarse, n] or [n_coarse, na, n]
    bond: np.ndarray                     # [n_coarse]
    S_final: torch.Tensor                # [n] or [na, n]  terminal fine value
    vol: torch.Tensor | None = None      # [n_coarse, n] (SV / Heston)
    nfrac: torch.Tensor | None = None    # [n_coarse, n] N_t/N (pension)
    lam: torch.Tensor | None = None      # [n_coarse, n]
    nfrac_final: torch.Tensor | None = None
    norm: float = 1.0
    na: int = 1
    meta: dict = field(default_factory=dict)

    @property
    def n_coarse(self) -> int:
        return self.S.shape[0]

    def asset(self, t: int, a: int = 0) -> torch.Tensor:
        return self.S[t, a] if self.S.dim() == 3 else self.S[t]

    def prices(self, t: int) -> list:
        return [self.asset(t, a) for a in range(self.na)]

    def features(self, t: int) -> list:
        if self.kind == "pension":
            return [self.S[t], self.nfrac[t], self.lam[t]]
        if self.kind in ("heston", "sv"):
            return [self.S[t], self.vol[t]]
        return self.prices(t)


def _dev_is_gpu(device) -> bool:
    return torch.device(device).type == "cuda"


# ---------------------------------------------------------------------------
# device simulation
# ---------------------------------------------------------------------------
def path_indices(n_local: int, offset: int, index_map=None) -> np.ndarray:
    """Global (Sobol / Philox) indices of the local paths: ``offset + p``, or
    with ``index_map = (blk, stride)`` ``offset + (p // blk) * stride + p % blk``
    (the LM Gram subsample: the first ``blk`` paths of aligned global blocks,
    simulated on every rank; csrc/paths.hip sim_gidx)."""
    p = np.arange(int(n_local), dtype=np.uint64)
    if index_map is None:
        return p + np.uint64(offset)
    blk, stride = (int(v) for v in index_map)
    return np.uint64(offset) + (p // np.uint64(blk)) * np.uint64(stride) + p % np.uint64(blk)


def _desc(model, n_local, offset, grid: Grid, fp64, parity, index_map=None):
    from . import native

    d = native.SimDesc()
    d.model = model
    d.n_local = int(n_local)
    d.path_offset = int(offset)
    if index_map is not None:
        d.map_blk, d.map_stride = (int(v) for v in index_map)
    d.n_fine = grid.n_fine
    d.reduction = grid.reduction
    d.n_coarse = grid.n_coarse
    d.na = 1
    d.fp64 = 1 if fp64 else 0
    d.parity = 1 if parity else 0
    d.dt = float(grid.dt)
    return d


def simulate_gbm(grid: Grid, n_local: int, s0: float, mu: float, sigma: float, scheme: str = "arith",
                 norm: float = 1.0, device="cuda", offset: int = 0, fp64: bool = False, seed: int = SEED_W1,
                 stream=None, out: Paths | None = None, index_map=None) -> Paths:
    """Fund/stock GBM on the fine grid, stored on the coarse grid (K1+K2+K3).

    ``out``: re-simulate into the buffers of an existing :class:`Paths`
    (no allocation: graph-capturable).  ``index_map``: (blk, stride) global
    path-index map (:func:`path_indices`)."""
    dev = torch.device(device)
    S = out.S if out is not None else torch.empty(grid.n_coarse, n_local, dtype=torch.float32, device=dev)
    fin = out.S_final if out is not None else torch.empty(n_local, dtype=torch.float32, device=dev)
    if _dev_is_gpu(dev):
        from . import native

        sv, sh, dims = device_table(grid.n_fine, seed, dev)
        d = _desc(L.SIM_GBM_LOG if scheme == "log" else L.SIM_GBM_ARITH, n_local, offset, grid, fp64, False,
                  index_map)
        d.sv1, d.shift1, d.dims1 = sv.data_ptr(), sh.data_ptr(), dims
        d.s0[0], d.mu[0], d.sigma[0], d.inv_norm[0] = s0, mu, sigma, 1.0 / norm
        d.out, d.final_out = S.data_ptr(), fin.data_ptr()
        native.simulate(d, stream)
    else:
        s_np, f_np = _cpu_gbm(grid, n_local, s0, mu, sigma, scheme, offset, seed, index_map)
        S.copy_(torch.from_numpy((s_np / norm).astype(np.float32)))
        fin.copy_(torch.from_numpy((f_np / norm).astype(np.float32)))
    if out is not None:
        return out
    p = Paths(kind="gbm", grid=grid, n_local=n_local, path_offset=offset, S=S, bond=grid.bond(0.0),
              S_final=fin, norm=norm)
    p.meta["index_map"] = index_map
    return p


def simulate_sv(grid: Grid, n_local: int, s0: float, mu: float, v0: float, model: str = "sv_ref",
                a=0.0, b=0.0, c=0.0, kappa=0.0, theta=0.0, xi=0.0, rho=0.0, norm: float = 1.0,
                device="cuda", offset: int = 0, fp64: bool = False, parity_nan: bool = False,
                seed1: int = SEED_W1, seed2: int = SEED_W2, stream=None, out: Paths | None = None,
                scheme: str = "qe", sv_tscale: float = 0.0, joint: bool | None = None, index_map=None) -> Paths:
    """Reference CIR-on-sigma SV (RP:282-289) or Heston (K4).

    ``scheme`` (Heston): "qe" = Andersen quadratic-exponential variance step
    with the martingale-corrected log-price step (default: no visible
    discretisation bias at 10 steps per date), "euler" = full-truncation Euler.
    ``sv_tscale`` (SV_REF): 0 = the reference recursion (Q5); > 0 = corrected
    CIR-on-sigma with the calibrated daily (a, b, c) applied over
    ``dt * sv_tscale`` calibration days per fine step."""
    if scheme not in ("qe", "euler"):
        raise ValueError(f"heston scheme must be qe | euler, got {scheme!r}")
    if model == "heston" and scheme == "qe" and not (kappa > 0 and xi > 0):
        scheme = "euler"  # QE needs a mean-reverting, stochastic variance
    # The reference draws W1 and W_SV from two separately scrambled Sobol
    # sequences of the SAME dimensions (RP:274-275): dimension t of both is a
    # bijective re-scrambling of one coordinate, so the two shocks of a step are
    # deterministically paired, not independent (it biased the Heston price by
    # about -1 % with QE, +1.3 % with Euler).  Heston and the corrected SV model
    # draw both shocks from ONE sequence of 2 n_fine dimensions instead; the
    # reference SV recursion keeps the reference's two sequences.
    # (``joint``: None = by model; ParityFlags.paired_sobol selects it in the API)
    if joint is None:
        joint = model == "heston" or (model == "sv_ref" and sv_tscale > 0)
    dev = torch.device(device)
    S = out.S if out is not None else torch.empty(grid.n_coarse, n_local, dtype=torch.float32, device=dev)
    V = out.vol if out is not None else torch.empty(grid.n_coarse, n_local, dtype=torch.float32, device=dev)
    fin = out.S_final if out is not None else torch.empty(n_local, dtype=torch.float32, device=dev)
    mcode = L.SIM_SV_REF if model == "sv_ref" else L.SIM_HESTON
    if _dev_is_gpu(dev):
        from . import native

        d = _desc(mcode, n_local, offset, grid, fp64, parity_nan, index_map)
        nf = grid.n_fine
        if joint:
            # ONE Sobol sequence of 2 n_fine dimensions: price shocks at dims
            # [0, nf), variance shocks at [nf, 2 nf) - jointly equidistributed
            sv, sh, dd = device_table(2 * nf, seed1, dev)
            d.sv1, d.shift1, d.dims1 = sv.data_ptr(), sh.data_ptr(), nf
            d.sv2, d.shift2, d.dims2 = sv.data_ptr() + nf * 32 * 4, sh.data_ptr() + nf * 4, nf
        else:
            sv1, sh1, d1 = device_table(nf, seed1, dev)
            sv2, sh2, d2 = device_table(nf, seed2, dev)
            d.sv1, d.shift1, d.dims1 = sv1.data_ptr(), sh1.data_ptr(), d1
            d.sv2, d.shift2, d.dims2 = sv2.data_ptr(), sh2.data_ptr(), d2
        d.s0[0], d.mu[0], d.inv_norm[0] = s0, mu, 1.0 / norm
        d.v0, d.a, d.b, d.c = v0, a, b, c
        d.kappa, d.theta, d.xi, d.rho = kappa, theta, xi, rho
        d.sv_tscale = float(sv_tscale) if model == "sv_ref" else 0.0
        d.scheme = L.HESTON_QE if scheme == "qe" else L.HESTON_EULER
        d.out, d.out2, d.final_out = S.data_ptr(), V.data_ptr(), fin.data_ptr()
        native.simulate(d, stream)
    else:
        s_np, v_np, f_np = _cpu_sv(grid, n_local, s0, mu, v0, model, a, b, c, kappa, theta, xi, rho, offset,
                                   parity_nan, seed1, seed2, scheme=scheme,
                                   sv_tscale=float(sv_tscale) if model == "sv_ref" else 0.0, joint=joint,
                                   index_map=index_map)
        S.copy_(torch.from_numpy((s_np / norm).astype(np.float32)))
        V.copy_(torch.from_numpy(v_np.astype(np.float32)))
        fin.copy_(torch.from_numpy((f_np / norm).astype(np.float32)))
    if out is not None:
        return out
    p = Paths(kind="heston" if model == "heston" else "sv", grid=grid, n_local=n_local, path_offset=offset,
              S=S, vol=V, bond=grid.bond(0.0), S_final=fin, norm=norm)
    p.meta["index_map"] = index_map
    return p


def simulate_basket(grid: Grid, n_local: int, s0, mu, sigma, corr, norm=None, device="cuda", offset: int = 0,
                    seed: int = SEED_W1, stream=None, out: Paths | None = None, index_map=None) -> Paths:
    """Correlated log-GBM basket (K3 basket variant)."""
    na = len(s0)
    norm = np.asarray(norm if norm is not None else s0, dtype=np.float64)
    C = np.asarray(corr, dtype=np.float64)
    chol = np.linalg.cholesky(C)
    dev = torch.device(device)
    S = out.S if out is not None else torch.empty(grid.n_coarse, na, n_local, dtype=torch.float32, device=dev)
    fin = out.S_final if out is not None else torch.empty(na, n_local, dtype=torch.float32, device=dev)
    if _dev_is_gpu(dev):
        from . import native

        sv, sh, dims = device_table(na * grid.n_fine, seed, dev)
        d = _desc(L.SIM_BASKET, n_local, offset, grid, False, False, index_map)
        d.na = na
        d.sv1, d.shift1, d.dims1 = sv.data_ptr(), sh.data_ptr(), dims
        for i in range(na):
            d.s0[i], d.mu[i], d.sigma[i], d.inv_norm[i] = float(s0[i]), float(mu[i]), float(sigma[i]), 1.0 / norm[i]
        for i in range(na):
            for j in range(na):
                d.chol[i * 8 + j] = float(chol[i, j])
        d.out, d.final_out = S.data_ptr(), fin.data_ptr()
        native.simulate(d, stream)
    else:
        s_np, f_np = _cpu_basket(grid, n_local, s0, mu, sigma, chol, offset, seed, index_map)
        S.copy_(torch.from_numpy((s_np / norm[None, :, None]).astype(np.float32)))
        fin.copy_(torch.from_numpy((f_np / norm[:, None]).astype(np.float32)))
    if out is not None:
        return out
    p = Paths(kind="basket", grid=grid, n_local=n_local, path_offset=offset, S=S, bond=grid.bond(0.0),
              S_final=fin, norm=float(norm[0]), na=na)
    p.meta["norms"] = norm
    p.meta["index_map"] = index_map
    return p


def simulate_mortality(paths: Paths, l0: float, c: float, eta: float, n0: int, lambda_fine_index: bool = False,
                       device=None, fp64: bool = False, seed: int = SEED_W2, philox_seed: int = 1234,
                       numpy_binomial: bool = False, stream=None) -> Paths:
    """Mortality intensity + binomial survivors (K5+K6); attaches nfrac/lam to ``paths``."""
    grid, n_local, offset = paths.grid, paths.n_local, paths.path_offset
    dev = paths.S.device if device is None else torch.device(device)
    reuse = paths.nfrac is not None and paths.lam is not None and paths.meta.get("nfrac_final_buf") is not None
    NF = paths.nfrac if reuse else torch.empty(grid.n_coarse, n_local, dtype=torch.float32, device=dev)
    LM = paths.lam if reuse else torch.empty(grid.n_coarse, n_local, dtype=torch.float32, device=dev)
    NT = paths.meta["nfrac_final_buf"] if reuse else torch.empty(n_local, dtype=torch.float32, device=dev)
    if _dev_is_gpu(dev):
        from . import native

        sv, sh, dims = device_table(grid.n_fine, seed, dev)
        d = _desc(L.SIM_MORTALITY, n_local, offset, grid, fp64, lambda_fine_index, paths.meta.get("index_map"))
        d.sv2, d.shift2, d.dims2 = sv.data_ptr(), sh.data_ptr(), dims
        d.l0, d.lc, d.eta, d.n0, d.seed = l0, c, eta, int(n0), int(philox_seed)
        d.out2, d.out3, d.final2_out = NF.data_ptr(), LM.data_ptr(), NT.data_ptr()
        native.simulate(d, stream)
    else:
        nf, lm, nt = _cpu_mortality(grid, n_local, l0, c, eta, n0, lambda_fine_index, offset, seed, philox_seed,
                                    numpy_binomial, paths.meta.get("index_map"))
        NF.copy_(torch.from_numpy(nf.astype(np.float32)))
        LM.copy_(torch.from_numpy(lm.astype(np.float32)))
        NT.copy_(torch.from_numpy(nt.astype(np.float32)))
    paths.kind = "pension"
    paths.nfrac, paths.lam, paths.nfrac_final = NF, LM, NT
    paths.meta["nfrac_final_buf"] = NT
    return paths


def payoff(kind: str, paths: Paths, strike: float, weights=None, stream=None, out: torch.Tensor | None = None
           ) -> torch.Tensor:
    """Terminal value V_T in normalised units (K7); ``out`` reuses a buffer."""
    S = paths.S_final
    n = paths.n_local
    if out is None:
        out = torch.empty(n, dtype=torch.float32, device=S.device)
    code = {"guarantee": 0, "call": 1, "put": 2, "basket_call": 3}[kind]
    if S.is_cuda:
        from . import native

        w = None
        if code == 3:  # cached per Paths: no host->device copy on re-simulation (graph capture)
            key = ("basket_w", tuple(float(x) for x in weights))
            w = paths.meta.get(key)
            if w is None:
                w = paths.meta[key] = torch.tensor(np.asarray(weights, np.float32), device=S.device)
        native.payoff(code, S, out, strike, nfrac=paths.nfrac_final if code == 0 else None, wts=w, na=paths.na,
                      stream=stream)
        return out
    if code == 0:
        y = S
        out.copy_(torch.where(y > strike, y, torch.full_like(y, strike)) *
                  (paths.nfrac_final if paths.nfrac_final is not None else 1.0))
    elif code == 1:
        out.copy_((S - strike).clamp_min(0))
    elif code == 2:
        out.copy_((strike - S).clamp_min(0))
    else:
        w = torch.tensor(np.asarray(weights, np.float32))
        out.copy_(((S * w[:, None]).sum(0) - strike).clamp_min(0))
    return out


# ---------------------------------------------------------------------------
# numpy oracles (same Sobol points; fp64 recursion)
# ---------------------------------------------------------------------------
def _normals(table_dims, seed, n_local, offset, dims, f32=False, index_map=None):
    tab = sobol_table(table_dims, seed)
    x = tab.points_u30(path_indices(n_local, offset, index_map), dims=dims).astype(np.int64)
    return ndtri_u30_f32(np.maximum(x, 1)).astype(np.float64) if f32 else ndtri_u30_f64(x)


def _cpu_gbm(grid, n, s0, mu, sigma, scheme, offset, seed, index_map=None):
    W = _normals(grid.n_fine, seed, n, offset, grid.n_fine, index_map=index_map)
    dt = grid.dt
    y = np.full(n, math.log(s0) if scheme == "log" else s0, dtype=np.float64)
    out = np.empty((grid.n_coarse, n))
    out[0] = s0
    for t in range(1, grid.n_fine):
        if scheme == "log":
            y = y + (mu - 0.5 * sigma ** 2) * dt + sigma * math.sqrt(dt) * W[:, t]
        else:
            y = y + y * (mu * dt + sigma * math.sqrt(dt) * W[:, t])
        if t % grid.reduction == 0 and t // grid.reduction < grid.n_coarse:
            out[t // grid.reduction] = np.exp(y) if scheme == "log" else y
    fin = np.exp(y) if scheme == "log" else y
    return out, fin


def _u30(table_dims, seed, n_local, offset, dims, index_map=None):
    tab = sobol_table(table_dims, seed)
    return tab.points_u30(path_indices(n_local, offset, index_map), dims=dims).astype(np.int64)


def _qe_step(v, z1, x2, dt, mu, kappa, theta, xi, rho):
    """One Andersen (2008) QE step (martingale-corrected K0*) — numpy twin of
    the k_sim_scan HESTON_QE branch.  Returns (d log S, v_next)."""
    ekd = math.exp(-kappa * dt)
    m = theta + (v - theta) * ekd
    s2 = v * xi * xi * ekd * (1 - ekd) / kappa + theta * xi * xi * (1 - ekd) ** 2 / (2 * kappa)
    psi = s2 / (m * m)
    k1 = 0.5 * dt * (kappa * rho / xi - 0.5) - rho / xi
    k2 = 0.5 * dt * (kappa * rho / xi - 0.5) + rho / xi
    k3 = 0.5 * dt * (1 - rho * rho)
    A = k2 + 0.5 * k3
    k0u = -rho * kappa * theta * dt / xi
    quad = psi <= 1.5
    with np.errstate(invalid="ignore", divide="ignore"):
        z2 = ndtri_u30_f64(x2)
        ip = 2.0 / psi
        b2 = ip - 1 + np.sqrt(ip) * np.sqrt(np.maximum(ip - 1, 0.0))
        qa = m / (1 + b2)
        vq = qa * (np.sqrt(b2) + z2) ** 2
        den = 1 - 2 * A * qa
        k0q = np.where(den > 0, -A * b2 * qa / den + 0.5 * np.log(np.maximum(den, 1e-300)) - (k1 + 0.5 * k3) * v, k0u)
        p = (psi - 1) / (psi + 1)
        beta = (1 - p) / m
        u = x2 * 2.0 ** -30
        ve = np.where(u <= p, 0.0, np.log((1 - p) / np.maximum(1 - u, 1e-300)) / beta)
        k0e = np.where(beta > A, -np.log(p + beta * (1 - p) / (beta - A)) - (k1 + 0.5 * k3) * v, k0u)
    vn = np.where(quad, vq, ve)
    k0 = np.where(quad, k0q, k0e)
    dly = mu * dt + k0 + k1 * v + k2 * vn + np.sqrt(np.maximum(k3 * (v + vn), 0.0)) * z1
    return dly, vn


def _cpu_sv(grid, n, s0, mu, v0, model, a, b, c, kappa, theta, xi, rho, offset, parity_nan, seed1, seed2,
            scheme="euler", sv_tscale=0.0, joint=None, index_map=None):
    if joint is None:
        joint = model == "heston" or (model == "sv_ref" and sv_tscale > 0)
    nf = grid.n_fine
    if joint:  # one 2 n_fine-dimensional sequence (see simulate_sv)
        X = _u30(2 * nf, seed1, n, offset, 2 * nf, index_map)
        W1, X2 = ndtri_u30_f64(X[:, :nf]), X[:, nf:]
    else:
        W1 = _normals(nf, seed1, n, offset, nf, index_map=index_map)
        X2 = _u30(nf, seed2, n, offset, nf, index_map)
    W2 = ndtri_u30_f64(X2)
    dt = grid.dt
    ly = np.full(n, math.log(s0))
    v = np.full(n, float(v0))
    S = np.empty((grid.n_coarse, n))
    V = np.empty((grid.n_coarse, n))
    S[0], V[0] = s0, v0
    rhoc = math.sqrt(1 - rho * rho)
    tau = sv_tscale * dt
    with np.errstate(invalid="ignore"):
        for t in range(1, grid.n_fine):
            if model == "sv_ref" and sv_tscale > 0:
                vp = np.maximum(v, 0.0)
                ly = ly + (mu - 0.5 * vp * vp) * dt + vp * math.sqrt(dt) * W1[:, t]
                v = v + a * (b - vp) * tau + c * np.sqrt(vp * tau) * W2[:, t]
            elif model == "sv_ref":
                arg = v * dt
                sq = np.sqrt(arg) if parity_nan else np.sqrt(np.maximum(arg, 0.0))
                v = v + a * (b - v) + c * sq * W2[:, t]
                ly = ly + (mu - 0.5 * v * v) * dt + v * math.sqrt(dt) * W1[:, t]
            elif scheme == "qe":
                dly, v = _qe_step(v, W1[:, t], X2[:, t], dt, mu, kappa, theta, xi, rho)
                ly = ly + dly
            else:
                vp = np.maximum(v, 0.0)
                sv = np.sqrt(vp * dt)
                ly = ly + (mu - 0.5 * vp) * dt + sv * (rho * W2[:, t] + rhoc * W1[:, t])
                v = v + kappa * (theta - vp) * dt + xi * sv * W2[:, t]
            if t % grid.reduction == 0 and t // grid.reduction < grid.n_coarse:
                S[t // grid.reduction] = np.exp(ly)
                V[t // grid.reduction] = v
    return S, V, np.exp(ly)


def _cpu_basket(grid, n, s0, mu, sigma, chol, offset, seed, index_map=None):
    na = len(s0)
    dims = na * grid.n_fine
    tab = sobol_table(dims, seed)
    idx = path_indices(n, offset, index_map)
    x = tab.points_u30(idx, dims=dims).astype(np.int64)
    Wall = ndtri_u30_f64(np.maximum(x, 1))
    dt = grid.dt
    ly = np.log(np.asarray(s0, dtype=np.float64))[:, None].repeat(n, 1)
    out = np.empty((grid.n_coarse, na, n))
    out[0] = np.asarray(s0)[:, None]
    mu, sigma = np.asarray(mu), np.asarray(sigma)
    for t in range(1, grid.n_fine):
        w = np.stack([Wall[:, a * grid.n_fine + t] for a in range(na)])
        z = chol @ w
        ly = ly + ((mu - 0.5 * sigma ** 2) * dt)[:, None] + (sigma * math.sqrt(dt))[:, None] * z
        if t % grid.reduction == 0 and t // grid.reduction < grid.n_coarse:
            out[t // grid.reduction] = np.exp(ly)
    return out, np.exp(ly)


def _cpu_mortality(grid, n, l0, c, eta, n0, q3, offset, seed, philox_seed, numpy_binomial, index_map=None):
    W2 = _normals(grid.n_fine, seed, n, offset, grid.n_fine, index_map=index_map)
    dt = grid.dt
    lam = np.full(n, float(l0))
    N = np.full(n, int(n0), dtype=np.int64)
    NF = np.empty((grid.n_coarse, n))
    LM = np.empty((grid.n_coarse, n))
    NF[0], LM[0] = 1.0, l0
    gidx = path_indices(n, offset, index_map)
    for t in range(1, grid.n_fine):
        lam = lam + (c * lam * dt + eta * math.sqrt(dt) * W2[:, t])
        p = np.exp(-lam * dt)
        if numpy_binomial:  # Q20: reference draw (MT19937 reseeded each fine step)
            np.random.seed(1234 + t)
            N = np.random.binomial(N, np.clip(p, 0, 1))
        else:
            q = np.clip(1.0 - p, 0.0, 1.0)
            r = philox4x32_10((gidx & np.uint64(0xFFFFFFFF)).astype(np.uint32),
                              (gidx >> np.uint64(32)).astype(np.uint32), np.uint32(t), np.uint32(0xB1A0),
                              philox_seed, 0x1234)
            u = u01d(r[0], r[1])
            D = np.zeros(n, dtype=np.int64)
            f = np.exp(N * np.log1p(-np.minimum(q, 1 - 1e-16)))
            F = f.copy()
            ratio = q / np.maximum(1.0 - q, 1e-300)
            active = (u > F) & (N > 0) & (q > 0)
            while active.any():
                f = np.where(active, f * (N - D) / (D + 1) * ratio, f)
                D = np.where(active, D + 1, D)
                F = np.where(active, F + f, F)
                active = active & (u > F) & (D < N)
            N = N - D
        if q3 and t < grid.n_coarse:
            LM[t] = lam
        if t % grid.reduction == 0 and t // grid.reduction < grid.n_coarse:
            NF[t // grid.reduction] = N / n0
            if not q3:
                LM[t // grid.reduction] = lam
    return NF, LM, N / n0
