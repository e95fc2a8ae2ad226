"""Scrambled Sobol quasi-Monte-Carlo (K1) + inverse normal (K2).

The reference draws ``qmc.Sobol(d, scramble=True, seed).random_base2(m)`` and
maps it through ``norm.ppf`` (``Replicating_Portfolio.py:54-57``).  scipy's
points are index-addressable:

    point(i) = shift XOR  XOR_{k in bits(gray(i))} sv[:, k],   gray(i) = i ^ (i >> 1)

so the host only builds the scrambled direction numbers ``sv`` ([d, 30] u32)
and the digital ``shift`` ([d] u32) once — with scipy itself, hence bit-exact —
and the GPU regenerates any (path, dim) coordinate on the fly inside the path
kernels.  No [paths x dims] normal matrix is ever materialised on the device.
"""
from __future__ import annotations

import functools
import math
from dataclasses import dataclass

import numpy as np

from .ndtri import ndtri_u30_f32, ndtri_u30_f64

BITS = 30
SCALE = 2.0 ** -BITS


@dataclass(frozen=True)
class SobolTable:
    """Scrambled direction numbers for ``dims`` dimensions (scipy seed)."""

    sv: np.ndarray      # [dims, 32] uint32 (columns 30,31 zero)
    shift: np.ndarray   # [dims] uint32
    seed: int
    dims: int

    def points_u30(self, idx: np.ndarray, dims=None) -> np.ndarray:
        """Raw 30-bit integers of points ``idx`` for the first ``dims`` dims -> [len(idx), dims]."""
        dims = self.dims if dims is None else dims
        idx = np.asarray(idx, dtype=np.uint64)
        g = (idx ^ (idx >> np.uint64(1))).astype(np.uint64)
        out = np.broadcast_to(self.shift[:dims], (len(idx), dims)).copy()
        for k in range(BITS):
            bit = ((g >> np.uint64(k)) & np.uint64(1)).astype(bool)
            if bit.any():
                out[bit] ^= self.sv[:dims, k]
        return out


@functools.lru_cache(maxsize=64)
def sobol_table(dims: int, seed: int) -> SobolTable:
    """scipy-identical scrambled Sobol table (Joe–Kuo numbers, LMS + shift)."""
    from scipy.stats import qmc

    s = qmc.Sobol(int(dims), scramble=True, seed=int(seed))
    assert s.bits == BITS, "rphedge assumes scipy's default 30-bit Sobol"
    sv = np.zeros((dims, 32), dtype=np.uint32)
    sv[:, :BITS] = s._sv.astype(np.uint32)
    shift = s._shift.astype(np.uint32).copy()
    sv.setflags(write=False)
    shift.setflags(write=False)
    return SobolTable(sv=sv, shift=shift, seed=int(seed), dims=int(dims))


def sobol_uniform_cpu(m: int, d: int, seed: int = 1234, offset: int = 0, n=None) -> np.ndarray:
    n = 2 ** m if n is None else n
    tab = sobol_table(d, seed)
    return tab.points_u30(np.arange(offset, offset + n, dtype=np.uint64)) * SCALE


def sobol_norm_cpu(m: int, d: int = 1, seed: int = 1234, dtype=np.float64, offset: int = 0, n=None) -> np.ndarray:
    """CPU oracle of the device generator: ``norm.ppf(Sobol.random_base2(m))``."""
    n = 2 ** m if n is None else n
    tab = sobol_table(d, seed)
    x = tab.points_u30(np.arange(offset, offset + n, dtype=np.uint64)).astype(np.int64)
    if dtype == np.float32:
        return ndtri_u30_f32(x)
    return ndtri_u30_f64(x)


def sobol_norm(m: int, d: int = 1, seed: int = 1234, device=None, dtype=None, offset: int = 0):
    """Drop-in for the reference ``sobol_norm(m, d, seed)`` (RP:54-57).

    ``m`` is log2 of the number of points.  On a GPU device the
    normals are produced by the K1+K2 HIP kernel; on CPU by the numpy oracle.
    Returns a torch tensor of shape [2**m, d].
    """
    import torch

    dev = torch.device(device) if device is not None else (
        torch.device("cuda") if torch.cuda.is_available() else torch.device("cpu"))
    dtype = dtype or torch.float64
    n = 2 ** int(m)
    if dev.type == "cpu":
        arr = sobol_norm_cpu(m, d, seed, np.float32 if dtype == torch.float32 else np.float64, offset)
        return torch.from_numpy(np.ascontiguousarray(arr)).to(dtype)
    from . import native

    tab = device_table(d, seed, dev)
    out = torch.empty((n, d), dtype=dtype, device=dev)
    native.sobol_normal(out, tab, offset=offset)
    return out


_DEVICE_TABLES: dict = {}


def device_table(dims: int, seed: int, device):
    """Upload (and cache) a Sobol table to ``device`` -> (sv, shift, dims)."""
    import torch

    key = (int(dims), int(seed), str(device))
    hit = _DEVICE_TABLES.get(key)
    if hit is not None:
        return hit
    tab = sobol_table(dims, seed)
    sv = torch.from_numpy(tab.sv.view(np.int32).copy()).to(device)
    sh = torch.from_numpy(tab.shift.view(np.int32).copy()).to(device)
    _DEVICE_TABLES[key] = (sv, sh, int(dims))
    return _DEVICE_TABLES[key]


def log2_paths(n_paths: int) -> int:
    """Reference path-count convention: ``ceil(log2(N))``."""
    return int(math.ceil(math.log2(n_paths)))
