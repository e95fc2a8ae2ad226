"""Host (numpy) twin of the device Philox4x32-10 generator and of the keyed
minibatch chunk permutation used by the fused training step (K11).

Bit-exact with ``csrc/rph_common.h::philox4x32_10`` and
``csrc/hedge_mlp.hip::make_perm`` so the CPU reference trainer draws exactly
the same minibatches as the GPU kernels.
"""
from __future__ import annotations

import numpy as np

M0 = np.uint64(0xD2511F53)
M1 = np.uint64(0xCD9E8D57)
W0 = np.uint32(0x9E3779B9)
W1 = np.uint32(0xBB67AE85)
MASK32 = np.uint64(0xFFFFFFFF)


def philox4x32_10(c0, c1, c2, c3, k0, k1):
    """Vectorised Philox4x32-10.  Inputs are uint32 arrays/scalars; returns a
    tuple of four uint32 arrays."""
    x = [np.asarray(v, dtype=np.uint32).astype(np.uint64) for v in (c0, c1, c2, c3)]
    key0 = np.asarray(k0, dtype=np.uint32).astype(np.uint64)
    key1 = np.asarray(k1, dtype=np.uint32).astype(np.uint64)
    for _ in range(10):
        p0 = M0 * x[0]
        p1 = M1 * x[2]
        hi0, lo0 = p0 >> np.uint64(32), p0 & MASK32
        hi1, lo1 = p1 >> np.uint64(32), p1 & MASK32
        x = [(hi1 ^ x[1] ^ key0) & MASK32, lo1, (hi0 ^ x[3] ^ key1) & MASK32, lo0]
        key0 = (key0 + np.uint64(W0)) & MASK32
        key1 = (key1 + np.uint64(W1)) & MASK32
    return tuple(v.astype(np.uint32) for v in x)


def u01d(hi, lo):
    """53-bit (0,1) double from two u32 words (device ``u01d``)."""
    hi = np.asarray(hi, dtype=np.uint64)
    lo = np.asarray(lo, dtype=np.uint64)
    m = ((hi << np.uint64(21)) ^ (lo >> np.uint64(11))) & np.uint64((1 << 53) - 1)
    return (m.astype(np.float64) + 0.5) * (1.0 / 9007199254740992.0)


class ChunkPerm:
    """Keyed bijection on ``range(n_chunks)`` (device ``Perm``)."""

    def __init__(self, n_chunks: int, seed: int, epoch: int, on: bool = True):
        m, bits = 1, 0
        while m < n_chunks:
            m <<= 1
            bits += 1
        self.mask = np.uint32(m - 1)
        self.n = int(n_chunks)
        r = philox4x32_10(epoch, 0x5EED, 0, 0, seed, 0xC0FFEE)
        s = philox4x32_10(epoch, 0x5EED, 1, 0, seed, 0xC0FFEE)
        self.k1 = np.uint32(int(r[0]) & int(self.mask))
        self.a1 = np.uint32(int(r[1]) | 1)
        self.b1 = np.uint32(int(r[2]))
        self.a2 = np.uint32(int(r[3]) | 1)
        self.b2 = np.uint32(int(s[0]))
        self.sh = np.uint32(bits // 2 if bits > 1 else 1)
        self.on = bool(on) and n_chunks > 1

    def _f(self, x: np.ndarray) -> np.ndarray:
        with np.errstate(over="ignore"):
            x = (((x ^ self.k1) * self.a1) + self.b1) & self.mask
            x = x ^ (x >> self.sh)
            x = ((x * self.a2) + self.b2) & self.mask
        return x

    def __call__(self, x) -> np.ndarray:
        x = np.asarray(x, dtype=np.uint32)
        if not self.on:
            return x.copy()
        y = self._f(x)
        bad = y >= self.n
        while np.any(bad):
            y[bad] = self._f(y[bad])
            bad = y >= self.n
        return y


def epoch_order(n_local: int, chunk_log2: int, seed: int, epoch: int, shuffle: bool = True) -> np.ndarray:
    """Path index visited at epoch-order position j for j in range(n_local)."""
    ch = 1 << chunk_log2
    n_chunks = (n_local + ch - 1) // ch
    perm = ChunkPerm(n_chunks, seed, epoch, shuffle)
    j = np.arange(n_local, dtype=np.uint32)
    p = (perm(j >> np.uint32(chunk_log2)) << np.uint32(chunk_log2)) | (j & np.uint32(ch - 1))
    p = np.where(p >= n_local, j, p)
    return p.astype(np.int64)
