"""Pseudo-random Brownian helpers (C42, ``brownian_motion.py:6-24``).

Kept for API completeness (the reference never imports them).  Same draws as
the reference: ``get_dW`` reseeds numpy's legacy global MT19937 stream with
``random_state`` and samples T iid N(0,1) increments from it (so the values
AND the global-RNG side effect match ``np.random.seed(s); np.random.normal``);
``get_W`` is the cumulative sum shifted to start at 0 (same length T).
"""
from __future__ import annotations

import numpy as np


def get_dW(T: int, random_state: int | None = None) -> np.ndarray:
    """Sample T times from a normal distribution (Brownian increments)."""
    np.random.seed(random_state)          # legacy global RandomState, as brownian_motion.py:12
    return np.random.normal(0.0, 1.0, T)


def get_W(T: int, random_state: int | None = None) -> np.ndarray:
    """Simulated Brownian motion at unit time steps: W_0 = 0, W_t = dW_1 + ... + dW_t."""
    dW = get_dW(T, random_state)
    return np.insert(dW.cumsum(), 0, 0.0)[:-1]
