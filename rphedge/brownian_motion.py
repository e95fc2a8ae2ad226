"""Pseudo-random Brownian helpers (C42, ``brownian_motion.py:6-24``).

Kept for API completeness (the reference never imports them): ``get_dW`` draws
T iid N(0,1) increments, ``get_W`` is their cumulative sum starting at 0.
"""
from __future__ import annotations

import numpy as np


def get_dW(T: int, random_state: int | None = None) -> np.ndarray:
    """Sample T times from a normal distribution (Brownian increments)."""
    rng = np.random.default_rng(random_state)
    return rng.normal(0.0, 1.0, T)


def get_W(T: int, random_state: int | None = None) -> np.ndarray:
    """Simulated Brownian motion W_0 = 0, W_t = sum of the first t increments."""
    dW = get_dW(T, random_state)
    return np.insert(np.cumsum(dW)[:-1], 0, 0.0)
