"""Global seeding (C01, ``Replicating_Portfolio.py:24-27``): the reference calls
``tf_seed(1234); seed(1234)``.  Device kernels are counter-based (Philox keyed
by explicit seeds) so they need no global state; this seeds numpy/torch for
host-side helpers."""
from __future__ import annotations

import os
import random

import numpy as np
import torch


def seed_everything(seed: int = 1234):
    random.seed(seed)
    np.random.seed(seed)
    torch.manual_seed(seed)
    os.environ.setdefault("TF_CPP_MIN_LOG_LEVEL", "3")  # parity with RP:2 (harmless without TF)
    return seed
