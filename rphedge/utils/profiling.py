"""Per-phase timers (simulate / train / report) with hipEvents on the GPU.

``RPH_PROFILE=1`` dumps the phase table as JSON at interpreter exit (SURVEY
§5.1).  Kernel-level evidence comes from ``rocprofv3 --kernel-trace --stats``:
every kernel has a distinct name (k_sim_scan / k_hedge_train_step /
k_hedge_eval / k_radix_hist / ...)."""
from __future__ import annotations

import atexit
import json
import os
import time
from contextlib import contextmanager

import torch

_ALL = []


class PhaseTimer:
    def __init__(self, enabled: bool = True, device=None):
        self.enabled = enabled
        self.device = device
        self.cpu = {}
        self.events = {}
        _ALL.append(self)

    @contextmanager
    def phase(self, name: str):
        if not self.enabled:
            yield
            return
        gpu = self.device is not None and torch.device(self.device).type == "cuda" and torch.cuda.is_available()
        if gpu:
            a = torch.cuda.Event(enable_timing=True)
            b = torch.cuda.Event(enable_timing=True)
            a.record()
        t0 = time.perf_counter()
        try:
            yield
        finally:
            self.cpu[name] = self.cpu.get(name, 0.0) + time.perf_counter() - t0
            if gpu:
                b.record()
                self.events.setdefault(name, []).append((a, b))

    def summary(self) -> dict:
        out = {f"host_{k}_s": v for k, v in self.cpu.items()}
        for k, lst in self.events.items():
            try:
                out[f"gpu_{k}_ms"] = sum(a.elapsed_time(b) for a, b in lst)
            except Exception:
                pass
        return out


def _dump():
    if os.environ.get("RPH_PROFILE") == "1" and _ALL:
        path = os.environ.get("RPH_PROFILE_OUT", "rph_profile.json")
        with open(path, "w") as f:
            json.dump([t.summary() for t in _ALL], f, indent=1)


atexit.register(_dump)
