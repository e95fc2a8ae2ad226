"""Per-phase timers (simulate / train / report) with hipEvents on the GPU.

``RPH_PROFILE=1`` dumps the phase table as JSON at interpreter exit (SURVEY
§5.1).  Kernel-level evidence comes from ``rocprofv3 --kernel-trace --stats``:
every kernel has a distinct name (k_sim_scan / k_hedge_step_lag /
k_hedge_eval / k_radix_hist / ...).

Timers register through a weak set, so a sweep that creates one run after
another does not keep every run's timer (and its recorded GPU events) alive;
the exit dump reports the timers still alive plus the summaries of the ones
collected earlier (bounded).
"""
from __future__ import annotations

import atexit
import json
import os
import time
import weakref
from contextlib import contextmanager

import torch

_LIVE: "weakref.WeakSet[PhaseTimer]" = weakref.WeakSet()
_DONE: list = []          # summaries of collected timers (RPH_PROFILE=1 only)
_DONE_MAX = 1024


class PhaseTimer:
    def __init__(self, enabled: bool = True, device=None):
        self.enabled = enabled
        self.device = device
        self.cpu = {}
        self.events = {}
        _LIVE.add(self)

    def __del__(self):
        if os.environ.get("RPH_PROFILE") == "1" and len(_DONE) < _DONE_MAX:
            try:
                _DONE.append(self.summary())
            except Exception:
                pass

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


def live_timers() -> int:
    return len(_LIVE)


def _dump():
    if os.environ.get("RPH_PROFILE") == "1" and (_LIVE or _DONE):
        path = os.environ.get("RPH_PROFILE_OUT", "rph_profile.json")
        with open(path, "w") as f:
            json.dump(list(_DONE) + [t.summary() for t in list(_LIVE)], f, indent=1)


atexit.register(_dump)
