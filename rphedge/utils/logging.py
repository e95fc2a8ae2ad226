"""Rank-0 console logging + structured JSONL per-date records."""
from __future__ import annotations

import json
import logging
import os
import time

_LOGGER = None


def _rank() -> int:
    return int(os.environ.get("RANK", "0"))


def get_logger(name: str = "rphedge") -> logging.Logger:
    global _LOGGER
    if _LOGGER is None:
        lg = logging.getLogger(name)
        if not lg.handlers:
            h = logging.StreamHandler()
            h.setFormatter(logging.Formatter(f"[%(asctime)s rank{_rank()}] %(message)s", "%H:%M:%S"))
            lg.addHandler(h)
        lg.setLevel(logging.INFO if _rank() == 0 else logging.WARNING)
        lg.propagate = False
        _LOGGER = lg
    return _LOGGER


class JsonlWriter:
    """Append structured records (loss, epochs, VaR, holdings, time) to a file."""

    def __init__(self, path: str | None):
        self.path = path
        self.f = open(path, "a") if (path and _rank() == 0) else None

    def write(self, **rec):
        if self.f is None:
            return
        rec.setdefault("ts", time.time())
        self.f.write(json.dumps(rec, default=float) + "\n")
        self.f.flush()

    def close(self):
        if self.f is not None:
            self.f.close()
            self.f = None
