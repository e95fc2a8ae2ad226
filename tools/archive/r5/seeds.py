"""Seed sweep of a bench.py preset in ONE process (no per-seed torch import /
library load): one JSON line per seed with the timing and quality fields.

usage: python tools/archive/r5/seeds.py OUT.jsonl SEEDS [bench.py args...]
  SEEDS: comma list or a-b range, e.g. 1-8
"""
import contextlib
import io
import json
import os
import sys
import time

sys.path.insert(0, os.path.abspath(os.path.join(os.path.dirname(__file__), "..", "..")))
import bench  # noqa: E402


def seeds(spec: str):
    if "-" in spec:
        a, b = spec.split("-")
        return list(range(int(a), int(b) + 1))
    return [int(x) for x in spec.split(",")]


def main():
    out, spec, rest = sys.argv[1], sys.argv[2], sys.argv[3:]
    with open(out, "a") as f:
        for s in seeds(spec):
            buf = io.StringIO()
            t0 = time.perf_counter()
            with contextlib.redirect_stdout(buf):
                bench.main(rest + ["--seed", str(s)])
            line = [l for l in buf.getvalue().splitlines() if l.startswith("{")][-1]
            r = json.loads(line)
            q = r["quality"]
            ha = q.get("hedge_anchor") or {}
            rec = {"seed": s, "args": " ".join(rest), "ms": r["ms_per_step"], "pnl": q["terminal_pnl_std"],
                   "resid": q["terminal_residual_std"], "V0": q["V0"], "anchor_pnl": ha.get("pnl_std"),
                   "anchor_price": (q.get("anchor") or {}).get("price"),
                   "first_best": ((r.get("lm") or {}).get("first_date") or {}).get("best_loss"),
                   "ms_pick": ((r.get("lm") or {}).get("multistart") or {}).get("pick"),
                   "wall_s": time.perf_counter() - t0}
            f.write(json.dumps(rec) + "\n")
            f.flush()
            print(json.dumps(rec), flush=True)


if __name__ == "__main__":
    main()
