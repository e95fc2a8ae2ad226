"""Quality/throughput sweep of the flagship bench configuration (one process).

Prints one JSON line per configuration: ms per full run, V0 vs Black-Scholes,
terminal P&L std.  Used to choose bench.py defaults (see BENCHMARKS.md)."""
import itertools
import json
import sys
import time

import torch

sys.path.insert(0, ".")
import bench  # noqa: E402


FLAG = {"ef": "--epochs-first", "er": "--epochs-rest", "lr_rest": "--lr-rest", "decay": "--lr-decay"}


def one(graph=True, **kw):
    """One bench.py run; keys are bench flags (underscores) or the short names in FLAG."""
    argv = ["--steps", str(kw.pop("steps", 2)), "--warmup", "1", "--json-out", "/tmp/_sweep.json"]
    for k, v in kw.items():
        argv += [FLAG.get(k, "--" + k.replace("_", "-")), str(v)]
    if not graph:
        argv.append("--no-graph")
    import contextlib
    import io

    buf = io.StringIO()
    with contextlib.redirect_stdout(buf):
        bench.main(argv)
    r = json.loads(open("/tmp/_sweep.json").read())
    q = r["quality"]
    return dict(kw, ms=round(r["ms_per_step"], 2), V0=round(q["V0"], 4), pnl_std=round(q["terminal_pnl_std"], 4),
                phi0=round(q["phi0"], 4), anchor=q["anchor"].get("price"), mc=round(q["mc_discounted_payoff"], 4),
                value=r["value"])


if __name__ == "__main__":
    grid = json.loads(sys.argv[1]) if len(sys.argv) > 1 else None
    combos = grid or [dict(batch_log2=b, ef=ef, er=er, lr=lr, lr_rest=lrr, decay=dc, graph=False)
                      for b in (14, 16, 18) for (ef, er) in ((32, 6), (64, 12), (128, 24))
                      for (lr, lrr) in ((1e-2, 2e-3), (2e-2, 5e-3)) for dc in (1.0, 0.1)]
    for c in combos:
        t = time.time()
        try:
            res = one(**c)
        except Exception as e:  # keep sweeping
            res = dict(c, error=repr(e))
        res["wall_s"] = round(time.time() - t, 2)
        print(json.dumps(res), flush=True)
