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


def one(batch_log2, ef, er, lr, lr_rest, decay, graph, paths_log2=20, dates=30):
    argv = ["--paths-log2", str(paths_log2), "--dates", str(dates), "--epochs-first", str(ef), "--epochs-rest",
            str(er), "--batch-log2", str(batch_log2), "--lr", str(lr), "--lr-rest", str(lr_rest), "--steps", "2",
            "--warmup", "1", "--lr-decay", str(decay), "--json-out", "/tmp/_sweep.json"]
    if not graph:
        argv.append("--no-graph")
    import contextlib
    import io

    buf = io.StringIO()
    with contextlib.redirect_stdout(buf):
        bench.main(argv)
    r = json.loads(open("/tmp/_sweep.json").read())
    return {"batch_log2": batch_log2, "ef": ef, "er": er, "lr": lr, "lr_rest": lr_rest, "decay": decay,
            "ms": round(r["ms_per_step"], 2), "V0": round(r["quality"]["V0"], 4),
            "pnl_std": round(r["quality"]["terminal_pnl_std"], 4), "phi0": round(r["quality"]["phi0"], 4),
            "value": r["value"]}


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
