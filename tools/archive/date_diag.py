"""Diagnostic: per-date fit record of one bench configuration (eager run):
best loss, passes, accepted trials, one-step residual std and the fitted
holdings' means, to find the date that breaks a self-financing P&L.
usage: python tools/archive/date_diag.py <bench args...>"""
import json
import sys

import torch

sys.path.insert(0, ".")
import bench  # noqa: E402
from rphedge.api import HedgeRun  # noqa: E402


def main(argv):
    a = bench.parse(argv)
    cfg = bench.build_run(a, 1)
    run = HedgeRun(cfg)
    run.build()
    run.enqueue()
    if torch.cuda.is_available():
        torch.cuda.synchronize()
    res = run.collect()
    ind = res.induction
    nh = run.spec.nhold
    for d in ind.dates:
        f = d.fit_mse
        h = [x for x in f["history"] if x == x]
        acc = sum(1 for i in range(1, len(h)) if h[i] < min(h[:i]))
        print(json.dumps({"date": d.index, "best": f["best_loss"], "start": h[0] if h else None, "passes": len(h) - 1,
                          "acc": acc, "res_std": d.residual_std, "res_mean": d.residual_mean,
                          "hold": [float(x) for x in d.mean_holdings(nh)]}))
    print(json.dumps({"pnl": res.terminal_pnl, "V0": res.v0}))


if __name__ == "__main__":
    main(sys.argv[1:])
