"""Per-date diagnosis of a multi-asset hedge run (basket5): for every
rebalancing date t, the std of the hedge's discounted P&L increment
sum_k phi_t,k (S_t+1,k - S_t,k B_t+1/B_t), the largest |holding| and the mean
|phi| - a date whose fit went wrong stands out against its neighbours.
Reductions run on the device (the holdings of 2^23 paths x 252 dates do not
leave the GPU).

usage: python tools/archive/r5/basket_diag.py OUT.jsonl <bench args...>"""
import json
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.abspath(os.path.join(os.path.dirname(__file__), "..", "..")))
import bench  # noqa: E402
from rphedge.api import HedgeRun  # noqa: E402


def main(argv):
    out, argv = argv[0], argv[1:]
    a = bench.parse(argv)
    cfg = bench.build_run(a, 1)
    cfg.keep_paths = True
    run = HedgeRun(cfg)
    res = run.run()
    if torch.cuda.is_available():
        torch.cuda.synchronize()
    p = run.paths
    B = np.asarray(p.bond, np.float64)
    hold = res.induction.holdings  # [nc-1, nhold, n]
    na = p.na
    rows = []
    for t in range(p.n_coarse - 1):
        inc = torch.zeros_like(p.asset(t, 0), dtype=torch.float64)
        for k in range(na):
            inc += hold[t, k].double() * (p.asset(t + 1, k).double() - p.asset(t, k).double() * (B[t + 1] / B[t]))
        h = hold[t].abs()
        rows.append({"t": t, "inc_std": float(inc.std()) * cfg.Y, "max_abs_hold": float(h.max()),
                     "mean_abs_phi": float(h[:na].mean()), "mean_abs_psi": float(h[na:].mean())})
    st = np.array([r["inc_std"] for r in rows])
    med = float(np.median(st))
    summary = {"args": " ".join(argv), "seed": a.seed, "pnl_std": res.terminal_pnl["std"],
               "inc_std_median": med, "worst_inc_dates": sorted(rows, key=lambda r: -r["inc_std"])[:6],
               "worst_hold_dates": sorted(rows, key=lambda r: -r["max_abs_hold"])[:6]}
    print(json.dumps(summary))
    with open(out, "a") as f:
        f.write(json.dumps({"summary": summary, "rows": rows}) + "\n")


if __name__ == "__main__":
    main(sys.argv[1:])
