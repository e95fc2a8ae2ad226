"""Where the learnt hedge's self-financing P&L loses to the Black-Scholes
delta hedge (GBM presets): per rebalancing date t, the contribution of the
hedge-ratio error e_t = phi_t - Delta_BS(t, S_t) to the P&L difference,
  P&L_NN - P&L_BS = sum_t e_t (S_{t+1} - S_t B_{t+1}/B_t) + (V0_NN - V0_BS) B_T/B_0,
reported as E[(e_t dS_t)^2] per date (the terms are uncorrelated across dates
under the martingale measure up to the drift) and the RMS of e_t, grouped into
date bands, plus the totals.  Needs the per-date holdings (keep_paths).

usage: python tools/hedge_diag.py OUT.json <bench args...>"""
import json
import math
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.abspath(os.path.join(os.path.dirname(__file__), "..")))
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
    S = p.S.double()  # [nc, n] normalised
    nc = S.shape[0]
    B = np.asarray(p.bond, np.float64)
    tt = np.asarray(run.grid.times(), np.float64)
    K, r, sg, T = cfg.K / cfg.Y, cfg.r, cfg.sigma, cfg.T
    hold = res.induction.holdings  # [nc-1, nhold, n]
    rows = []
    tot_e2 = 0.0
    for t in range(nc - 1):
        tau = T - tt[t]
        sq = sg * math.sqrt(tau)
        d1 = (torch.log(S[t] / K) + (r + 0.5 * sg * sg) * tau) / sq
        dl = 0.5 * torch.erfc(-d1 / math.sqrt(2.0))
        phi = hold[t, 0].double()
        e = phi - dl
        dS = S[t + 1] - S[t] * (B[t + 1] / B[t])
        c = float(((e * dS) ** 2).mean()) * cfg.Y ** 2
        tot_e2 += c
        rows.append({"t": t, "tau": tau, "rms_err": float((e * e).mean().sqrt()), "mean_err": float(e.mean()),
                     "contrib": c})
    n_d = nc - 1
    bands = [(0, n_d // 2), (n_d // 2, int(n_d * 0.9)), (int(n_d * 0.9), n_d - 5), (n_d - 5, n_d)]
    summary = {"preset": a.preset, "seed": a.seed, "n_dates": n_d, "pnl_std": res.terminal_pnl["std"],
               "sum_contrib": tot_e2, "sqrt_sum_contrib": math.sqrt(tot_e2), "bands": []}
    for lo, hi in bands:
        cs = sum(x["contrib"] for x in rows[lo:hi])
        summary["bands"].append({"dates": [lo, hi], "contrib": cs, "share": cs / tot_e2,
                                 "rms_err_mean": float(np.mean([x["rms_err"] for x in rows[lo:hi]]))})
    summary["worst_dates"] = sorted(rows, key=lambda x: -x["contrib"])[:8]
    print(json.dumps(summary))
    with open(out, "a") as f:
        f.write(json.dumps({"summary": summary, "rows": rows}) + "\n")


if __name__ == "__main__":
    main(sys.argv[1:])
