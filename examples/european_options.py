"""'European Options.ipynb' end to end: simulate, hedge backward, report.

    python examples/european_options.py [--parity] [--paths 3000] [--plots]
"""
import argparse
import json

import rphedge
from rphedge.utils import reports

ap = argparse.ArgumentParser()
ap.add_argument("--parity", action="store_true", help="reference psi = 1 - phi head and B/S0 bonds (Q13)")
ap.add_argument("--paths", type=int, default=3000)
ap.add_argument("--rebalancing", type=float, default=1 / 52)
ap.add_argument("--plots", action="store_true")
a = ap.parse_args()

res = rphedge.european_option(N_paths=a.paths, rebalancing_frequency=a.rebalancing, parity=a.parity,
                              verbose=True, poll_every=10)
val = reports.valuation_report(res, 0.08, 1.0, eo_artifact=a.parity)
print(json.dumps({"V0": res.v0, "BS": res.summary["bs_price"], "phi0": res.phi, "psi0": res.psi,
                  "delta_BS": res.summary["bs_delta"], "terminal_PnL": res.terminal_pnl, "VaR": res.var,
                  "valuation": val}, indent=1, default=float))
if a.plots:
    print(reports.plot_run(res, out_prefix="european"))
