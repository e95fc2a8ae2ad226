"""Corrected-mode pension (the RP-module liability, default semantics: two
networks, standardised inputs, self-financing P&L, exact mean refit) against
the closed-form anchor of SURVEY §6.1: N·P·max(1, Y_T) under Q with
independent mortality ≈ 917,112 EUR (Δ-hedge ≈ 696,036 fund + 221,076 bond).
One JSON line per (optimizer, capital-charge blend, paths, seed): V0, phi0, psi0, VaR, P&L.

usage: python tools/archive/pension_corrected.py [n_seeds] [log2 paths ...]
"""
import json
import sys
import time

sys.path.insert(0, ".")
from rphedge.api import run_params  # noqa: E402
from rphedge.experiments import mts_parameters  # noqa: E402


def main(n_seeds=4, paths=(12, 16)):
    for n in paths:
        for opt, coc in (("adam", 0.1), ("lm", 0.1), ("lm", 0.0)):
            for k in range(n_seeds):
                t0 = time.perf_counter()
                over = dict(verbose=False, poll_every=10, seed=1234 + k, n_paths=n, optimizer=opt)
                if coc == 0.0:  # pure MSE hedge: no capital-charge blend (the closed form's counterpart)
                    over.update(cost_of_capital=0.0, q99=False)
                res = run_params(mts_parameters(**over))
                print(json.dumps({"optimizer": opt, "cost_of_capital": coc, "n_paths": n, "seed": 1234 + k,
                                  "V0": res.v0, "phi0": res.phi,
                                  "psi0": res.psi, "VaR": res.var, "pnl": res.terminal_pnl,
                                  "s": time.perf_counter() - t0}, default=float), flush=True)


if __name__ == "__main__":
    main(int(sys.argv[1]) if len(sys.argv) > 1 else 4, [int(a) for a in sys.argv[2:]] or (12, 16))
