"""Seed scatter of the "Multi Time Step.ipynb" headline run (Q15 paths) on the
GPU: V0 / phi0 / psi0 / VaR for several training seeds (Keras-Adam, the
reference's optimiser) and for the full-batch LM fit, one JSON line each.

usage: python tools/archive/mts_seeds.py [n_seeds] [log2 paths ...] > out.jsonl
"""
import json
import sys
import time

sys.path.insert(0, ".")
from rphedge.experiments import mts_notebook  # noqa: E402


def main(n_seeds=8, paths=()):
    runs = [dict(seed=1234 + k) for k in range(n_seeds)] + [dict(optimizer="lm")]
    for n in paths:  # path-count convergence of both optimisers
        runs += [dict(n_paths=n), dict(n_paths=n, optimizer="lm")]
    for over in runs:
        t0 = time.perf_counter()
        out = mts_notebook(verbose=False, poll_every=10, **over)
        rec = {"over": over, "V0": out["V0"], "phi0": out["phi0"], "psi0": out["psi0"], "VaR": out.get("VaR"),
               "s": time.perf_counter() - t0}
        print(json.dumps(rec), flush=True)


if __name__ == "__main__":
    main(int(sys.argv[1]) if len(sys.argv) > 1 else 8, [int(a) for a in sys.argv[2:]])
