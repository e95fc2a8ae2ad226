"""sigma sweep of "Multi Time Step.ipynb" (cells 104-111, RP module, 4096 paths)
over training seeds, in parity mode (the reference's quirks: shared Q99 model,
raw features, Keras schedule) and in the corrected default mode: one JSON line
per (mode, seed) with the [sigma, Phi, Psi, sum] rows.

usage: python tools/archive/sigma_sweep_seeds.py [n_seeds] > out.jsonl
"""
import json
import sys

sys.path.insert(0, ".")
from rphedge.experiments import volatility_sweep  # noqa: E402


def main(n_seeds=4):
    for parity in (True, False):
        for k in range(n_seeds):
            rows = volatility_sweep(parity=parity, seed=1234 + k, verbose=False, poll_every=10)
            print(json.dumps({"parity": parity, "seed": 1234 + k,
                              "rows": [[r["sigma"], r["Phi"], r["Psi"], r["sum"]] for r in rows]}), flush=True)


if __name__ == "__main__":
    main(int(sys.argv[1]) if len(sys.argv) > 1 else 4)
