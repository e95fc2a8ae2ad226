"""'Multi Time Step.ipynb': the module call, the sigma sweep and the SV run.

    python examples/multi_time_step.py [--parity] [--sweep] [--sv]
"""
import argparse
import json

from rphedge import Replicating_Portfolio, Replicating_Portfolio_SV
from rphedge.experiments import mts_parameters, sanity_checks, sv_parameters, volatility_sweep

ap = argparse.ArgumentParser()
ap.add_argument("--parity", action="store_true")
ap.add_argument("--sweep", action="store_true")
ap.add_argument("--sv", action="store_true")
a = ap.parse_args()

params = mts_parameters(parity=a.parity, poll_every=10)
print(json.dumps(sanity_checks(dict(params, verbose=False)), default=float, indent=1))
phi, psi = Replicating_Portfolio(params)
print(f"Phi t=0 : {phi:,.0f} Stocks\nPsi t=0 : {psi:,.0f} Bonds   (reference: 634,349 / 350,176)")
if a.sweep:
    for row in volatility_sweep(parity=a.parity, poll_every=10, verbose=False):
        print(row)
if a.sv:
    phi, psi = Replicating_Portfolio_SV(sv_parameters(parity=True, poll_every=10))
    print(f"SV: Phi {phi:,.0f}  Psi {psi:,.0f}   (reference: 626,123 / 371,854)")
