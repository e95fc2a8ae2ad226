"""'Single Time Step.ipynb': one 10-year hedge, MSE vs cost-of-capital holdings."""
import json

from rphedge.experiments import single_time_step

out = single_time_step(parity=True, poll_every=10, verbose=False)
out.pop("result")
print(json.dumps(out, indent=1, default=float))
print("reference: Res1 VaR99 = 0.25823, Res2 VaR99 = 0.00085 (per unit N*P); phi0/psi0 = 819,539 / 257,308")
