"""Wall time of the reference-scale API calls (4096 paths, batch 512) per GPU
step schedule: the reference's own configurations, latency-bound (2 workgroups
per step).  One JSON line per (experiment, step_mode)."""
import json
import sys
import time

import torch

sys.path.insert(0, ".")
from rphedge.api import run_params  # noqa: E402
from rphedge.experiments import mts_parameters, sv_parameters  # noqa: E402


def cases():
    yield "pension_parity", mts_parameters(parity=True, verbose=False), False
    yield "pension_corrected", mts_parameters(verbose=False), False
    yield "sv_parity", sv_parameters(parity=True, verbose=False), True
    eo = dict(Y=100.0, K=100.0, T=1.0, mu=0.08, r=0.08, sigma=0.15, rebalancing=1 / 52, N=1, P=1.0, x=0.0, l0=0.0,
              c=0.0, ita=0.0, dt=1 / 365, n_paths=12, payoff="call", option_type="CALL", model="gbm_log",
              mortality=False, q99=False, verbose=False)
    yield "eo_corrected", eo, False


if __name__ == "__main__":
    modes = sys.argv[1].split(",") if len(sys.argv) > 1 else ["lag", "persistent", "ticket"]
    for name, p, sv in cases():
        for m in modes:
            q = dict(p, step_mode=m)
            run_params(dict(q, epochs_first=5, epochs_rest=2), sv=sv)  # warm caches / JIT tables
            torch.cuda.synchronize()
            t0 = time.perf_counter()
            res = run_params(q, sv=sv)
            torch.cuda.synchronize()
            dt = time.perf_counter() - t0
            print(json.dumps({"case": name, "step_mode": m, "wall_s": round(dt, 3), "phi0": res.phi, "psi0": res.psi,
                              "V0": res.v0, "epochs": res.summary.get("epochs_mse")[:6]}), flush=True)
