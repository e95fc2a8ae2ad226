"""Corrected-mode pension (Replicating_Portfolio semantics, "Multi Time Step.ipynb"
:1329-1351 parameters, two networks) at 2^n paths, 40 quarterly dates: both fits
(MSE and the Q99 pinball fit, Replicating_Portfolio.py:138-145, :211, :217) on
Levenberg-Marquardt (q99_optimizer="lm") vs both on Keras-Adam (the reference
optimiser).  Per run: wall time of the whole API call (graph-free, one sync at
the end), V0 / phi0 / psi0, and the Q99 net's one-step residual quantiles per
date (the sign condition of "Single Time Step.ipynb":656-662: the 99 % quantile
of V_{t+1} - h_q(state_t) . prices_{t+1} should sit at ~0).

usage: python tools/archive/r5/pension_lm.py OUT.jsonl n_log2 seeds opt [opt ...]
  opt: lm | adam
"""
import json
import os
import sys
import time

import torch

sys.path.insert(0, os.path.abspath(os.path.join(os.path.dirname(__file__), "..", "..")))


def q99_residual_quantiles(run, res):
    """99 % quantile of the Q99 net's one-step residual at every date (and the
    fraction of paths above zero)."""
    from rphedge.models.hedge_mlp import torch_forward

    ind = run.induction
    spec = run.spec
    p = run.paths
    P = spec.nparams
    out = []
    with torch.no_grad():
        for t in range(ind.n_dates):
            w = ind.snap[t, 1, :P].float()
            X = torch.stack([f.float() for f in p.features(t)], 1)
            if ind.norms:
                mu, isd = ind.norms[t]
                X = (X - torch.tensor(mu, dtype=torch.float32, device=X.device)) * \
                    torch.tensor(isd, dtype=torch.float32, device=X.device)
            pr = torch.stack([q.float() for q in p.prices(t + 1)] + [torch.full_like(X[:, 0], float(p.bond[t + 1]))], 1)
            r = (ind.values[t + 1].float() - (torch_forward(spec, w, X) * pr).sum(1)).double()
            k = max(1, int(0.01 * r.numel()))
            q99 = float(torch.topk(r, k).values.min())  # 99 % quantile (torch.quantile caps the input size)
            out.append((q99, float((r > 0).double().mean())))
    return out


def main():
    out, n, seeds, opts = sys.argv[1], int(sys.argv[2]), sys.argv[3], sys.argv[4:]
    from rphedge import experiments
    from rphedge.api import HedgeRun
    from rphedge.config import parse_params
    from rphedge.driver import DateResult

    seeds = [int(s) for s in seeds.split(",")]
    with open(out, "a") as f:
        for opt in opts:
            for s in seeds:
                p = experiments.mts_parameters()
                p.update(n_paths=n, seed=s, verbose=False, device="cuda:0")
                if opt.startswith("preset"):  # experiments.mts_lm_parameters (+ variants as below)
                    p = experiments.mts_lm_parameters(n_paths=n, seed=s, verbose=False, device="cuda:0")
                    keys = {"qr": "lm_q_passes_rest", "qf": "lm_q_passes_first", "mr": "lm_passes_rest",
                            "mf": "lm_passes_first", "st": "lm_starts", "ep": "lm_explore_passes"}
                    for kv in opt.split(",")[1:]:
                        k, v = kv.split("=")
                        p[keys[k]] = int(v)
                elif opt.startswith("lm"):
                    p.update(optimizer="lm", q99_optimizer="lm", lm_passes_first=40, lm_passes_rest=3,
                             lm_q_passes_first=40, lm_q_passes_rest=4, lm_lam_carry=3.0, lm_out_fix=True)
                    # variants: lm,qr=10,qf=60,k=1.0,d=1e-4,mr=3
                    keys = {"qr": "lm_q_passes_rest", "qf": "lm_q_passes_first", "k": "lm_q_kappa",
                            "d": "lm_q_delta", "mr": "lm_passes_rest", "qs": "lm_q_start", "mf": "lm_passes_first",
                            "st": "lm_starts", "ep": "lm_explore_passes", "el": "lm_explore_log2"}
                    for kv in opt.split(",")[1:]:
                        k, v = kv.split("=")
                        p[keys[k]] = float(v) if k in ("k", "d") else (v if k == "qs" else int(v))
                cfg = parse_params(p)
                run = HedgeRun(cfg)
                torch.cuda.synchronize()
                t0 = time.perf_counter()
                res = run.run()
                torch.cuda.synchronize()
                dt = time.perf_counter() - t0
                qs = q99_residual_quantiles(run, res)
                rec = {"opt": opt, "seed": s, "n_log2": n, "wall_s": dt, "V0": res.v0, "phi0": res.phi,
                       "psi0": res.psi, "pnl_std": res.terminal_pnl["std"],
                       "q99_resid_q99_max": max(q for q, _ in qs), "q99_resid_q99_mean": sum(q for q, _ in qs) / len(qs),
                       "q99_frac_above_mean": sum(a for _, a in qs) / len(qs),
                       "q99_resid_q99_first_last": [qs[0][0], qs[-1][0]], "scale": run.scale,
                       "var": res.var, "terminal_residual_std": res.terminal_residual["std"]}
                d0 = res.induction.dates[0]  # the last date (the first fit of the induction)
                rec["last_mse_resid_std"] = (DateResult(0, 0.0, stats=d0.stats_mse).residual_std * run.scale
                                             if d0.stats_mse is not None else None)
                rec["mse_loss_first_fit"] = d0.fit_mse["best_loss"]
                rec["q_loss_first_fit"] = d0.fit_q99["best_loss"] if d0.fit_q99 else None
                rec["mse_loss_mean"] = sum(d.fit_mse["best_loss"] for d in res.induction.dates) / len(res.induction.dates)
                rec["q_loss_mean"] = sum(d.fit_q99["best_loss"] for d in res.induction.dates) / len(res.induction.dates)
                f.write(json.dumps(rec) + "\n")
                f.flush()
                print(json.dumps(rec), flush=True)
                del run, res
                torch.cuda.empty_cache()


if __name__ == "__main__":
    main()
