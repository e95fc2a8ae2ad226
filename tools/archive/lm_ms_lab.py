"""CPU laboratory: multi-start first-date LM fits and damping carried across
dates (float64 torch oracle, bench.py --cpu).

  python tools/archive/lm_ms_lab.py --seeds 1,2,3 --variants base,ms4,ms4+carry3

Variant flags ('+'-joined):
  msK        first date: K starts (init seeds seed, seed+1, ...) explored for
             N1 passes on the first 2^SUB paths (ms_n1=, ms_sub=), the best
             (lowest best loss) polished for N2 passes on every path (ms_n2=)
  carryF     later dates start at the previous fit's final damping x F
  lfX        first date's initial damping X
  adaptT     later dates: stop once a pass lowers the best loss by < T (relative)
One JSON line per (variant, seed): SF P&L std, one-step residual std, V0,
first-date best loss, accepted trials on later dates.
"""
from __future__ import annotations

import argparse
import io
import json
import os
import sys
from contextlib import redirect_stdout

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

from rphedge import engine as E  # noqa: E402
from rphedge.models import hedge_mlp as hm  # noqa: E402
from rphedge.models.hedge_mlp import torch_forward  # noqa: E402
from rphedge.ops import layout as L  # noqa: E402

CFG = {"flags": {}, "log": [], "seed": 1234}


def lm_core(spec, t, w0, X, pr, y, ns_req, passes, lam, tol=0.0, kmin=2):
    """The HIP solver's sequence (simple damping rule) on the paths (X, pr, y)."""
    from torch.func import jacrev, vmap

    n = X.shape[0]
    ns = max(L.LM_TILE, min(int(ns_req), n)) // L.LM_TILE * L.LM_TILE
    blk, bstride = E.lm_gram_geometry(n, ns, 1)
    sub = torch.tensor([(j // blk) * bstride + j % blk for j in range(ns)], dtype=torch.long)

    def v_one(w, x, p):
        return (torch_forward(spec, w, x[None])[0] * p).sum()

    def evaluate(w):
        wg = w.detach().clone().requires_grad_(True)
        e = (torch_forward(spec, wg, X) * pr).sum(1) - y
        lsum = (e * e).sum()
        (lsum / n).backward()
        J = vmap(jacrev(v_one), in_dims=(None, 0, 0))(w.detach(), X[sub], pr[sub])
        return (J.T @ J) / ns, wg.grad.detach(), float(lsum) / n

    w_best = w0.clone()
    G, g, Lb = evaluate(w_best)
    hist, nacc = [Lb], 0
    for k in range(1, passes + 1):
        Lb_prev = Lb
        A = 2.0 * G
        dg = torch.diagonal(A).clone()
        dmp = dg * lam + float(t.lm_ridge) * float(dg.mean())
        Lc, info = torch.linalg.cholesky_ex(A + torch.diag(dmp))
        if int(info) != 0:
            lam = min(lam * t.lm_lam_up * t.lm_lam_up, t.lm_lam_max)
            hist.append(Lb)
            continue
        trial = w_best + torch.cholesky_solve(-g[:, None], Lc)[:, 0]
        Gt, gt, Lt = evaluate(trial)
        hist.append(Lt)
        if Lt == Lt and Lt < Lb:
            nacc += 1
            lam = max(lam * t.lm_lam_down, t.lm_lam_min)
            w_best, G, g, Lb = trial, Gt, gt, Lt
        else:
            lam = min(lam * t.lm_lam_up, t.lm_lam_max)
        if tol > 0.0 and k >= kmin and not (Lb_prev - Lb > tol * Lb):
            break
    return w_best, G, g, Lb, lam, hist, nacc


def lab_lm_fit(self, wts, fit, data, fcfg):
    fl = CFG["flags"]
    spec, t = self.spec, self.tcfg
    P = spec.nparams
    dt = torch.float64
    X = E._normalise(torch.stack([f.to(dt) for f in data.feats], dim=1), data)
    pr = torch.stack([p.to(dt) for p in data.prices_next] +
                     [torch.full_like(data.target, float(data.bond_next), dtype=dt)], dim=1)
    y = data.target.to(dt)
    first = not CFG["log"]
    cur = int(wts[L.W_CUR].item())
    w0 = wts[cur * L.PMAX: cur * L.PMAX + P].to(dt).clone()
    lam = float(t.lm_lam0)
    if first and "lf" in fl:
        lam = fl["lf"]
    if not first and "carry" in fl:
        lam = max(CFG["lam_end"] * fl["carry"], t.lm_lam_min)
    rec = {}
    if first and "ms" in fl:
        K, n1 = int(fl["ms"]), int(fl.get("ms_n1", 50))
        nsub = min(X.shape[0], 1 << int(fl.get("ms_sub", 14)))
        o = spec.offsets
        starts = [w0]
        for k in range(1, K):
            wk = hm.init_weights(spec, w0[o["b3"]:o["P"]].numpy(), seed=CFG["seed"] + 1000 * k)
            starts.append(torch.tensor(wk, dtype=dt))
        res = [lm_core(spec, t, s, X[:nsub], pr[:nsub], y[:nsub], t.lm_gram_paths, n1, lam) for s in starts]
        kb = int(np.argmin([r[3] for r in res]))
        rec["ms_losses"] = [r[3] for r in res]
        rec["ms_pick"] = kb
        w_best, G, g, Lb, lam, hist, nacc = lm_core(spec, t, res[kb][0], X, pr, y, t.lm_gram_paths,
                                                    int(fl.get("ms_n2", 25)), res[kb][4])
    else:
        w_best, G, g, Lb, lam, hist, nacc = lm_core(spec, t, w0, X, pr, y, t.lm_gram_paths, int(fcfg.epochs), lam,
                                                    tol=0.0 if first else fl.get("adapt", 0.0))
    bi = E._lm_bias_index(spec, t)
    if "outfix" in fl:
        # exact Newton step on the whole (linear) output layer at the final
        # point: 2 G_oo d = -g_o (Gram of the subsample, full-batch gradient)
        P_ = spec.nparams
        n_out = spec.hidden * spec.nout + spec.nout
        oi = torch.arange(P_ - n_out, P_)
        Goo = G[oi][:, oi]
        mu = fl.get("ofmu", 0.0)
        A = 2.0 * Goo + torch.diag(2.0 * Goo.diagonal() * mu) + 1e-10 * torch.eye(n_out, dtype=G.dtype) * Goo.diagonal().mean()
        dlt = torch.linalg.solve(A, -g[oi])
        w_best = w_best.clone()
        w_best[oi] += fl["outfix"] * dlt
    elif bi >= 0 and float(G[bi, bi]) > 0.0:
        w_best = w_best.clone()
        w_best[bi] -= g[bi] / (2.0 * G[bi, bi])
    w32 = w_best.to(torch.float32)
    wts[:P] = w32
    wts[L.PMAX:L.PMAX + P] = w32
    wts[L.W_CUR] = 0.0
    fit.zero_()
    fit[L.F_WBEST:L.F_WBEST + P] = w32
    fit[L.F_BEST] = Lb
    fit[L.F_LAST_LOSS] = Lb
    fit[L.F_EPOCH] = len(hist)
    fit[L.F_STOPPED] = 1.0
    fit[L.F_HASBEST] = 1.0
    CFG["lam_end"] = lam
    rec.update({"passes": len(hist) - 1, "acc": nacc, "L": Lb, "lam": lam})
    CFG["log"].append(rec)


def parse_flags(v):
    out = {}
    for f in v.split("+"):
        if f == "base":
            continue
        for key in ("ms_n1", "ms_n2", "ms_sub", "ms", "carry", "lf", "adapt", "outfix", "ofmu"):
            if f.startswith(key):
                out[key] = float(f[len(key):].lstrip("="))
                break
        else:
            raise SystemExit(f"unknown flag {f}")
    return out


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--variants", default="base")
    ap.add_argument("--seeds", default="1234")
    ap.add_argument("--preset", default="euro30")
    ap.add_argument("--paths-log2", type=int, default=16)
    ap.add_argument("--extra", default="")
    a = ap.parse_args()
    import bench

    E.TorchBackend._lm_fit = lab_lm_fit
    for v in a.variants.split(","):
        for s in a.seeds.split(","):
            CFG.update(flags=parse_flags(v), log=[], seed=int(s))
            buf = io.StringIO()
            argv = ["--cpu", "--preset", a.preset, "--paths-log2", str(a.paths_log2), "--steps", "1",
                    "--warmup", "0", "--seed", s] + a.extra.split()
            with redirect_stdout(buf):
                bench.main(argv)
            q = json.loads(buf.getvalue().strip().splitlines()[-1])["quality"]
            log = CFG["log"]
            print(json.dumps({"variant": v, "seed": int(s), "pnl_std": round(q["terminal_pnl_std"], 4),
                              "resid_std": round(q["terminal_residual_std"], 4), "V0": round(q["V0"], 4),
                              "first_L": log[0]["L"], "ms": log[0].get("ms_losses"), "pick": log[0].get("ms_pick"),
                              "acc_rest": sum(x["acc"] for x in log[1:]),
                              "passes_rest": sum(x["passes"] for x in log[1:])}), flush=True)


if __name__ == "__main__":
    main()
