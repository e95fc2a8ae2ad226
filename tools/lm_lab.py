"""CPU laboratory for Levenberg-Marquardt variants of the hedge fits.

Runs ``bench.py --cpu`` (torch backend, float64 LM oracle) with
``TorchBackend._lm_fit`` replaced by a variant and prints one JSON line per
variant: SF P&L std, residual std, V0 and the per-date acceptance counts.

  python tools/lm_lab.py --variants base,stale --paths-log2 16

Variants (combinable with '+'):
  base    the HIP solver's sequence (csrc/hedge_lm.hip)
  stale   pipelined factorisation: the accept branch steps with the PREVIOUS
          best point's Gram matrix (factorised while the pass runs), the
          reject branch is exact (its Gram is the best point's)
  varpro  accept / reject on the loss projected over the (linear) output
          layer: the exact output-layer minimiser is applied to every
          evaluated point before the comparison
  outfix  lm_out_fix's final output-layer Newton step (full-batch output
          Gram, fp64); omu=<x>: its relative damping (TrainConfig.lm_out_mu);
          ogtail=<k>: only when the best point is one of the last k
          evaluations (else the bias step); ogsub=<k>: output Gram over
          every k-th path only (the gradient stays full-batch)
  oglast  with outfix: the output Gram of the last evaluation only; a
          rejected last trial + its out step is published when it beats
          the best point (else the bias step at the best point)
"""
from __future__ import annotations

import argparse
import io
import json
import os
import sys
from contextlib import redirect_stdout

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

from rphedge import engine as E  # noqa: E402
from rphedge.ops import layout as L  # noqa: E402
from rphedge.models.hedge_mlp import torch_forward  # noqa: E402

VARIANT = {"flags": set(), "log": []}


def _out_slice(spec):
    """Indices of the output layer (W3, b3) in the flat parameter vector."""
    P = spec.nparams
    n_out = spec.hidden * spec.nout + spec.nout
    return list(range(P - n_out, P))


def lab_lm_fit(self, wts, fit, data, fcfg):
    from torch.func import jacrev, vmap

    flags = VARIANT["flags"]
    if "fo" in flags and VARIANT["log"]:
        # first-date-only variant: later dates run the base sequence
        flags = {f for f in flags if f in ("fo",) or f.startswith("carry=") or f.startswith("adapt=")}
    spec, t = self.spec, self.tcfg
    P = spec.nparams
    dt = torch.float64
    X = E._normalise(torch.stack([f.to(dt) for f in data.feats], dim=1), data)
    pr = torch.stack([p.to(dt) for p in data.prices_next] +
                     [torch.full_like(data.target, float(data.bond_next), dtype=dt)], dim=1)
    y = data.target.to(dt)
    n_glob = float(self.n_local)
    ns = max(L.LM_TILE, min(int(t.lm_gram_paths), self.n_local)) // L.LM_TILE * L.LM_TILE
    blk, bstride = E.lm_gram_geometry(self.n_local, ns, 1)
    sub = torch.tensor([(j // blk) * bstride + j % blk for j in range(ns)], dtype=torch.long)

    oi = torch.tensor(_out_slice(spec))
    kvf = dict(f.split("=") for f in flags if "=" in f)
    vpk = int(kvf["vp"]) if "vp" in kvf else (10**9 if "varpro" in flags else 0)

    def v_one(w, x, p):
        return (torch_forward(spec, w, x[None])[0] * p).sum()

    def evaluate(w):
        wg = w.detach().clone().requires_grad_(True)
        e = (torch_forward(spec, wg, X) * pr).sum(1) - y
        lsum = (e * e).sum()
        (lsum / n_glob).backward()
        J = vmap(jacrev(v_one), in_dims=(None, 0, 0))(w.detach(), X[sub], pr[sub])
        G = (J.T @ J) / ns
        if "varpro" in flags or "vp" in kvf:
            # output-layer Gram over EVERY path (the loss is exactly quadratic
            # in the output layer): its features are a2 x (price combination)
            with torch.no_grad():
                Jo = vmap(jacrev(v_one), in_dims=(None, 0, 0))(w.detach(), X, pr)[:, oi]
                G = G.clone()
                G[oi[:, None], oi[None, :]] = (Jo.T @ Jo) / n_glob
        return G, wg.grad.detach(), float(lsum) / n_glob

    def project(w, G, g, Lv, Gsub=None, mu=0.0):
        """Exact minimiser over the output layer (loss quadratic in it, Gram
        from the subsample): w_o += -G_oo^-1 g_o / 2, loss and gradient
        updated to first order (mu: lm_out_newton's relative damping)."""
        Goo = (Gsub if Gsub is not None else G)[oi][:, oi]
        try:
            do = torch.linalg.solve(2.0 * Goo + torch.diag(2.0 * mu * Goo.diagonal()) +
                                    1e-9 * torch.eye(len(oi), dtype=dt) * Goo.diagonal().mean(), -g[oi])
        except RuntimeError:
            return w, g, Lv
        w2 = w.clone()
        w2[oi] += do
        g2 = g + 2.0 * G[:, oi] @ do
        L2 = Lv + 0.5 * float(g[oi] @ do)
        return w2, g2, L2

    def factor(G, lam, k=0):
        A = 2.0 * G
        dg = torch.diagonal(A).clone()
        fl = float(kvf.get("floor", t.lm_diag_floor))
        dmp = torch.clamp_min(dg, fl * float(dg.mean())) * lam + float(t.lm_ridge) * float(dg.mean())
        if "nodo" in flags or k < int(kvf.get("nodo", 0)):
            dmp[oi] = float(t.lm_ridge) * float(dg.mean())
        Lc, info = torch.linalg.cholesky_ex(A + torch.diag(dmp))
        return (Lc if int(info) == 0 else None), dmp

    cur = int(wts[L.W_CUR].item())
    w_best = wts[cur * L.PMAX: cur * L.PMAX + P].to(dt).clone()
    prev = VARIANT.get("norm")
    if "renorm" in flags and prev is not None and data.fmu:
        # keep the warm start's function of the RAW features: x_new = (s - mu_n) isd_n
        o = spec.offsets
        W1 = w_best[o["W1"]:o["b1"]].view(spec.nin, spec.hidden)
        b1 = w_best[o["b1"]:o["W2"]]
        for f in range(spec.nin):
            mo, io = prev[0][f], prev[1][f]
            mn, inn = data.fmu[f], data.fisd[f]
            b1 += W1[f] * io * (mn - mo)
            W1[f] *= io / inn
    VARIANT["norm"] = (tuple(data.fmu), tuple(data.fisd)) if data.fmu else None
    kv = kvf
    first = not VARIANT["log"]
    lam = float(kv["lf"]) if (first and "lf" in kv) else float(t.lm_lam0)
    if not first and "carry" in kv:
        lam = max(VARIANT["lam_end"] * float(kv["carry"]), t.lm_lam_min)
    G, g, Lb = evaluate(w_best)
    if vpk > 0:
        w_best, g, Lb = project(w_best, G, g, Lb)
    hist = [Lb]
    last = (w_best, G, g, Lb)  # the last evaluated point
    kbest = 0  # the evaluation the best point came from
    nacc = 0
    stale = "stale" in flags or ("stale_rest" in VARIANT["flags"] and not first)
    pend = None  # stale accept-branch factor (pipelined variant)
    for k in range(1, int(fcfg.epochs) + 1):
        if pend is not None:
            Lc, pend = pend, None
        else:
            Lc, _ = factor(G, lam, k)
        if Lc is None:
            trial = w_best.clone()
            lam = min(lam * t.lm_lam_up * t.lm_lam_up, t.lm_lam_max)
        else:
            trial = w_best + torch.cholesky_solve(-g[:, None], Lc)[:, 0]
        Gt, gt, Lt = evaluate(trial)
        if k < vpk:
            trial, gt, Lt = project(trial, Gt, gt, Lt)
        elif k == vpk and vpk > 0:
            # leaving the projected phase: re-evaluate the best point exactly
            pass
        hist.append(Lt)
        last = (trial, Gt, gt, Lt)
        Lb_prev = Lb
        if Lt == Lt and Lt < Lb:
            nacc += 1
            lam = max(lam * t.lm_lam_down, t.lm_lam_min)
            if stale:
                # factorised while this pass ran: the previous best Gram
                pend, _ = factor(G, lam)
            w_best, G, g, Lb = trial, Gt, gt, Lt
            kbest = k
        else:
            lam = min(lam * t.lm_lam_up, t.lm_lam_max)
        if "adapt" in kv and not first and k >= int(kv.get("kmin", 2)):
            # adaptive budget: stop once a pass improves the best loss by less than tol
            if (Lb_prev - Lb) / max(Lb, 1e-300) < float(kv["adapt"]):
                break
    if os.environ.get("LAB_DEBUG"): print("HIST", json.dumps([float("%.4g" % h) for h in hist]), file=sys.stderr)
    bi = E._lm_bias_index(spec, t)
    ntail = int(kvf.get("ogtail", 10**9))  # the output Gram exists for the last ntail evaluations only
    if "oglast" in flags and kbest != len(hist) - 1:
        # the output Gram of the LAST evaluation only: the out step at the
        # rejected last trial (its own exact Gram and gradient) is published
        # when it beats the best point
        lw, lG, lg, lL = last
        with torch.no_grad():
            Jo = vmap(jacrev(v_one), in_dims=(None, 0, 0))(lw.detach(), X, pr)[:, oi]
            Gf = lG.clone()
            Gf[oi[:, None], oi[None, :]] = (Jo.T @ Jo) / n_glob
        w2, g2, L2 = project(lw, Gf, lg, lL, mu=float(kvf.get("omu", 0.0)))
        if L2 < Lb:
            w_best, g, Lb = w2, g2, L2
        elif bi >= 0 and float(G[bi, bi]) > 0.0:
            w_best = w_best.clone()
            w_best[bi] -= g[bi] / (2.0 * G[bi, bi])
    elif "outfix" in flags and kbest > len(hist) - 1 - ntail:
        # lm_out_fix: exact output-layer Newton step with the full-batch output Gram
        with torch.no_grad():
            Jo = vmap(jacrev(v_one), in_dims=(None, 0, 0))(w_best.detach(), X, pr)[:, oi]
            Gf = G.clone()
            ks = int(kvf.get("ogsub", 1))  # output Gram over every ks-th path only
            Js = Jo[::ks]
            Gf[oi[:, None], oi[None, :]] = (Js.T @ Js) / float(len(Js))
        w_best, g, Lb = project(w_best, Gf, g, Lb, mu=float(kvf.get("omu", 0.0)))
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
    VARIANT["lam_end"] = lam
    VARIANT["log"].append({"passes": len(hist) - 1, "acc": nacc, "L0": hist[0], "L": Lb, "lam": lam, "hist": hist})



def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--variants", default="base")
    ap.add_argument("--preset", default="euro30")
    ap.add_argument("--paths-log2", type=int, default=16)
    ap.add_argument("--extra", default="", help="extra bench.py args")
    a = ap.parse_args()
    import bench

    for v in a.variants.split(","):
        VARIANT["flags"] = set(v.split("+"))
        VARIANT["log"] = []
        VARIANT["norm"] = None
        E.TorchBackend._lm_fit = lab_lm_fit
        buf = io.StringIO()
        argv = ["--cpu", "--preset", a.preset, "--paths-log2", str(a.paths_log2), "--steps", "1", "--warmup", "0"]
        argv += a.extra.split()
        with redirect_stdout(buf):
            bench.main(argv)
        res = json.loads(buf.getvalue().strip().splitlines()[-1])
        q = res["quality"]
        log = VARIANT["log"]
        if os.environ.get("LAB_HIST"):
            with open(os.environ["LAB_HIST"], "w") as fh:
                json.dump(log, fh)
        print(json.dumps({"variant": v, "extra": a.extra, "pnl_std": round(q["terminal_pnl_std"], 4),
                          "resid_std": round(q["terminal_residual_std"], 4), "V0": round(q["V0"], 4),
                          "first": log[0] if log else None,
                          "acc_rest": sum(x["acc"] for x in log[1:]), "fits": len(log),
                          "passes_rest": sum(x["passes"] for x in log[1:])}), flush=True)


if __name__ == "__main__":
    main()
