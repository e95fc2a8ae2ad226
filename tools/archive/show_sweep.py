"""Print one summary line per bench JSON line of a sweep file."""
import json
import sys

for path in sys.argv[1:]:
    for l in open(path):
        d = json.loads(l)
        q, c, lm = d["quality"], d["config"], d.get("lm") or {}
        ms = c.get("lm_multistart") or {}
        anc = q.get("hedge_anchor") or {}
        print("%-9s %7.2f ms  pnl %.4f (anchor %s)  res %.4f  V0 %.4f  starts %s/%s/%s carry %s rest %s stop %s acc %.2f first %s pick %s" % (
            c.get("preset"), d["ms_per_step"], q["terminal_pnl_std"], ("%.4f" % anc["pnl_std"]) if anc.get("pnl_std") else "-",
            q["terminal_residual_std"], q["V0"], ms.get("starts_per_rank"), ms.get("explore_passes"),
            ms.get("explore_paths_per_rank"), c.get("lm_lam_carry"), c.get("lm_passes_rest"), c.get("lm_stop"),
            lm.get("acceptance_rate", float("nan")), "%.3g" % lm.get("first_date", {}).get("best_loss", float("nan")),
            (lm.get("multistart") or {}).get("pick")))
