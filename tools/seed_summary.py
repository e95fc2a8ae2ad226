"""Summarise tools/seeds.py JSONL files: per file, P&L / analytic-hedge ratio
(mean, worst, per seed), last one-step residual (worst), ms (mean).
usage: python tools/seed_summary.py FILE.jsonl [...]"""
import json
import sys


def main():
    for fn in sys.argv[1:]:
        recs, seen = [], set()
        for line in open(fn):
            if not line.startswith("{"):
                continue
            r = json.loads(line)
            if "seed" not in r or "pnl" not in r:  # (hedge_diag records)
                continue
            k = (r["seed"], r["args"])
            if k in seen:
                continue
            seen.add(k)
            recs.append(r)
        if not recs:
            print(f"{fn}: empty")
            continue
        rat = [r["pnl"] / r["anchor_pnl"] if r.get("anchor_pnl") else float("nan") for r in recs]
        res = [r["resid"] for r in recs]
        ms = sum(r["ms"] for r in recs) / len(recs)
        dv0 = max(abs(r["V0"] - r["anchor_price"]) for r in recs if r.get("anchor_price"))  if any(r.get("anchor_price") for r in recs) else float("nan")
        print(f"{fn.split('/')[-1]:28s} n={len(recs):2d} ms={ms:8.2f} ratio mean={sum(rat)/len(rat):.4f} "
              f"worst={max(rat):.4f} resid worst={max(res):.4f} |dV0|max={dv0:.2e} pnl mean={sum(r['pnl'] for r in recs)/len(recs):.4f} "
              f"worst={max(r['pnl'] for r in recs):.4f}")
        print("    " + " ".join(f"{x:.3f}" for x in rat))


if __name__ == "__main__":
    main()
