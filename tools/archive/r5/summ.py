"""Summarise seed-sweep JSONL files (tools/archive/r5/seeds.py): per file mean / worst
P&L std, residual, |V0 - analytic|, ms."""
import json
import sys

import numpy as np

for fn in sys.argv[1:]:
    rs = [json.loads(l) for l in open(fn) if l.strip()]
    if not rs:
        continue
    p = np.array([r["pnl"] for r in rs])
    res = np.array([r["resid"] for r in rs])
    ms = np.array([r["ms"] for r in rs])
    dv = np.array([abs(r["V0"] - r["anchor_price"]) if r.get("anchor_price") else np.nan for r in rs])
    anc = rs[0].get("anchor_pnl")
    print(f"{fn.split('/')[-1]:34s} n={len(rs)} ms {ms.mean():.3f} | pnl mean {p.mean():.4f} worst {p.max():.4f} "
          f"({p.mean() / anc if anc else float('nan'):.3f}x) | resid mean {res.mean():.4f} worst {res.max():.4f} | "
          f"|dV0| max {np.nanmax(dv):.5f} | seeds>0.915: {[r['seed'] for r in rs if r['pnl'] > 0.915]}")
