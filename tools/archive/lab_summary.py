import json,collections,sys,statistics as st
rows=[json.loads(l) for f in sys.argv[1:] for l in open(f)]
by=collections.defaultdict(list)
for r in rows: by[(r['v'],r.get('ex'))].append(r)
for (v,pf),rs in by.items():
  print(f"{v:28s} {pf} n={len(rs)} pnl {st.mean(r['pnl'] for r in rs):.4f} max {max(r['pnl'] for r in rs):.4f} res {st.mean(r['res'] for r in rs):.4f} L {st.mean(r['L'] for r in rs):.3e}", [r['reach']['1.2e-05'] for r in rs],[r['reach']['3e-05'] for r in rs])
