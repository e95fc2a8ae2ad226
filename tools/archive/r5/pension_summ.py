"""Summarise tools/archive/r5/pension_lm.py records: per run and per variant
(mean +- sd over seeds of V0 / phi0 / psi0, last-date one-step residual std,
self-financing P&L std, Q99 fraction above, median wall time).

usage: python tools/archive/r5/pension_summ.py FILE.jsonl [FILE ...]"""
import collections
import json
import sys

import numpy as np


def main():
    g = collections.OrderedDict()
    for fn in sys.argv[1:]:
        for line in open(fn):
            r = json.loads(line)
            g.setdefault(r["opt"], []).append(r)
    for k, v in g.items():
        def f(key):
            return np.array([x[key] for x in v], np.float64)
        sd = (lambda a: a.std(ddof=1) if len(a) > 1 else 0.0)
        print(f"{k:44s} n={len(v)} V0 {f('V0').mean():8.0f}±{sd(f('V0')):6.0f} phi {f('phi0').mean():7.0f}±{sd(f('phi0')):6.0f}"
              f" psi {f('psi0').mean():7.0f}±{sd(f('psi0')):6.0f} resid {f('terminal_residual_std').mean() if 'terminal_residual_std' in v[0] else float('nan'):6.0f}"
              f" pnl {f('pnl_std').mean():6.0f} q99max {f('q99_resid_q99_max').max():.4f} above {f('q99_frac_above_mean').mean():.4f}"
              f" wall {np.median(f('wall_s')):.3f}s")


if __name__ == "__main__":
    main()
