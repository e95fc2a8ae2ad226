"""Durations of the LM kernels by position inside each later date of ONE
replay (rocprofv3 results db): which solve / pass / reduce of a date costs
what.  usage: python tools/solve_positions.py RESULTS.db"""
import collections
import sqlite3
import sys


def main():
    c = sqlite3.connect(sys.argv[1])
    rows = list(c.execute("select s.kernel_name, d.start, d.end from rocpd_kernel_dispatch d "
                          "join rocpd_info_kernel_symbol s on d.kernel_id = s.id order by d.start"))
    sims = [i for i, r in enumerate(rows) if "k_sim_scan" in r[0]]
    start = sims[-2]
    end = next(i for i in range(start, len(rows)) if "k_hedge_pnl" in rows[i][0])
    rep = rows[start:end + 1]
    fe = next(i for i, r in enumerate(rep) if "k_hedge_eval" in r[0])
    pos = collections.defaultdict(list)
    cnt = collections.Counter()
    for name, t0, t1 in rep[fe:]:
        k = next((x for x in ("k_lm_solve", "k_lm_pass", "k_lm_reduce", "k_hedge_eval") if x in name), None)
        if k is None:
            continue
        if k == "k_hedge_eval":
            cnt.clear()
        pos[(k, cnt[k])].append((t1 - t0) / 1e3)
        cnt[k] += 1
    for (k, i), v in sorted(pos.items()):
        print(f"{k:14s} #{i}  n={len(v):3d}  mean {sum(v) / len(v):7.2f} us  min {min(v):7.2f}  max {max(v):7.2f}")


if __name__ == "__main__":
    main()
