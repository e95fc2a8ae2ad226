"""Phase breakdown of ONE graph replay of the euro30 bench from a rocprofv3
results database: kernels of the first date's multi-start exploration (grid
y > 1), the first date's polish, and the later dates, with totals / counts /
means per kernel, and the idle time between kernels.
usage: python tools/phases.py RESULTS.db"""
import collections
import sqlite3
import sys


def main():
    c = sqlite3.connect(sys.argv[1])
    rows = list(c.execute("select s.kernel_name, d.start, d.end, d.grid_size_y from rocpd_kernel_dispatch d "
                          "join rocpd_info_kernel_symbol s on d.kernel_id = s.id order by d.start"))
    sims = [i for i, r in enumerate(rows) if "k_sim_scan" in r[0]]
    start = sims[-2]  # the last replay (each replay simulates the main paths and the exploration prefix)
    end = next(i for i in range(start, len(rows)) if "k_hedge_pnl" in rows[i][0])
    rep = rows[start:end + 1]
    first_eval = next(i for i, r in enumerate(rep) if "k_hedge_eval" in r[0])
    agg, cnt = collections.defaultdict(float), collections.Counter()
    for i, (name, t0, t1, gy) in enumerate(rep):
        seg = "explore" if gy > 1 else ("first" if i < first_eval else "later")
        k = name.split("(")[0].replace("_ZN3rph", "").split("E")[0][:24]
        agg[(seg, k)] += (t1 - t0) / 1e3
        cnt[(seg, k)] += 1
    print(f"replay {(rep[-1][2] - rep[0][1]) / 1e3:.1f} us, {len(rep)} kernels, first date "
          f"{(rep[first_eval][1] - rep[0][1]) / 1e3:.1f} us, idle "
          f"{sum(max(0, rep[i + 1][1] - rep[i][2]) for i in range(len(rep) - 1)) / 1e3:.1f} us")
    for k in sorted(agg):
        print(f"  {k[0]:8s} {k[1]:26s} n={cnt[k]:3d} total {agg[k]:8.1f} us  mean {agg[k] / cnt[k]:6.2f} us")


if __name__ == "__main__":
    main()
