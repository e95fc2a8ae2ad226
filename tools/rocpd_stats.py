"""Per-kernel statistics from a rocprofv3 SQLite database (rocpd format,
the default output of ``rocprofv3 --kernel-trace``): name, calls, total /
mean / min / max µs and share, sorted by total time; optional CSV output.

    python tools/rocpd_stats.py gpurun_out/prof/run_results.db [out.csv] [--calls-per N]

``--calls-per N`` divides calls and total by N (per-step numbers for a run of
N timed replays)."""
import csv
import sqlite3
import sys


def stats(db):
    c = sqlite3.connect(db)
    rows = c.execute("select name, count(*), sum(end - start), avg(end - start), min(end - start), "
                     "max(end - start) from kernels group by name order by sum(end - start) desc").fetchall()
    tot = sum(r[2] for r in rows) or 1
    return [dict(name=r[0], calls=r[1], total_us=r[2] / 1e3, mean_us=r[3] / 1e3, min_us=r[4] / 1e3,
                 max_us=r[5] / 1e3, share=r[2] / tot) for r in rows]


def main(argv):
    args = [a for a in argv if not a.startswith("--")]
    per = 1
    if "--calls-per" in argv:
        per = int(argv[argv.index("--calls-per") + 1])
        args = [a for a in args if a != str(per)]
    st = stats(args[0])
    if len(args) > 1:
        with open(args[1], "w", newline="") as f:
            w = csv.DictWriter(f, fieldnames=list(st[0]))
            w.writeheader()
            w.writerows(st)
    for r in st[:25]:
        print(f"{r['calls'] / per:9.1f} {r['total_us'] / per:11.1f} us {r['mean_us']:9.2f} mean "
              f"{r['min_us']:8.2f} min {100 * r['share']:5.1f}%  {r['name'][:110]}")


if __name__ == "__main__":
    main(sys.argv[1:])
