"""Per-kernel statistics (calls, total / mean / min us, share) from a rocprofv3
results database (rocpd sqlite, the default output format) or a
kernel_stats.csv.  usage: python tools/kstats.py FILE [name-filter]"""
import collections
import csv
import sqlite3
import sys


def from_db(fn):
    c = sqlite3.connect(fn)
    q = ("select s.kernel_name, d.end - d.start from rocpd_kernel_dispatch d "
         "join rocpd_info_kernel_symbol s on d.kernel_id = s.id")
    out = collections.defaultdict(list)
    for name, dur in c.execute(q):
        out[name].append(dur)
    return out


def main():
    fn = sys.argv[1]
    filt = sys.argv[2] if len(sys.argv) > 2 else ""
    if fn.endswith(".csv"):
        rows = {r["Name"]: (int(r["Calls"]), float(r["TotalDurationNs"]), float(r["AverageNs"]), float(r["MinNs"]))
                for r in csv.DictReader(open(fn))}
    else:
        rows = {k: (len(v), float(sum(v)), sum(v) / len(v), float(min(v))) for k, v in from_db(fn).items()}
    tot = sum(r[1] for r in rows.values())
    for k, (n, t, a, m) in sorted(rows.items(), key=lambda kv: -kv[1][1]):
        if filt and filt not in k:
            continue
        short = k.split("(")[0].replace("void ", "").replace("rph::", "")[:70]
        print(f"{short:70s} n={n:5d} tot={t / 1e3:9.1f}us mean={a / 1e3:7.2f}us min={m / 1e3:7.2f}us {100 * t / tot:5.1f}%")


if __name__ == "__main__":
    main()
