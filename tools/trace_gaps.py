"""Kernel timeline of one replay from a rocprofv3 SQLite trace: per kernel
name the mean duration and the mean idle gap before it (end of the previous
kernel on the queue -> its start), to price launch / dependency gaps.

    python tools/trace_gaps.py gpurun_out/prof/x_results.db [kernel-substring]
"""
import collections
import sqlite3
import sys


def main(db, filt=""):
    c = sqlite3.connect(db)
    rows = c.execute("select name, start, end from kernels order by start").fetchall()
    gap = collections.defaultdict(list)
    dur = collections.defaultdict(list)
    prev_end = None
    for name, s, e in rows:
        short = name.split("(")[0].replace("void rph::", "")[:70]
        if prev_end is not None and filt in short:
            gap[short].append((s - prev_end) / 1e3)
        dur[short].append((e - s) / 1e3)
        prev_end = e
    tot_gap = sum(sum(v) for v in gap.values())
    print(f"kernels {len(rows)}, summed gaps {tot_gap:.1f} us, summed busy {sum(sum(v) for v in dur.values()):.1f} us")
    for k in sorted(dur, key=lambda k: -sum(dur[k]))[:12]:
        g = gap.get(k, [0.0])
        gs = sorted(g)
        print(f"{k:70s} n={len(dur[k]):6d} dur {sum(dur[k]) / len(dur[k]):7.2f} us  gap before: mean {sum(g) / len(g):6.2f} median {gs[len(gs) // 2]:6.2f} us")


if __name__ == "__main__":
    main(sys.argv[1], sys.argv[2] if len(sys.argv) > 2 else "")
