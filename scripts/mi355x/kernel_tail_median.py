"""Median duration (us) of the last N dispatches of every kernel whose name contains PATTERN in a rocprofv3 rocpd db
(the first sweeps over freshly initialised fields run slower).
    python scripts/mi355x/kernel_tail_median.py DB PATTERN [N]"""
import sqlite3
import statistics
import sys

db, pat = sys.argv[1], sys.argv[2]
n = int(sys.argv[3]) if len(sys.argv) > 3 else 6
rows = sqlite3.connect(db).execute("select name, start, end from kernels order by start").fetchall()
d = [(e - s) / 1e3 for name, s, e in rows if pat in name]
tail = d[-n:]
print(f"{len(d)} dispatches, last {len(tail)}: median {statistics.median(tail):.1f} us, min {min(tail):.1f}, "
      f"first {d[0]:.1f}" if d else "no dispatch")
