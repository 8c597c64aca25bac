#!/usr/bin/env python3
"""Summarise a rocprofv3 rocpd SQLite trace (kernel + memory-copy tracing): per-kernel and per-copy-kind counts,
median / total durations, and the last `--tail` events of the timeline on each stream (relative microseconds).

    python scripts/mi355x/rocpd_summary.py gpurun_out/r4b/eng_r0/eng_results.db [--tail 30] > summary.txt"""
import argparse
import sqlite3
import statistics as stats
from collections import defaultdict


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("db")
    ap.add_argument("--tail", type=int, default=30)
    a = ap.parse_args()
    cur = sqlite3.connect(a.db).cursor()
    ks = cur.execute("select name, start, end, stream_id from kernels order by start").fetchall()
    cs = cur.execute("select name, start, end, stream_id, size from memory_copies order by start").fetchall()
    print(f"# {a.db}: {len(ks)} kernel dispatches, {len(cs)} memory copies")
    agg = defaultdict(list)
    for n, s, e, _ in ks:
        agg[n.split("(")[0][:90]].append((e - s) / 1e3)
    print(f"{'kernel':90s} {'n':>5s} {'med_us':>9s} {'total_us':>10s}")
    for n, v in sorted(agg.items(), key=lambda kv: -sum(kv[1])):
        print(f"{n:90s} {len(v):5d} {stats.median(v):9.1f} {sum(v):10.1f}")
    cagg = defaultdict(list)
    for n, s, e, _, sz in cs:
        cagg[(n, sz)].append((e - s) / 1e3)
    print(f"\n{'copy kind':40s} {'bytes':>10s} {'n':>5s} {'med_us':>9s} {'min_us':>9s} {'max_us':>9s} {'med_GBps':>9s}")
    for (n, sz), v in sorted(cagg.items(), key=lambda kv: -sum(kv[1])):
        m = stats.median(v)
        print(f"{n:40s} {sz:10d} {len(v):5d} {m:9.1f} {min(v):9.1f} {max(v):9.1f} {sz / m / 1e3 if m else 0:9.1f}")
    ev = [("K " + n.split("(")[0][-40:], s, e, st) for n, s, e, st in ks] + \
         [(f"C {n[12:]} {sz}", s, e, st) for n, s, e, st, sz in cs]
    ev.sort(key=lambda x: x[1])
    tail = ev[-a.tail:] if a.tail > 0 else []
    if tail:
        t0 = tail[0][1]
        print(f"\nlast {len(tail)} events (us from the first shown)")
        for n, s, e, st in tail:
            print(f"  {n:60s} stream {st!s:>3s} {(s - t0) / 1e3:9.1f} .. {(e - t0) / 1e3:9.1f}  ({(e - s) / 1e3:7.1f})")


if __name__ == "__main__":
    main()
