"""Idle gaps in rocprofv3 kernel traces (one CSV per process under a directory).

    python3 scripts/mi355x/gaps.py gpurun_out/r3b/mp8 [--last-ms 20]

For each process: kernels, busy time (union of its kernels' intervals), the gaps between consecutive kernels of the
process and their distribution; then the same over all processes merged (how much of the window the GPU ran any
kernel). Used to tell queue time-slicing (long gaps while other processes' kernels run) from launch overhead.
"""
import argparse
import csv
import glob
import os
import statistics


def load(path):
    rows = []
    with open(path) as f:
        for r in csv.DictReader(f):
            name = r.get("Kernel_Name", "")
            if "rocclr" in name:
                continue
            rows.append((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), name, r.get("Queue_Id", "?")))
    rows.sort()
    return rows


def union(iv):
    tot, cur_s, cur_e = 0, None, None
    for s, e in sorted(iv):
        if cur_e is None or s > cur_e:
            if cur_e is not None:
                tot += cur_e - cur_s
            cur_s, cur_e = s, e
        else:
            cur_e = max(cur_e, e)
    if cur_e is not None:
        tot += cur_e - cur_s
    return tot


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("dir")
    ap.add_argument("--last-ms", type=float, default=0, help="only the last N ms of the trace (the timed loop)")
    a = ap.parse_args()
    files = sorted(glob.glob(os.path.join(a.dir, "**", "*kernel_trace.csv"), recursive=True))
    allrows = []
    per = []
    for f in files:
        rows = load(f)
        if rows:
            per.append((f, rows))
            allrows += rows
    if not allrows:
        print("no kernel traces under", a.dir)
        return
    tend = max(r[1] for r in allrows)
    tlo = tend - int(a.last_ms * 1e6) if a.last_ms > 0 else min(r[0] for r in allrows)
    print(f"window {(tend - tlo) / 1e6:.3f} ms, {len(per)} process trace(s)")
    for f, rows in per:
        rows = [r for r in rows if r[0] >= tlo]
        if not rows:
            continue
        busy = union([(s, e) for s, e, _, _ in rows])
        gaps = [rows[i + 1][0] - rows[i][1] for i in range(len(rows) - 1)]
        gaps = [g for g in gaps if g > 0]
        big = sorted(gaps)[-5:]
        print(f"{os.path.relpath(f, a.dir)}: {len(rows)} kernels, busy {busy / 1e6:.3f} ms "
              f"({100 * busy / max(1, tend - tlo):.1f} % of the window), gaps: n={len(gaps)} "
              f"median {statistics.median(gaps) / 1e3 if gaps else 0:.1f} us, max {[round(g / 1e3, 1) for g in big]} us")
        byname = {}
        for s, e, n, _ in rows:
            byname.setdefault(n[:60], []).append(e - s)
        for n, d in sorted(byname.items(), key=lambda kv: -sum(kv[1]))[:6]:
            print(f"    {sum(d) / 1e3:10.1f} us total  {statistics.median(d) / 1e3:8.1f} us median  x{len(d):<5} {n}")
    allw = [(s, e) for s, e, _, _ in allrows if s >= tlo]
    print(f"all processes: GPU running some kernel {100 * union(allw) / max(1, tend - tlo):.1f} % of the window")


if __name__ == "__main__":
    main()
