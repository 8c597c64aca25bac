"""Average each PMC counter per kernel over its dispatches (rocprofv3 --pmc csv output under DIR/p*/)."""
import collections
import csv
import glob
import sys

d = sys.argv[1]
acc = collections.defaultdict(lambda: collections.defaultdict(list))
for f in glob.glob(f"{d}/p*/**/*counter_collection.csv", recursive=True):
    per = collections.defaultdict(float)
    for r in csv.DictReader(open(f)):
        per[(r["Kernel_Name"], r["Dispatch_Id"], r["Counter_Name"])] += float(r["Counter_Value"])
    for (k, _, c), v in per.items():
        acc[k][c].append(v)
for k, cs in acc.items():
    if "rocclr" in k or "fill_region" in k:
        continue
    print(k[:90])
    for c in sorted(cs):
        v = cs[c]
        print(f"  {c:24s} {sum(v) / len(v):16.0f}  (n={len(v)})")
