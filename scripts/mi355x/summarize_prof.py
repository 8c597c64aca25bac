import csv, glob, collections, sys
d = sys.argv[1]
for f in glob.glob(d + "/kt/**/*kernel_stats.csv", recursive=True):
    print("== kernel stats")
    for r in csv.DictReader(open(f)):
        print(f"  {float(r['AverageNs'])/1e3:9.1f} us x{r['Calls']:>4}  {r['Name'][:90]}")
for f in glob.glob(d + "/kt/**/*kernel_trace.csv", recursive=True):
    rows = list(csv.DictReader(open(f)))
    seen = set()
    for r in rows:
        k = r['Kernel_Name'][:60]
        if k in seen: continue
        seen.add(k)
        print(f"  vgpr={r['VGPR_Count']:>4} sgpr={r['SGPR_Count']:>4} lds={r['LDS_Block_Size']:>6} scratch={r['Scratch_Size']} grid={r['Grid_Size_X']}x{r['Grid_Size_Y']} wg={r['Workgroup_Size_X']}x{r['Workgroup_Size_Y']} {k}")
agg = collections.defaultdict(lambda: collections.defaultdict(list))
for f in glob.glob(d + "/p*/**/*counter_collection.csv", recursive=True):
    for r in csv.DictReader(open(f)):
        agg[r['Kernel_Name'][:70]][r['Counter_Name']].append(float(r['Counter_Value']))
for k, v in agg.items():
    if 'rocclr' in k or 'fill' in k: continue
    print("== " + k)
    for c, vals in v.items():
        print(f"   {c:16s} {sum(vals)/len(vals):.4g}")
