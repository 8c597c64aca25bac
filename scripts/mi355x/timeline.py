import csv, glob, sys
d = sys.argv[1]
f = glob.glob(d + "/**/*kernel_trace.csv", recursive=True)[0]
rows = sorted(csv.DictReader(open(f)), key=lambda r: int(r['Start_Timestamp']))
rows = [r for r in rows if 'rocclr' not in r['Kernel_Name'] and 'fill_region' not in r['Kernel_Name']]
t0 = int(rows[0]['Start_Timestamp'])
for r in rows[-int(sys.argv[2]) if len(sys.argv) > 2 else -24:]:
    s = int(r['Start_Timestamp']) - t0
    e = int(r['End_Timestamp']) - t0
    print(f"{s/1e3:10.1f} -> {e/1e3:10.1f}  {(e-s)/1e3:8.1f}us q{r['Queue_Id']} {r['Kernel_Name'][:70]}")
