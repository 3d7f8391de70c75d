"""Summarise rocprofv3 --pmc CSVs: per kernel name, average of each counter over dispatches."""
import csv, glob, os, sys
from collections import defaultdict
d = sys.argv[1]
filt = sys.argv[2] if len(sys.argv) > 2 else "gemm"
vals = defaultdict(lambda: defaultdict(list))
durs = defaultdict(list)
for f in sorted(glob.glob(os.path.join(d, "*_counter_collection.csv"))):
    for r in csv.DictReader(open(f)):
        if filt not in r["Kernel_Name"]:
            continue
        vals[r["Kernel_Name"][:70]][r["Counter_Name"]].append(float(r["Counter_Value"]))
for f in sorted(glob.glob(os.path.join(d, "*_kernel_trace.csv"))):
    for r in csv.DictReader(open(f)):
        if filt in r["Kernel_Name"]:
            durs[r["Kernel_Name"][:70]].append(int(r["End_Timestamp"]) - int(r["Start_Timestamp"]))
for k, cs in vals.items():
    print(k)
    dd = sorted(durs.get(k, [0]))
    print(f"  median dur us {dd[len(dd)//2]/1e3:.1f}")
    for c, v in sorted(cs.items()):
        print(f"  {c:32s} {sum(v)/len(v):.4g}")
