#!/usr/bin/env python3
"""Average PMC counter values per kernel from rocprofv3 counter_collection.csv files."""
import csv
import glob
import sys
from collections import defaultdict

root = sys.argv[1] if len(sys.argv) > 1 else "gpurun_out"
filt = sys.argv[2] if len(sys.argv) > 2 else "olap_scan"
pat = sys.argv[3] if len(sys.argv) > 3 else "pmc*"   # run directories, e.g. pmcab_p1_*
by_kernel = len(sys.argv) > 4 and sys.argv[4] == "by-kernel"  # one block per kernel name
vals = defaultdict(list)
for f in glob.glob(f"{root}/{pat}/**/*counter_collection.csv", recursive=True):
    for r in csv.DictReader(open(f)):
        if filt in r.get("Kernel_Name", ""):
            k = (r["Kernel_Name"][:60] if by_kernel else "", r["Counter_Name"])
            vals[k].append(float(r["Counter_Value"]))
last = None
for kn, c in sorted(vals):
    if by_kernel and kn != last:
        print(f"--- {kn}")
        last = kn
    v = vals[(kn, c)]
    print(f"{c:28s} n={len(v):3d} mean={sum(v)/len(v):16.1f} last={v[-1]:16.1f}")
