#!/usr/bin/env python3
"""Sum rocprofv3 --pmc counter CSVs of tools/sqprof.sh per counter for the chain kernel."""
import csv
import glob
import os
import sys
from collections import defaultdict

d = sys.argv[1]
tot = defaultdict(float)
disp = defaultdict(set)
for f in glob.glob(os.path.join(d, "g*", "**", "*counter_collection.csv"), recursive=True):
    with open(f) as fh:
        for r in csv.DictReader(fh):
            if "chain_viterbi" not in r.get("Kernel_Name", ""):
                continue
            name = r.get("Counter_Name")
            tot[name] += float(r.get("Counter_Value", 0) or 0)
            disp[name].add(r.get("Dispatch_Id"))
for k in sorted(tot):
    n = max(len(disp[k]), 1)
    print(f"{k:28s} total {tot[k]:16.0f}  dispatches {n:3d}  per-dispatch {tot[k] / n:14.0f}")
