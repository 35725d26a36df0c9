#!/usr/bin/env python3
"""Average per-dispatch counter values of the checksum kernel from rocprofv3
counter_collection.csv files under a directory.  python tools/pmc_summary.py DIR [kernel-substring]"""
import csv
import glob
import sys
from collections import defaultdict

d = sys.argv[1]
pat = sys.argv[2] if len(sys.argv) > 2 else "crc32"
vals = defaultdict(list)
for f in glob.glob(f"{d}/**/*counter_collection.csv", recursive=True):
    for row in csv.DictReader(open(f)):
        if pat not in row.get("Kernel_Name", ""):
            continue
        vals[row["Counter_Name"]].append(float(row["Counter_Value"]))
for k in sorted(vals):
    v = vals[k]
    print(f"{k:28s} n={len(v):3d} mean={sum(v) / len(v):,.0f}")
