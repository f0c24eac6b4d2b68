#!/usr/bin/env python3
"""Average every PMC counter per kernel over a rocprofv3 --pmc directory."""
import collections
import csv
import glob
import os
import sys

agg = collections.defaultdict(lambda: collections.defaultdict(list))
for f in glob.glob(os.path.join(sys.argv[1], "**", "*counter_collection.csv"), recursive=True):
    for r in csv.DictReader(open(f)):
        agg[r["Kernel_Name"].split("(")[0]][r["Counter_Name"]].append(float(r["Counter_Value"]))
for k in sorted(agg):
    cs = agg[k]
    n = max(len(v) for v in cs.values())
    print(f"{k}  ({n} launches)")
    for c in sorted(cs):
        v = cs[c]
        print(f"    {c:24s} {sum(v) / len(v):16.1f}")
