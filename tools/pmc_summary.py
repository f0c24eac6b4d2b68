#!/usr/bin/env python3
"""Average every PMC counter per kernel over a rocprofv3 --pmc directory."""
import collections
import csv
import glob
import os
import re
import sys


def short(name):
    """'void pm::k_down<(pm::Mode)0, true>(pm::DownArgs)' -> 'k_down'."""
    m = re.search(r"\b(k_\w+)", name)
    return m.group(1) if m else name.split("(")[0]


agg = collections.defaultdict(lambda: collections.defaultdict(list))
for f in glob.glob(os.path.join(sys.argv[1], "**", "*counter_collection.csv"), recursive=True):
    for r in csv.DictReader(open(f)):
        agg[short(r["Kernel_Name"])][r["Counter_Name"]].append(float(r["Counter_Value"]))
for k in sorted(agg):
    cs = agg[k]
    n = max(len(v) for v in cs.values())
    print(f"{k}  ({n} launches)")
    for c in sorted(cs):
        v = cs[c]
        print(f"    {c:24s} {sum(v) / len(v):16.1f}")
