#!/usr/bin/env python3
"""Merge per-run PMC traffic files (tools/pmc_traffic.py outputs, every entry stamped with the
build id it was measured on) into profiles/traffic_fitch.json, dropping entries without a
build stamp:  tools/merge_traffic.py OUT.json IN.json..."""
import json
import sys

out = sys.argv[1]
res = {}
for path in sys.argv[2:]:
    for k, v in json.load(open(path)).items():
        res.setdefault(k, {}).update(v)
clean = {}
for k, v in res.items():
    base = lambda kk: kk.rsplit(":", 1)[0] if kk.endswith((":step", ":fetch_step")) else kk
    keep = {kk: vv for kk, vv in v.items() if (base(kk) + ":build") in v or kk.endswith(":build")}
    keep = {kk: vv for kk, vv in keep.items() if not kk.endswith(":build") or kk[:-6] in keep}
    if keep:
        clean[k] = keep
json.dump(clean, open(out, "w"), indent=1, sort_keys=True)
print(f"{out}: {len(clean)} kernels")
