#!/usr/bin/env python3
"""Turn rocprofv3 --pmc FETCH_SIZE / WRITE_SIZE passes into HBM bytes per launch.

Usage: tools/pmc_traffic.py FETCH_DIR WRITE_DIR WORKLOAD_KEY OUT_JSON BUILD_ID
  FETCH_DIR / WRITE_DIR: rocprofv3 -d directories (…_counter_collection.csv inside)
  WORKLOAD_KEY: e.g. fitch:1000000x30000 (mode:leaves x sites-per-GPU), the key bench.py looks up.
  BUILD_ID: pm_build_id() of the profiled library (bench.py's "build_id"); written beside every
  entry as "<key>:build", and bench.py reports no traffic when the loaded library differs.

gfx950 corrections (MI355X_MICROARCH.md §HBM): FETCH_SIZE (KiB) reports half of the bytes
of a wide coalesced 16-B-per-lane stream -> doubled; WRITE_SIZE (KiB) is exact for 16-B
streaming stores.  Both kernels load and store uint4 per lane.
"""
import collections
import csv
import glob
import json
import os
import re
import sys


def short(name):
    """'void pm::k_down<(pm::Mode)0, true>(pm::DownArgs)' -> 'k_down' (the bench's key)."""
    m = re.search(r"\b(k_\w+)", name)
    return m.group(1) if m else name


def per_kernel(d, counter):
    agg = collections.defaultdict(lambda: [0, 0.0])
    for f in glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True):
        for r in csv.DictReader(open(f)):
            if r["Counter_Name"] != counter:
                continue
            a = agg[short(r["Kernel_Name"])]
            a[0] += 1
            a[1] += float(r["Counter_Value"]) * 1024.0
    return agg


def main():
    fetch_dir, write_dir, key, out, build = sys.argv[1:6]
    fetch = per_kernel(fetch_dir, "FETCH_SIZE")
    write = per_kernel(write_dir, "WRITE_SIZE")
    res = json.load(open(out)) if os.path.exists(out) else {}
    # runs of the profiled command: k_site_score is launched exactly once per parsimony run,
    # so "<key>:step" = a kernel's HBM bytes per run (all its launches: levels, bands, tail)
    runs = fetch.get("k_site_score", [0])[0]
    for k in sorted(set(fetch) & set(write)):
        nf, bf = fetch[k]
        nw, bw = write[k]
        per_launch = 2.0 * bf / nf + bw / nw
        res.setdefault(k, {})[key] = per_launch
        res[k][key + ":build"] = build
        step = ""
        if runs:
            res[k][key + ":step"] = (2.0 * bf + bw * nf / nw) / runs
            res[k][key + ":fetch_step"] = 2.0 * bf / runs
            step = f"  {res[k][key + ':step'] / 1e9:8.3f} GB/run ({nf / runs:.1f} launches)"
        print(f"{k:32s} launches {nf:5d}  fetch(x2) {2 * bf / nf / 1e6:10.2f} MB  write {bw / nw / 1e6:10.2f} MB"
              f"  -> {per_launch / 1e6:10.2f} MB/launch{step}")
    json.dump(res, open(out, "w"), indent=1, sort_keys=True)


if __name__ == "__main__":
    main()
