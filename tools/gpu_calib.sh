#!/bin/bash
# FETCH_SIZE calibration on known access patterns (tools/calib_fetch.hip):
#   tools/gpu_calib.sh TAG  ->  gpurun_out/calib_TAG/{stats,fetch,req,req64}, calib_TAG.txt
set -o pipefail
cd "$(dirname "$0")/.."
export TMPDIR=/tmp
tag=$1
out=gpurun_out/calib_$tag
mkdir -p $out
timeout -s KILL 60 rocprofv3 --kernel-trace --stats --output-format csv -d $out/stats -o run -- ./tools/calib_fetch > $out/run.txt 2> $out/stats.log || exit 2
timeout -s KILL 60 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $out/fetch -o run -- ./tools/calib_fetch > /dev/null 2> $out/fetch.log || exit 3
timeout -s KILL 60 rocprofv3 --pmc TCC_EA0_RDREQ_sum TCC_BUBBLE_sum TCC_EA0_RDREQ_32B_sum --output-format csv -d $out/req -o run -- ./tools/calib_fetch > /dev/null 2> $out/req.log || exit 4
timeout -s KILL 60 rocprofv3 --pmc TCC_EA0_RDREQ_64B_sum --output-format csv -d $out/req64 -o run -- ./tools/calib_fetch > /dev/null 2> $out/req64.log || exit 5
python3 - $out > gpurun_out/calib_$tag.txt <<'P'
import collections, csv, glob, os, sys
d = sys.argv[1]
def dispatches(sub):
    rows = []
    for f in glob.glob(os.path.join(d, sub, "**", "*counter_collection.csv"), recursive=True):
        rows += list(csv.DictReader(open(f)))
    by = collections.defaultdict(dict)
    for r in rows:
        by[(int(r["Dispatch_Id"]), r["Kernel_Name"].split("(")[0])][r["Counter_Name"]] = float(r["Counter_Value"])
    return [(k[1], v) for k, v in sorted(by.items())]
names = ["fill"] + ["stream", "s128", "s64", "s64x2", "row64", "rand"] * 2
cols = {}
for sub in ("fetch", "req", "req64"):
    for i, (kn, v) in enumerate(dispatches(sub)):
        cols.setdefault(i, {"kernel": kn}).update(v)
for line in open(os.path.join(d, "run.txt")):
    print("#", line.rstrip())
for i in sorted(cols):
    print(i, names[i] if i < len(names) else "?", {k: (round(v) if k != "kernel" else v) for k, v in cols[i].items()})
t = [r for f in glob.glob(os.path.join(d, "stats", "**", "*kernel_trace.csv"), recursive=True) for r in csv.DictReader(open(f))]
for i, r in enumerate(sorted(t, key=lambda r: int(r["Dispatch_Id"]))):
    print("time", i, names[i] if i < len(names) else "?", (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3, "us")
P
cat gpurun_out/calib_$tag.txt
