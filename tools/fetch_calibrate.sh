#!/bin/bash
# FETCH_SIZE / WRITE_SIZE per launch of scattered 16-B reads (GPU box, repo root):
#   tools/fetch_calibrate.sh  ->  gpurun_out/fetchcal/{fetch_S,write_S}/..., fetchcal.txt
set -o pipefail
cd "$(dirname "$0")/.."
export TMPDIR=/tmp
out=gpurun_out/fetchcal
mkdir -p $out
lanes=8388608
for st in 16 32 64 128 256; do
  for c in FETCH_SIZE WRITE_SIZE; do
    timeout -s KILL 120 rocprofv3 --pmc $c --output-format csv -d $out/${c}_$st -o run -- python3 -c "
import ctypes as C, sys; sys.path.insert(0, '.')
import panman_amd
ms = C.c_double(0); rc = panman_amd.load().pm_gather_probe(0, $lanes, $st, 3, C.byref(ms)); assert rc == 0, rc
print($st, ms.value)" > $out/${c}_$st.log 2>&1 || { echo "probe $st $c failed"; tail -5 $out/${c}_$st.log; exit 1; }
  done
done
python3 - $out $lanes <<'P' | tee $out/fetchcal.txt
import csv, glob, sys
out, lanes = sys.argv[1], int(sys.argv[2])
print("stride_B  launches  FETCH_SIZE_KiB/launch  bytes/lane(read 4x16B)  WRITE_SIZE_KiB/launch  ms/launch")
for st in (16, 32, 64, 128, 256):
    vals = {}
    for c in ("FETCH_SIZE", "WRITE_SIZE"):
        rows = [r for f in glob.glob(f"{out}/{c}_{st}/**/*counter_collection.csv", recursive=True)
                for r in csv.DictReader(open(f)) if "k_gather_probe" in r["Kernel_Name"] and r["Counter_Name"] == c]
        vals[c] = (len(rows), sum(float(r["Counter_Value"]) for r in rows) / max(len(rows), 1))
    ms = open(f"{out}/FETCH_SIZE_{st}.log").read().split()[-1]
    n, f = vals["FETCH_SIZE"]
    print(f"{st:8d} {n:9d} {f:22.1f} {f * 1024 / lanes:22.2f} {vals['WRITE_SIZE'][1]:22.1f}  {ms}")
P
