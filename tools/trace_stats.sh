#!/bin/bash
# rocprofv3 kernel-trace --stats of one bench command: tools/trace_stats.sh TAG [bench args]
#   -> gpurun_out/trace_TAG/kernel_stats.csv (+ the bench line in gpurun_out/trace_TAG.json)
set -euo pipefail
cd "$(dirname "$0")/.."
export TMPDIR=/tmp
tag=$1; shift
out=gpurun_out/trace_$tag
mkdir -p "$out"
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d "$out" -o run -- python3 bench.py --no-cpu --with none "$@" \
  > "$out.json" 2> "$out.log"
find "$out" -name "*kernel_stats.csv" -exec cp {} "$out/kernel_stats.csv" \;
python3 - "$out/kernel_stats.csv" <<'P'
import csv, re, sys
rows = list(csv.DictReader(open(sys.argv[1])))
for r in sorted(rows, key=lambda r: -float(r["TotalDurationNs"]))[:12]:
    m = re.search(r"\b(k_\w+(<[^(]*>)?)", r["Name"]); n = m.group(0) if m else r["Name"][:40]
    n = n.replace("(pm::Mode)", "M")
    print(f'{n:40s} calls {int(r["Calls"]):6d} total {float(r["TotalDurationNs"])/1e6:9.2f} ms  avg {float(r["AverageNs"])/1e3:9.1f} us')
P
