#!/bin/bash
# One PMC pass per (variant, counter group) over a short bench run:
#   tools/pmc_variants.sh "COUNTERS" NAME... [-- bench args]   -> gpurun_out/pmc_NAME_G/
set -o pipefail
export TMPDIR=/tmp
counters=$1; shift
names=(); args=()
while [ $# -gt 0 ]; do
  if [ "$1" = "--" ]; then shift; args=("$@"); break; fi
  names+=("$1"); shift
done
tag=$(echo "$counters" | tr ' ' '_' | cut -c1-40)
for n in "${names[@]}"; do
  if [ "$n" = base ]; then lib=""; else lib=build_var/$n/libpanman_amd.so; fi
  out=gpurun_out/pmc_${n}_$tag
  PANMAN_AMD_LIB=$lib timeout -s KILL 200 rocprofv3 --pmc $counters --output-format csv -d "$out" -o run -- python3 bench.py --no-cpu --with none --steps 2 --warmup 1 "${args[@]}" > "$out.json" 2> "$out.log" || { echo "$n failed"; tail -5 "$out.log"; exit 1; }
  python3 tools/pmc_summary.py "$out" | grep -A12 -E "^k_(down|fitch_up)" > "$out.txt" || true
  echo "== $n"; cat "$out.txt"
done
