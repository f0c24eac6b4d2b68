#!/bin/bash
# Replay-mode bench of library variants (tools/build_variant.sh), "base" = in-tree:
#   tools/replay_variants.sh NAME...
set -o pipefail
mkdir -p gpurun_out
for n in "$@"; do
  if [ "$n" = base ]; then lib=""; else lib=build_var/$n/libpanman_amd.so; fi
  PANMAN_AMD_LIB=$lib timeout -k 10 300 python bench.py --no-cpu --mode replay --replay-tree ${TREE:-random-join} --steps 20 > gpurun_out/rv_$n.json 2> gpurun_out/rv_$n.err || { echo "$n failed"; tail -3 gpurun_out/rv_$n.err; exit 1; }
  python3 -c "import json; d=json.load(open('gpurun_out/rv_$n.json')); print('$n', round(d['ms_per_step'], 3))"
done
