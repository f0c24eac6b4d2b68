#!/bin/bash
# Bench experimental library variants (tools/build_variant.sh) side by side:
#   tools/variants.sh NAME... [-- bench args]   ("base" = the in-tree library)
set -o pipefail
mkdir -p gpurun_out
names=(); args=()
while [ $# -gt 0 ]; do
  if [ "$1" = "--" ]; then shift; args=("$@"); break; fi
  names+=("$1"); shift
done
for n in "${names[@]}"; do
  if [ "$n" = base ]; then lib=""; else lib=build_var/$n/libpanman_amd.so; fi
  PANMAN_AMD_LIB=$lib timeout -k 10 300 python bench.py --no-cpu --with none "${args[@]}" > gpurun_out/var_$n.json 2> gpurun_out/var_$n.err || { echo "$n failed"; tail -5 gpurun_out/var_$n.err; exit 1; }
  python3 -c "
import json; d=json.load(open('gpurun_out/var_$n.json')); r=d['roofline']
print('$n', 'ms', round(d['ms_per_step'],3), r['kernel'], 'kern_ms', r['kernel_ms_per_step'], r['other_kernels_ms_per_step'])"
done
