#!/bin/bash
# r05w: non-temporal loads of k_tail's subtree leaf words / of Fitch set records (A/B)
set -o pipefail
cd "$(dirname "$0")/.."
tools/ab_variants.sh fitch 2 default subnt fsetnt && tools/ab_variants.sh sankoff 1 default subnt
for rep in 1 2; do
for t in random-join sars-like; do
for v in base u256 u256l32; do
  lib=""; [ $v != base ] && lib=build_var/$v/libpanman_amd.so
  PANMAN_AMD_LIB=$lib timeout -k 10 300 python bench.py --no-cpu --mode replay --replay-tree $t --steps 20 --warmup 3 > gpurun_out/rw_${v}_$t.json 2> gpurun_out/rw_${v}_$t.err || { echo "$v $t failed"; tail -3 gpurun_out/rw_${v}_$t.err; exit 1; }
  python3 -c "import json; d=json.load(open('gpurun_out/rw_${v}_$t.json')); r=d['roofline']; print('$v $t', round(d['ms_per_step'], 3), r['kernel'], r['avg_launch_ms'], r['leaf_groups'])"
done
done
done
