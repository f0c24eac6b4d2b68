#!/bin/bash
# r05ad: k_replay_dfs write-out unrolled for whole tiles without absent blocks (A/B)
set -o pipefail
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
for rep in 1 2; do
for t in random-join sars-like; do
for v in base dfswo; do
  lib=""; [ $v != base ] && lib=build_var/$v/libpanman_amd.so
  PANMAN_AMD_LIB=$lib timeout -k 10 300 python bench.py --no-cpu --mode replay --replay-tree $t --steps 20 --warmup 3 > gpurun_out/rd_${v}_$t.json 2> gpurun_out/rd_${v}_$t.err || { echo "$v $t failed"; tail -3 gpurun_out/rd_${v}_$t.err; exit 1; }
  python3 -c "import json; d=json.load(open('gpurun_out/rd_${v}_$t.json')); r=d['roofline']; print('$v $t', round(d['ms_per_step'], 3), r['kernel'], r['avg_launch_ms'])"
done
done
done
tools/ab_variants.sh fitch 2 default scorent
