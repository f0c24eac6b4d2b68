#!/bin/bash
# r05q: k_replay_dfs shape with non-temporal rows: tile 2 / 8 KiB, 32 leaves per group, 5 waves per SIMD
set -o pipefail
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
for rep in 1 2; do
for t in random-join sars-like; do
for v in base dfs_t8k dfs_t2k dfs_l32 dfs_w5; do
  lib=""; [ $v != base ] && lib=build_var/$v/libpanman_amd.so
  PANMAN_AMD_LIB=$lib timeout -k 10 300 python bench.py --no-cpu --mode replay --replay-tree $t --steps 20 --warmup 3 > gpurun_out/rq_${v}_$t.json 2> gpurun_out/rq_${v}_$t.err || { echo "$v $t failed"; tail -3 gpurun_out/rq_${v}_$t.err; exit 1; }
  python3 -c "import json; d=json.load(open('gpurun_out/rq_${v}_$t.json')); r=d['roofline']; print('$v $t', round(d['ms_per_step'], 3), r['kernel'], r['avg_launch_ms'], 'frac_w', r.get('frac_of_measured_write'))"
done
done
done
