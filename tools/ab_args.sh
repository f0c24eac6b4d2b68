#!/bin/bash
# Interleaved A/B of bench argument sets on the in-tree library:
#   tools/ab_args.sh REPS "ARGS A" "ARGS B" ...   (common args in $BENCH_ARGS)
set -o pipefail
cd "$(dirname "$0")/.."
reps=$1; shift
mkdir -p gpurun_out/ab_args
for r in $(seq $reps); do
  i=0
  for a in "$@"; do
    i=$((i + 1))
    timeout -k 10 300 python bench.py --no-cpu --with none --steps 10 --warmup 3 ${BENCH_ARGS:-} $a > gpurun_out/ab_args/$i.json 2> gpurun_out/ab_args/$i.err || { echo "bench [$a] failed"; tail -5 gpurun_out/ab_args/$i.err; exit 2; }
    python3 -c "import json;d=json.load(open('gpurun_out/ab_args/$i.json'));r=d['roofline'];print('[$a]', round(d['ms_per_step'],3), r['kernel'], r['kernel_ms_per_step'], r['other_kernels_ms_per_step'])"
  done
done
