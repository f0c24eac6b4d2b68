#!/bin/bash
# Interleaved A/B of variant libraries on the GPU box:
#   tools/ab_variants.sh MODE REPS VARIANT...   (VARIANT = default or a build_var/NAME)
set -o pipefail
cd "$(dirname "$0")/.."
mode=$1; reps=$2; shift 2
mkdir -p gpurun_out
for r in $(seq $reps); do
  for v in "$@"; do
    lib=""; [ "$v" != default ] && lib="PANMAN_AMD_LIB=build_var/$v/libpanman_amd.so"
    env $lib timeout -k 10 300 python bench.py --no-cpu --with none --steps 10 --warmup 3 --mode $mode ${BENCH_ARGS:-} > gpurun_out/ab_${mode}_$v.json 2> gpurun_out/ab_${mode}_$v.err || { echo "bench $v failed"; tail -5 gpurun_out/ab_${mode}_$v.err; exit 2; }
    python3 -c "import json;d=json.load(open('gpurun_out/ab_${mode}_$v.json'));r=d['roofline'];print('$mode $v', round(d['ms_per_step'],3), r['kernel'], r['kernel_ms_per_step'], r['other_kernels_ms_per_step'])"
  done
done
