#!/bin/bash
# Sweep-kernel variants and thresholds (bench lines only): tools/gpu_cl_sweep.sh TAG
set -o pipefail
cd "$(dirname "$0")/.."
tag=$1
mkdir -p gpurun_out
run() {  # run NAME LIB ARGS...
  local name=$1 lib=$2; shift 2
  local env=""; [ "$lib" != default ] && env="PANMAN_AMD_LIB=build_var/$lib/libpanman_amd.so"
  env $env timeout -k 10 300 python bench.py --no-cpu --with none --steps 10 --warmup 3 "$@" > gpurun_out/${tag}_$name.json 2> gpurun_out/${tag}_$name.err || { echo "$name failed"; tail -5 gpurun_out/${tag}_$name.err; exit 3; }
  python3 -c "import json;d=json.load(open('gpurun_out/${tag}_$name.json'));r=d['roofline'];print('$name', round(d['ms_per_step'],3), 'up', r['kernel_ms_per_step'] if r['kernel'].startswith('k_fitch_up') else r['other_kernels_ms_per_step'], r['launches_per_step'])"
}
C3="--tree sars-like --leaves 100000"
for v in ${VARIANTS:-default}; do
  for cl in ${C3CL:-1}; do run c3_${v}_$cl $v $C3 --cluster $cl; done
done
for cl in ${NSCL:-}; do run ns_$cl default --cluster $cl; done
