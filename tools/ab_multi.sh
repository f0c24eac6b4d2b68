#!/bin/bash
# N* bench of the current library and experiment builds, one line each: tools/ab_multi.sh V1 V2 ...
set -o pipefail
mkdir -p gpurun_out/ab
for v in cur "$@"; do
  if [ $v = cur ]; then L=panman_amd/libpanman_amd.so; else L=build_var/$v/libpanman_amd.so; fi
  PANMAN_AMD_LIB=$L timeout -k 10 200 python bench.py --no-cpu --with none --steps 10 --warmup 3 $BENCH_ARGS > gpurun_out/ab/$v.json 2> gpurun_out/ab/$v.err || { tail -3 gpurun_out/ab/$v.err; exit 1; }
  python3 -c "import json;d=json.load(open('gpurun_out/ab/$v.json'));r=d['roofline'];print('$v', round(d['ms_per_step'],3), r['kernel'], r['kernel_ms_per_step'], r['other_kernels_ms_per_step'])"
done
