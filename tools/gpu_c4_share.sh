#!/bin/bash
# C4 rank share (8M leaves x 3750 sites: one rank of bench.py --gpus 8), by set-record load
# policy: gpurun_out/c4_share_nt{-1,0,1}.json
set -o pipefail
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
for rep in 1 2; do
  for nt in -1 0 1; do
    timeout -k 10 400 python bench.py --no-cpu --with none --leaves 8000000 --sites 3750 --steps 10 --warmup 3 --nt-loads $nt \
      > gpurun_out/c4_share_nt$nt.json 2> gpurun_out/c4_share_nt$nt.err || { tail -5 gpurun_out/c4_share_nt$nt.err; exit 2; }
    python3 -c "import json;d=json.load(open('gpurun_out/c4_share_nt$nt.json'));r=d['roofline'];print('C4 share nt=$nt', round(d['ms_per_step'],3), r['kernel'], r['kernel_ms_per_step'], r['other_kernels_ms_per_step'])"
  done
done
