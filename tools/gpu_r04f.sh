#!/bin/bash
# Which change broke the narrow-band test: the working tree vs builds without the wide-node
# mask prefetch / without the mixed kernel / before the prefetch
set -o pipefail
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
for v in ${VARIANTS:-default nopf nomixed}; do
  lib=""; [ "$v" != default ] && lib="PANMAN_AMD_LIB=build_var/$v/libpanman_amd.so"
  env $lib timeout -k 10 300 python -u -m pytest tests/test_gpu_narrow.py tests/test_gpu_group.py -q --timeout 120 --timeout-method thread > gpurun_out/narrow_$v.log 2>&1
  rc=$?
  echo "$v rc=$rc $(tail -1 gpurun_out/narrow_$v.log)"
  grep FAILED gpurun_out/narrow_$v.log | head -4
  [ $rc -ge 124 ] && exit 3
done
exit 0
