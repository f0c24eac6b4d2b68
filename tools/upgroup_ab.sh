#!/bin/bash
# A/B of the grouped post-order launches (PM_OPT_UP_GROUP) and PM_UP_GROUP_NODES variants on
# C3 / C2 / N* (GPU box, repo root): VARIANTS="v1 v2" tools/upgroup_ab.sh
set -o pipefail
mkdir -p gpurun_out/ug
run() {  # tag lib args...
  local tag=$1 lib=$2; shift 2
  PANMAN_AMD_LIB=$lib timeout -k 10 240 python bench.py --no-cpu --with none --steps 10 --warmup 3 "$@" > gpurun_out/ug/$tag.json 2> gpurun_out/ug/$tag.err || { echo "FAIL $tag"; tail -5 gpurun_out/ug/$tag.err; exit 1; }
  python3 -c "import json;d=json.load(open('gpurun_out/ug/$tag.json'));print('$tag', round(d['ms_per_step'],3), '%.3e'%d['value'])"
}
for v in off cur ${VARIANTS:-}; do
  a=""; L=panman_amd/libpanman_amd.so
  if [ $v = off ]; then a="--no-up-group"; elif [ $v != cur ]; then L=build_var/$v/libpanman_amd.so; fi
  run c3_$v $L --tree sars-like --leaves 100000 --sites 30000 $a
  run c2_$v $L --leaves 4096 --sites 15000 $a
  run ns_$v $L $a
done
exit 0
