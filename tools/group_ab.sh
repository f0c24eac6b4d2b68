#!/bin/bash
# A/B of the pre-order level groups (PM_OPT_GROUP_WAVES / _LEVELS) on C3 / C2 / N* (GPU box,
# repo root): VARIANTS="v1 v2" GRP="0 32768" LEVELS="2 3" NS=1 tools/group_ab.sh
set -o pipefail
mkdir -p gpurun_out/group
run() {  # tag lib args...
  local tag=$1 lib=$2; shift 2
  PANMAN_AMD_LIB=$lib timeout -k 10 240 python bench.py --no-cpu --with none --steps 10 --warmup 3 "$@" > gpurun_out/group/$tag.json 2> gpurun_out/group/$tag.err || { echo "FAIL $tag"; tail -5 gpurun_out/group/$tag.err; exit 1; }
  python3 -c "import json;d=json.load(open('gpurun_out/group/$tag.json'));print('$tag', round(d['ms_per_step'],3), '%.3e'%d['value'])"
}
for v in cur ${VARIANTS:-}; do
  if [ $v = cur ]; then L=panman_amd/libpanman_amd.so; else L=build_var/$v/libpanman_amd.so; fi
  for p in ${GRP:-0 32768}; do
    for lv in ${LEVELS:-3}; do
      [ $p = 0 ] && [ $lv != 3 ] && continue
      [ $v != cur ] && [ $p = 0 ] && continue
      run c3_${v}_g${p}_l$lv $L --tree sars-like --leaves 100000 --sites 30000 --group $p --group-levels $lv
      run c2_${v}_g${p}_l$lv $L --leaves 4096 --sites 15000 --group $p --group-levels $lv
      [ -n "${NS:-}" ] && run ns_${v}_g${p}_l$lv $L --group $p --group-levels $lv
    done
  done
done
exit 0
