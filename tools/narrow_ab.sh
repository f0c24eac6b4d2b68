#!/bin/bash
# A/B of PM_OPT_NARROW on C2 / C3 / N* (GPU box, repo root): one bench line per (config, narrow)
set -o pipefail
mkdir -p gpurun_out/narrow
run() {  # tag args...
  local tag=$1; shift
  timeout -k 10 240 python bench.py --no-cpu --with none --steps 10 --warmup 3 "$@" > gpurun_out/narrow/$tag.json 2> gpurun_out/narrow/$tag.err || { echo "FAIL $tag"; tail -5 gpurun_out/narrow/$tag.err; exit 1; }
  python3 -c "import json;d=json.load(open('gpurun_out/narrow/$tag.json'));print('$tag', round(d['ms_per_step'],3), '%.3e'%d['value'])"
}
for n in ${NARROW:-0 16}; do
  run c3_n$n --tree sars-like --leaves 100000 --sites 30000 --narrow $n
  run c2_n$n --leaves 4096 --sites 15000 --narrow $n
done
for n in ${NARROW_NS:-0 16}; do
  run ns_n$n --narrow $n
done
