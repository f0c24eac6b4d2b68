#!/bin/bash
# Profile the bench workload on a GPU box (run from the repo root):
#   tools/profile_fitch.sh TAG [bench.py args]   ->  gpurun_out/prof_TAG/
# Passes (separate runs, as the MI355X guide prescribes): kernel-trace stats, FETCH_SIZE,
# WRITE_SIZE, SQ cycle/instruction counters.  Then HBM bytes per launch and SQ summaries.
set -euo pipefail
cd "$(dirname "$0")/.."
export TMPDIR=/tmp
tag=$1; shift
out=gpurun_out/prof_$tag
mkdir -p "$out"
mode=fitch
for a in "$@"; do case $a in sankoff) mode=sankoff;; esac; done
run() {  # run NAME ROCPROF_ARGS... -- (bench args appended)
  local name=$1; shift
  timeout -k 10 400 rocprofv3 "$@" --output-format csv -d "$out/$name" -o run -- python3 bench.py --no-cpu --with none "${BENCH[@]}" \
    > "$out/$name.json" 2> "$out/$name.log"
}
BENCH=(--steps 4 --warmup 1 "$@")
run stats --kernel-trace --stats
BENCH=(--steps 2 --warmup 1 "$@")
run fetch --pmc FETCH_SIZE
run write --pmc WRITE_SIZE
run sq --pmc SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_SMEM SQ_INSTS_LDS
leaves=$(python3 -c "import json;d=json.load(open('$out/stats.json'));print(d['config']['leaves'])")
sites=$(python3 -c "import json;d=json.load(open('$out/stats.json'));print(d['config']['sites_per_gpu'])")
# (the tree family joins the key unless random-join: bench.py traffic_key)
tsuf=$(python3 -c "import json;t=json.load(open('$out/stats.json'))['config']['tree'];print('' if t=='random-join' else ':'+t)")
build=$(python3 -c "import json;print(json.load(open('$out/stats.json'))['build_id'])")
python3 tools/pmc_traffic.py "$out/fetch" "$out/write" "$mode:${leaves}x${sites}$tsuf" "$out/traffic.json" "$build" > "$out/traffic.txt"
python3 tools/pmc_summary.py "$out/sq" > "$out/sq.txt"
find "$out" -name "*kernel_stats.csv" -exec cp {} "$out/kernel_stats.csv" \;
echo "profile $tag done"
