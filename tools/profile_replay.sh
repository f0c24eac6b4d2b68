#!/bin/bash
# PMC HBM traffic of the replay kernel (separate FETCH_SIZE / WRITE_SIZE passes):
#   tools/profile_replay.sh TAG  ->  gpurun_out/prof_replay_TAG/{traffic.txt,traffic.json}
set -euo pipefail
cd "$(dirname "$0")/.."
export TMPDIR=/tmp
out=gpurun_out/prof_replay_$1
mkdir -p "$out"
for c in FETCH_SIZE WRITE_SIZE; do
  timeout -k 10 300 rocprofv3 --pmc $c --output-format csv -d "$out/$c" -o run -- python3 bench.py --no-cpu --mode replay --steps 2 --warmup 1 \
    > "$out/$c.json" 2> "$out/$c.log"
done
key=$(python3 -c "import json;d=json.load(open('$out/FETCH_SIZE.json'));c=d['config'];print(f\"replay:{c['leaves_per_gpu']}x{c['columns']}\")")
build=$(python3 -c "import json;print(json.load(open('$out/FETCH_SIZE.json'))['build_id'])")
python3 tools/pmc_traffic.py "$out/FETCH_SIZE" "$out/WRITE_SIZE" "$key" "$out/traffic.json" "$build" > "$out/traffic.txt"
cat "$out/traffic.txt"
