#!/bin/bash
# C4 per-rank share, Sankoff (8M leaves x 3750 sites: one rank of --gpus 8)
set -o pipefail
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
timeout -k 10 600 python bench.py --no-cpu --with none --mode sankoff --leaves 8000000 --sites 3750 --steps 5 --warmup 2 > gpurun_out/c4share_sankoff_r04.json 2> gpurun_out/c4share_sankoff_r04.err || { tail -5 gpurun_out/c4share_sankoff_r04.err; exit 2; }
python3 -c "import json;d=json.load(open('gpurun_out/c4share_sankoff_r04.json'));print('C4 share sankoff', round(d['ms_per_step'],3), '%.3g' % d['value'], json.dumps(d.get('footprint'))[:300])"
