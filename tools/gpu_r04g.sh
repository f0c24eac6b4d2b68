#!/bin/bash
# Pre-order traffic attribution (PMC per variant, timing-only variants) and the C4 rank share's
# footprint.
set -o pipefail
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
(cd /tmp && timeout -k 5 60 rocprofv3 -L > $GRAFT_REPO_ROOT/gpurun_out/rocprof_counters.txt 2>&1) || true
bash tools/pmc_variants.sh FETCH_SIZE base nodirty nopfinal || exit 2
bash tools/ab_variants.sh fitch 1 default nodirty nopfinal || exit 3
timeout -k 10 600 python bench.py --no-cpu --with none --leaves 8000000 --sites 3750 --steps 5 --warmup 2 > gpurun_out/c4share_r04g.json 2> gpurun_out/c4share_r04g.err || { tail -5 gpurun_out/c4share_r04g.err; exit 4; }
python3 -c "import json;d=json.load(open('gpurun_out/c4share_r04g.json'));print('C4 share', round(d['ms_per_step'],3), json.dumps(d['footprint']))"
