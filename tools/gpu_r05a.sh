#!/bin/bash
# r05a: deep replay tests first, then every GPU test, C5 replay on both tree families, default bench.
set -o pipefail
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_replay_deep.py tests/test_gpu_replay.py tests/test_gpu_reroot.py -x -v --timeout 120 --timeout-method thread > gpurun_out/r05a_deep.log 2>&1 \
  || { echo "DEEP TESTS FAILED"; tail -60 gpurun_out/r05a_deep.log; exit 1; }
tail -2 gpurun_out/r05a_deep.log
for t in random-join sars-like; do
  timeout -k 10 300 python bench.py --mode replay --replay-tree $t --no-cpu --steps 20 --warmup 3 > gpurun_out/r05a_replay_$t.json 2> gpurun_out/r05a_replay_$t.err \
    || { echo "replay bench $t failed"; tail -20 gpurun_out/r05a_replay_$t.err; exit 2; }
  python3 -c "import json;d=json.load(open('gpurun_out/r05a_replay_$t.json'));r=d['roofline'];print('$t', d['config']['workload'], round(d['ms_per_step'],3), r.get('kernel_ms'), r['frac'])"
done
tools/gpu_round_check.sh r05a
