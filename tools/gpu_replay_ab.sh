#!/bin/bash
# Replay A/B: deep + replay GPU tests, then the C5 replay on both tree families (TAG names the outputs).
set -o pipefail
cd "$(dirname "$0")/.."
tag=${1:-ab}
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_replay_deep.py tests/test_gpu_replay.py tests/test_gpu_reroot.py -x -q --timeout 120 --timeout-method thread > gpurun_out/${tag}_tests.log 2>&1 \
  || { echo "REPLAY TESTS FAILED"; tail -60 gpurun_out/${tag}_tests.log; exit 1; }
tail -1 gpurun_out/${tag}_tests.log
for rep in 1 2; do
for t in random-join sars-like; do
  timeout -k 10 300 python bench.py --mode replay --replay-tree $t --no-cpu --steps 20 --warmup 3 > gpurun_out/${tag}_replay_$t.json 2> gpurun_out/${tag}_replay_$t.err \
    || { echo "replay bench $t failed"; tail -20 gpurun_out/${tag}_replay_$t.err; exit 2; }
  python3 -c "import json;d=json.load(open('gpurun_out/${tag}_replay_$t.json'));r=d['roofline'];print('$t', round(d['ms_per_step'],3), r['frac'], r.get('traffic'))"
done
done
