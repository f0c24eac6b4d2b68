#!/bin/bash
# r05ac: set-record load policy per run (two builds of the passes) -- full GPU suite, then N* and
# C3 with the policy forced each way
set -o pipefail
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/gputests_r05ac.log 2>&1 \
  || { echo "GPU TESTS FAILED"; tail -60 gpurun_out/gputests_r05ac.log; exit 1; }
tail -1 gpurun_out/gputests_r05ac.log
for rep in 1 2; do
  for nt in -1 0 1; do
    for shape in "" "--tree sars-like --leaves 100000"; do
      for mode in fitch sankoff; do
        timeout -k 10 300 python bench.py --no-cpu --with none --steps 10 --warmup 3 --mode $mode --nt-loads $nt $shape > gpurun_out/ac.json 2> gpurun_out/ac.err || { echo "bench failed"; tail -5 gpurun_out/ac.err; exit 2; }
        python3 -c "import json;d=json.load(open('gpurun_out/ac.json'));print('nt=$nt', '$mode', d['config']['workload'][:24], round(d['ms_per_step'],3))"
      done
    done
  done
done
