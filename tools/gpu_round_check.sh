#!/bin/bash
# GPU box: every -m gpu test, then the default bench line (driver-style).
#   tools/gpu_round_check.sh TAG  ->  gpurun_out/gputests_TAG.log, gpurun_out/bench_default_TAG.json
set -o pipefail
cd "$(dirname "$0")/.."
tag=$1
mkdir -p gpurun_out
(while true; do date >> gpurun_out/heartbeat_$tag.txt; sleep 30; done) &
hb=$!
trap "kill $hb" EXIT
if [ -z "${ONLY_LINES:-}" ]; then
if [ -z "${NOTESTS:-}" ]; then
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 900 --timeout-method thread > gpurun_out/gputests_$tag.log 2>&1 \
  || { echo "GPU TESTS FAILED"; tail -60 gpurun_out/gputests_$tag.log; exit 1; }
tail -2 gpurun_out/gputests_$tag.log
fi
timeout -k 10 900 python bench.py > gpurun_out/bench_default_$tag.json 2> gpurun_out/bench_default_$tag.err \
  || { echo "bench failed"; tail -20 gpurun_out/bench_default_$tag.err; exit 2; }
python3 -c "
import json;d=json.load(open('gpurun_out/bench_default_$tag.json'));r=d['roofline']
print('N*', round(d['ms_per_step'],3), 'ms', r['kernel'], r['kernel_ms_per_step'], r['other_kernels_ms_per_step'], 'frac', r['frac'], 'traffic', r['traffic'])
print('cmds', json.dumps(d.get('commands'))[:1500])
print('replay cpu', json.dumps(d['secondary']['replay']['cpu_baseline'])[:400])
"
fi
# the other configs' lines (bench.py's labels), each against the same traffic file
line() {  # NAME ARGS...
  local name=$1; shift
  timeout -k 10 600 python bench.py --no-cpu --with none --steps 10 --warmup 3 "$@" > gpurun_out/bench_${name}_$tag.json 2> gpurun_out/bench_${name}_$tag.err \
    || { echo "bench $name failed"; tail -20 gpurun_out/bench_${name}_$tag.err; exit 3; }
  python3 -c "
import json;d=json.load(open('gpurun_out/bench_${name}_$tag.json'));r=d['roofline']
print('$name', round(d['ms_per_step'],3), 'ms', r['kernel'], r['kernel_ms_per_step'], r['other_kernels_ms_per_step'], 'launches', r['launches_per_step'], 'frac', r['frac'], 'traffic', r['traffic'], r.get('traffic_over_design'))"
}
[ -n "${LINES:-1}" ] || exit 0
line c3 --tree sars-like --leaves 100000
line c3_sankoff --tree sars-like --leaves 100000 --mode sankoff
line c4t2 --tree sars-like --leaves 8000000 --sites 3750
line c4 --leaves 8000000 --sites 3750
