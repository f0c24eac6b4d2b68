#!/bin/bash
# The LDS-staged post-order sweeps on a GPU box: parity (tests/test_gpu_cluster.py), then
# C3 / C4-T2 share / N* with the sweeps off and on (BENCH_ARGS appended), then a kernel trace
# of C3 with the sweeps:  tools/gpu_cluster_ab.sh TAG
set -o pipefail
cd "$(dirname "$0")/.."
tag=$1
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_gpu_cluster.py ${EXTRA_TESTS:-} -x -v --timeout 300 --timeout-method thread > gpurun_out/${tag}_tests.log 2>&1
rc=$?
tail -3 gpurun_out/${tag}_tests.log
[ $rc -eq 0 ] || { grep -E "Error|assert|FAIL" gpurun_out/${tag}_tests.log | head -30; exit $rc; }
for args in "--tree sars-like --leaves 100000" ${BIG:+"--tree sars-like --leaves 8000000 --sites 3750"} "--leaves 1000000"; do
  for cl in ${CLS:-0 1}; do
    t=$(echo "$args cl$cl" | tr -c 'a-z0-9' '_')
    timeout -k 10 300 python bench.py --no-cpu --with none --steps 10 --warmup 3 $args --cluster $cl ${BENCH_ARGS:-} > gpurun_out/${tag}_$t.json 2> gpurun_out/${tag}_$t.err || { tail -5 gpurun_out/${tag}_$t.err; exit 3; }
    python3 -c "import json;d=json.load(open('gpurun_out/${tag}_$t.json'));r=d['roofline'];print('$args cl$cl', round(d['ms_per_step'],3), r['kernel'], r['kernel_ms_per_step'], r['launches_per_step'], r['other_kernels_ms_per_step'])"
  done
done
if [ -n "${TRACE:-}" ]; then
  bash tools/trace_stats.sh ${tag}_c3 --tree sars-like --leaves 100000 --steps 5 --warmup 2 --cluster 1 || exit 4
fi
