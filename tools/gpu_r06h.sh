#!/bin/bash
# full GPU suite, then the cluster A/B on C3 / C4-T2 share / N*
set -o pipefail
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
tag=${1:-r06h}
(while true; do date >> gpurun_out/${tag}_heartbeat.txt; sleep 30; done) &
hb=$!
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 900 --timeout-method thread > gpurun_out/${tag}_gputests.log 2>&1
rc=$?
kill $hb
tail -3 gpurun_out/${tag}_gputests.log
[ $rc -eq 0 ] || { grep -E "Error|assert|FAIL" gpurun_out/${tag}_gputests.log | head -30; exit $rc; }
BIG=1 CLS="0 1" bash tools/gpu_cluster_ab.sh ${tag}ab
