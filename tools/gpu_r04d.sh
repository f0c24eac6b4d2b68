#!/bin/bash
set -o pipefail
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_gpu_fitch.py tests/test_gpu_narrow.py tests/test_gpu_group.py tests/test_gpu_graph.py tests/test_gpu_replay.py tests/test_gpu_reroot.py tests/test_gpu_subdown.py tests/test_gpu_fullsize.py -x -q --timeout 120 --timeout-method thread > gpurun_out/gputests_r04d.log 2>&1 || { echo TESTS FAILED; tail -30 gpurun_out/gputests_r04d.log; exit 3; }
tail -1 gpurun_out/gputests_r04d.log
bash tools/ab_variants.sh fitch 2 default noslots occ3 sub5 sub6 || exit 2
bash tools/ab_args.sh 2 "--sub-down 0" "--sub-down 1" || exit 7
