#!/bin/bash
# Tests after the branch-free child sets / slots; A/B: branch-free (prebf), slots (noslots), plain split
set -o pipefail
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_gpu_sankoff.py tests/test_gpu_fitch.py tests/test_gpu_group.py tests/test_gpu_narrow.py tests/test_gpu_fullsize.py -x -q --timeout 120 --timeout-method thread > gpurun_out/gputests_r04d2.log 2>&1 || { echo TESTS FAILED; tail -30 gpurun_out/gputests_r04d2.log; exit 3; }
tail -1 gpurun_out/gputests_r04d2.log
bash tools/ab_variants.sh fitch 2 default prebf noslots || exit 12
bash tools/ab_args.sh 2 "--plain-up 0" "--plain-up 1" || exit 11
bash tools/ab_variants.sh sankoff 2 default prebf noslots || exit 9
