#!/bin/bash
# Tests after the plain threshold + Sankoff plain kernel + replay double buffer; replay DB A/B;
# then the round's N* Fitch evidence (rocprofv3 stats + FETCH / WRITE / SQ passes)
set -o pipefail
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_gpu_group.py tests/test_gpu_sankoff.py tests/test_gpu_fitch.py tests/test_gpu_narrow.py tests/test_gpu_fullsize.py tests/test_gpu_replay.py -x -q --timeout 120 --timeout-method thread > gpurun_out/gputests_r04i.log 2>&1 || { echo TESTS FAILED; tail -30 gpurun_out/gputests_r04i.log; exit 3; }
tail -1 gpurun_out/gputests_r04i.log
bash tools/replay_variants.sh base nodb base nodb || exit 8
bash tools/profile_fitch.sh r04 || exit 9
cat gpurun_out/prof_r04/traffic.txt | head -20
