set -o pipefail
timeout -k 10 300 python -u -m pytest tests/test_gpu_replay_deep.py tests/test_gpu_replay.py tests/test_gpu_reroot.py -x -q --timeout 120 --timeout-method thread > gpurun_out/rv_tests.log 2>&1 || { echo "REPLAY TESTS FAILED"; tail -40 gpurun_out/rv_tests.log; exit 1; }
tail -1 gpurun_out/rv_tests.log
tools/replay_variants.sh base dfsne base dfsne && TREE=sars-like tools/replay_variants.sh base
