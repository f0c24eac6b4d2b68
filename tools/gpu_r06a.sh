set -o pipefail
mkdir -p gpurun_out
(while true; do date >> gpurun_out/r06a_heartbeat.txt; sleep 30; done) &
hb=$!
timeout -k 10 1000 python -u -m pytest tests/test_gpu_replay_deep.py tests/test_gpu_fullsize.py -k "dfs_stack or forced_load or c4shard_t2" -x -v --timeout 900 --timeout-method thread > gpurun_out/r06a_tests.log 2>&1
rc=$?
tail -15 gpurun_out/r06a_tests.log
if [ $rc -eq 0 ]; then
  timeout -k 10 300 python bench.py --no-cpu --with none --tree sars-like --leaves 8000000 --sites 3750 --steps 10 --warmup 3 > gpurun_out/r06a_c4t2.json 2> gpurun_out/r06a_c4t2.err
  rc=$?
  python3 -c "import json;d=json.load(open('gpurun_out/r06a_c4t2.json'));r=d['roofline'];print(d['config']['workload'], round(d['ms_per_step'],3), r['kernel'], r['kernel_ms_per_step'], r['launches_per_step'], r['other_kernels_ms_per_step'])"
fi
kill $hb
exit $rc
