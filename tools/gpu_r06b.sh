# cluster sweeps: GPU parity, then C3 / C4-T2 / N* with the sweeps off and on
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_gpu_cluster.py -x -v --timeout 300 --timeout-method thread > gpurun_out/r06b_tests.log 2>&1
rc=$?
tail -5 gpurun_out/r06b_tests.log
[ $rc -eq 0 ] || { grep -E "Error|assert|FAIL" gpurun_out/r06b_tests.log | head -30; exit $rc; }
for args in "--tree sars-like --leaves 100000" "--tree sars-like --leaves 8000000 --sites 3750" "--leaves 1000000"; do
  for cl in 0 1; do
    tag=$(echo "$args cl$cl" | tr -c 'a-z0-9' '_')
    timeout -k 10 300 python bench.py --no-cpu --with none --steps 10 --warmup 3 $args --cluster $cl > gpurun_out/r06b_$tag.json 2> gpurun_out/r06b_$tag.err || { tail -5 gpurun_out/r06b_$tag.err; exit 3; }
    python3 -c "import json;d=json.load(open('gpurun_out/r06b_$tag.json'));r=d['roofline'];print('$args cl$cl', round(d['ms_per_step'],3), r['kernel'], r['kernel_ms_per_step'], r['launches_per_step'], r['other_kernels_ms_per_step'])"
  done
done
