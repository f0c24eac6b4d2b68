set -o pipefail
mkdir -p gpurun_out
timeout -k 10 500 python -u -m pytest tests/test_gpu_fitch.py tests/test_gpu_graph.py tests/test_gpu_fullsize.py -x -q --timeout 200 --timeout-method thread > gpurun_out/t_sub.log 2>&1
rc=$?; tail -25 gpurun_out/t_sub.log; echo tests_rc=$rc
[ $rc -eq 0 ] || exit 1
timeout -k 10 200 python bench.py --no-cpu --with none --steps 5 > gpurun_out/b_sub.json 2> gpurun_out/b_sub.err || exit 2
timeout -k 10 200 python bench.py --no-cpu --with none --steps 5 --no-subtree > gpurun_out/b_nosub.json 2> gpurun_out/b_nosub.err || exit 3
python3 - <<'P'
import json
for f in ('gpurun_out/b_sub.json','gpurun_out/b_nosub.json'):
    d=json.load(open(f)); r=d['roofline']
    print(f, 'ms %.3f'%d['ms_per_step'], r['kernel'], 'launch', r['avg_launch_ms'], 'kern', r['kernel_ms_per_step'], r['other_kernels_ms_per_step'], 'design GB %.1f'%(r['step_design_bytes']/1e9), r['step_design_parts'])
P
