#!/bin/bash
# r05l: CLI walls -- fast exit + size-dependent xz blocks vs the previous behaviour (env)
set -o pipefail
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
show() { python3 -c "
import json,sys;d=json.load(open(sys.argv[1]))
for r in d['commands']['runs']:
    p=r.get('gpu_cli_phases_s',{})
    print(sys.argv[2], r['command'][:60], r.get('workload','')[:40], 'cli', r.get('gpu_cli_wall_s'), 'oracle', r.get('oracle_driver_s'), 'x', r.get('speedup_cli'), 'total', p.get('cli.total'), 'xz', p.get('panman.xz_encode'), 'ctx', p.get('hip.create_context'))
" "$1" "$2"; }
for rep in 1 2; do
  timeout -k 10 600 python bench.py --no-cpu --with commands --steps 2 --warmup 1 > gpurun_out/cli_new.json 2> gpurun_out/cli_new.err || { tail -5 gpurun_out/cli_new.err; exit 2; }
  show gpurun_out/cli_new.json new
  PM_CLI_FULL_EXIT=1 PM_XZ_BLOCK=1048576 timeout -k 10 600 python bench.py --no-cpu --with commands --steps 2 --warmup 1 > gpurun_out/cli_old.json 2> gpurun_out/cli_old.err || { tail -5 gpurun_out/cli_old.err; exit 2; }
  show gpurun_out/cli_old.json old
  PM_CLI_FULL_EXIT=1 timeout -k 10 600 python bench.py --no-cpu --with commands --steps 2 --warmup 1 > gpurun_out/cli_xzonly.json 2> gpurun_out/cli_xzonly.err || { tail -5 gpurun_out/cli_xzonly.err; exit 2; }
  show gpurun_out/cli_xzonly.json xzonly
done
