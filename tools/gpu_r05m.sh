#!/bin/bash
# r05m: CLI walls with the HIP warm-up thread vs without (PM_CLI_NO_WARMUP=1)
set -o pipefail
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
show() { python3 -c "
import json,sys;d=json.load(open(sys.argv[1]))
for r in d['commands']['runs']:
    p=r.get('gpu_cli_phases_s',{})
    print(sys.argv[2], r['command'][14:58], r.get('workload','')[:16], 'cli', r.get('gpu_cli_wall_s'), 'oracle', r.get('oracle_driver_s'), 'x', r.get('speedup_cli'), 'total', p.get('cli.total'), 'warm', p.get('hip.warmup'), 'ctx', p.get('hip.create_context'), 'up', p.get('msa.upload'), p.get('tree.device upload'), 'fetch', p.get('msa.fetch_records'))
" "$1" "$2"; }
for rep in 1 2; do
  timeout -k 10 600 python bench.py --no-cpu --with commands --steps 2 --warmup 1 > gpurun_out/cli_warm.json 2> gpurun_out/cli_warm.err || { tail -5 gpurun_out/cli_warm.err; exit 2; }
  show gpurun_out/cli_warm.json warm
  PM_CLI_NO_WARMUP=1 timeout -k 10 600 python bench.py --no-cpu --with commands --steps 2 --warmup 1 > gpurun_out/cli_nowarm.json 2> gpurun_out/cli_nowarm.err || { tail -5 gpurun_out/cli_nowarm.err; exit 2; }
  show gpurun_out/cli_nowarm.json nowarm
done
