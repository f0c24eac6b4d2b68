#!/bin/bash
set -o pipefail
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
BENCH_ARGS="--tree sars-like --leaves 100000" bash tools/ab_variants.sh fitch 2 default noslots base || exit 4
BENCH_ARGS="--tree sars-like --leaves 100000" bash tools/ab_args.sh 2 "--sub-down 0" "--sub-down 1" || exit 8
bash tools/replay_variants.sh base rp_e4w5 rp_e8w5 rp_e16w4 || exit 6
bash tools/fetch_calibrate.sh || exit 5
(cd /tmp && timeout -k 5 60 rocprofv3 -L > $GRAFT_REPO_ROOT/gpurun_out/rocprof_counters.txt 2>&1) || true
grep -i "TCC_EA0_RD\|TCC_EA_RD\|TCC_BUBBLE\|TCC_REQ" gpurun_out/rocprof_counters.txt | head -40 || true
