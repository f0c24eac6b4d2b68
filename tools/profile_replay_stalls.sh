#!/bin/bash
# Why the replay kernel writes at ~3 TB/s (review item 6): PMC passes over the C5 replay bench,
# each its own run (counter limits per pass: 4 TCC, 8 SQ, 2 TA, 2 GRBM):
#   tools/profile_replay_stalls.sh TAG  ->  gpurun_out/replay_stalls_TAG/{tcc,sq,ta}.txt
set -o pipefail
cd "$(dirname "$0")/.."
export TMPDIR=/tmp
out=gpurun_out/replay_stalls_$1
mkdir -p "$out"
pass() {  # NAME COUNTERS...
  local name=$1; shift
  timeout -s KILL 150 rocprofv3 --pmc "$@" --output-format csv -d "$out/$name" -o run -- python3 bench.py --no-cpu --mode replay --steps 2 --warmup 1 \
    > "$out/$name.json" 2> "$out/$name.log" || { echo "pass $name failed"; tail -5 "$out/$name.log"; return 1; }
  python3 tools/pmc_summary.py "$out/$name" | grep -A12 "^k_replay" > "$out/$name.txt" || true
  echo "== $name"; cat "$out/$name.txt"
}
pass tcc TCC_EA0_WRREQ_sum TCC_EA0_WRREQ_STALL_sum TCC_EA0_WRREQ_DRAM_CREDIT_STALL_sum TCC_BUSY_avr || exit 2
pass sq SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_LDS SQ_ACTIVE_INST_LDS SQ_INSTS_LDS SQ_INSTS_VMEM_WR SQ_INSTS_VALU SQ_BUSY_CYCLES || exit 3
pass ta TA_BUSY_avr TA_DATA_STALLED_BY_TC_CYCLES_sum SQ_LDS_BANK_CONFLICT GRBM_GUI_ACTIVE || exit 4
