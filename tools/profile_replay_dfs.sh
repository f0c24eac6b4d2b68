#!/bin/bash
# SQ / TCC counters of the replay kernel (k_replay_dfs or k_replay) over the C5 replay bench,
# each pass its own run:  tools/profile_replay_dfs.sh TAG [LIB]  ->  gpurun_out/rdfs_TAG/*.txt
set -o pipefail
cd "$(dirname "$0")/.."
export TMPDIR=/tmp
out=gpurun_out/rdfs_$1
lib=${2:-}
mkdir -p "$out"
pass() {  # NAME COUNTERS...
  local name=$1; shift
  PANMAN_AMD_LIB=$lib timeout -s KILL 150 rocprofv3 --pmc "$@" --output-format csv -d "$out/$name" -o run -- python3 bench.py --no-cpu --mode replay --steps 2 --warmup 1 \
    > "$out/$name.json" 2> "$out/$name.log" || { echo "pass $name failed"; tail -5 "$out/$name.log"; return 1; }
  python3 tools/pmc_summary.py "$out/$name" | grep -A12 "^k_replay" > "$out/$name.txt" || true
  echo "== $name"; cat "$out/$name.txt"
}
pass sq SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VMEM_WR SQ_INSTS_VALU SQ_BUSY_CYCLES SQ_WAVES || exit 3
pass sq2 SQ_INSTS_LDS SQ_INSTS_SALU SQ_INSTS_SMEM SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_WAIT_INST_LDS SQ_INST_CYCLES_VMEM_WR SQ_LDS_BANK_CONFLICT || exit 4
pass tcc TCC_EA0_WRREQ_sum TCC_EA0_WRREQ_STALL_sum TCC_BUSY_avr GRBM_GUI_ACTIVE || exit 5
