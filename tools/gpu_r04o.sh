#!/bin/bash
# Replay tile size / tiles per workgroup / double buffer (compile-time variants, C5)
set -o pipefail
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
bash tools/replay_variants.sh base t8k t8kdb t8kdbg8 g16 g4 base t8k t8kdb t8kdbg8 g16 g4 || exit 2
