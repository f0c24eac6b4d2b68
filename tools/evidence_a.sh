#!/bin/bash
# Round evidence, part A (GPU box): N* Fitch rocprofv3 stats + PMC passes -> gpurun_out/prof_TAG
set -o pipefail
cd "$(dirname "$0")/.."
bash tools/profile_fitch.sh $1 || exit 2
