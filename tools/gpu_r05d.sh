#!/bin/bash
# r05d: replay parity (deep + shallow + reroot), then C5 replay on both trees x2.
set -o pipefail
cd "$(dirname "$0")/.."
tools/gpu_replay_ab.sh r05d
