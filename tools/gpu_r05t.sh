#!/bin/bash
# r05t: record shards partitioned by XCD A/B
set -o pipefail
cd "$(dirname "$0")/.."
tools/ab_variants.sh fitch 2 default xcdshard && tools/ab_variants.sh sankoff 1 default xcdshard
