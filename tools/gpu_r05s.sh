#!/bin/bash
# r05s: record shard count (the pre-order's reservation atomic) A/B
set -o pipefail
cd "$(dirname "$0")/.."
tools/ab_variants.sh fitch 2 default sh256 sh4k sh16k && tools/ab_variants.sh sankoff 1 default sh4k sh16k
