#!/bin/bash
# Copy one evidence set (tools/round_evidence.sh TAG, merged back into gpurun_out/) into
# profiles/ under the round's names:  tools/collect_evidence.sh TAG
set -euo pipefail
cd "$(dirname "$0")/.."
tag=$1
g=gpurun_out
p=profiles/$tag
cp $g/bench_default_$tag.json ${p}_bench_default.json
for m in fitch sankoff; do
  s=$g/prof_$tag; [ $m = sankoff ] && s=$g/prof_${tag}_sankoff
  cp $s/kernel_stats.csv ${p}_${m}_ns_kernel_stats.csv
  cp $s/stats.json ${p}_${m}_ns_bench_under_rocprof.json
  cp $s/traffic.txt ${p}_${m}_ns_pmc_traffic.txt
  cp $s/sq.txt ${p}_${m}_ns_pmc_sq.txt
done
for t in c3 c3_sankoff c2; do
  cp $g/trace_${tag}_$t/kernel_stats.csv ${p}_${t}_kernel_stats.csv
  cp $g/trace_${tag}_$t.json ${p}_${t}_bench_under_rocprof.json
done
cp $g/prof_replay_$tag/traffic.txt ${p}_replay_pmc_traffic.txt
cp $g/traffic_fitch_$tag.json profiles/traffic_fitch.json
ls ${p}_* | wc -l
