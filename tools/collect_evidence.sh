#!/bin/bash
# Copy one evidence set (tools/round_evidence.sh profile / merge / check TAG, merged back into
# gpurun_out/) into profiles/ under the round's names:  tools/collect_evidence.sh TAG
set -euo pipefail
cd "$(dirname "$0")/.."
tag=$1
g=gpurun_out
p=profiles/$tag
cp $g/bench_default_$tag.json ${p}_bench_default.json
cp $g/gputests_$tag.log ${p}_gputests.log
for w in c3 c3_sankoff c4t2 c4; do
  [ -f $g/bench_${w}_$tag.json ] && cp $g/bench_${w}_$tag.json ${p}_${w}_bench_line.json
done
# PMC profile sets: N* Fitch / Sankoff, C3 Fitch / Sankoff, C4 (T2) rank share
for s in "" _sankoff _c3 _c3_sankoff _c4t2; do
  d=$g/prof_$tag$s; [ -d $d ] || continue
  n=${s#_}; n=${n:-fitch}; [ "$s" = _sankoff ] && n=sankoff
  case $s in ""|_sankoff) n=${n}_ns;; esac
  cp $d/kernel_stats.csv ${p}_${n}_kernel_stats.csv
  cp $d/stats.json ${p}_${n}_bench_under_rocprof.json
  cp $d/traffic.txt ${p}_${n}_pmc_traffic.txt
  cp $d/sq.txt ${p}_${n}_pmc_sq.txt
done
for t in c2 c4; do
  d=$g/trace_${tag}_$t; [ -d $d ] || continue
  cp $d/kernel_stats.csv ${p}_${t}_kernel_stats.csv
  cp $g/trace_${tag}_$t.json ${p}_${t}_bench_under_rocprof.json
done
cp $g/prof_replay_$tag/traffic.txt ${p}_replay_pmc_traffic.txt
ls ${p}_* | wc -l
