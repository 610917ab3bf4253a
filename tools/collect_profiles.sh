#!/bin/bash
# Copies one round's GPU results (tools/gpu.sh profile R / lines R, merged back under gpurun_out/R/) into
# profiles/R/: the rocprofv3 kernel stats of the default bench command, the PMC pass CSVs of every kernel instance
# with their summaries and the per-launch traffic JSON bench.py reads, and the bench JSON lines.
#   tools/collect_profiles.sh r05
set -eu
cd "$(dirname "$0")/.."
R=${1:?round}
G=gpurun_out/$R
mkdir -p profiles/$R
if [ -f $G/stats/trace_kernel_stats.csv ]; then
  cp $G/stats/trace_kernel_stats.csv profiles/$R/ant65536_kernel_stats.csv
  cp $G/stats/bench.log profiles/$R/ant65536_bench.log
fi
for d in $G/pmc_*_*_*/; do
  [ -d "$d" ] || continue
  name=$(basename "$d")                       # pmc_<Task>_<n>_<obj>
  set -- $(echo "$name" | tr '_' ' ')         # pmc Task n obj
  task=$2; n=$3; obj=$4
  kern=k_env_step; [ "$task" = ShadowHand ] && kern=k_hand_step
  tag=$task; [ "$obj" != block ] && tag=$task-$obj
  mkdir -p profiles/$R/$name
  cp "$d"pass*_counter_collection.csv profiles/$R/$name/
  python tools/pmc_summary.py "$d" $kern --json profiles/$R/pmc_${tag}_$n.json > profiles/$R/$name/summary.txt
done
if [ -d $G/bench ]; then
  mkdir -p profiles/$R/bench
  cp $G/bench/*.json profiles/$R/bench/
fi
