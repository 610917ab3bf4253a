#!/bin/bash
# Copies one GPU session's results (gpurun_out/, from tools/gpu_bench_all.sh, gpu_check.sh prof and
# gpu_prof.sh <task> <n>) into profiles/<round>/: bench JSON lines, the rocprofv3 kernel stats, the PMC
# pass CSVs with their summaries and the per-launch traffic JSON bench.py reads.
set -eu
cd "$(dirname "$0")/.."
R=${1:-r01}
mkdir -p profiles/$R
for f in gpurun_out/bench/*.json; do cp "$f" profiles/$R/; done
cp gpurun_out/prof/trace_kernel_stats.csv profiles/$R/ant65536_kernel_stats.csv
[ -f gpurun_out/rocprof_trace.log ] && cp gpurun_out/rocprof_trace.log profiles/$R/ant65536_bench.log
for spec in "Ant 65536 k_env_step" "Humanoid 32768 k_env_step" "ShadowHand 16384 k_hand_step" "ShadowHand-egg 16384 k_hand_step" "ShadowHand-pen 16384 k_hand_step"; do
  set -- $spec
  [ -d gpurun_out/pmc/$1 ] || continue
  mkdir -p profiles/$R/pmc_$1
  cp gpurun_out/pmc/$1/pass*_counter_collection.csv profiles/$R/pmc_$1/
  python tools/pmc_summary.py gpurun_out/pmc/$1 $3 --json profiles/$R/pmc_$1_$2.json > profiles/$R/pmc_$1/summary.txt
done
