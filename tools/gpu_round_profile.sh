#!/bin/bash
# A round's full GPU evidence in one call, self-consistent: rocprof kernel stats + PMC passes per kernel
# instance (tools/gpu_prof_all.sh), their per-launch traffic summaries installed where bench.py reads them
# (profiles/<round>/pmc_*.json, on the box), then the bench lines of every config (tools/gpu_bench_all.sh),
# which therefore cite this build's traffic.  Copy back with tools/collect_profiles.sh <round>.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
R=${1:-r03}
bash tools/gpu_prof_all.sh > gpurun_out/prof_all.log 2>&1 || { tail -5 gpurun_out/prof_all.log; exit 1; }
for spec in "Ant 65536 k_env_step" "Humanoid 32768 k_env_step" "ShadowHand 16384 k_hand_step" \
            "ShadowHand-egg 16384 k_hand_step" "ShadowHand-pen 16384 k_hand_step"; do
  set -- $spec
  python tools/pmc_summary.py gpurun_out/pmc/$1 $3 --json profiles/$R/pmc_$1_$2.json > /dev/null || exit 1
done
bash tools/gpu_bench_all.sh > gpurun_out/bench_all.log 2>&1 || { tail -5 gpurun_out/bench_all.log; exit 1; }
grep -h '"value"' gpurun_out/bench/*.json | python -c "import sys,json; [print(d['config']['workload'][:60], round(d['value']/1e6,2), (d['roofline'].get('traffic_bytes_per_launch') or 0)/1e6) for d in map(json.loads, sys.stdin)]"
