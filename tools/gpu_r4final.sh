#!/bin/bash
# Round 4 final evidence in one call: GPU tests + smoke, rocprofv3 kernel stats + PMC passes (tools/gpu_prof_all.sh),
# then the bench lines of every config (tools/gpu_bench_all.sh) and the phase timing.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
bash tools/gpu_r4a.sh || exit $?
rm -rf gpurun_out/pmc gpurun_out/prof gpurun_out/bench
bash tools/gpu_prof_all.sh > gpurun_out/prof_all.log 2>&1 || { tail -5 gpurun_out/prof_all.log; exit 1; }
# bench lines cite the traffic of this build: install the passes' summaries where bench.py reads them
for spec in "Ant 65536 k_env_step" "Humanoid 32768 k_env_step" "ShadowHand 16384 k_hand_step" \
            "ShadowHand-egg 16384 k_hand_step" "ShadowHand-pen 16384 k_hand_step"; do
  set -- $spec
  python tools/pmc_summary.py gpurun_out/pmc/$1 $3 --json profiles/r04/pmc_$1_$2.json > /dev/null || exit 1
done
bash tools/gpu_bench_all.sh > gpurun_out/bench_all.log 2>&1 || { tail -5 gpurun_out/bench_all.log; exit 1; }
grep -h '"value"' gpurun_out/bench/*.json | python -c "import sys,json; [print(d['config']['workload'][:70], round(d['value']/1e6,2), round(d['roofline']['kernel_ms'],4), d['roofline'].get('traffic_bytes_per_launch')) for d in map(json.loads, sys.stdin)]"
mkdir -p gpurun_out/phase
for spec in Humanoid:32768 Ant:65536 ShadowHand:16384:block ShadowHand:16384:pen ShadowHand:16384:egg; do
  IFS=: read t n o <<< "$spec"; o=${o:-block}
  timeout -k 10 200 python -u tools/phase_timing.py --task $t --num-envs $n --object-type $o --steps 20 --warmup 5 \
    > gpurun_out/phase/${t}_${n}_$o.txt 2>&1 || { echo "phase $t rc=$?"; exit 1; }
done
