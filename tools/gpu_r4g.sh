#!/bin/bash
# Round 4 final: GPU tests + smoke, the bench lines of every config (tools/gpu_bench_all.sh), phase timing.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
bash tools/gpu_r4a.sh || exit $?
rm -rf gpurun_out/bench
bash tools/gpu_bench_all.sh > gpurun_out/bench_all.log 2>&1 || { tail -5 gpurun_out/bench_all.log; exit 1; }
grep -h '"value"' gpurun_out/bench/*.json | python -c "import sys,json; [print(d['config']['workload'][:60], round(d['value']/1e6,2), d['roofline'].get('kernel_ms')) for d in map(json.loads, sys.stdin)]"
mkdir -p gpurun_out/phase
for spec in Humanoid:32768 Ant:65536 ShadowHand:16384:block ShadowHand:16384:pen ShadowHand:16384:egg; do
  IFS=: read t n o <<< "$spec"; o=${o:-block}
  timeout -k 10 200 python -u tools/phase_timing.py --task $t --num-envs $n --object-type $o --steps 20 --warmup 5 \
    > gpurun_out/phase/${t}_${n}_$o.txt 2>&1 || { echo "phase $t rc=$?"; exit 1; }
done
