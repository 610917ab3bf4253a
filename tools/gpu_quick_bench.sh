#!/bin/bash
# Quick throughput check of every config (no CPU baseline), one line each: tools/gpu_quick_bench.sh [tag]
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
tag=${1:-q}
mkdir -p gpurun_out/$tag
for spec in "Ant 65536" "Humanoid 32768" "MAAnt 8192" "ShadowHand 16384" "ShadowHand 16384 egg" "ShadowHand 16384 pen" "Cartpole 256"; do
  set -- $spec
  obj=${3:-block}; t=$1_$2_$obj
  timeout -k 10 300 python bench.py --task $1 --num-envs $2 --object-type $obj --steps 50 --warmup 10 --no-cpu-baseline > gpurun_out/$tag/$t.json 2> gpurun_out/$tag/$t.err
  rc=$?
  python -c "import json,sys;d=json.loads(open('gpurun_out/$tag/$t.json').read().strip().splitlines()[-1]);print('$t', round(d['value']/1e6,2), 'M', d['ms_per_step'])" || { tail -5 gpurun_out/$tag/$t.err; exit $rc; }
done
