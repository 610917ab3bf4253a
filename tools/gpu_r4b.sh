#!/bin/bash
# Round 4: wider teams on small shards (MIGYM_MIN_TEAM A/B) + parity of the T=64 hand instance.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out/ab
MIGYM_MIN_TEAM=64 timeout -k 10 300 python -u -m pytest tests/test_gpu_hand.py -q --timeout 240 --timeout-method thread \
  -p no:cacheprovider -k "physics_step or fused_env_step" > gpurun_out/ab/t64_hand_tests.log 2>&1
echo "t64 hand tests rc=$?"; tail -3 gpurun_out/ab/t64_hand_tests.log
for spec in "ShadowHand 4096 0" "ShadowHand 4096 64" "ShadowHand 16384 0" "ShadowHand 16384 64" \
            "Ant 16384 0" "Ant 16384 32" "Ant 65536 0" "Humanoid 32768 0" "Humanoid 32768 64"; do
  set -- $spec
  tag=$1_$2_t$3
  MIGYM_MIN_TEAM=$3 timeout -k 10 300 python bench.py --task $1 --num-envs $2 --steps 100 --warmup 10 --no-cpu-baseline \
    > gpurun_out/ab/$tag.json 2> gpurun_out/ab/$tag.err
  rc=$?
  echo "$tag rc=$rc $(python -c "import json,sys; d=json.load(open('gpurun_out/ab/$tag.json')); print(round(d['value']/1e6,2), 'M', d['ms_per_step'])" 2>/dev/null)"
  [ $rc -ne 0 ] && { tail -3 gpurun_out/ab/$tag.err; exit $rc; }
done
exit 0
