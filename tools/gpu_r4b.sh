#!/bin/bash
# Round 4 A/B: wider teams on small shards (MIGYM_MIN_TEAM) and work ordering (MIGYM_ORDER_EVERY), plus the
# parity of the T=64 hand instance and of an ordered run.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out/ab
MIGYM_MIN_TEAM=64 timeout -k 10 300 python -u -m pytest tests/test_gpu_hand.py -q --timeout 240 --timeout-method thread \
  -p no:cacheprovider -k "physics_step or fused_env_step" > gpurun_out/ab/t64_hand_tests.log 2>&1
echo "t64 hand tests rc=$?"; tail -3 gpurun_out/ab/t64_hand_tests.log
MIGYM_ORDER_EVERY=1 timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_hand.py -q --timeout 240 \
  --timeout-method thread -p no:cacheprovider -k "fused_env_step or multi_agent_env_step" > gpurun_out/ab/order_tests.log 2>&1
echo "ordered tests rc=$?"; tail -3 gpurun_out/ab/order_tests.log
for spec in "ShadowHand 4096 0 0" "ShadowHand 4096 64 0" "ShadowHand 16384 0 0" "ShadowHand 16384 64 0" "ShadowHand 16384 0 8" \
            "Ant 16384 0 0" "Ant 16384 32 0" "Ant 16384 0 8" "Ant 65536 0 0" "Ant 65536 0 8" "Ant 65536 0 32" \
            "Humanoid 32768 0 0" "Humanoid 32768 64 0" "Humanoid 32768 0 8" "MAAnt 8192 0 0" "MAAnt 8192 0 8"; do
  set -- $spec
  tag=$1_$2_t$3_o$4
  MIGYM_MIN_TEAM=$3 MIGYM_ORDER_EVERY=$4 timeout -k 10 300 python bench.py --task $1 --num-envs $2 --steps 100 --warmup 10 \
    --no-cpu-baseline > gpurun_out/ab/$tag.json 2> gpurun_out/ab/$tag.err
  rc=$?
  echo "$tag rc=$rc $(python -c "import json,sys; d=json.load(open('gpurun_out/ab/$tag.json')); print(round(d['value']/1e6,2), 'M', d['ms_per_step'])" 2>/dev/null)"
  [ $rc -ne 0 ] && { tail -3 gpurun_out/ab/$tag.err; exit $rc; }
done
exit 0
