#!/bin/bash
# ShadowHand object types on one GPU: the hand GPU tests, then bench lines for block / egg / pen.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out/bench
timeout -k 10 600 python -u -m pytest tests/test_gpu_hand.py -x -v --timeout 120 --timeout-method thread \
  -p no:cacheprovider > gpurun_out/pytest_hand.log 2>&1
rc=$?; tail -n 30 gpurun_out/pytest_hand.log; [ $rc -eq 0 ] || exit $rc
for k in block egg pen; do
  timeout -k 10 300 python bench.py --task ShadowHand --num-envs 16384 --object-type $k --steps 100 --warmup 10 \
    --no-cpu-baseline > gpurun_out/bench/ShadowHand_16384_$k.json 2> gpurun_out/bench/ShadowHand_16384_$k.err
  rc=$?; echo "$k rc=$rc"; python -c "import json;d=json.load(open('gpurun_out/bench/ShadowHand_16384_$k.json'));print('$k', round(d['value']/1e6,2),'M/s')"
  [ $rc -eq 0 ] || exit $rc
done
