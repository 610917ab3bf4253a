#!/bin/bash
# Bench lines for every BASELINE config that fits one GPU (per-GPU shard sizes for the 8-GPU ones).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out/bench
for spec in "Ant 65536" "Ant 16384" "Humanoid 32768" "MAAnt 8192" "ShadowHand 16384" "ShadowHand 4096" "Cartpole 256" \
            "ShadowHand 16384 egg" "ShadowHand 16384 pen"; do
  set -- $spec
  obj=${3:-block}; tag=$1_$2; [ "$obj" != block ] && tag=$1_$2_$obj
  steps=100; [ "$1" = Cartpole ] && steps=1000   # BASELINE.json configs[0]: 1000 steps
  echo "== bench $1 $2 $obj"
  timeout -k 10 400 python bench.py --task $1 --num-envs $2 --object-type $obj --steps $steps --warmup 10 --cpu-seconds 10 > gpurun_out/bench/$tag.json 2> gpurun_out/bench/$tag.err
  rc=$?; echo "rc=$rc"; cat gpurun_out/bench/$tag.json
  if [ $rc -ne 0 ]; then tail -5 gpurun_out/bench/$tag.err; exit $rc; fi
done
