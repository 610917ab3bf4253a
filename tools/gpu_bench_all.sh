#!/bin/bash
# Bench lines for every BASELINE config that fits one GPU (per-GPU shard sizes for the 8-GPU ones).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out/bench
for spec in "Ant 65536" "Ant 16384" "Humanoid 32768" "MAAnt 8192" "ShadowHand 16384" "ShadowHand 4096" "Cartpole 256"; do
  set -- $spec
  echo "== bench $1 $2"
  timeout -k 10 400 python bench.py --task $1 --num-envs $2 --steps 100 --warmup 10 --cpu-seconds 10 > gpurun_out/bench/$1_$2.json 2> gpurun_out/bench/$1_$2.err
  rc=$?; echo "rc=$rc"; cat gpurun_out/bench/$1_$2.json
  if [ $rc -ne 0 ]; then tail -5 gpurun_out/bench/$1_$2.err; exit $rc; fi
done
