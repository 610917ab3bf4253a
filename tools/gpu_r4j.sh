#!/bin/bash
# small-shard phase timing (round 4): where the single-round grids spend their cycles
set -o pipefail
mkdir -p gpurun_out/phase_small
for spec in "ShadowHand 4096 block" "ShadowHand 16384 block" "Ant 16384 block" "Ant 65536 block"; do
  set -- $spec
  timeout -k 10 200 python -u tools/phase_timing.py --task $1 --num-envs $2 --object-type $3 --steps 20 --warmup 5 \
    > gpurun_out/phase_small/$1_$2_$3.txt 2>&1 || { echo "phase $1 $2 rc=$?"; exit 1; }
done
echo done
