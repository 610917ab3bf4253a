#!/bin/bash
# Round 4: phase timing (ABA and collide split) of the team instances, then the same-box A/B of the variants.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out/phase
for spec in Humanoid:32768 Ant:65536 ShadowHand:16384:block ShadowHand:16384:pen ShadowHand:16384:egg; do
  IFS=: read t n o <<< "$spec"; o=${o:-block}
  timeout -k 10 200 python -u tools/phase_timing.py --task $t --num-envs $n --object-type $o --steps 20 --warmup 5 \
    > gpurun_out/phase/${t}_${n}_$o.txt 2>&1 || { echo "phase $t rc=$?"; tail -5 gpurun_out/phase/${t}_${n}_$o.txt; exit 1; }
done
VAR_SPECS=${VAR_SPECS:-"Humanoid:32768 ShadowHand:16384 Ant:65536"} STEPS=${STEPS:-200} timeout -k 10 900 bash tools/gpu_variants.sh
