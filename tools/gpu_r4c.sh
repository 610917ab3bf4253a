#!/bin/bash
# Round 4: GPU tests + smoke (gpu_r4a.sh), then the phase-timing split of the ABA for the team instances.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out/phase
bash tools/gpu_r4a.sh || exit $?
for spec in Humanoid:32768 Ant:65536 ShadowHand:16384; do
  IFS=: read t n <<< "$spec"
  timeout -k 10 200 python -u tools/phase_timing.py --task $t --num-envs $n --steps 20 --warmup 5 \
    > gpurun_out/phase/${t}_$n.txt 2>&1 || { echo "phase $t rc=$?"; tail -5 gpurun_out/phase/${t}_$n.txt; exit 1; }
  cat gpurun_out/phase/${t}_$n.txt | tail -20
done
# same-box A/B of the variant libraries (migym/_lib/var/*.so) against the default build
VAR_SPECS="Humanoid:32768 ShadowHand:16384 Ant:65536" STEPS=${STEPS:-200} bash tools/gpu_variants.sh
