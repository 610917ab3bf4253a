#!/bin/bash
# Round 4: GPU tests + smoke (gpu_r4a.sh), then the same-box A/B of the variant libraries.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
bash tools/gpu_r4a.sh || exit $?
VAR_SPECS=${VAR_SPECS:-"Humanoid:32768 ShadowHand:16384 ShadowHand:16384:egg ShadowHand:16384:pen Ant:65536"} STEPS=${STEPS:-200} \
  timeout -k 10 900 bash tools/gpu_variants.sh
