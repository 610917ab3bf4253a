#!/bin/bash
# Round 4: same-box A/B of the variant libraries, then the GPU parity tests against each variant (MIGYM_LIB).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out/var
VAR_SPECS=${VAR_SPECS:-"Humanoid:32768 ShadowHand:16384 Ant:65536 Ant:16384 ShadowHand:4096"} STEPS=${STEPS:-200} \
  timeout -k 10 900 bash tools/gpu_variants.sh || exit $?
for lib in $(ls isaacgymenvs-ma_amd/migym/_lib/var/*.so 2>/dev/null); do
  name=$(basename "$lib" .so)
  MIGYM_LIB=$PWD/$lib timeout -k 10 300 python -u -m pytest tests -m gpu -q -p no:cacheprovider --timeout 120 \
    --timeout-method thread -k "${TESTK:-physics or teacher or fused or dr_}" > gpurun_out/var/tests_$name.log 2>&1
  rc=$?
  echo "$name tests rc=$rc: $(tail -1 gpurun_out/var/tests_$name.log)"
  if [ $rc -gt 1 ]; then exit $rc; fi
done
