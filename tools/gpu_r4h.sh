#!/bin/bash
# Round 4: same-box A/B of the variant libraries (throughput), then their GPU parity tests.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
VAR_SPECS=${VAR_SPECS:-"Humanoid:32768 ShadowHand:16384 Ant:65536 Ant:16384"} STEPS=${STEPS:-200} \
  timeout -k 10 900 bash tools/gpu_variants.sh || exit $?
for lib in $(ls isaacgymenvs-ma_amd/migym/_lib/var/*.so 2>/dev/null); do
  name=$(basename "$lib" .so)
  MIGYM_LIB=$PWD/$lib timeout -k 10 300 python -u -m pytest tests -m gpu -q -p no:cacheprovider --timeout 120 \
    --timeout-method thread -k "${TESTK:-physics or teacher or fused}" > gpurun_out/var/tests_$name.log 2>&1
  rc=$?
  echo "$name tests rc=$rc: $(tail -1 gpurun_out/var/tests_$name.log)"
  if [ $rc -gt 1 ]; then exit $rc; fi
done
