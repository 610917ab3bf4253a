#!/bin/bash
# Same-box A/B of the default build against the variant libraries (tools/gpu_variants.sh) after the whole GPU
# suite on the default build.  Stops at the first fault / abort / timeout.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out/var
timeout -k 10 600 python -u -m pytest tests -m gpu -q -p no:cacheprovider --timeout 120 --timeout-method thread \
  ${PYTEST_ARGS:-} > gpurun_out/var/tests_default.log 2>&1
rc=$?
echo "default tests rc=$rc: $(tail -1 gpurun_out/var/tests_default.log)"
grep -E "^FAILED|^ERROR" gpurun_out/var/tests_default.log | head -20
if [ $rc -gt 1 ]; then exit $rc; fi
VAR_SPECS=${VAR_SPECS:-ShadowHand:16384:egg} STEPS=${STEPS:-200} timeout -k 10 900 bash tools/gpu_variants.sh || exit $?
