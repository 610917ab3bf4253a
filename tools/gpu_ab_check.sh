#!/bin/bash
# One GPU call for a kernel change: the GPU tests selected by PYTEST_K (all of -m gpu by default), then the
# same-box A/B of the default build against the variants under migym/_lib/var/ (tools/gpu_variants.sh).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
timeout -k 10 ${PYTEST_LIMIT:-600} python -u -m pytest tests -m gpu -x -v ${PYTEST_K:+-k "$PYTEST_K"} -p no:cacheprovider \
  --timeout 300 --timeout-method thread > gpurun_out/ab_tests.log 2>&1
rc=$?; tail -3 gpurun_out/ab_tests.log
[ $rc -eq 0 ] || exit $rc
bash tools/gpu_variants.sh
