#!/bin/bash
# One GPU-box session: parity tests -> smoke -> bench -> rocprof.  Stops at the
# first fault/abort/timeout (exit codes other than 0/1 from pytest).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
STAGE=${1:-all}
run() {  # name timeout cmd...
  local name=$1 to=$2; shift 2
  echo "== $name"
  timeout -k 10 "$to" "$@" > "gpurun_out/$name.log" 2>&1
  local rc=$?
  echo "== $name rc=$rc"
  tail -n 25 "gpurun_out/$name.log"
  return $rc
}
if [ "$STAGE" = all ] || [ "$STAGE" = tests ]; then
  run pytest_gpu 900 python -m pytest tests -m gpu -x -q -p no:cacheprovider
  rc=$?; if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
  run smoke 300 python __graft_entry__.py smoke || exit $?
fi
if [ "$STAGE" = all ] || [ "$STAGE" = bench ]; then
  run bench 600 python bench.py --steps 100 --warmup 10 || exit $?
fi
if [ "$STAGE" = all ] || [ "$STAGE" = prof ]; then
  export TMPDIR=/tmp
  run rocprof_trace 600 rocprofv3 --kernel-trace --stats -d gpurun_out/prof -o trace --output-format csv -- python bench.py --steps 50 --warmup 5 --no-cpu-baseline || exit $?
fi
