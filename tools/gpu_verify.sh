#!/bin/bash
# Round verification on one GPU box: the driver's own GPU tiers (pytest -m gpu, smoke, default bench), each
# under its own limit, stopping at the first fault / abort / timeout.  Logs -> gpurun_out/verify/ (copied into
# profiles/r03/ with the HEAD sha by the caller).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
out=gpurun_out/verify; mkdir -p $out
step() {  # name limit cmd...
  local name=$1 to=$2; shift 2
  echo "== $name ($(date +%T))"
  timeout -k 10 "$to" "$@" > "$out/$name.log" 2>&1
  local rc=$?
  echo "== $name rc=$rc ($(date +%T))"; tail -n 6 "$out/$name.log"
  return $rc
}
step pytest_gpu ${PYTEST_LIMIT:-1000} python -u -m pytest tests -m gpu -v -p no:cacheprovider --timeout 300 --timeout-method thread ${PYTEST_ARGS:-}
rc=$?; if [ $rc -gt 1 ]; then exit $rc; fi
step smoke 300 python -u __graft_entry__.py smoke || exit $?
[ "${SKIP_BENCH:-0}" = 1 ] || step bench 400 python -u bench.py || exit $?
exit $rc
