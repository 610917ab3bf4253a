#!/bin/bash
# Egg narrowphase variants (csrc/convex.hpp's note): k_simulate twice on the same states
# (run-to-run difference) and against the fp64 oracle.  Stops at the first failing / timed-out variant.
# The round-3 experiment (before the narrowphase became a real call built without IPRA) used
#   build.py --variant egg_inline_w1 -DMG_WAVES=1                       (inlined, 1-wave blocks)
#   build.py --variant egg_noinline_w1 -DMG_CVX_INLINE=noinline -DMG_WAVES=1   (real call, IPRA on)
#   build.py --variant egg_noinline -DMG_CVX_INLINE=noinline            (real call, IPRA on, 8-wave blocks)
#   build.py --variant egg_noinline_noipra ... --flag=-mllvm --flag=-enable-ipra=false
# with those switches in the sources of that commit; results in profiles/r03/egg_ab/.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out/egg_ab
for v in ${VARIANTS:-default egg_inline_w1 egg_noinline_w1 egg_noinline}; do
  if [ $v = default ]; then unset MIGYM_LIB; else export MIGYM_LIB=$PWD/isaacgymenvs-ma_amd/migym/_lib/var/$v.so; fi
  echo "== $v"
  timeout -k 5 90 python -u tools/egg_diag.py egg > gpurun_out/egg_ab/$v.log 2>&1
  rc=$?
  cat gpurun_out/egg_ab/$v.log | grep -v amdgpu.ids
  echo "== $v rc=$rc"
  [ $rc -eq 0 ] || exit $rc
done
