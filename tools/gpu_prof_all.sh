#!/bin/bash
# Round profiling: rocprofv3 kernel stats of the default bench line, then the four PMC passes of every
# kernel instance the bench lines time (tools/gpu_prof.sh).  Stops at the first failure.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out/prof
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof -o trace --output-format csv -- python bench.py --steps 50 --warmup 5 --no-cpu-baseline > gpurun_out/rocprof_trace.log 2>&1 || exit 1
for spec in "Ant 65536 block" "Humanoid 32768 block" "ShadowHand 16384 block" "ShadowHand 16384 egg" "ShadowHand 16384 pen"; do
  set -- $spec
  bash tools/gpu_prof.sh $1 $2 $3 || exit 1
done
