#!/bin/bash
# FETCH_SIZE / WRITE_SIZE passes (one counter set per run) of the bench workloads: tools/gpu_traffic.sh <tag>
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
tag=${1:-tr}
mkdir -p gpurun_out/$tag
for spec in ${TR_SPECS:-Ant:65536:block Humanoid:32768:block ShadowHand:16384:block}; do
  IFS=: read t n o <<< "$spec"
  for c in FETCH_SIZE WRITE_SIZE; do
    timeout -k 10 120 rocprofv3 --pmc $c -d gpurun_out/$tag/${t}_${o} -o $c --output-format csv -- python bench.py --task $t --num-envs $n --object-type $o --steps 10 --warmup 2 --no-cpu-baseline > gpurun_out/$tag/${t}_${o}_$c.log 2>&1 || exit 1
  done
  python tools/pmc_summary.py gpurun_out/$tag/${t}_${o} "_step<" --json gpurun_out/$tag/${t}_${o}.json | sed "s/^/$t $o /"
done
