#!/bin/bash
# Egg instance A/B: throughput (tools/gpu_variants.sh) and FETCH_SIZE / WRITE_SIZE per variant library.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
VAR_SPECS=${VAR_SPECS:-ShadowHand:16384:egg} bash tools/gpu_variants.sh || exit 1
for lib in default $(ls isaacgymenvs-ma_amd/migym/_lib/var/*.so 2>/dev/null); do
  name=$(basename "$lib" .so)
  if [ "$lib" = default ]; then unset MIGYM_LIB; else export MIGYM_LIB=$PWD/$lib; fi
  d=gpurun_out/vtr/$name; mkdir -p $d
  for c in FETCH_SIZE WRITE_SIZE; do
    timeout -k 10 120 rocprofv3 --pmc $c -d $d -o $c --output-format csv -- python bench.py --task ShadowHand --num-envs 16384 --object-type egg --steps 10 --warmup 2 --no-cpu-baseline > $d/$c.log 2>&1 || exit 1
  done
  python tools/pmc_summary.py $d "_step<" --json $d/t.json | sed "s/^/$name /"
done
