#!/bin/bash
# A/B throughput of the variant libraries plus the FETCH_SIZE / WRITE_SIZE passes of each on the egg instance.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out/var
VAR_SPECS=${VAR_SPECS:-ShadowHand:16384:egg} STEPS=${STEPS:-200} timeout -k 10 900 bash tools/gpu_variants.sh || exit $?
for lib in default $(ls isaacgymenvs-ma_amd/migym/_lib/var/*.so 2>/dev/null); do
  name=$(basename "$lib" .so)
  if [ "$lib" = default ]; then unset MIGYM_LIB; else export MIGYM_LIB=$PWD/$lib; fi
  for C in FETCH_SIZE WRITE_SIZE; do
    timeout -s KILL 120 rocprofv3 --pmc $C -d gpurun_out/var/pmc_$name -o $C --output-format csv -- python bench.py --task ShadowHand --num-envs 16384 --object-type egg --steps 10 --warmup 2 --no-cpu-baseline > gpurun_out/var/pmc_${name}_$C.log 2>&1 || exit 1
  done
  python tools/pmc_summary.py gpurun_out/var/pmc_$name k_hand_step --json gpurun_out/var/pmc_$name.json | grep -E "FETCH|WRITE"
  echo "$name $(python -c "import json; print(round(json.load(open('gpurun_out/var/pmc_$name.json'))['traffic_bytes_per_launch']/1e6,1))") MB/launch"
done
