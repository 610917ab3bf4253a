#!/bin/bash
# A/B of library variants (migym/_lib/var/*.so via MIGYM_LIB) on throughput AND per-launch HBM traffic:
# one bench line plus a FETCH_SIZE and a WRITE_SIZE pass per variant and workload.  Stops at the first failure.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out/vt
for lib in default $(ls isaacgymenvs-ma_amd/migym/_lib/var/*.so 2>/dev/null); do
  name=$(basename "$lib" .so)
  if [ "$lib" = default ]; then unset MIGYM_LIB; else export MIGYM_LIB=$PWD/$lib; fi
  for spec in ${VAR_SPECS:-Humanoid:32768 Ant:65536}; do
    IFS=: read t n o <<< "$spec"; o=${o:-block}
    tag=${name}_${t}_$o
    timeout -k 10 200 python bench.py --task $t --num-envs $n --object-type $o --steps 100 --warmup 10 --no-cpu-baseline \
      > gpurun_out/vt/$tag.json 2> gpurun_out/vt/$tag.err || { echo "$tag bench failed"; tail -3 gpurun_out/vt/$tag.err; exit 1; }
    for c in FETCH_SIZE WRITE_SIZE; do
      timeout -k 10 120 rocprofv3 --pmc $c -d gpurun_out/vt/$tag -o $c --output-format csv -- python bench.py --task $t --num-envs $n --object-type $o --steps 20 --warmup 3 --no-cpu-baseline > gpurun_out/vt/${tag}_$c.log 2>&1 || { echo "$tag $c failed"; exit 1; }
    done
    python tools/pmc_summary.py gpurun_out/vt/$tag "_step<" --json gpurun_out/vt/${tag}_traffic.json > /dev/null
    python -c "import json,sys; d=json.load(open(sys.argv[1])); t=json.load(open(sys.argv[2])); print(f'{sys.argv[3]:36s} {d[\"value\"]/1e6:8.2f} M/s  kernel {d[\"roofline\"][\"kernel_ms\"]:.3f} ms  traffic {t[\"traffic_bytes_per_launch\"]/1e6:7.1f} MB')" gpurun_out/vt/$tag.json gpurun_out/vt/${tag}_traffic.json $tag
  done
done
