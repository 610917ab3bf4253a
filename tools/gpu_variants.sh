#!/bin/bash
# A/B throughput of library variants (isaacgymenvs-ma_amd/migym/_lib/var/*.so, selected through MIGYM_LIB)
# against the default build, on the bench workloads.  One GPU call; stops at the first failing run.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out/var
SPECS=${VAR_SPECS:-Ant:65536 Humanoid:32768 ShadowHand:16384}
for lib in default $(ls isaacgymenvs-ma_amd/migym/_lib/var/*.so 2>/dev/null); do
  name=$(basename "$lib" .so)
  for spec in $SPECS; do
    IFS=: read t n o <<< "$spec"; o=${o:-block}
    if [ "$lib" = default ]; then unset MIGYM_LIB; else export MIGYM_LIB=$PWD/$lib; fi
    timeout -k 10 200 python bench.py --task $t --num-envs $n --object-type $o --steps ${STEPS:-100} --warmup 10 --no-cpu-baseline \
      > gpurun_out/var/${name}_${t}_$o.json 2> gpurun_out/var/${name}_${t}_$o.err
    rc=$?
    if [ $rc -ne 0 ]; then echo "$name $t rc=$rc"; tail -3 gpurun_out/var/${name}_${t}_$o.err; exit $rc; fi
    python -c "import json,sys; d=json.load(open(sys.argv[1])); print(f'{sys.argv[2]:24s} {sys.argv[3]:10s} {d[\"value\"]/1e6:8.2f} M/s  kernel {d[\"roofline\"][\"kernel_ms\"]:.3f} ms')" gpurun_out/var/${name}_${t}_$o.json $name $t-$o
  done
done
