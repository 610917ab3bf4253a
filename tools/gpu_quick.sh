#!/bin/bash
# Parity tests + a few bench lines (one GPU call): stops at the first fault/timeout.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out/bench
timeout -k 10 600 python -m pytest tests -m gpu -q -p no:cacheprovider > gpurun_out/pytest_gpu.log 2>&1
rc=$?; tail -15 gpurun_out/pytest_gpu.log; if [ $rc -gt 1 ]; then exit $rc; fi
for spec in ${QUICK_SPECS:-Ant:65536 Humanoid:32768 ShadowHand:16384}; do
  t=${spec%%:*}; n=${spec##*:}
  timeout -k 10 300 python bench.py --task $t --num-envs $n --steps 100 --warmup 10 --no-cpu-baseline > gpurun_out/bench/${t}_${n}.json 2> gpurun_out/bench/${t}_${n}.err
  rc=$?; echo "$t $n rc=$rc"; python -c "import json,sys; d=json.load(open(sys.argv[1])); print(sys.argv[1], round(d['value']/1e6,2), 'M/s', round(d['ms_per_step'],3), 'ms')" gpurun_out/bench/${t}_${n}.json 2>/dev/null
  if [ $rc -ne 0 ]; then tail -5 gpurun_out/bench/${t}_${n}.err; exit $rc; fi
done
