#!/bin/bash
# GPU parity tests, then bench lines of the main configs (no CPU baseline).  Stops at the first failure.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out/q
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q -p no:cacheprovider --timeout 120 --timeout-method thread > gpurun_out/q/pytest.log 2>&1
rc=$?; tail -3 gpurun_out/q/pytest.log; [ $rc -eq 0 ] || exit $rc
for spec in ${Q_SPECS:-Ant:65536 Humanoid:32768 ShadowHand:16384 ShadowHand:16384:egg MAAnt:8192}; do
  IFS=: read t n o <<< "$spec"; o=${o:-block}
  timeout -k 10 200 python bench.py --task $t --num-envs $n --object-type $o --steps 100 --warmup 10 --no-cpu-baseline > gpurun_out/q/${t}_$o.json 2> gpurun_out/q/${t}_$o.err || { tail -3 gpurun_out/q/${t}_$o.err; exit 1; }
  python -c "import json,sys; d=json.load(open(sys.argv[1])); print(f'{sys.argv[2]:24s} {d[\"value\"]/1e6:8.2f} M/s  kernel {d[\"roofline\"][\"kernel_ms\"]:.3f} ms')" gpurun_out/q/${t}_$o.json $t-$o
done
