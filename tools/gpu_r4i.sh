#!/bin/bash
# Round 4: GPU tests + smoke, then bench lines of the main configs (no CPU leg)
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
bash tools/gpu_r4a.sh || exit $?
mkdir -p gpurun_out/quick
for spec in "Ant 65536" "Ant 16384" "Humanoid 32768" "ShadowHand 16384" "ShadowHand 4096" "MAAnt 8192"; do
  set -- $spec
  timeout -k 10 200 python bench.py --task $1 --num-envs $2 --steps 200 --warmup 10 --no-cpu-baseline > gpurun_out/quick/$1_$2.json 2> gpurun_out/quick/$1_$2.err || exit 1
  python -c "import json,sys; d=json.load(open(sys.argv[1])); print(sys.argv[1], round(d['value']/1e6,2), round(d['roofline']['kernel_ms'],3))" gpurun_out/quick/$1_$2.json
done
