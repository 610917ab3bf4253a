#!/bin/bash
# round 4: pose-only FK in the fused locomotion step's outputs (pose) and two-instruction friction bounds in the
# PGS visit (fric, on top of pose) -- GPU suite on the in-tree build (fric), then same-box A/B base / pose / fric
set -o pipefail
mkdir -p gpurun_out/r4l
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread \
  > gpurun_out/r4l/pytest.txt 2>&1 || { echo "pytest rc=$?"; tail -30 gpurun_out/r4l/pytest.txt; exit 1; }
tail -3 gpurun_out/r4l/pytest.txt
for rep in 1 2; do
for spec in "Ant 65536" "Ant 16384" "Humanoid 32768" "MAAnt 8192" "ShadowHand 16384 block" "ShadowHand 4096 block" "ShadowHand 16384 pen"; do
  set -- $spec; obj=${3:-block}
  for v in base pose fric; do
    MIGYM_LIB=$PWD/ab_libs/libmigym_$v.so timeout -k 10 200 python bench.py --task $1 --num-envs $2 --object-type $obj \
      --steps 200 --warmup 20 --no-cpu-baseline > gpurun_out/r4l/b.json 2>/dev/null || { echo "bench $spec $v rc=$?"; exit 1; }
    python -c "import json,sys; d=json.load(open('gpurun_out/r4l/b.json')); print('%-26s %-5s %8.2f M  kernel %.4f ms' % (sys.argv[1], sys.argv[2], d['value']/1e6, d['roofline']['kernel_ms']))" "$1_$2_$obj" $v | tee -a gpurun_out/r4l/ab.txt
  done
done
done
