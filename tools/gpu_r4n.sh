#!/bin/bash
# round 4: the DOF force's limit impulses from the node's own limit rows (index kept by build_rows) instead of a
# scan over every limit row -- GPU suite on the in-tree build, then same-box A/B base / lrow
set -o pipefail
mkdir -p gpurun_out/r4n
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread \
  > gpurun_out/r4n/pytest.txt 2>&1 || { echo "pytest rc=$?"; tail -30 gpurun_out/r4n/pytest.txt; exit 1; }
tail -3 gpurun_out/r4n/pytest.txt
for rep in 1 2; do
for spec in "Humanoid 32768" "ShadowHand 16384 block" "ShadowHand 4096 block" "ShadowHand 16384 pen"; do
  set -- $spec; obj=${3:-block}
  for v in base lrow; do
    MIGYM_LIB=$PWD/ab_libs/libmigym_$v.so timeout -k 10 200 python bench.py --task $1 --num-envs $2 --object-type $obj \
      --steps 200 --warmup 20 --no-cpu-baseline > gpurun_out/r4n/b.json 2>/dev/null || { echo "bench $spec $v rc=$?"; exit 1; }
    python -c "import json,sys; d=json.load(open('gpurun_out/r4n/b.json')); print('%-26s %-5s %8.2f M  kernel %.4f ms' % (sys.argv[1], sys.argv[2], d['value']/1e6, d['roofline']['kernel_ms']))" "$1_$2_$obj" $v | tee -a gpurun_out/r4n/ab.txt
  done
done
done
