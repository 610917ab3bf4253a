#!/bin/bash
# Rehearsal of the driver's multi-rank bench launch on a one-GPU box: torchrun with N ranks that all share
# cuda:0 (RCCL refuses two ranks on one device, so the collectives go over gloo here).  Exercises bench.py's
# rank setup, the kernel's global env offsets, PackedGather in both modes, the barriers and the max over
# ranks; the RCCL transport itself is only exercised on a multi-GPU node.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
N=${1:-2}
for mode in all root; do
  echo "== torchrun x$N gather=$mode"
  timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node "$N" --master-addr 127.0.0.1 \
    --master-port $((29500 + RANDOM % 1000)) bench.py --gpus "$N" --steps 20 --warmup 5 --backend gloo \
    --gather $mode > gpurun_out/multirank_${N}_$mode.log 2>&1
  rc=$?
  echo "rc=$rc"; tail -n 4 gpurun_out/multirank_${N}_$mode.log
  [ $rc -eq 0 ] || exit $rc
done
