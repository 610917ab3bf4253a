#!/bin/bash
# Counter passes for the bench workload (separate --pmc runs, no trace domains).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out/pmc
TASK=${1:-Ant}; NENV=${2:-65536}; OBJ=${3:-block}
ARGS="--task $TASK --num-envs $NENV --object-type $OBJ --steps 20 --warmup 3 --no-cpu-baseline"
TAG=$TASK; [ "$OBJ" != block ] && TAG=$TASK-$OBJ
i=0
for C in "FETCH_SIZE" "WRITE_SIZE" "SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_INSTS_LDS" "SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT SQ_INSTS_SMEM SQ_ACTIVE_INST_VALU SQ_INSTS_BRANCH"; do
  i=$((i+1))
  echo "== pmc pass $i: $C"
  timeout -k 10 300 rocprofv3 --pmc $C -d gpurun_out/pmc/$TAG -o pass$i --output-format csv -- python bench.py $ARGS > gpurun_out/pmc/${TAG}_pass$i.log 2>&1
  rc=$?; echo "rc=$rc"; tail -n 2 gpurun_out/pmc/${TAG}_pass$i.log
  if [ $rc -ne 0 ]; then exit $rc; fi
done
