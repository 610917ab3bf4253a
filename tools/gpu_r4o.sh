#!/bin/bash
# round 4: no dof_actuation view bound by the locomotion VecTask (the fused step's effort write-back skipped)
# -- same-box A/B against the bound view (re-enabled by sed on the box copy), bench + FETCH/WRITE pass
set -o pipefail
mkdir -p gpurun_out/r4o
ab() {
  for spec in "Ant 65536" "Humanoid 32768" "MAAnt 8192" "Ant 16384"; do
    set -- $spec
    timeout -k 10 200 python bench.py --task $1 --num-envs $2 --steps 200 --warmup 20 --no-cpu-baseline \
      > gpurun_out/r4o/b.json 2>/dev/null || { echo "bench $spec rc=$?"; exit 1; }
    python -c "import json,sys; d=json.load(open('gpurun_out/r4o/b.json')); print('%-20s %-6s %8.2f M  kernel %.4f ms' % (sys.argv[1], sys.argv[2], d['value']/1e6, d['roofline']['kernel_ms']))" "$1_$2" $v | tee -a gpurun_out/r4o/ab.txt
  done
}
for rep in 1 2; do
  v=nobind; ab
  sed -i 's/        v.dof_actuation, v.sensors = None, _abi.ptr(self.sensor_tensor)/        v.dof_actuation, v.sensors = _abi.ptr(self.dof_actuation), _abi.ptr(self.sensor_tensor)/' isaacgymenvs-ma_amd/migym/tasks/base/vec_task.py
  v=bind; ab
  git checkout -q isaacgymenvs-ma_amd/migym/tasks/base/vec_task.py 2>/dev/null || sed -i 's/        v.dof_actuation, v.sensors = _abi.ptr(self.dof_actuation), _abi.ptr(self.sensor_tensor)/        v.dof_actuation, v.sensors = None, _abi.ptr(self.sensor_tensor)/' isaacgymenvs-ma_amd/migym/tasks/base/vec_task.py
done
grep -c "v.dof_actuation, v.sensors = None" isaacgymenvs-ma_amd/migym/tasks/base/vec_task.py
