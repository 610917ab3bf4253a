set -u
export TMPDIR=/tmp
mkdir -p gpurun_out/wq
for v in default kr0; do
  if [ $v = default ]; then unset MIGYM_LIB; else export MIGYM_LIB=$PWD/isaacgymenvs-ma_amd/migym/_lib/var/$v.so; fi
  for T in "Ant 65536" "Humanoid 32768"; do
    set -- $T
    timeout -k 10 120 rocprofv3 --pmc WRITE_SIZE -d gpurun_out/wq/${v}_$1 -o p --output-format csv -- python bench.py --task $1 --num-envs $2 --steps 10 --warmup 2 --no-cpu-baseline > gpurun_out/wq/${v}_$1.log 2>&1 || exit 1
    python tools/pmc_summary.py gpurun_out/wq/${v}_$1 | sed "s/^/$v $1 /"
  done
done
