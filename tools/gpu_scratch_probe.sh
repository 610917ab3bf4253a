set -u
cd "${GRAFT_REPO_ROOT}"
for envs in "" "HSA_NO_SCRATCH_THREAD_LIMITER=1" "HSA_SCRATCH_SINGLE_LIMIT=4294967296"; do
  for lib in default base; do
    if [ $lib = default ]; then unset MIGYM_LIB; else export MIGYM_LIB=$PWD/isaacgymenvs-ma_amd/migym/_lib/var/$lib.so; fi
    r=$(env $envs timeout -k 10 120 python bench.py --task ShadowHand --num-envs 16384 --steps 200 --warmup 10 --no-cpu-baseline 2>/dev/null | python -c "import json,sys; d=json.loads(sys.stdin.read()); print(round(d['value']/1e6,2))")
    echo "[$envs] $lib block $r"
  done
done
