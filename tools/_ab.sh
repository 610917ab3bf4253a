mkdir -p gpurun_out/var
for lib in default isaacgymenvs-ma_amd/migym/_lib/var/*.so; do
  name=$(basename "$lib" .so)
  if [ "$lib" = default ]; then unset MIGYM_LIB; else export MIGYM_LIB=$PWD/$lib; fi
  for o in ${OBJS:-egg}; do
    timeout -k 10 200 python bench.py --task ShadowHand --num-envs 16384 --object-type $o --steps 60 --warmup 5 --no-cpu-baseline > gpurun_out/var/${name}_$o.json 2>/dev/null || exit 1
    python -c "import json,sys; d=json.load(open(sys.argv[1])); print(sys.argv[2], sys.argv[3], round(d['value']/1e6,2))" gpurun_out/var/${name}_$o.json $name $o
  done
done
