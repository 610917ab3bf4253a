cd "${GRAFT_REPO_ROOT}"
for lib in default egginl head; do
  if [ $lib = default ]; then unset MIGYM_LIB; else export MIGYM_LIB=$PWD/isaacgymenvs-ma_amd/migym/_lib/var/$lib.so; fi
  timeout -k 10 300 python -u -m pytest tests/test_gpu_dr.py tests/test_gpu_hand.py -m gpu -q -k egg -p no:cacheprovider --timeout 200 --timeout-method thread > gpurun_out/eggchk_$lib.log 2>&1
  rc=$?; echo "$lib rc=$rc $(tail -1 gpurun_out/eggchk_$lib.log)"
  if [ $rc -gt 1 ]; then exit $rc; fi
done
