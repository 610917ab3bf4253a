set -o pipefail
cd /root/repo
MIGYM_PARITY_REPORT=gpurun_out/parity_r4a.json timeout -k 10 600 python -u -m pytest tests -m gpu -q --timeout 300 --timeout-method thread -p no:cacheprovider > gpurun_out/r4a_gpu.log 2>&1
rc=$?
echo "pytest rc=$rc"
tail -40 gpurun_out/r4a_gpu.log
if [ $rc -eq 0 ] || [ $rc -eq 1 ]; then
  timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/r4a_smoke.log 2>&1; echo "smoke rc=$?"; tail -5 gpurun_out/r4a_smoke.log
fi
