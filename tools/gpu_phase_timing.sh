set -e
mkdir -p gpurun_out/pt
for spec in "Ant 65536 block" "Humanoid 32768 block" "ShadowHand 16384 block" "ShadowHand 16384 egg" "ShadowHand 16384 pen" "MAAnt 8192 block"; do
  set -- $spec
  timeout -k 10 240 python -u tools/phase_timing.py --task $1 --num-envs $2 --object-type $3 > gpurun_out/pt/phase_timing_$1_$2_$3.txt 2>&1
  echo done $spec
done
