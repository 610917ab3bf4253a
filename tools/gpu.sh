#!/bin/bash
# One parametrised driver for every GPU-box job (run it through gpurun; results land under gpurun_out/<OUT>/).
# Library variants for A/Bs are built HERE, on the CPU, beforehand:
#     python isaacgymenvs-ma_amd/build.py --variant NAME -D MACRO[=V] [--flag ...]   -> migym/_lib/var/NAME.so
# and selected on the box through MIGYM_LIB; no step edits tracked source.
#
#   tools/gpu.sh tests [PYTEST ARGS...]         pytest -m gpu (verbose, per-test timeout, stops at the first failure)
#   tools/gpu.sh smoke                          __graft_entry__.smoke()
#   tools/gpu.sh bench OUT SPEC...              bench lines, SPEC = Task:N[:objectType[:steps]] -> OUT/<tag>.json
#   tools/gpu.sh ab OUT REPS "VAR..." SPEC...   same-box A/B: the default library and each prebuilt variant VAR,
#                                               alternating, REPS passes over the SPECs -> OUT/ab.txt
#   tools/gpu.sh stats OUT [BENCH ARGS...]      rocprofv3 --kernel-trace --stats of one bench command
#   tools/gpu.sh pmc OUT Task N [obj] [VAR]     the four separate --pmc passes + tools/pmc_summary.py JSON
#   tools/gpu.sh traffic OUT "VAR..." SPEC      FETCH_SIZE / WRITE_SIZE passes (and a bench line) per variant
#   tools/gpu.sh phase OUT SPEC...              per-phase cycle profile (the --timing build)
#   tools/gpu.sh multirank N                    torchrun x N ranks sharing the one GPU (gloo), both gather modes
#   tools/gpu.sh profile R                      a round's kernel stats and PMC passes per kernel instance
#   tools/gpu.sh lines R                        a round's bench lines of every config
#
# Every GPU step runs under its own timeout and the first failure ends the job (no retries).
set -u
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mode=${1:?mode}; shift

uselib() {  # $1 = default | variant name, either with an optional %MODE suffix (MIGYM_ORDER=off|lists|sort)
  local name=${1%%\%*}
  if [ "$name" != "$1" ]; then export MIGYM_ORDER=${1#*%}; else unset MIGYM_ORDER; fi
  if [ "$name" = default ]; then unset MIGYM_LIB; else export MIGYM_LIB=$PWD/isaacgymenvs-ma_amd/migym/_lib/var/$name.so
    [ -f "$MIGYM_LIB" ] || { echo "no variant library $MIGYM_LIB (build it on the CPU first)"; exit 2; }; fi
}

bench_one() {  # $1 = out file, $2 = SPEC, rest = extra bench args
  local out=$1 spec=$2; shift 2
  IFS=: read -r t n o k <<< "$spec"; o=${o:-block}; k=${k:-200}
  timeout -k 10 400 python bench.py --task "$t" --num-envs "$n" --object-type "$o" --steps "$k" --warmup 20 \
    "$@" > "$out" 2> "${out%.json}.err"
  local rc=$?
  if [ $rc -ne 0 ]; then echo "bench $spec rc=$rc"; tail -5 "${out%.json}.err"; exit $rc; fi
}

summ() {  # one-line summary of a bench JSON: $1 file, $2 label
  python - "$1" "$2" <<'EOF'
import json, sys
d = json.load(open(sys.argv[1]))
r = d["roofline"]
print(f"{sys.argv[2]:34s} {d['value'] / 1e6:9.2f} M env-steps/s  {d['ms_per_step']:.4f} ms/step  kernel {r['kernel_ms']:.4f} ms"
      f"  frac {r['frac']:.4%}")
EOF
}

pmc_passes() {  # $1 dir, $2 task, $3 n, $4 obj
  local i=0
  for C in "FETCH_SIZE" "WRITE_SIZE" \
           "SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_INSTS_LDS" \
           "SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT SQ_INSTS_SMEM SQ_ACTIVE_INST_VALU SQ_INSTS_BRANCH"; do
    i=$((i+1))
    [ "${PMC_PASSES:-4}" -lt $i ] && break
    echo "== pmc pass $i ($2 $3 $4): $C"
    timeout -k 10 300 rocprofv3 --pmc $C -d "$1" -o pass$i --output-format csv -- python bench.py --task "$2" \
      --num-envs "$3" --object-type "$4" --steps 20 --warmup 3 --no-cpu-baseline --no-strong > "$1/pass$i.log" 2>&1
    local rc=$?; echo "rc=$rc"
    [ $rc -eq 0 ] || { tail -3 "$1/pass$i.log"; exit $rc; }
  done
}

case $mode in
  tests)
    mkdir -p gpurun_out
    timeout -k 10 1100 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread "$@" \
      > gpurun_out/gpu_tests.log 2>&1
    rc=$?; tail -n 15 gpurun_out/gpu_tests.log; exit $rc ;;
  smoke)
    timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" ;;
  bench)
    OUT=gpurun_out/${1:?out}; shift; mkdir -p "$OUT"
    for spec in "$@"; do
      tag=$(echo "$spec" | tr ':' '_'); echo "== bench $spec"
      bench_one "$OUT/$tag.json" "$spec" ${BENCH_ARGS:-}
      summ "$OUT/$tag.json" "$spec"
    done ;;
  ab)
    OUT=gpurun_out/${1:?out}; REPS=${2:?reps}; VARS=${3:?variants}; shift 3; mkdir -p "$OUT"
    for rep in $(seq 1 "$REPS"); do
      for v in default $VARS; do
        uselib "$v"
        for spec in "$@"; do
          tag=$(echo "$spec" | tr ':' '_')
          bench_one "$OUT/${v}_$tag.json" "$spec" --no-cpu-baseline --no-strong
          summ "$OUT/${v}_$tag.json" "$v $spec" | tee -a "$OUT/ab.txt"
        done
      done
    done ;;
  stats)
    OUT=gpurun_out/${1:?out}; shift; mkdir -p "$OUT"
    timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$OUT" -o trace --output-format csv -- python bench.py "$@" \
      > "$OUT/bench.log" 2>&1
    rc=$?; tail -n 3 "$OUT/bench.log"; exit $rc ;;
  pmc)
    OUT=gpurun_out/${1:?out}; t=${2:?task}; n=${3:?n}; o=${4:-block}; v=${5:-default}; mkdir -p "$OUT"
    uselib "$v"
    pmc_passes "$OUT" "$t" "$n" "$o"
    kern=k_env_step; [ "$t" = ShadowHand ] && kern=k_hand_step
    tag=$t; [ "$o" != block ] && tag=$t-$o
    python tools/pmc_summary.py "$OUT" $kern --json "$OUT/pmc_${tag}_$n.json" ;;
  traffic)
    OUT=gpurun_out/${1:?out}; VARS=${2:?variants}; spec=${3:?spec}; mkdir -p "$OUT"
    IFS=: read -r t n o k <<< "$spec"; o=${o:-block}
    kern=k_env_step; [ "$t" = ShadowHand ] && kern=k_hand_step
    for v in default $VARS; do
      uselib "$v"; mkdir -p "$OUT/$v"
      bench_one "$OUT/$v/bench.json" "$spec" --no-cpu-baseline --no-strong
      PMC_PASSES=2 pmc_passes "$OUT/$v" "$t" "$n" "$o"
      python tools/pmc_summary.py "$OUT/$v" $kern --json "$OUT/$v/traffic.json" > /dev/null
      summ "$OUT/$v/bench.json" "$v $spec" | tee -a "$OUT/traffic.txt"
      python -c "import json,sys; d=json.load(open(sys.argv[1])); print('   traffic per launch %.1f MB' % (d['traffic_bytes_per_launch'] / 1e6))" \
        "$OUT/$v/traffic.json" | tee -a "$OUT/traffic.txt"
    done ;;
  phase)
    OUT=gpurun_out/${1:?out}; shift; mkdir -p "$OUT"
    for spec in "$@"; do
      IFS=: read -r t n o k <<< "$spec"; o=${o:-block}
      timeout -k 10 240 python -u tools/phase_timing.py --task "$t" --num-envs "$n" --object-type "$o" \
        > "$OUT/phase_timing_${t}_${n}_$o.txt" 2>&1 || { echo "phase $spec failed"; exit 1; }
      echo "done $spec"
    done ;;
  multirank)
    N=${1:-2}; mkdir -p gpurun_out/multirank
    for gm in all root; do
      echo "== torchrun x$N gather=$gm"
      timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node "$N" --master-addr 127.0.0.1 \
        --master-port $((29500 + RANDOM % 1000)) bench.py --gpus "$N" --steps 20 --warmup 5 --backend gloo --steady-steps 0 \
        --gather $gm > gpurun_out/multirank/x${N}_$gm.log 2>&1
      rc=$?; echo "rc=$rc"; tail -n 2 gpurun_out/multirank/x${N}_$gm.log
      [ $rc -eq 0 ] || exit $rc
    done ;;
  profile)   # a round's kernel stats + PMC passes per kernel instance (copy the pmc_*.json into profiles/R after)
    R=${1:?round}; OUT=gpurun_out/$R; mkdir -p "$OUT"
    "$0" stats "$R/stats" --steps 50 --warmup 5 --no-cpu-baseline --no-strong || exit 1
    for spec in "Ant 65536 block" "Humanoid 32768 block" "ShadowHand 16384 block" "ShadowHand 16384 egg" \
                "ShadowHand 16384 pen" "MAAnt 8192 block" "ShadowHand 4096 block"; do
      set -- $spec
      "$0" pmc "$R/pmc_$1_$2_$3" "$1" "$2" "$3" > "$OUT/pmc_$1_$2_$3.log" 2>&1 || { tail -5 "$OUT/pmc_$1_$2_$3.log"; exit 1; }
      tag=$1; [ "$3" != block ] && tag=$1-$3
      mkdir -p "profiles/$R"; cp "$OUT/pmc_$1_$2_$3/pmc_${tag}_$2.json" "profiles/$R/"   # bench lines cite this build
      echo "pmc $spec done"
    done ;;
  lines)     # the round's bench lines of every config (cpu baselines included)
    R=${1:?round}
    BENCH_ARGS="--cpu-seconds 10 --no-strong" "$0" bench "$R/bench" Ant:65536 Ant:32768 Ant:16384 Ant:8192 \
      Humanoid:32768 MAAnt:8192 MAAnt:65536 ShadowHand:16384 ShadowHand:4096 ShadowHand:32768 Cartpole:256::1000 \
      ShadowHand:16384:egg ShadowHand:16384:pen ;;
  *) echo "unknown mode $mode"; exit 2 ;;
esac
