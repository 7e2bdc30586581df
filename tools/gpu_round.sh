#!/bin/bash
# One GPU-box measurement session (round 2): bench line, rocprofv3 kernel-trace stats, PMC passes
# (FETCH_SIZE, WRITE_SIZE, MFMA busy / MOPS + GRBM clock) on the split conv kernels, and the
# FETCH/WRITE calibration micro-kernels. Each GPU step has its own time limit; stops at the first failure.
set -u
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out
TAG=${1:-r02}
STEPS=${STEPS:-5}
mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp
timeout -k 10 500 python $R/bench.py --steps $STEPS --warmup 1 > $OUT/bench_$TAG.json 2> $OUT/bench_$TAG.err || { echo "bench failed rc=$?"; exit 1; }
echo "bench ok"; tail -c 600 $OUT/bench_$TAG.json
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d $OUT/prof_$TAG -o trace --output-format csv -- \
   python $R/bench.py --steps 1 --warmup 1 --cpu-baseline-seconds 0 --fp32-exact-steps 0 --train-steps 0 > $OUT/prof_$TAG.log 2>&1 || { echo "rocprof trace failed rc=$?"; exit 1; }
echo "trace ok"
BARGS="--steps 1 --warmup 0 --ddim-steps 10 --no-profile --cpu-baseline-seconds 0 --fp32-exact-steps 0 --f16-steps 0 --train-steps 0"
i=0
for P in "FETCH_SIZE" "WRITE_SIZE" "SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_VALU_MFMA_MOPS_F16 SQ_BUSY_CYCLES SQ_WAVE_CYCLES GRBM_GUI_ACTIVE GRBM_COUNT"; do
  i=$((i+1))
  timeout -s KILL 300 rocprofv3 --pmc $P --kernel-include-regex "conv_" -d $OUT/pmc${i}_$TAG -o pmc --output-format csv -- \
     python $R/bench.py $BARGS > $OUT/pmc${i}_$TAG.log 2>&1 || { echo "pmc pass $i failed rc=$?"; tail -3 $OUT/pmc${i}_$TAG.log; exit 1; }
  echo "pmc pass $i ok"
done
for P in FETCH_SIZE WRITE_SIZE; do
  timeout -s KILL 120 rocprofv3 --pmc $P -d $OUT/cal_${P}_$TAG -o cal --output-format csv -- $R/tools/micro/pmc_cal > $OUT/cal_${P}_$TAG.log 2>&1 || { echo "cal $P failed rc=$?"; exit 1; }
done
echo "calibration ok"
