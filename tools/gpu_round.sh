#!/bin/bash
# One GPU-box session: bench line, rocprofv3 kernel-trace stats, two PMC passes. Stops at the first failure.
set -u
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out
TAG=${1:-r01}
mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp
timeout -k 10 400 python $R/bench.py > $OUT/bench_$TAG.json 2> $OUT/bench_$TAG.err || { echo "bench failed rc=$?"; exit 1; }
echo "bench ok"
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d $OUT/prof_$TAG -o trace --output-format csv -- \
   python $R/bench.py --steps 1 --warmup 1 --cpu-baseline-seconds 0 --fp32-exact-steps 0 > $OUT/prof_$TAG.log 2>&1 || { echo "rocprof trace failed rc=$?"; exit 1; }
echo "trace ok"
timeout -k 10 400 rocprofv3 --pmc FETCH_SIZE -d $OUT/pmc_fetch_$TAG -o pmc --output-format csv -- \
   python $R/bench.py --steps 1 --warmup 0 --ddim-steps 10 --no-profile --cpu-baseline-seconds 0 --fp32-exact-steps 0 > $OUT/pmc_fetch_$TAG.log 2>&1 || { echo "pmc fetch failed rc=$?"; exit 1; }
echo "pmc fetch ok"
timeout -k 10 400 rocprofv3 --pmc WRITE_SIZE -d $OUT/pmc_write_$TAG -o pmc --output-format csv -- \
   python $R/bench.py --steps 1 --warmup 0 --ddim-steps 10 --no-profile --cpu-baseline-seconds 0 --fp32-exact-steps 0 > $OUT/pmc_write_$TAG.log 2>&1 || { echo "pmc write failed rc=$?"; exit 1; }
echo "pmc write ok"
