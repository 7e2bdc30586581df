#!/bin/bash
# round 4: training kernel profile (rocprofv3 stats) of the 3xf16 train bench
set -u
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out; mkdir -p $OUT
cd $R
export TMPDIR=/tmp
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d $OUT/prof_train -o run --output-format csv -- python bench.py --workload train --batch 32 --steps 3 --warmup 1 --fp32-exact-steps 0 --f16-steps 0 > $OUT/prof_train.log 2>&1 || exit $?
f=$(find $OUT/prof_train -name "*kernel_stats.csv" | head -1); cp $f $OUT/train_kernel_stats.csv; echo ok
