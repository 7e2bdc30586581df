#!/bin/bash
# round 6 session g2: kernel traces of the training step with gnb_act off / on
set -u
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/r06g; mkdir -p $O
cd /tmp && export TMPDIR=/tmp
T="--workload train --batch 32 --steps 2 --warmup 1 --fp32-exact-steps 0 --f16-steps 0"
for v in 0 1; do
  IFD_TRAIN_GNB_ACT=$v timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/trace_act$v -o trace --output-format csv -- python $R/bench.py $T > $O/trace_act$v.log 2>&1 || { echo "trace $v failed"; exit 1; }
  echo "trace $v ok"
done
