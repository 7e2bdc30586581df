#!/bin/bash
# round 6 session j: LDS counters of the split conv kernels (bank conflicts, LDS-array busy, LDS instruction waits)
set -u
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/r06j; mkdir -p $O
cd /tmp && export TMPDIR=/tmp
B="--steps 1 --warmup 0 --ddim-steps 10 --no-profile --cpu-baseline-seconds 0 --fp32-exact-steps 0 --f16-steps 0 --train-steps 0"
timeout -s KILL 300 rocprofv3 --pmc SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INSTS_LDS SQ_WAIT_INST_LDS SQ_VALU_MFMA_BUSY_CYCLES SQ_BUSY_CYCLES SQ_WAVE_CYCLES GRBM_GUI_ACTIVE \
  --kernel-include-regex "conv_x3|skip_x3|conv_head" -d $O/lds -o pmc --output-format csv -- python $R/bench.py $B > $O/lds.log 2>&1 || { echo "lds pass failed rc=$?"; tail -3 $O/lds.log; exit 1; }
echo "lds pass ok"
