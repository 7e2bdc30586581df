#!/bin/bash
# SQ counter passes (one --pmc set per pass, kernel-trace off) on the stream conv vs the per-tile conv.
set -u
R=${GRAFT_REPO_ROOT:-$(pwd)}; OUT=$R/gpurun_out; mkdir -p $OUT; cd /tmp && export TMPDIR=/tmp
P1="SQ_VMEM_TA_ADDR_FIFO_FULL SQ_VMEM_TA_CMD_FIFO_FULL SQ_INST_CYCLES_VMEM_RD SQ_INSTS_VMEM_RD SQ_WAIT_INST_ANY SQ_IFETCH"
P2="SQ_LDS_CMD_FIFO_FULL SQ_LDS_DATA_FIFO_FULL SQ_INST_LEVEL_VMEM SQ_INSTS_SALU SQ_ACTIVE_INST_SCA SQ_WAVE_CYCLES"
P3="SQ_INSTS_VALU SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_VMEM SQ_ACTIVE_INST_LDS SQ_WAIT_ANY SQ_BUSY_CYCLES"
i=0
for S in 1 0; do
for P in "$P1" "$P2" "$P3"; do
  i=$((i+1))
  IFD_CONV_STREAM=$S timeout -k 10 300 rocprofv3 --pmc $P --kernel-include-regex conv_ -d $OUT/cs$i -o ctr --output-format csv -- python $R/tools/one_eval.py 16 2 > $OUT/cs$i.log 2>&1 || { echo "pass $i failed rc=$?"; tail -5 $OUT/cs$i.log; exit 1; }
done
done
echo counters done
