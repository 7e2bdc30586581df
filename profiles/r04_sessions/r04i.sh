#!/bin/bash
# round 4: PMC pass over the weight-gradient kernels (MFMA busy, LDS, clocks)
set -u
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out; mkdir -p $OUT
cd $R
export TMPDIR=/tmp
C="SQ_VALU_MFMA_BUSY_CYCLES SQ_BUSY_CYCLES SQ_WAIT_INST_LDS SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE GRBM_GUI_ACTIVE"
IFD_WGRAD_WS=1 timeout -s KILL 120 rocprofv3 --kernel-trace --pmc $C -d $OUT/pmc_ws1 -o run --output-format csv -- python tools/diag/wgrad_time.py > $OUT/pmc_ws1.log 2>&1 || exit $?
IFD_WGRAD_WS=0 timeout -s KILL 120 rocprofv3 --kernel-trace --pmc $C -d $OUT/pmc_ws0 -o run --output-format csv -- python tools/diag/wgrad_time.py > $OUT/pmc_ws0.log 2>&1 || exit $?
IFD_LIB_PATH=$R/tools/abl/libifd_pd3a1.so timeout -s KILL 120 rocprofv3 --kernel-trace --pmc $C -d $OUT/pmc_a1 -o run --output-format csv -- python tools/diag/wgrad_time.py > $OUT/pmc_a1.log 2>&1 || exit $?
echo done
