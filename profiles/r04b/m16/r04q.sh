#!/bin/bash
# round 4: accuracy of the one-accumulator M16 variant (full-trajectory and per-eval parity tests)
set -u
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out; mkdir -p $OUT
cd $R
export IFD_LIB_PATH=$R/tools/abl/libifd_${V:-m16a}.so
timeout -k 10 500 python -u -m pytest -q --timeout 120 --timeout-method thread tests/test_gpu_x3.py tests/test_gpu_full.py tests/test_gpu_blocks.py tests/test_gpu_f16.py > $OUT/m16q_tests.txt 2>&1
rc=$?; grep -E "c1_full|FAILED|passed|failed" $OUT/m16q_tests.txt | cut -c1-400; [ $rc -le 1 ] || exit 1
