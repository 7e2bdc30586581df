#!/bin/bash
# round 4: Gray-ordered MFMA walk (one operand changes per MFMA) vs the shipped order; parity first
set -u
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out; mkdir -p $OUT
cd $R
export IFD_LIB_PATH=$R/tools/abl/libifd_gray.so
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_x3.py tests/test_gpu_blocks.py > $OUT/gray_tests.txt 2>&1
rc=$?; tail -2 $OUT/gray_tests.txt; [ $rc -le 1 ] || exit 1
for rep in 1 2 3; do
  for v in base gray; do
    if [ $v = base ]; then unset IFD_LIB_PATH; else export IFD_LIB_PATH=$R/tools/abl/libifd_$v.so; fi
    r=$(QT_N=20 timeout -k 10 120 python tools/quick_time.py 16 3xf16 2>/dev/null | tail -1) || exit 1
    echo "$v $r" | tee -a $OUT/gray.txt
  done
done
