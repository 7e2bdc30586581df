#!/bin/bash
# round 4: shifted-lane column fragments (v2: masked edge-lane reads; v2n: same without the residual
# prefetch, timing only) vs the shipped build and its no-residual-prefetch probe (norpf); v2 parity first
set -u
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out; mkdir -p $OUT
cd $R
export IFD_LIB_PATH=$R/tools/abl/libifd_v2.so
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_x3.py tests/test_gpu_blocks.py > $OUT/v2_tests.txt 2>&1
rc=$?; tail -3 $OUT/v2_tests.txt; [ $rc -le 1 ] || exit 1
for rep in 1 2; do
  for v in base v2 norpf v2n; do
    if [ $v = base ]; then unset IFD_LIB_PATH; else export IFD_LIB_PATH=$R/tools/abl/libifd_$v.so; fi
    r=$(QT_N=20 timeout -k 10 120 python tools/quick_time.py 16 3xf16 2>/dev/null | tail -1) || exit 1
    echo "$v $r" | tee -a $OUT/v2.txt
  done
done
