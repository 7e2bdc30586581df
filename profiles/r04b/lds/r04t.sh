#!/bin/bash
# round 4: DPP-built middle-column A fragments (dppA: shipped residual prefetch, 12-14 spills; dppB:
# no residual prefetch, timing only; norpf: the shipped consumer without residual prefetch, timing
# only) vs the shipped build; parity tests on dppA first
set -u
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out; mkdir -p $OUT
cd $R
export IFD_LIB_PATH=$R/tools/abl/libifd_dppA.so
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_x3.py tests/test_gpu_blocks.py > $OUT/dpp_tests.txt 2>&1
rc=$?; tail -3 $OUT/dpp_tests.txt; [ $rc -le 1 ] || exit 1
for rep in 1 2; do
  for v in base dppA dppB norpf; do
    if [ $v = base ]; then unset IFD_LIB_PATH; else export IFD_LIB_PATH=$R/tools/abl/libifd_$v.so; fi
    r=$(QT_N=20 timeout -k 10 120 python tools/quick_time.py 16 3xf16 2>/dev/null | tail -1) || exit 1
    echo "$v $r" | tee -a $OUT/dpp.txt
  done
done
for v in base dppA; do
  if [ $v = base ]; then unset IFD_LIB_PATH; else export IFD_LIB_PATH=$R/tools/abl/libifd_$v.so; fi
  timeout -k 10 120 python tools/layer_prof.py 16 3xf16 > $OUT/lp_$v.txt 2>&1 || exit 1
  echo "$v $(tail -1 $OUT/lp_$v.txt) | $(grep 'r256 128+0->128 skip0' $OUT/lp_$v.txt | head -1 | cut -c60-)"
done
