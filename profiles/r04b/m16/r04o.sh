#!/bin/bash
# round 4: the 16x16x32 conv_x3 consumer (X3_M16 build, tools/abl/libifd_m16.so): parity tests, then
# same-box interleaved timing against the shipped lib and the dominant layer's profile
set -u
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out; mkdir -p $OUT
cd $R
export IFD_LIB_PATH=$R/tools/abl/libifd_m16.so
timeout -k 10 500 python -u -m pytest -q --timeout 120 --timeout-method thread tests/test_gpu_x3.py tests/test_gpu_full.py tests/test_gpu_blocks.py tests/test_gpu_f16.py tests/test_gpu_parity.py > $OUT/m16_tests.txt 2>&1
rc=$?; tail -8 $OUT/m16_tests.txt; [ $rc -le 1 ] || exit 1
for rep in 1 2; do
  for v in new m16; do
    if [ $v = new ]; then unset IFD_LIB_PATH; else export IFD_LIB_PATH=$R/tools/abl/libifd_$v.so; fi
    r=$(QT_N=20 timeout -k 10 120 python tools/quick_time.py 16 3xf16 2>/dev/null | tail -1) || exit 1
    echo "$v $r" | tee -a $OUT/m16.txt
  done
done
for v in new m16; do
  if [ $v = new ]; then unset IFD_LIB_PATH; else export IFD_LIB_PATH=$R/tools/abl/libifd_$v.so; fi
  timeout -k 10 120 python tools/layer_prof.py 16 3xf16 > $OUT/lp_$v.txt 2>&1 || exit 1
  echo "$v $(tail -1 $OUT/lp_$v.txt) | $(grep 'r256 128+0->128 skip0' $OUT/lp_$v.txt | head -1 | cut -c60-)"
done
